#!/usr/bin/env python3
"""Golden fixtures for the text-encoder front-end of GradTTS.forward, produced by running the
REAL reference in the build container (fixtures are data: inputs + expected outputs; the reference does not travel).

* ``model.text_encoder.TextEncoder`` (/root/reference/model/text_encoder.py:285-335) with GradTTS's configuration
  (params.py: 149 symbols, 192 channels, 768 filter, 256 duration-predictor filter, 2 heads, 6 layers, kernel 3,
  window 4; speaker-agnostic as GradTTS builds it, tts.py:49-51), eval mode (dropout off), synthetic weights
  (``gradtts_amd.params.synthetic_text_encoder_state_dict``; the seed and a SHA-256 are stored), float32 and float64.
* The front-end of ``GradTTS.forward`` after the encoder (tts.py:86-101): durations, ``y_lengths``,
  ``fix_len_compatibility``, ``generate_path`` (utils.py:26-39) and ``mu_y``, with the reference's own utils, at
  length_scale 1.0 and 1.25.

Usage:  make -C oracle ref && PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_tts.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402
from gradtts_amd.params import state_dict_sha256, synthetic_text_encoder_state_dict  # noqa: E402

SEED = 5


def main():
    mg.import_reference()
    import model.text_encoder as te  # noqa: E402
    import model.utils as mu  # noqa: E402
    sd = synthetic_text_encoder_state_dict(SEED)
    sha = state_dict_sha256(sd)
    cases = [("te_B3_T37", [37, 25, 11], 37, 101), ("te_B2_T130", [130, 97], 130, 102)]
    for name, lengths, Tx, seed in cases:
        rng = np.random.default_rng(seed)
        B = len(lengths)
        tokens = rng.integers(0, 149, size=(B, Tx)).astype(np.int64)
        x_lengths = np.array(lengths, dtype=np.int64)
        out = {"tokens": tokens, "x_lengths": x_lengths, "weights_seed": np.array(SEED), "weights_sha256": np.array(sha)}
        for tag, dt in (("f32", torch.float32), ("f64", torch.float64)):
            enc = te.TextEncoder(149, 80, 192, 768, 256, 2, 6, 3, 0.1, 4).to(dt).eval()
            enc.load_state_dict({k: torch.from_numpy(v).to(dt) for k, v in sd.items()}, strict=True)
            with torch.no_grad():
                mu_x, logw, x_mask = enc(torch.from_numpy(tokens), torch.from_numpy(x_lengths))
            out[f"mu_x_{tag}"] = mu_x.numpy()
            out[f"logw_{tag}"] = logw.numpy()
            out[f"x_mask_{tag}"] = x_mask.numpy()
            if tag == "f32":
                for ls in (1.0, 1.25):
                    # tts.py:86-101, verbatim order of operations with the reference's utils
                    w = torch.exp(logw) * x_mask
                    w_ceil = torch.ceil(w) * ls
                    y_lengths = torch.clamp_min(torch.sum(w_ceil, [1, 2]), 1).long()
                    y_max_length = int(y_lengths.max())
                    y_max_length_ = mu.fix_len_compatibility(y_max_length)
                    y_mask = mu.sequence_mask(y_lengths, y_max_length_).unsqueeze(1).to(x_mask.dtype)
                    attn_mask = x_mask.unsqueeze(-1) * y_mask.unsqueeze(2)
                    attn = mu.generate_path(w_ceil.squeeze(1), attn_mask.squeeze(1)).unsqueeze(1)
                    mu_y = torch.matmul(attn.squeeze(1).transpose(1, 2), mu_x.transpose(1, 2)).transpose(1, 2)
                    k = f"ls{int(ls * 100)}"
                    out[f"{k}_w"] = w.numpy()
                    out[f"{k}_w_ceil"] = w_ceil.numpy()
                    out[f"{k}_y_lengths"] = y_lengths.numpy()
                    out[f"{k}_y_max_length"] = np.array(y_max_length)
                    out[f"{k}_y_mask"] = y_mask.numpy()
                    out[f"{k}_attn"] = attn.numpy().astype(np.uint8)
                    out[f"{k}_mu_y"] = mu_y.numpy()
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        print(name, {k: v.shape for k, v in out.items() if hasattr(v, "shape")})


if __name__ == "__main__":
    main()
