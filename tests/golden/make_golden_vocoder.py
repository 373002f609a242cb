#!/usr/bin/env python3
"""Golden fixtures for the HiFi-GAN generator (the vocoder consuming the decoder's mel), produced by
running the REAL reference in the build container: /root/reference/hifi-gan/models.py ``Generator`` (:77-128) with
the configuration of checkpts/hifigan-config.json (V1), synthetic weights (``synthetic_vocoder_state_dict``; seed
and SHA-256 stored) loaded as weight_g / weight_v / bias, ``remove_weight_norm()`` as inference.py:76 does, eval,
float32 and float64. Also records the state_dict layout (keys + shapes) of the reference Generator. A second set
(voc3_*) runs the same reference Generator with the HiFi-GAN V3 configuration (resblock '2': ResBlock2,
models.py:53-74), which the reference code supports although its checkpts ship only the V1 config.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_vocoder.py
"""
import importlib.util
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("GRADTTS_REFERENCE", "/root/reference")
sys.path.insert(0, os.path.join(REPO, "grad-tts_amd"))
from gradtts_amd.params import HIFIGAN_V1, HIFIGAN_V3, state_dict_sha256, synthetic_vocoder_state_dict  # noqa: E402

sys.dont_write_bytecode = True
SEED = 7


def load_reference():
    sys.path.insert(0, os.path.join(REF, "hifi-gan"))
    spec = importlib.util.spec_from_file_location("ref_hifigan_models", os.path.join(REF, "hifi-gan", "models.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    from env import AttrDict  # noqa: E402  (hifi-gan/env.py)
    with open(os.path.join(REF, "checkpts", "hifigan-config.json")) as f:
        h = AttrDict(json.load(f))
    return mod, h


def main():
    mod, h = load_reference()
    for k in HIFIGAN_V1:
        assert h[k] == HIFIGAN_V1[k], k
    sd = synthetic_vocoder_state_dict(SEED)
    layout = [[k, list(v.shape)] for k, v in mod.Generator(h).state_dict().items()]
    assert [k for k, _ in layout] == list(sd), "synthetic layout != reference Generator layout"
    assert all(list(sd[k].shape) == s for k, s in layout)
    with open(os.path.join(HERE, "hifigan_layout.json"), "w") as f:
        json.dump(layout, f)
    from env import AttrDict  # noqa: E402  (hifi-gan/env.py)
    h3 = AttrDict(dict(HIFIGAN_V3))
    sd3 = synthetic_vocoder_state_dict(SEED, HIFIGAN_V3)
    assert list(mod.Generator(h3).state_dict()) == list(sd3), "synthetic V3 layout != reference Generator layout"
    for name, B, T, seed, hh, sdd in (("voc_B2_T6", 2, 6, 11, h, sd), ("voc_B1_T13", 1, 13, 12, h, sd),
                                      ("voc3_B2_T7", 2, 7, 13, h3, sd3)):
        rng = np.random.default_rng(seed)
        mel = (rng.standard_normal((B, 80, T)) * 2.0 - 5.0).astype(np.float32)   # log-mel-like range
        out = {"mel": mel, "weights_seed": np.array(SEED), "weights_sha256": np.array(state_dict_sha256(sdd))}
        for tag, dt in (("f32", torch.float32), ("f64", torch.float64)):
            g = mod.Generator(hh)
            g.load_state_dict({k: torch.from_numpy(v) for k, v in sdd.items()}, strict=True)
            g = g.to(dt).eval()
            g.remove_weight_norm()
            with torch.no_grad():
                out[f"audio_{tag}"] = g(torch.from_numpy(mel).to(dt)).numpy()
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        print(name, out["audio_f32"].shape, float(np.abs(out["audio_f32"] - out["audio_f64"]).max()))


if __name__ == "__main__":
    main()
