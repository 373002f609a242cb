#!/usr/bin/env python3
"""Record the state_dict layout of the reference's full GradTTS model (build container only).

The reference saves checkpoints as ``torch.save(model.state_dict(), f"{log_dir}/grad_{epoch}.pt")``
(/root/reference/train.py:174-175) and loads them with ``generator.load_state_dict(torch.load(path))``
(/root/reference/inference.py:66). This script instantiates the unmodified reference ``model.tts.GradTTS``
with the configuration of /root/reference/params.py (n_vocab = len(symbols) + 1 = 149; n_spks 1, 247, -1)
and writes every key's shape, in order, to tests/golden/gradtts_layout.json -- the data the checkpoint tests
use to build reference-layout checkpoints without the reference.

Usage:  make -C oracle ref && PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_gradtts_layout.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402


def main():
    mg.import_reference()
    import model.tts as tts  # noqa: E402  (GradTTS: tts.py:20-52)
    out = {}
    for n_spks in (1, 247, -1):
        m = tts.GradTTS(149, n_spks, 64, 192, 768, 256, 2, 6, 3, 0.1, 4, 80, 64, 0.05, 20.0, 1000)
        out[str(n_spks)] = [[k, list(v.shape)] for k, v in m.state_dict().items()]
        dec = [k for k, _ in out[str(n_spks)] if k.startswith("decoder.")]
        print(f"n_spks={n_spks}: {len(out[str(n_spks)])} keys, {len(dec)} decoder keys")
    with open(os.path.join(HERE, "gradtts_layout.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
