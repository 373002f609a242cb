#!/usr/bin/env python3
"""Record the REFERENCE's own bf16 error envelope on the golden fixtures (build container only).

For every estimator / sampler fixture, the unmodified reference (/root/reference/model/diffusion.py, imported as
make_golden.py does) is run under ``torch.autocast("cpu", dtype=torch.bfloat16)`` on the fixture's inputs and
weights, and its max|y_bf16 - y_f32| / max|y_f32| against the fixture's fp32 output is written to
tests/golden/ref_bf16_envelope.json. The GPU tests gate the HIP bf16 path against this envelope: a bf16 decoder
is held to the accuracy the reference itself reaches in bf16, not to an arbitrary constant.

Usage:  make -C oracle ref && PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_bf16_envelope.py
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402

EST = ["estimator_s1.npz", "estimator_s247.npz", "estimator_sm1.npz", "estimator_s1_T132.npz", "estimator_s1_T20.npz"]
REV = ["reverse_s1_N10.npz", "reverse_s247_N10.npz", "reverse_s1_N50.npz"]


def load(name):
    with np.load(os.path.join(HERE, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def rel(a, b):
    return float(np.max(np.abs(a.astype(np.float64) - b)) / np.max(np.abs(b)))


def main():
    diffusion, _ = mg.import_reference()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    out = {}
    for name in EST + REV:
        g = load(name)
        n_spks = int(g["n_spks"])
        dec, _ = mg.build_reference_decoder(diffusion, n_spks, int(g["seed_w"]), torch.float32)
        spk = torch.from_numpy(g["spk"]) if n_spks != 1 else None
        with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
            if name.startswith("estimator"):
                y = dec.estimator(*(torch.from_numpy(g[k]) for k in ("x", "mask", "mu", "t")), spk)
            else:
                y = dec(torch.from_numpy(g["z"]), torch.from_numpy(g["mask"]), torch.from_numpy(g["mu"]),
                        int(g["n_timesteps"]), False, spk)
        out[name] = {"ref_bf16_vs_f32": rel(y.float().numpy(), g["out"]),
                     "ref_f32_vs_f64": rel(g["out"], g["out_f64"]) if g["out_f64"].size else None}
        print(name, out[name])
    with open(os.path.join(HERE, "ref_bf16_envelope.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
