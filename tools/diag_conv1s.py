"""conv1s vs conv_kernel at a bench-sized batch: per-stage mismatch fraction and non-finite counts (GPU box).
usage: python tools/diag_conv1s.py [B T]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "grad-tts_amd"))
from gpu_util import make_decoder, probe  # noqa: E402
from gradtts_amd import _lib  # noqa: E402
from gradtts_amd.params import synthetic_inputs  # noqa: E402

B, T = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (32, 512)
STAGES = [("downs.1.0", 128, 40), ("downs.1.2", 128, 40), ("downs.2.0", 256, 20), ("downs.2.2", 256, 20),
          ("mid_attn", 256, 20), ("ups.0.0", 128, 20), ("ups.0.2", 128, 20), ("ups.1.0", 64, 40)]
mu, z, mask, _ = synthetic_inputs(5, B, T)
cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
args = (cu(z), cu(mask), cu(mu), cu(np.linspace(0.9, 0.1, B).astype(np.float32)), None)
res = {}
for c1s in (1, 0):
    os.environ["GT_CONV1S"] = str(c1s)
    dec, _ = make_decoder(1, 3, torch.bfloat16)
    _lib.check(_lib.lib().gt_decoder_set_small_batch(dec.estimator._native(), 0), "small")
    out = {"estimator": dec.estimator(*args).cpu().numpy()}
    for st, C, F in STAGES:
        _, pr = probe(dec.estimator, torch.bfloat16, *args, st, (B, C, F, T // 2 if F == 40 else T // 4))
        out[st] = pr.cpu().numpy()
    res[c1s] = out
for k in res[1]:
    a, b = res[1][k], res[0][k]
    bad = ~np.isfinite(a)
    print(f"{k:12s} mismatch {np.mean(a != b):.3e} nonfinite(c1s) {int(bad.sum())} nonfinite(ref) {int((~np.isfinite(b)).sum())}")
    if bad.any():
        idx = np.argwhere(bad)
        print("   first non-finite (b, c, f, t):", idx[:5].tolist(), " utterances:", np.unique(idx[:, 0]).tolist()[:10])
    elif np.any(a != b):
        idx = np.argwhere(a != b)
        print("   first mismatches (b, c, f, t):", idx[:5].tolist(), " utterances:", np.unique(idx[:, 0]).tolist()[:10])
