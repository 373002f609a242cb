"""Locate differences between the fused (conv64 IN_X0) and unfused input-conv paths: per-stage error maps over
(mel row, frame) . Usage (GPU box): python tools/diag_x0.py [B T small]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "grad-tts_amd"))
from gpu_util import make_decoder, probe  # noqa: E402
from gradtts_amd import _lib  # noqa: E402
from gradtts_amd.params import synthetic_inputs  # noqa: E402

B, T, small = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (3, 132, 0)
mu, z, mask, _ = synthetic_inputs(41, B, T, lengths=[T - 7 * i for i in range(B)])
t = np.linspace(0.9, 0.2, B).astype(np.float32)
cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
args = (cu(z), cu(mask), cu(mu), cu(t), None)
res = {}
for fuse in (1, 0):
    os.environ["GT_X0_FUSE"] = str(fuse)
    dec, _ = make_decoder(1, 23, torch.bfloat16)
    _lib.check(_lib.lib().gt_decoder_set_small_batch(dec.estimator._native(), 16 if small else 0), "small")
    out = {}
    for st in ("downs.0.0.pre1", "downs.0.0.pre2"):
        _, pr = probe(dec.estimator, torch.bfloat16, *args, st, (B, 64, 80, T))
        out[st] = pr.cpu().numpy()
    res[fuse] = out
for st in ("downs.0.0.pre1", "downs.0.0.pre2"):
    a, b = res[1][st], res[0][st]
    d = np.abs(a - b).max(axis=1)   # [B, F, T]
    scale = np.abs(b).max()
    print(f"{st}: max rel {d.max() / scale:.3e}")
    bad = d > 1e-2 * scale
    if bad.any():
        bb, ff, tt = np.nonzero(bad)
        print("  bad count", bad.sum(), "of", bad.size)
        print("  rows f%4 hist", np.bincount(ff % 4, minlength=4), "f hist (first 12)", np.bincount(ff, minlength=80)[:12])
        print("  frames t%32 hist", np.bincount(tt % 32, minlength=32))
        print("  utterance hist", np.bincount(bb, minlength=B))
        print("  first bad (b, f, t):", list(zip(bb[:10], ff[:10], tt[:10])))
