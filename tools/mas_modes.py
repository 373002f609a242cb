"""A/B helper for the MAS kernel variants (GT_MAS_MODE bits, csrc/mas.hip): mismatches vs the golden paths
and the C oracle on random / tie-heavy grids. usage: GT_MAS_MODE=<m> python tools/mas_modes.py"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "grad-tts_amd"), os.path.join(REPO, "tests")]
from conftest import load_golden  # noqa: E402
from gradtts_amd.monotonic_align import maximum_path  # noqa: E402

bad = []
for n in ["mas_random.npz", "mas_ties.npz", "mas_logprior.npz"]:
    g = load_golden(n)
    p = maximum_path(torch.from_numpy(g["value"]).cuda(), torch.from_numpy(g["mask"]).cuda()).cpu().numpy()
    d = (p.astype(np.int8) != g["path"])
    bad.append((n, int(d.sum()), [int(x) for x in np.nonzero(d.any(axis=(1, 2)))[0]]))
print(os.environ.get("GT_MAS_MODE"), bad)
