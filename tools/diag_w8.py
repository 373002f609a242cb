"""Error distribution of one estimator call (W8 or bf16) vs the oracle on a golden fixture, for the library
named by GRADTTS_LIB (same-box comparison of two builds). usage: python tools/diag_w8.py <fixture> <dtype>"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "grad-tts_amd"), REPO, os.path.join(REPO, "tests")]
from conftest import load_golden  # noqa: E402
from gpu_util import make_decoder  # noqa: E402
from oracle import decoder as odec  # noqa: E402

name, dt = sys.argv[1], sys.argv[2]
g = load_golden(name)
n_spks = int(g["n_spks"])
cdt = {"bf16": torch.bfloat16, "w8": "bf16_w8"}[dt]
dec, sd = make_decoder(n_spks, int(g["seed_w"]), cdt)
c = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
spk = c(g["spk"]) if n_spks != 1 else None
y = dec.estimator(c(g["x"]), c(g["mask"]), c(g["mu"]), c(g["t"]), spk).cpu().numpy().astype(np.float64)
if dt == "w8":
    with torch.no_grad():
        ref = odec.estimator(odec.fp8_params(sd), *(torch.from_numpy(g[k]) for k in ("x", "mask", "mu", "t")),
                             torch.from_numpy(g["spk"]) if n_spks != 1 else None, n_spks).numpy().astype(np.float64)
else:
    ref = g["out"].astype(np.float64)
d = np.abs(y - ref) / np.abs(ref).max()
s = np.sort(d.ravel())[::-1]
print(f"{os.environ.get('GRADTTS_LIB', 'tree')[-30:]:30s} {name} {dt}: max {s[0]:.3e} 2nd {s[1]:.3e} 10th {s[9]:.3e} "
      f"p99.9 {np.quantile(d, 0.999):.3e} mean {d.mean():.3e} at {np.unravel_index(d.argmax(), d.shape)}")
