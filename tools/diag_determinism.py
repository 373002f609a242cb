"""Find the first U-Net stage whose output differs between two identical runs (GPU diagnostic)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "grad-tts_amd"), os.path.join(REPO, "tests"), REPO]
from gpu_util import STAGES, make_decoder, probe  # noqa: E402
from gradtts_amd.params import synthetic_inputs  # noqa: E402

cdt = {"bf16": torch.bfloat16, "fp32": torch.float32, "w8": "bf16_w8"}[sys.argv[1] if len(sys.argv) > 1 else "bf16"]
B, T = int(os.environ.get("B", 32)), int(os.environ.get("T", 512))
dec, _ = make_decoder(1, 0, cdt)
mu, z, mask, _ = synthetic_inputs(1234, B, T)
t = np.full(B, 0.5, np.float32)
args = [torch.from_numpy(a).cuda() for a in (z, mask, mu, t)]
shapes = {}
C = {0: 64, 1: 128, 2: 256}
for st in STAGES:
    lvl = 0 if st.startswith(("downs.0", "final", "ups.1.3")) else (1 if st.startswith(("downs.1", "ups.1", "downs.0.3", "ups.0.3")) else 2)
    if st == "downs.0.3": lvl = 1
    if st == "downs.1.3": lvl = 2
    ch = {"downs.0.0": 64, "ups.0.0": 128, "ups.0.1": 128, "ups.0.2": 128, "ups.0.3": 128, "ups.1.0": 64, "ups.1.1": 64,
          "ups.1.2": 64, "ups.1.3": 64, "downs.1.3": 128, "downs.0.3": 64}.get(st.split(".pre")[0], C[lvl])
    if st.startswith("ups.0.0.pre"): ch = 128
    shape = (B, ch, 80 >> lvl, T >> lvl)
    outs = []
    for rep in range(3):
        o, pr = probe(dec.estimator, cdt, *args, None, st, shape)
        outs.append(pr.cpu())
    same = all(torch.equal(outs[0], o) for o in outs[1:])
    nan = torch.isnan(outs[0]).any().item()
    d = max((outs[0] - o).abs().max().item() for o in outs[1:])
    print(f"{st:18s} {tuple(shape)} identical={same} maxdiff={d:.3e} nan={nan}", flush=True)
