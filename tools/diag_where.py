"""Locate the elements of one stage that differ between identical runs (GPU diagnostic)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "grad-tts_amd"), os.path.join(REPO, "tests"), REPO]
from gpu_util import make_decoder, probe  # noqa: E402
from gradtts_amd.params import synthetic_inputs  # noqa: E402

stage = sys.argv[1] if len(sys.argv) > 1 else "downs.1.0"
shape = tuple(int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "32,128,40,256").split(","))
B, T = shape[0], shape[3] * (512 // shape[3]) if shape[3] < 512 else shape[3]
T = int(os.environ.get("T", 512))
dec, _ = make_decoder(1, 0, torch.bfloat16)
mu, z, mask, _ = synthetic_inputs(1234, B, T)
t = np.full(B, 0.5, np.float32)
args = [torch.from_numpy(a).cuda() for a in (z, mask, mu, t)]
outs = []
for rep in range(6):
    _, pr = probe(dec.estimator, torch.bfloat16, *args, None, stage, shape)
    outs.append(pr.cpu().numpy())
ref = outs[0]
for i, o in enumerate(outs[1:], 1):
    d = np.argwhere(o != ref)
    print(f"rep {i}: {len(d)} differing elements")
    if len(d):
        for ax, name in enumerate("bcft"):
            u, c = np.unique(d[:, ax], return_counts=True)
            print(f"   {name}: {len(u)} distinct, e.g. {list(zip(u[:12].tolist(), c[:12].tolist()))}")
        print("   first:", d[:6].tolist(), "vals", [(float(ref[tuple(x)]), float(o[tuple(x)])) for x in d[:3]])
