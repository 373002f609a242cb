"""Per-stage error of the bf16 estimator against the fp32 oracle on the inputs of
tests/test_decoder_gpu.py::test_estimator_vs_oracle_other_shapes (B=3, T=256) -- A/B of library switches via env.
usage: python tools/diag_stage_err.py"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "grad-tts_amd"), os.path.join(REPO, "tests")]
from gpu_util import STAGES, make_decoder, probe, rel_err  # noqa: E402
from oracle import decoder as odec  # noqa: E402
from gradtts_amd.params import synthetic_inputs  # noqa: E402

B, T = 3, 256
dec, sd = make_decoder(1, 1, torch.bfloat16)
mu, z, mask, _ = synthetic_inputs(7, B, T, lengths=[256, 200, 64])
t = np.linspace(0.9, 0.1, B).astype(np.float32)
taps = {}
with torch.no_grad():
    ref = odec.estimator(odec.to_torch_params(sd), torch.from_numpy(z), torch.from_numpy(mask), torch.from_numpy(mu),
                         torch.from_numpy(t), taps=taps).numpy()
args = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (z, mask, mu, t)]
y = dec.estimator(*args).cpu().numpy()
print("estimator", rel_err(y, ref))
for st in ["downs.0.0.pre1", "downs.0.0.pre2", "downs.0.0", "downs.0.1", "downs.0.2", "mid_block2", "ups.1.2",
           "final_block.pre"]:
    r = taps[st].numpy()
    _, pr = probe(dec.estimator, torch.bfloat16, *args, None, st, r.shape)
    print(st, rel_err(pr.cpu().numpy(), r))
