"""Localise the large-logit attention mismatch: per-stage errors vs the oracle (fp32) for the
test_attention_large_logits_fp32 setup."""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "grad-tts_amd"), REPO, os.path.join(REPO, "tests")]
from oracle import decoder as odec
from gradtts_amd.diffusion import Diffusion
from gradtts_amd.params import synthetic_inputs, synthetic_state_dict
from gpu_util import STAGES, probe, rel_err

scale = float(sys.argv[1]) if len(sys.argv) > 1 else 300.0
g = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
sd = synthetic_state_dict(seed=2)
for k in list(sd):
    if k.endswith("to_qkv.weight"):
        w = sd[k].copy(); w[128:256] *= scale; sd[k] = w
    elif k.endswith("fn.g"):
        sd[k] = np.full_like(sd[k], g)
dec = Diffusion(80, 64, 1, 64, 0.05, 20, 1000, compute_dtype=torch.float32)
dec.estimator.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
dec = dec.cuda()
B, T = 2, 256
mu, z, mask, _ = synthetic_inputs(17, B, T, lengths=[256, 190])
t = np.linspace(0.8, 0.3, B).astype(np.float32)
taps = {}
with torch.no_grad():
    ref = odec.estimator(odec.to_torch_params(sd), torch.from_numpy(z), torch.from_numpy(mask),
                         torch.from_numpy(mu), torch.from_numpy(t), taps=taps).numpy()
args = [torch.from_numpy(a).cuda() for a in (z, mask, mu, t)]
for st in STAGES:
    r = taps[st].numpy()
    _, pr = probe(dec.estimator, torch.float32, *args, None, st, r.shape)
    p = pr.cpu().numpy()
    per_b = [rel_err(p[b], r[b]) for b in range(B)]
    print(f"{st:18s} {rel_err(p, r):.3e}  per utt {per_b[0]:.2e} {per_b[1]:.2e}  max|ref| {np.abs(r).max():.3e}")
