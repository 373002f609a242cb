"""Run the HIP training step (Diffusion.loss_t + backward, fp32) at the reference's training shape for profiling:
rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -- python tools/train_step.py [--B 16 --T 172 --steps 5]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "grad-tts_amd"))
from gradtts_amd.diffusion import Diffusion  # noqa: E402
from gradtts_amd.params import synthetic_inputs, synthetic_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--T", type=int, default=172)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--n_spks", type=int, default=1)
    a = ap.parse_args()
    dec = Diffusion(80, 64, a.n_spks, 64, 0.05, 20, 1000)
    sd = synthetic_state_dict(seed=0, n_spks=a.n_spks)
    dec.estimator.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    dec = dec.cuda()
    mu, z, mask, spk = synthetic_inputs(1, a.B, a.T)
    c = lambda x: torch.from_numpy(x).cuda()
    x0 = c(mu + 0.5 * np.random.default_rng(2).standard_normal(mu.shape).astype(np.float32))
    t = torch.rand(a.B, device="cuda").clamp(1e-5, 1 - 1e-5)
    s = c(spk) if a.n_spks > 1 else None
    args = (x0, c(mask), c(mu), t, s)
    zz = c(z)
    for i in range(a.steps + 2):
        if i == 2:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        dec.zero_grad(set_to_none=True)
        loss, _ = dec.loss_t(*args, z=zz)
        loss.backward()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    print(f"training step B={a.B} T={a.T}: {ms:.2f} ms, {a.B * a.T / ms * 1e3:.0f} frames/s, loss {float(loss):.5f}")


if __name__ == "__main__":
    main()
