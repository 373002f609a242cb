"""Run the HIP HiFi-GAN generator for profiling: B utterances x T mel frames (synthetic weights).
rocprofv3 --kernel-trace --stats -d gpurun_out/prof_voc -- python tools/vocoder_run.py [--B 16 --T 172 --iters 3]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "grad-tts_amd"))
from gradtts_amd.params import HIFIGAN_V1, synthetic_vocoder_state_dict  # noqa: E402
from gradtts_amd.vocoder import Generator  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=16)
ap.add_argument("--T", type=int, default=172)
ap.add_argument("--iters", type=int, default=3)
a = ap.parse_args()
g = Generator(HIFIGAN_V1)
g.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_vocoder_state_dict(1).items()})
g = g.cuda().eval()
mel = torch.randn(a.B, 80, a.T, device="cuda") * 2 - 5
g(mel)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.iters):
    g(mel)
torch.cuda.synchronize()
print(f"vocoder B={a.B} T={a.T}: {(time.perf_counter() - t0) / a.iters * 1e3:.2f} ms")
