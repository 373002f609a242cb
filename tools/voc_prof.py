"""Vocoder timing workload for rocprofv3 (fp32 HiFi-GAN V1, B = 16, T = 172 = 2 s of audio per utterance): a few
forward calls of the HIP generator, then (with --eager) the same algorithm as torch eager ops (oracle restatement,
MIOpen) so one kernel trace shows both.   usage: python tools/voc_prof.py [--eager] [--bf16]"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "grad-tts_amd")]
from gradtts_amd.params import HIFIGAN_V1, synthetic_vocoder_state_dict  # noqa: E402
from gradtts_amd.vocoder import Generator  # noqa: E402

dt = torch.bfloat16 if "--bf16" in sys.argv else torch.float32
g = Generator(HIFIGAN_V1, compute_dtype=dt)
sd = synthetic_vocoder_state_dict(4)
g.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
g = g.cuda().eval()
mel = torch.randn(16, 80, 172, device="cuda") * 2.0 - 5.0
with torch.no_grad():
    for _ in range(2):
        g(mel)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        g(mel)
    torch.cuda.synchronize()
    print(f"ours {dt}: {(time.perf_counter() - t0) / 3 * 1e3:.1f} ms", flush=True)
    if "--eager" in sys.argv:
        from oracle import vocoder as ov
        p = {k: v.cuda() for k, v in ov.to_torch_params(sd).items()}
        ov.generator(p, mel)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            ov.generator(p, mel)
        torch.cuda.synchronize()
        print(f"eager fp32: {(time.perf_counter() - t0) / 3 * 1e3:.1f} ms", flush=True)
