"""Wall time of the bench workload with and without the per-launch HIP-event profiling."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "grad-tts_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from gradtts_amd import _lib  # noqa: E402
from gradtts_amd.params import synthetic_inputs  # noqa: E402
from gpu_util import make_decoder  # noqa: E402

dt = sys.argv[1] if len(sys.argv) > 1 else "bf16"
dec, _ = make_decoder(1, 0, {"bf16": torch.bfloat16, "bf16_w8": "bf16_w8"}[dt])
mu, z, mask, _ = synthetic_inputs(1234, 32, 512)
zc, mc, muc = (torch.from_numpy(a).cuda() for a in (z, mask, mu))
L = _lib.lib()
h = dec.estimator._native()
import ctypes
buf = ctypes.create_string_buffer(1 << 20)
for prof in (0, 1, 0, 1):
    L.gt_decoder_profile_enable(h, prof)
    dec(zc, mc, muc, 10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        dec(zc, mc, muc, 50)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 3 * 1e3
    if prof:
        L.gt_decoder_profile_read(h, buf, len(buf))
    print(f"{dt} events={prof}: {ms:.2f} ms per 50-step decode, {32 * 512 / ms * 1e3:.0f} mel-frames/s", flush=True)
