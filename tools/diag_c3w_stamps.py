"""conv3w phase-wait stamps (diagnostic build: tools/build_variant1.sh conv3w.hip st -DGT_C3W_STAMP=1; run with
GRADTTS_LIB=ab/st/libgradtts.so; A8=1: conv3w_a8, built with conv3w_a8.hip -DGT_C3W8_STAMP=1, on an fp8 decoder). One bf16 estimator call at the bench shape; the last launch of the stamped
instantiation (default <IN_GN, 256, 2>: mid_block2's block2 at level 2) leaves per-wave cycle counts: DMA wait, phase
barrier, item waits, item transform + write, the whole chunk loop, phases."""
import ctypes
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "grad-tts_amd"))
sys.path.insert(0, os.path.join(R, "tests"))
from gpu_util import make_decoder  # noqa: E402
from gradtts_amd import _lib  # noqa: E402
from gradtts_amd.params import synthetic_inputs  # noqa: E402

B, T = int(os.environ.get("B", "32")), 512
A8 = os.environ.get("A8") == "1"
dec, _ = make_decoder(1, 0, "fp8" if A8 else torch.bfloat16)
mu, z, mask, _ = synthetic_inputs(1234, B, T)
z, mask, mu = (torch.from_numpy(a).cuda() for a in (z, mask, mu))
t = torch.full((B,), 0.5, device="cuda")
for _ in range(3):
    dec.estimator(z, mask, mu, t)
torch.cuda.synchronize()
L = _lib.lib()
f = L.gt_diag_conv3w_a8_stamps if A8 else L.gt_diag_conv3w_stamps
f.argtypes = [ctypes.c_void_p, ctypes.c_long]
buf = np.zeros(512 * 8 * 8, dtype=np.uint64)
assert f(buf.ctypes.data, buf.size) == 0
a = buf.reshape(512, 8, 8).astype(np.float64)
used = a[:, :, 5] > 0
names = ["dma_wait", "barrier", "item_wait", "item_put", "loop", "phases", "prologue", "epilogue"]
print(f"workgroups with stamps: {int(used.any(1).sum())}")
for i, n in enumerate(names):
    v = a[:, :, i][used]
    print(f"{n:10s} mean {v.mean():12.0f}  min {v.min():12.0f}  max {v.max():12.0f}")
loop = a[:, :, 4][used]
for i, n in enumerate(names[:4]):
    print(f"{n:10s} share of loop {(a[:, :, i][used] / loop).mean():.3f}")
ph = a[:, :, 5][used].mean()
tot = (a[:, :, 4] + a[:, :, 6] + a[:, :, 7])[used]
print(f"prologue {(a[:, :, 6][used] / tot).mean():.3f}  loop {(loop / tot).mean():.3f}  epilogue {(a[:, :, 7][used] / tot).mean():.3f} of {tot.mean():.0f} cycles")
print(f"cycles per phase {loop.mean() / ph:.0f} (MFMA floor per SIMD: 2 waves x " +
      ("10 x 64" if A8 else "40 x 16") + " = 1280)")
