"""conv64 stamps (diagnostic build: tools/build_variant1.sh conv64.hip c64st -DGT_C64_STAMP=1 [-DGT_C64_STAMP_IN=2];
run with GRADTTS_LIB=ab/c64st/libgradtts.so). One bf16 estimator call at the bench shape; the last level-0 (F = 80)
launch of the stamped instantiation leaves per-wave cycle counts: prologue, tile loop, end-of-tile barrier waits, the
passes' MFMA streams (staging items included), the passes' epilogues, tiles, segment end."""
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
dec, _ = make_decoder(1, 0, torch.bfloat16)
mu, z, mask, _ = synthetic_inputs(1234, B, T)
z, mask, mu = (torch.from_numpy(a).cuda() for a in (z, mask, mu))
t = torch.full((B,), 0.5, device="cuda")
for _ in range(3):
    dec.estimator(z, mask, mu, t)
torch.cuda.synchronize()
f = _lib.lib().gt_diag_conv64_stamps
f.argtypes = [ctypes.c_void_p, ctypes.c_long]
buf = np.zeros(512 * 4 * 8, dtype=np.uint64)
assert f(buf.ctypes.data, buf.size) == 0
a = buf.reshape(512, 4, 8).astype(np.float64)
used = a[:, :, 5] > 0
names = ["prologue", "loop", "barrier", "mfma_pass", "epilogue", "tiles", "end", "-"]
print(f"waves with stamps: {int(used.sum())}")
for i, n in enumerate(names[:7]):
    v = a[:, :, i][used]
    print(f"{n:10s} mean {v.mean():12.0f}  min {v.min():12.0f}  max {v.max():12.0f}")
loop = a[:, :, 1][used]
for i in (2, 3, 4):
    print(f"{names[i]:10s} share of loop {(a[:, :, i][used] / loop).mean():.3f}")
tiles = a[:, :, 5][used].mean()
print(f"cycles per tile {loop.mean() / tiles:.0f} (MFMA floor 2 waves/SIMD x 72 x 32 = 4608)")
# where the slow segments are: blockIdx = col * kseg + part, col = b * n_tt + tt (kseg = 1 at level 0, T = 512)
lw = np.where(used, a[:, :, 1], np.nan)
wg = np.nanmax(lw, axis=1)
n_tt = T // 32
idx = np.arange(512)
ok = ~np.isnan(wg)
print("loop by tt   ", " ".join(f"{np.nanmean(wg[(idx % n_tt == k) & ok]) / 1e3:.0f}" for k in range(n_tt)))
print("loop by b    ", " ".join(f"{np.nanmean(wg[(idx // n_tt == k) & ok]) / 1e3:.0f}" for k in range(min(B, 32))))
print("loop by bid%8", " ".join(f"{np.nanmean(wg[(idx % 8 == k) & ok]) / 1e3:.0f}" for k in range(8)))
print("lengths", synthetic_inputs.__doc__ and "", (mask.sum(-1).flatten()[:32]).tolist())
print("histogram (k cycles)", np.histogram(wg[ok] / 1e3, bins=8))
