"""Phase timeline of the level-0 3x3 conv from a GT_STAMPS build (tools/build_variant.sh stamps -DGT_STAMPS=<IN>).

    GRADTTS_LIB=ab/stamps_mask/libgradtts.so python tools/stamps.py

Stamps (s_memtime, wave 0 of every workgroup): 0 start, 1 prologue done, per chunk c (k = 2 + 5c):
k   before the top barrier (= previous chunk's MFMAs done), k+1 after it, k+2 patch stored,
k+3 weight DMA waited, k+4 after the second barrier (MFMAs start); 40 epilogue start, 41 end.
"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "grad-tts_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from gradtts_amd import _lib  # noqa: E402
from gradtts_amd.params import synthetic_inputs  # noqa: E402
from gpu_util import make_decoder  # noqa: E402

ST_PER_WG, ST_WGS = 48, 8192


def main():
    dec, _ = make_decoder(1, 0, torch.bfloat16)
    mu, z, mask, _ = synthetic_inputs(1234, 32, 512)
    zc, mc, muc = (torch.from_numpy(a).cuda() for a in (z, mask, mu))
    for _ in range(3):
        dec(zc, mc, muc, 1)
    torch.cuda.synchronize()
    L = _lib.lib()
    L.gt_debug_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    st = np.zeros(ST_WGS * ST_PER_WG, np.uint64)
    hw = np.zeros(ST_WGS, np.uint32)
    assert L.gt_debug_read_stamps(st.ctypes.data, hw.ctypes.data) == 0
    st = st.reshape(ST_WGS, ST_PER_WG).astype(np.int64)
    used = st[:, 0] > 0
    st, hw = st[used], hw[used]
    nwg = len(st)
    nch = sum(1 for c in range(8) if (st[:, 2 + 5 * c] > 0).all())   # stamps cover up to 7 chunks
    t0 = st[:, 0].min()
    span = st[:, 41].max() - t0
    print(f"workgroups {nwg}, chunks {nch}, kernel span {span} cycles")
    med = lambda a: float(np.median(a))
    print(f"prologue (0->1)           {med(st[:, 1] - st[:, 0]):8.0f}")
    for c in range(nch):
        k = 2 + 5 * c
        prev_end = st[:, 1] if c == 0 else st[:, k]
        print(f"chunk {c}: barrier1 {med(st[:, k + 1] - st[:, k]):6.0f}  patch-store {med(st[:, k + 2] - st[:, k + 1]):6.0f}  "
              f"dma-wait {med(st[:, k + 3] - st[:, k + 2]):6.0f}  barrier2 {med(st[:, k + 4] - st[:, k + 3]):6.0f}  "
              f"mfma {med((st[:, k + 5] if c + 1 < nch else st[:, 40]) - st[:, k + 4]):6.0f}")
    print(f"epilogue (40->41)         {med(st[:, 41] - st[:, 40]):8.0f}:  transpose+store {med(st[:, 42] - st[:, 40]):.0f}, "
          f"stat shuffles {med(st[:, 43] - st[:, 42]):.0f}, barrier {med(st[:, 44] - st[:, 43]):.0f}, "
          f"final reduce {med(st[:, 41] - st[:, 44]):.0f}")
    life = st[:, 41] - st[:, 0]
    print(f"workgroup lifetime: median {med(life):.0f}, p10 {np.percentile(life, 10):.0f}, p90 {np.percentile(life, 90):.0f}")
    # concurrency: how many workgroups are alive on average (sum of lifetimes / span) per CU
    xcc = (hw >> 20) & 0x7 if False else None
    print(f"mean live workgroups across the chip: {life.sum() / span:.1f} (256 CUs)")
    starts = np.sort(st[:, 0] - t0)
    print("start-time deciles (cycles):", [int(np.percentile(starts, q)) for q in (0, 10, 25, 50, 75, 90, 100)])


if __name__ == "__main__":
    main()
