"""Phase timeline of conv64_kernel from a GT_C64_STAMPS build:

    bash tools/build_variant.sh s64 -DGT_C64_STAMPS=1      # 1 = IN_MASK, 2 = IN_GN
    GRADTTS_LIB=ab/s64/libgradtts.so python tools/stamps64.py

Per 4x32 tile (s_memtime, first and last wave of the first 256 workgroups): 0 loop top, 1 pass 0 (MFMAs of the
wave's first row, staging of the next tile interleaved), 2 pass 1 (+ pass 0's epilogue), 3 pass 1's epilogue +
GroupNorm partials + closing barrier + slot write.
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

WG, TILES, PH = 256, 24, 4
PER = 2 + TILES * PH
NAMES = ["pass0", "pass1", "stats+barrier+slot"]


def main():
    dec, _ = make_decoder(1, 0, torch.bfloat16)
    mu, z, mask, _ = synthetic_inputs(1234, 32, 512)
    zc, mc, muc = (torch.from_numpy(a).cuda() for a in (z, mask, mu))
    for _ in range(3):
        dec(zc, mc, muc, 1)
    torch.cuda.synchronize()
    L = _lib.lib()
    L.gt_debug_read_c64_stamps.argtypes = [ctypes.c_void_p]
    st = np.zeros(WG * 2 * PER, np.uint64)
    assert L.gt_debug_read_c64_stamps(st.ctypes.data) == 0
    st = st.reshape(WG, 2, PER).astype(np.int64)
    for w, name in ((0, "first wave"), (1, "last wave")):
        s = st[:, w, :]
        ntile = int(((s[:, 2::PH] > 0).sum(1)).min())
        t0 = s[:, 0].min()
        print(f"{name}: tiles/wg {ntile}, prologue {np.median(s[:, 1] - s[:, 0]):.0f} cycles, "
              f"span {s[:, 2 + (ntile - 1) * PH + 3].max() - t0} cycles")
        for t in range(min(ntile, 3)):
            k = 2 + t * PH
            d = [np.median(s[:, k + i + 1] - s[:, k + i]) for i in range(3)]
            print(f"  tile {t}: " + "  ".join(f"{n} {v:6.0f}" for n, v in zip(NAMES, d)))
        k0, k1 = 2 + PH, 2 + (ntile - 1) * PH
        d = [np.median((s[:, k1 + i + 1] - s[:, k1 + i] + s[:, k0 + i + 1] - s[:, k0 + i]) / 2) for i in range(3)]
        tot = np.median((s[:, k1 + 3] - s[:, k0]) / (ntile - 1))
        print(f"  steady (median of tiles 1 and last): " + "  ".join(f"{n} {v:6.0f}" for n, v in zip(NAMES, d)) +
              f"   per tile {tot:.0f}")


if __name__ == "__main__":
    main()
