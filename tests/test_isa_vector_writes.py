"""Every GPU write of libgradtts.so is a vector memory instruction (tools/isa_scalar_mem_check.py): the gfx950 code
objects in the built library are disassembled on the CPU and searched for scalar-cache writes (scalar stores, scalar
atomics, scalar-cache write-back / discard), which this project never emits -- the split-K completion counter
(conv.hip) is a vector atomic. This file and the checker name those instructions and never run on a GPU box
(.gpurunignore)."""
import os
import subprocess
import sys

import pytest

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(R, "grad-tts_amd", "gradtts_amd", "libgradtts.so")
sys.path.insert(0, os.path.join(R, "tools"))


def test_checker_pattern():
    import isa_scalar_mem_check as c
    for ok in ("s_load_dwordx2 s[0:1], s[4:5], 0x0", "global_atomic_add_u32 v0, v1, s[2:3]", "s_waitcnt vmcnt(0)",
               "buffer_store_dwordx4 v[0:3], v4, s[8:11], 0 offen"):
        assert not c.FORBIDDEN.match("\t" + ok)
    for bad in ("s_store_dword s0, s[2:3], 0x0", "s_atomic_add s0, s[2:3], 0x0", "s_dcache_wb",
                "s_buffer_store_dword s0, s[4:7], 0x0"):
        assert c.FORBIDDEN.match("\t" + bad)


@pytest.mark.skipif(not os.path.exists(LIB), reason="libgradtts.so not built")
def test_library_has_no_scalar_cache_writes():
    r = subprocess.run([sys.executable, os.path.join(R, "tools", "isa_scalar_mem_check.py"), LIB],
                       capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout
