"""CPU check of the hand-counted waits around inline-asm vector loads (tools/asm_load_audit.py).

conv3w (csrc/conv3w.hip) loads the next chunk's patch items with inline-asm `buffer_load_dwordx4` so that hipcc does not
drain the weight DMAs with a conservative `s_waitcnt vmcnt(0)`; the matching counted `s_waitcnt vmcnt(N)` is written by
hand. If the compiler (or a source edit) lets an instruction read or overwrite a load's destination registers before
the wait that retires it, the kernel reads stale data or -- as in round 4 -- faults the GPU with an illegal address.
This test compiles every csrc/*.hip file whose inline asm (its own or c3w_asm.h's) issues buffer loads to a gfx950 listing (hipcc -S, device
only) and runs the audit over each kernel: a hazard fails here, on the CPU, instead of on the GPU."""
import os
import re
import shutil
import subprocess
import sys

import pytest

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(R, "grad-tts_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ASM_LOAD = re.compile(r'asm\s+volatile\s*\(\s*"[^"]*buffer_load_dword', re.S)


# headers whose inline asm issues buffer loads (c3w_asm.h: asm_buffer_load / asm_buffer_load2)
ASM_HEADERS = [f for f in sorted(os.listdir(CSRC)) if f.endswith(".h") and ASM_LOAD.search(open(os.path.join(CSRC, f)).read())]


def _sources():
    out = []
    for f in sorted(os.listdir(CSRC)):
        if not f.endswith(".hip"):
            continue
        text = open(os.path.join(CSRC, f)).read()
        if ASM_LOAD.search(text) or any(f'#include "{h}"' in text and "asm_buffer_load" in text for h in ASM_HEADERS):
            out.append(f)
    return out


def test_asm_load_sources_found():
    # conv3w and its fp8-operand twin are the kernels whose inline-asm loads the audit guards (their loads live in
    # c3w_asm.h); if they stop using them, update this test
    assert "c3w_asm.h" in ASM_HEADERS
    assert "conv3w.hip" in _sources() and "conv3w_a8.hip" in _sources()


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src", _sources())
def test_inline_asm_loads_waited_before_use(src, tmp_path):
    listing = tmp_path / (src + ".s")
    cmd = [HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
           "-I", os.path.join(R, "include"), "-I", CSRC, "-Wno-unused-result",
           "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",   # the product build's flags (build.py)
           os.path.join(CSRC, src), "-o", str(listing)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    a = subprocess.run([sys.executable, os.path.join(R, "tools", "asm_load_audit.py"), str(listing)],
                       capture_output=True, text=True)
    print(a.stdout[-3000:])
    assert a.returncode == 0 and a.stdout.strip().endswith("OK"), a.stdout[-3000:]
    audited = [int(n) for n in re.findall(r": (\d+) asm loads audited", a.stdout)]
    assert audited and all(n > 0 for n in audited), "no inline-asm loads seen in the listing: audit did not run"


def _run_audit(text, tmp_path):
    f = tmp_path / "fake.s"
    f.write_text(text)
    return subprocess.run([sys.executable, os.path.join(R, "tools", "asm_load_audit.py"), str(f)],
                          capture_output=True, text=True)


FAKE = """_Z4fakev:
\ts_mov_b32 s0, 0
\t;;#ASMSTART
\tbuffer_load_dwordx4 v[4:7], v1, s[8:11], s2 offen
\t;;#ASMEND
\ts_cmp_gt_i32 s3, 3
\ts_cbranch_scc1 .LBB0_2
\t{wait}
.LBB0_2:
\tv_add_f32_e32 v9, v4, v5
\ts_endpgm
.Lfunc_end0:
"""


def test_audit_flags_a_wait_only_some_waves_execute(tmp_path):
    # the wait sits on the fall-through of a (wave-uniform) branch: waves taking the branch read v4 before the load
    # lands -- the round-4 fault. The audit must call it BAD, and OK once the wait is on every path.
    r = _run_audit(FAKE.format(wait="s_waitcnt vmcnt(0)"), tmp_path)
    assert r.returncode == 1 and "BAD" in r.stdout, r.stdout
    ok = FAKE.replace("\ts_cmp_gt_i32", "\ts_waitcnt vmcnt(0)\n\ts_cmp_gt_i32").format(wait="s_nop 0")
    r = _run_audit(ok, tmp_path)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout


# ---- split-K ordering (tools/sk_order_audit.py): the small plan's split tiles hand fp32 partials between workgroups
# through relaxed agent-scope atomics; the audit pins the lowering that makes that safe (sc1 stores and loads, the
# stores drained and the workgroup past a barrier before the counter increment).
@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_split_k_handoff_lowering(tmp_path):
    listing = tmp_path / "conv.s"
    cmd = [HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
           "-I", os.path.join(R, "include"), "-I", CSRC, "-Wno-unused-result",
           "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",
           os.path.join(CSRC, "conv.hip"), "-o", str(listing)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    a = subprocess.run([sys.executable, os.path.join(R, "tools", "sk_order_audit.py"), str(listing)],
                       capture_output=True, text=True)
    print(a.stdout[-3000:])
    assert a.returncode == 0 and a.stdout.strip().endswith("OK"), a.stdout[-3000:]


SK_FAKE = """_Z2skv:
\tglobal_store_dword v[2:3], v4, off {st}
\t{wait}
\ts_barrier
\tglobal_atomic_add v5, v5, v6, s[0:1] sc0
\ts_waitcnt vmcnt(0)
\tglobal_load_dword v7, v[2:3], off sc1
\ts_endpgm
.Lfunc_end0:
"""


def test_split_k_audit_flags_missing_order(tmp_path):
    f = tmp_path / "sk.s"
    for st, wait, good in (("sc1", "s_waitcnt vmcnt(0)", True), ("", "s_waitcnt vmcnt(0)", False),
                           ("sc1", "s_nop 0", False)):
        f.write_text(SK_FAKE.format(st=st, wait=wait))
        r = subprocess.run([sys.executable, os.path.join(R, "tools", "sk_order_audit.py"), str(f)],
                           capture_output=True, text=True)
        assert (r.returncode == 0) == good, r.stdout
