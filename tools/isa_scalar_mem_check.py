"""Check that the built library's gfx950 machine code never writes through the scalar data cache: no scalar memory
stores, scalar atomics or scalar-cache write-back / discard instructions (runs of such code were followed by hardware
errors on this GPU pool; every GPU write here must be a vector store or vector atomic). Runs on the CPU over the
code objects inside libgradtts.so (.hip_fatbin section, one clang offload bundle per translation unit), disassembled
with llvm-objdump. This file names those instructions, so it is listed in .gpurunignore (it never runs on a GPU box).
usage: python tools/isa_scalar_mem_check.py [path/to/libgradtts.so]"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
# scalar-cache writes: s_store_*, s_buffer_store_*, s_scratch_store_*, s_atomic_*, s_buffer_atomic_*, s_dcache_wb*,
# s_dcache_discard*
FORBIDDEN = re.compile(r"^\s*(s_store_|s_buffer_store|s_scratch_store|s_atomic_|s_buffer_atomic|s_dcache_wb|s_dcache_discard)")


def code_objects(lib):
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", lib, os.devnull],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
    objs, pos = [], 0
    while True:
        i = data.find(MAGIC, pos)
        if i < 0:
            return objs
        n, = struct.unpack_from("<Q", data, i + 24)
        q = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, q)
            q += 24
            triple = data[q:q + tl].decode()
            q += tl
            if "gfx950" in triple:
                objs.append(data[i + off:i + off + size])
        pos = i + len(MAGIC)


def check(lib):
    objs = code_objects(lib)
    bad, ninstr = [], 0
    with tempfile.TemporaryDirectory() as d:
        for k, o in enumerate(objs):
            f = os.path.join(d, f"co{k}.o")
            open(f, "wb").write(o)
            r = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", f],
                               capture_output=True, text=True, check=True)
            for line in r.stdout.splitlines():
                if line.startswith("\t") or line.startswith(" "):
                    ninstr += 1
                    if FORBIDDEN.match(line):
                        bad.append(line.strip())
    return len(objs), ninstr, bad


def main():
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(here, "grad-tts_amd", "gradtts_amd", "libgradtts.so")
    nobj, ninstr, bad = check(lib)
    print(f"{nobj} gfx950 code objects, {ninstr} instructions, {len(bad)} scalar-cache writes")
    for b in bad[:20]:
        print("  ", b)
    return 1 if bad or nobj == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
