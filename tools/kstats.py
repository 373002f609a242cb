"""Register / scratch / LDS usage of every kernel of one source: python tools/kstats.py [--src misc.hip] [-DFLAG ...]"""
import os
import re
import subprocess
import sys
import tempfile

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[2] if len(sys.argv) > 2 and sys.argv[1] == "--src" else "conv.hip"
flags = [a for a in sys.argv[1:] if a.startswith("-D")]
with tempfile.TemporaryDirectory() as d:
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                    "-I", f"{R}/include", "-I", f"{R}/grad-tts_amd/csrc", "-Xclang", "-target-feature", "-Xclang",
                    "-packed-fp32-ops", *flags, f"{R}/grad-tts_amd/csrc/{src}", "-o", f"{d}/k.s"], check=True)
    s = open(f"{d}/k.s").read()
for b in s.split(".end_amdhsa_kernel"):
    m = re.search(r"\.amdhsa_kernel (\S+)", b)
    if not m:
        continue
    g = lambda k: re.search(rf"\.amdhsa_{k} (\d+)", b).group(1)
    name = m.group(1)   # mangled (c++filt mis-decodes the bf16 template argument)
    print(f"{name[:70]:70s} vgpr {g('next_free_vgpr'):>3} agpr_off {g('accum_offset'):>3} "
          f"scratch {g('private_segment_fixed_size'):>3} lds {g('group_segment_fixed_size'):>6}")
