"""Build libgradtts.so (gfx950) in-tree with hipcc.

    python grad-tts_amd/build.py            # incremental
    python grad-tts_amd/build.py --force    # rebuild everything

Every HIP translation unit in csrc/ is compiled in parallel to an object next to the sources
(csrc/_obj/, git-ignored) and linked into grad-tts_amd/gradtts_amd/libgradtts.so, which travels
with the repository snapshot to the GPU box (no JIT cache involved).
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(CSRC, "_obj")
OUT = os.path.join(HERE, "gradtts_amd", "libgradtts.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("GRADTTS_ARCH", "gfx950")
SOURCES = ["conv.hip", "conv64.hip", "attn.hip", "misc.hip", "mas.hip", "decoder.cpp"]
# -packed-fp32-ops: keep the compiler from emitting v_pk_{fma,add,mul}_f32. With them the GroupNorm
# sum-of-squares chain in conv_kernel's epilogue produced timing-dependent (run-to-run different)
# results on MI355X while the plain sums stayed bit-exact (tools/diag_parts.py); without them every
# stage is bit-reproducible. (The host compile ignores the feature with a one-line note.)
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", os.path.join(REPO, "include"), "-I", CSRC,
         "-Wno-unused-result", "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]


def _deps_mtime():
    return max(os.path.getmtime(os.path.join(CSRC, f)) for f in os.listdir(CSRC) if f.endswith((".h", ".hip", ".cpp")))


def _compile(src, force):
    obj = os.path.join(OBJ, src + ".o")
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(_deps_mtime(), os.path.getmtime(os.path.join(REPO, "include", "gradtts.h"))):
        return obj, None
    lang = ["-x", "hip"] if src.endswith(".cpp") else []
    cmd = [HIPCC, *FLAGS, *lang, "-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    return obj, (None if r.returncode == 0 else f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    jobs = min(len(SOURCES), max(1, min(8, os.cpu_count() or 1)))
    with ThreadPoolExecutor(jobs) as ex:
        res = list(ex.map(lambda s: _compile(s, force), SOURCES))
    errs = [e for _, e in res if e]
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    objs = [o for o, _ in res]
    if force or not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {OUT}")
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
