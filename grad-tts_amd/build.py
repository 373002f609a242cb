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
OPS_OUT = os.path.join(HERE, "gradtts_amd", "libgradtts_ops.so")   # torch.ops.gradtts.* (csrc/torch_ops.cpp)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("GRADTTS_ARCH", "gfx950")
SOURCES = ["conv.hip", "conv1s.hip", "conv64.hip", "conv3w.hip", "conv3w_a8.hip", "attn.hip", "attn_down.hip", "misc.hip", "mas.hip", "train.hip", "bwd.hip", "textenc.hip", "textenc_train.hip",
           "decoder.cpp", "train_bwd.cpp", "textenc.cpp", "vocoder.cpp"]
# -packed-fp32-ops: keep the compiler from emitting v_pk_{fma,add,mul}_f32. Rounds 1-2 saw run-to-run differences
# with them (GroupNorm sum-of-squares partials, W8 decodes); round 3 found the cause -- the compiler paired the
# per-lane GroupNorm sum / sum-of-squares chains into packed ops whose op_sel_hi read a dword the previous VALU
# instruction had just written, which gfx950 can return stale -- and keeps those chains scalar in the source
# (DESIGN.md §3), after which a packed build is bit-reproducible. The flag stays because the packed build measured
# no faster. (The host compile ignores the feature with a one-line note.)
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", os.path.join(REPO, "include"), "-I", CSRC,
         "-Wno-unused-result", "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]


def _deps_mtime():
    return max(os.path.getmtime(os.path.join(CSRC, f)) for f in os.listdir(CSRC) if f.endswith((".h", ".hip", ".cpp")))


# per-source extra flags: conv64's pass loop (36 steps with the staging of 8 items, IN_RB0's ResnetBlock-output transform
# the largest) must unroll fully -- past LLVM's default pragma-unroll size threshold the IN_RB0 loop stayed rolled and
# indexed its register rings dynamically (thousands of v_cndmask)
SRC_FLAGS = {"conv64.hip": ["-mllvm", "-pragma-unroll-threshold=1000000"]}


def _compile(src, force):
    obj = os.path.join(OBJ, src + ".o")
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(_deps_mtime(), os.path.getmtime(os.path.join(REPO, "include", "gradtts.h"))):
        return obj, None
    lang = ["-x", "hip"] if src.endswith(".cpp") else []
    cmd = [HIPCC, *FLAGS, *SRC_FLAGS.get(src, []), *lang, "-c", os.path.join(CSRC, src), "-o", obj]
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
    build_ops(force)
    if verbose:
        print(f"built {OUT}, {OPS_OUT}")
    return OUT


def build_ops(force: bool = False) -> str:
    """The PyTorch custom-op registration (TORCH_LIBRARY(gradtts)): host code against torch's headers and
    libraries; it resolves the C ABI of libgradtts.so at run time (torch.ops.gradtts.bind)."""
    src = os.path.join(CSRC, "torch_ops.cpp")
    deps = max(os.path.getmtime(src), os.path.getmtime(os.path.join(REPO, "include", "gradtts.h")))
    if not force and os.path.exists(OPS_OUT) and os.path.getmtime(OPS_OUT) >= deps:
        return OPS_OUT
    import torch
    tdir = os.path.dirname(torch.__file__)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I", os.path.join(REPO, "include"), "-I", os.path.join(tdir, "include"),
           "-I", os.path.join(tdir, "include", "torch", "csrc", "api", "include"), "-I", "/opt/rocm/include", src,
           "-L", os.path.join(tdir, "lib"), "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
           f"-Wl,-rpath,{os.path.join(tdir, 'lib')}", "-ldl", "-o", OPS_OUT]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"torch ops build failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return OPS_OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
