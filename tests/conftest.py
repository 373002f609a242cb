import ctypes
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (os.path.join(REPO, "grad-tts_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def mas_oracle():
    """ctypes handle on the plain-C MAS restatement (oracle/mas.c), built on demand."""
    so = os.path.join(REPO, "oracle", "_build", "libmas_oracle.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "all"], check=True)
    lib = ctypes.CDLL(so)
    lib.oracle_maximum_path.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_float]
    lib.oracle_maximum_path.restype = None

    def run(values, t_xs, t_ys, max_neg_val=-1e9):
        values = np.ascontiguousarray(values, dtype=np.float32).copy()
        b, tx, ty = values.shape
        paths = np.zeros((b, tx, ty), dtype=np.int32)
        t_xs = np.ascontiguousarray(t_xs, dtype=np.int32)
        t_ys = np.ascontiguousarray(t_ys, dtype=np.int32)
        lib.oracle_maximum_path(paths.ctypes.data, values.ctypes.data, t_xs.ctypes.data, t_ys.ctypes.data,
                                b, tx, ty, max_neg_val)
        return paths, values
    return run
