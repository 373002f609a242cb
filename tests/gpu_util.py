"""Helpers shared by the GPU parity tests and tools: build the HIP-backed modules from the synthetic
weights a fixture names, and read intermediate stages through gt_estimator_probe."""
import ctypes
import json
import os

import numpy as np
import torch

from gradtts_amd import _lib
from gradtts_amd.diffusion import Diffusion, _dtype_code, _stream_ptr
from gradtts_amd.params import synthetic_state_dict

STAGES = (["downs.0.0.pre1", "downs.0.0.pre2", "downs.0.0", "downs.0.1", "downs.0.2", "downs.0.3",
           "downs.1.0.pre1", "downs.1.0.pre2", "downs.1.0", "downs.1.1.pre1", "downs.1.1.pre2", "downs.1.1", "downs.1.2", "downs.1.3",
           "downs.2.0", "downs.2.1", "downs.2.2", "mid_block1", "mid_attn", "mid_block2",
           "ups.0.0.pre1", "ups.0.0", "ups.0.1", "ups.0.2", "ups.0.3",
           "ups.1.0", "ups.1.1", "ups.1.2", "ups.1.3", "final_block.pre"])


def make_decoder(n_spks=1, seed=0, compute_dtype=torch.float32, device="cuda"):
    dec = Diffusion(80, 64, n_spks, 64, 0.05, 20, 1000, compute_dtype=compute_dtype)
    sd = synthetic_state_dict(seed=seed, n_spks=n_spks)
    dec.estimator.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return dec.to(device), sd


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def report(name, err, tol, gate=True, **extra):
    """Print the achieved parity error of one check (visible in the pytest log) and, when GRADTTS_PARITY_LOG
    names a file, append it there as one JSON line; then gate it."""
    rec = {"check": name, "err": float(err), "tol": float(tol), **extra}
    print(f"PARITY {name}: rel err {err:.3e} (gate {tol:.0e})")
    path = os.environ.get("GRADTTS_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")
    if gate:
        assert err <= tol, f"{name}: rel err {err:.3e} > {tol:.0e}"
    return err <= tol


def probe(est, compute_dtype, x, mask, mu, t, spk, stage, shape):
    """Run the estimator on device tensors and return (score, stage activation [B,C,F,T])."""
    dcode = _dtype_code(compute_dtype)
    B, _, T = x.shape
    h = est._native()
    out = torch.empty((B, 80, T), dtype=torch.float32, device=x.device)
    pr = torch.full(shape, float("nan"), dtype=torch.float32, device=x.device)
    ws = est._workspace(x.device, dcode, B, T, 0)
    _lib.check(_lib.lib().gt_estimator_probe(h, dcode, x.data_ptr(), mask.data_ptr(), mu.data_ptr(), t.data_ptr(),
                                             spk.data_ptr() if spk is not None else None, B, T, stage.encode(),
                                             pr.data_ptr(), out.data_ptr(), ws.data_ptr(), ws.numel(),
                                             _stream_ptr(x.device)), "gt_estimator_probe")
    torch.cuda.synchronize()
    return out, pr
