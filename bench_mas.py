#!/usr/bin/env python3
"""Benchmark of the monotonic-alignment-search kernel (SURVEY.md §8 rows a17-a19, §8d "MAS").

    python bench_mas.py [--steps 20] [--warmup 3] [--batch 32] [--tx 200] [--ty 800] [--ragged]
                        [--no-cpu-baseline]

A "step" is one ``maximum_path_c`` call (core.pyx:38-45 semantics, ``gt_maximum_path`` through the C ABI)
over a batch of log-prior grids already resident in HBM: fp32 values [b, t_x, t_y] in, int32 0/1 path out.
Default workload = the SURVEY §8a row-a18 measurement case (b = 32, t_x = 200, t_y = 800, full lengths);
``--ragged`` = a training batch (params.py:50 batch 16, t_x ~ U[100, 400], t_y ~ U[256, 1024]).

Printed: one JSON line. ``value`` = grid cells (b * t_x_max * t_y_max) per second; roofline = algorithmic
bytes (4 B read + 4 B written per cell, §8d) / the average call time, against 8 TB/s HBM.
``cpu_baseline`` = the C restatement oracle/mas.c ("port"), single-threaded as the reference's build is
(setup.py:7-11 compiles OpenMP out), on the same inputs.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "grad-tts_amd"))

from gradtts_amd.monotonic_align import maximum_path_c  # noqa: E402

HBM_PEAK = 8.0e12


def make_inputs(args):
    rng = np.random.default_rng(7)
    b = args.batch
    if args.ragged:
        t_x = rng.integers(100, 401, b).astype(np.int32)
        t_y = np.maximum(rng.integers(256, 1025, b), t_x).astype(np.int32)
    else:
        t_x = np.full(b, args.tx, np.int32)
        t_y = np.full(b, args.ty, np.int32)
    txm, tym = int(t_x.max()), int(t_y.max())
    # log-prior-like values (tts.py:143-149 is a sum of Gaussian log-densities: negative, O(100))
    v = (-0.5 * rng.standard_normal((b, txm, tym)) ** 2 * 80.0 - 73.5).astype(np.float32)
    m = (np.arange(txm)[None, :, None] < t_x[:, None, None]) & (np.arange(tym)[None, None, :] < t_y[:, None, None])
    return (v * m).astype(np.float32), t_x, t_y


def cpu_baseline(v, t_x, t_y, budget_s=3.0):
    """Time the C restatement of the reference MAS (oracle/mas.c, "port") on a bounded number of utterances
    of the same batch, single-threaded as the reference's build is (setup.py:7-11 compiles OpenMP out).
    The reference's own Cython core never travels to the GPU box: its timing, measured in the build
    container, is in BASELINE.md."""
    kind = "port"
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "_build", "libmas_oracle.so"))
    lib.oracle_maximum_path.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64] * 3 + [ctypes.c_float]

    def run(vv, xs, ys, pp):
        lib.oracle_maximum_path(pp.ctypes.data, vv.ctypes.data, xs.ctypes.data, ys.ctypes.data,
                                vv.shape[0], vv.shape[1], vv.shape[2], -1e9)
    b = v.shape[0]
    done, cells, dt = 0, 0, 0.0
    while dt < budget_s and done < 100000:   # cycle over the batch's utterances for ~budget_s of CPU work
        i = done % b
        vv = np.ascontiguousarray(v[i:i + 1]).copy()   # the core mutates its values in place (core.pyx:9-35)
        pp = np.zeros(vv.shape, np.int32)
        xs, ys = np.ascontiguousarray(t_x[i:i + 1]), np.ascontiguousarray(t_y[i:i + 1])
        t0 = time.perf_counter()
        run(vv, xs, ys, pp)
        dt += time.perf_counter() - t0
        cells += vv.size
        done += 1
    return {"value": cells / dt, "unit": "cells/s", "cores": 1, "kind": kind,
            "sample": f"{done} utterance calls cycling over the batch of {b} ({dt:.2f} s in the core), "
                      "oracle/mas.c"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--tx", type=int, default=200)
    ap.add_argument("--ty", type=int, default=800)
    ap.add_argument("--ragged", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    if args.ragged and args.batch == 32:
        args.batch = 16
    if not torch.cuda.is_available():
        raise SystemExit("bench_mas.py needs an MI355X")
    dev = torch.device("cuda", 0)
    v, t_x, t_y = make_inputs(args)
    b, txm, tym = v.shape
    vd = torch.from_numpy(v).to(dev)
    xs = torch.from_numpy(t_x).to(dev)
    ys = torch.from_numpy(t_y).to(dev)
    paths = torch.empty(v.shape, dtype=torch.int32, device=dev)
    for _ in range(args.warmup):
        maximum_path_c(paths, vd, xs, ys)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.steps):
        maximum_path_c(paths, vd, xs, ys)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    cells = b * txm * tym
    alg_bytes = 8.0 * cells
    achieved = alg_bytes / (ms * 1e-3)
    line = {
        "metric": "MAS grid cells/s (maximum_path, bit-exact to core.pyx)", "value": cells / (ms * 1e-3),
        "unit": "cells/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
        "higher_is_better": True, "dtype": "f32/i32", "data": "synthetic log-prior-like values (seed 7)",
        "config": {"workload": ("training batch, ragged lengths" if args.ragged else "SURVEY §8a row a18 case"),
                   "batch": b, "tx_max": txm, "ty_max": tym, "ragged": bool(args.ragged)},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK, "traffic": None,
                     "note": "whole call (DP + path write), 8 algorithmic bytes per grid cell"},
    }
    if not args.no_cpu_baseline:
        cb = cpu_baseline(v, t_x, t_y)
        ref_p = None
        # bit-exactness of this very run on the first utterance (the parity tests cover the rest)
        so = os.path.join(REPO, "oracle", "_build", "libmas_oracle.so")
        if os.path.exists(so):
            lib = ctypes.CDLL(so)
            lib.oracle_maximum_path.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64] * 3 + [ctypes.c_float]
            vv = np.ascontiguousarray(v[:1]).copy()
            ref_p = np.zeros(vv.shape, np.int32)
            lib.oracle_maximum_path(ref_p.ctypes.data, vv.ctypes.data, t_x[:1].ctypes.data, t_y[:1].ctypes.data,
                                    1, txm, tym, -1e9)
            cb["first_utterance_bit_exact"] = bool(np.array_equal(ref_p[0], paths[0].cpu().numpy()))
        line["cpu_baseline"] = cb
    print(json.dumps(line))


if __name__ == "__main__":
    main()
