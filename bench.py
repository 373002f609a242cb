#!/usr/bin/env python3
"""Benchmark: mel-frames/s of the N-step reverse-diffusion decoder on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 32] [--frames 512] [--n-timesteps 50]
                    [--dtype bf16|fp32|bf16_w8|fp8] [--n-spks 1] [--no-cpu-baseline] [--dry-run]

Launch: ``--gpus N`` with N > 1 and no ``WORLD_SIZE`` in the environment starts N ranks itself
(``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py ...``) from a
parent process that makes no HIP-runtime call at all (it does not even count devices: a rank that finds no GPU
fails and the parent exits with the ranks' status); rank 0's JSON line is relayed as the last line of stdout.
Under an external launcher (the driver's ``torch.distributed.run``) the world size comes from ``WORLD_SIZE``;
an explicit ``--gpus`` must match it. ``--dry-run`` exercises exactly this launch / rendezvous / gather /
max-over-ranks plumbing on CPU with gloo and no decoder (the line says ``"dry_run": true``; it is not a
measurement).

A "step" is one complete ``Diffusion.reverse_diffusion`` call (n_timesteps Euler steps of the U-Net)
over one batch of synthetic utterances already resident in HBM, followed by the RCCL all_gather of
the mel outputs when N > 1. Default workload = BASELINE config 2: LJSpeech single speaker, batch 32
per GPU, T = 512 frames, N = 50, bf16 compute. With N GPUs every rank decodes its own batch of 32
(weak scaling: the 8-GPU run is config 4, 256 utterances), ``value`` = all frames / max-rank time.

Printed (rank 0, one JSON line): the driver contract fields plus
  roofline      the dominant kernel's achieved algorithmic TFLOP/s vs the bf16 dense MFMA peak, measured
                live with a HIP event pair around each of its launches during the timed steps (the other
                launches run without events: an event pair on every launch costs ~11 % of the step);
  kernels/shapes per-kernel tables from the last warm-up step, run with an event pair on EVERY launch: its per-launch
                times include the events' stream overhead (~11 % of the step), so they rank kernels but do not add
                up to the timed step (the per-kernel times of the timed step are the rocprofv3 kernel trace of the
                same command, profiles/<round>/kernel_stats.csv);
  cpu_baseline  the oracle CPU restatement (oracle/decoder.py, "port") timed on this host for a bounded
                sample (one Euler step of a smaller batch at the same T), projected to mel-frames/s.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "grad-tts_amd"))

from gradtts_amd import _lib  # noqa: E402
from gradtts_amd.diffusion import Diffusion  # noqa: E402
from gradtts_amd.params import estimator_flops, synthetic_inputs, synthetic_state_dict  # noqa: E402
from gradtts_amd.shard import gather_shards  # noqa: E402

# dense MFMA peaks (MI355X_MICROARCH.md): bf16 2.5 PF; block-scaled e4m3 (v_mfma_scale_f32_32x32x64_f8f6f4) 5 PF.
# "fp8" runs its 3x3 convs over activations on the fp8 MFMA and the rest in bf16: its path fraction is quoted against
# the fp8 peak (the stricter figure), a kernel's roofline against the peak of the MFMA it issues.
PEAK = {"bf16": 2.5e15, "bf16_w8": 2.5e15, "fp8": 5.0e15, "fp32": 157.3e12}
HBM_PEAK = 8.0e12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks); default: WORLD_SIZE under an external launcher, else 1")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32, help="utterances per GPU")
    ap.add_argument("--frames", type=int, default=512)
    ap.add_argument("--n-timesteps", type=int, default=50)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "bf16_w8", "fp8"],
                    help="bf16_w8: fp8 e4m3 conv weights, bf16 MFMA operands; fp8: e4m3 weights and operands on the "
                         "block-scaled fp8 MFMA for the 3x3 convs over activations (BASELINE config 5)")
    ap.add_argument("--n-spks", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-batch", type=int, default=4)
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU/gloo rehearsal of the multi-rank launch and gather; no decoder, not a measurement")
    return ap.parse_args()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """Start args.gpus ranks of this script under torch.distributed.run (one process per GPU) and relay their
    output. The parent makes no HIP-runtime call (no device count either: with fewer GPUs than ranks a rank fails when it
    selects its device and the launcher's non-zero status is returned). Returns the launcher's exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    line = None
    for out in proc.stdout:          # stream the ranks' stdout (progress stays visible); hold back the JSON line
        if out.startswith("{") and '"metric"' in out:
            line = out.strip()
        else:
            sys.stdout.write(out)
            sys.stdout.flush()
    rc = proc.wait()
    if line is not None:
        print(line, flush=True)
    elif rc == 0:
        print("bench.py: ranks exited without a result line", file=sys.stderr)
        rc = 1
    return rc


def dry_run(args, world, rank):
    """The multi-rank skeleton of main() on CPU: gloo rendezvous, per-rank shard of synthetic inputs, the mel
    gather, barrier + max-over-ranks timing and the rank-0 line. The decode is replaced by a masked copy."""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    B, T = args.batch, args.frames
    mu, z, mask, _ = synthetic_inputs(1234 + rank, B, T)
    z, mask = torch.from_numpy(z), torch.from_numpy(mask)

    def step():
        y = z * mask
        return gather_shards(y, world * B, world) if world > 1 else y

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        y = step()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert y.shape == (world * B, 80, T), y.shape
    if rank == 0:
        sec = elapsed / max(args.steps, 1)
        print(json.dumps({
            "metric": METRIC, "value": world * B * T / sec, "unit": "mel-frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": sec * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype, "dry_run": True,
            "data": "dry run: CPU gloo plumbing only, decoder replaced by a masked copy (not a measurement)",
            "config": config_block(args, world)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


# GRADTTS_BENCH_SHARED_DEVICE=1: every rank on cuda:0 with gloo (rehearsal of the N-rank HIP path on a 1-GPU box;
# RCCL refuses two ranks on one device). Not for measurements.
SHARED_DEVICE = os.environ.get("GRADTTS_BENCH_SHARED_DEVICE", "0") == "1"
METRIC = "mel-frames/sec (reverse-diffusion, 80-mel, N=50) at 1/2/4/8 MI355X; RTF"


def config_block(args, world):
    B, T, N = args.batch, args.frames, args.n_timesteps
    return {"workload": f"LJSpeech single-speaker batch={B}/GPU, T={T} frames, n_timesteps={N}, "
                        f"{args.dtype} " + ("(BASELINE config 5: fp8 U-Net weights)" if args.dtype in ("bf16_w8", "fp8")
                                            else "(BASELINE config 2; N GPUs = config 4 weak-scaled)"),
            "global_batch": world * B, "seq_len": T, "n_timesteps": N, "n_spks": args.n_spks,
            "parallelism": f"dp{world} utterance shards, RCCL all_gather of mels" if world > 1 else "dp1"}


def pmc_traffic(kernel, args, world):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary (tools/make_profiles.py), or None
    when no summary exists or it was measured on another workload (batch per GPU, frames, dtype, speakers): a
    kernel's per-launch average depends on the shape mix of its launches."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    cfg = d.get("config", {})
    if (cfg.get("global_batch"), cfg.get("seq_len"), cfg.get("n_spks"), cfg.get("dtype")) != \
            (args.batch, args.frames, args.n_spks, args.dtype):
        return None
    return d.get("kernels", {}).get(kernel, {}).get("hbm_bytes_per_launch")


def host_cpus():
    """(threads to use, host CPU count, CPU model). BASELINE.md §5 runs the restatement on os.cpu_count() threads; a
    job whose CPU time is capped by its cgroup (cpu.max quota) or pinned to fewer CPUs gets that many instead, since
    threads beyond the quota only queue behind it."""
    n = os.cpu_count() or 1
    usable = n
    try:
        usable = min(usable, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            quota, period = open(path).read().split()[:2]
            if quota != "max":
                usable = min(usable, max(1, int(int(quota) // int(period))))
        except (OSError, ValueError):
            pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return usable, n, model


def cpu_baseline(args, sd):
    """Oracle restatement on the host cores, one Euler step of a bounded sample at the bench T."""
    from oracle import decoder as odec
    threads, ncpu, model = host_cpus()
    torch.set_num_threads(threads)
    Bs = args.cpu_sample_batch
    mu, z, mask, spk = synthetic_inputs(99, Bs, args.frames)
    p = odec.to_torch_params(sd)
    spk_t = torch.from_numpy(spk) if args.n_spks > 1 else None
    with torch.no_grad():
        odec.estimator(p, torch.from_numpy(z[:1]), torch.from_numpy(mask[:1]), torch.from_numpy(mu[:1]),
                       torch.tensor([0.5]), spk_t[:1] if spk_t is not None else None, n_spks=args.n_spks)   # warm-up
        t0 = time.perf_counter()
        odec.reverse_diffusion(p, torch.from_numpy(z), torch.from_numpy(mask), torch.from_numpy(mu), 1, spk_t,
                               n_spks=args.n_spks)
        dt = time.perf_counter() - t0
    frames_per_s = Bs * args.frames / (dt * args.n_timesteps)
    return {"value": frames_per_s, "unit": "mel-frames/s", "cores": threads, "kind": "port",
            "host_cpus": ncpu, "cpu_model": model, "label": "build CPU restatement",
            "sample": f"oracle/decoder.py (torch CPU fp32), 1 of {args.n_timesteps} Euler steps, B={Bs}, "
                      f"T={args.frames}: {dt:.2f} s, projected x{args.n_timesteps}"}


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus is None:
        args.gpus = int(env_world) if env_world else 1
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; launch with matching values")
    if args.dry_run:
        return dry_run(args, world, rank)
    if SHARED_DEVICE:
        local = 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("gloo" if SHARED_DEVICE else "nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    cdt = {"bf16": torch.bfloat16, "fp32": torch.float32, "bf16_w8": "bf16_w8", "fp8": "fp8"}[args.dtype]
    B, T, N = args.batch, args.frames, args.n_timesteps
    dec = Diffusion(80, 64, args.n_spks, 64, 0.05, 20, 1000, compute_dtype=cdt)
    sd = synthetic_state_dict(seed=0, n_spks=args.n_spks)
    dec.estimator.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    dec = dec.to(dev)
    mu, z, mask, spk = synthetic_inputs(1234 + rank, B, T)
    mu, z, mask = (torch.from_numpy(a).to(dev) for a in (mu, z, mask))
    spk = torch.from_numpy(spk).to(dev) if args.n_spks > 1 else None

    def step():
        y = dec(z, mask, mu, N, False, spk)
        if world > 1:   # every rank decodes its own shard of utterances; mels gathered in utterance order
            gather_shards(y, world * B, world)
        return y

    L = _lib.lib()
    handle = dec.estimator._native(dec.beta_min, dec.beta_max)
    buf = ctypes.create_string_buffer(1 << 20)

    def aggregate(entries):   # "<kernel>@<shape>" entries -> per kernel instantiation
        agg = {}
        for e in entries:
            k = e["kernel"].split("@")[0]
            a = agg.setdefault(k, {"kernel": k, "ms": 0.0, "launches": 0, "flop": 0.0, "bytes": 0.0})
            for f in ("ms", "launches", "flop", "bytes"):
                a[f] += e[f]
        return list(agg.values())

    # The last warm-up step runs with a HIP event pair around every launch: the per-kernel tables and the
    # choice of the dominant kernel come from it (earlier steps include one-time code loading). The timed
    # steps keep events on the dominant kernel's launches only (each event pair costs stream time: events
    # on every launch slow the whole decode by ~11 %). Without warm-up every timed launch is profiled.
    for i in range(args.warmup):
        if i == args.warmup - 1:          # the last warm-up step (steady state: code loaded, caches warm)
            torch.cuda.synchronize()
            L.gt_decoder_profile_enable(handle, 1)
        step()
    torch.cuda.synchronize()
    _lib.check(L.gt_decoder_profile_read(handle, buf, len(buf)), "gt_decoder_profile_read")
    shapes = json.loads(buf.value.decode())
    table_steps = 1
    prof = aggregate(shapes)
    # dominant kernel = the instantiation with the largest total time, over every kernel of the decode
    dom_name = max(prof, key=lambda p: p["ms"])["kernel"] if prof else None
    timed_events = os.environ.get("GRADTTS_BENCH_TIMED_EVENTS", "1") != "0"   # 0: A/B runs without events
    if not timed_events:
        L.gt_decoder_profile_enable(handle, 0)
    elif dom_name:
        L.gt_decoder_profile_filter(handle, (dom_name + "@").encode())
    else:
        L.gt_decoder_profile_enable(handle, 1)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        y = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    L.gt_decoder_profile_enable(handle, 0)
    L.gt_decoder_profile_filter(handle, None)
    _lib.check(L.gt_decoder_profile_read(handle, buf, len(buf)), "gt_decoder_profile_read")
    timed = aggregate(json.loads(buf.value.decode())) if timed_events else prof
    if not dom_name:   # no warm-up: every launch of the timed steps was profiled
        shapes, prof, table_steps = json.loads(buf.value.decode()), timed, args.steps
        dom_name = max(timed, key=lambda p: p["ms"])["kernel"]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    if not os.environ.get("GRADTTS_BENCH_NO_FINITE_CHECK"):   # timing-only experiment builds set this
        assert torch.isfinite(y).all(), "non-finite decoder output"

    if rank == 0:
        sec = elapsed / args.steps
        frames = world * B * T
        value = frames / sec
        flop_step = N * estimator_flops(B, T, args.n_spks)
        dom = next(p for p in timed if p["kernel"] == dom_name)   # events inside the timed region
        avg_s = dom["ms"] / dom["launches"] / 1e3
        # (fp8-operand kernels: conv_kernel's ",a8" instantiations and conv3w_a8_kernel issue the block-scaled fp8 MFMA)
        fp8_mfma = ",a8" in dom["kernel"] or dom["kernel"].startswith("conv3w_a8_kernel")
        kpeak = PEAK["fp8"] if fp8_mfma else PEAK["bf16" if args.dtype in ("bf16_w8", "fp8") else args.dtype]
        # bound: MFMA when the kernel's algorithmic FLOP per byte is past the ridge point (peak FLOP/s / 8 TB/s),
        # else HBM (achieved = algorithmic bytes per launch / launch time against 8 TB/s)
        mfma_bound = dom["flop"] > 0 and (dom["bytes"] <= 0 or dom["flop"] / dom["bytes"] >= kpeak / HBM_PEAK)
        if mfma_bound:
            achieved, peak_u, unit, scale = dom["flop"] / dom["launches"] / avg_s, kpeak, "TFLOP/s", 1e12
        else:
            achieved, peak_u, unit, scale = dom["bytes"] / dom["launches"] / avg_s, HBM_PEAK, "GB/s", 1e9
        total_kernel_ms = sum(p["ms"] for p in prof)
        out = {
            "metric": METRIC,
            "value": value, "unit": "mel-frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": sec * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic: mu~N(0,1), z=mu+N(0,1), full-length masks; random-init weights (seed 0), no checkpoint",
            "config": config_block(args, world),
            "rtf": sec * 22050 / (frames * 256),     # inference.py:91 formula
            "frame_steps_per_s": value * N,
            "path_tflops": flop_step * world / sec / 1e12,
            "path_mfma_frac": flop_step / sec / PEAK[args.dtype],
            "roofline": {"bound": "mfma" if mfma_bound else "hbm", "kernel": dom["kernel"],
                         "launches_per_step": dom["launches"] / args.steps,
                         "achieved": achieved / scale, "peak": peak_u / scale, "unit": unit,
                         "frac": achieved / peak_u, "avg_launch_us": avg_s * 1e6,
                         "flop_per_launch": dom["flop"] / dom["launches"],
                         "traffic": pmc_traffic(dom["kernel"], args, world),
                         "algorithmic_bytes_per_launch": dom["bytes"] / dom["launches"],
                         "timing": "HIP event pair around each launch of this kernel during the timed steps"},
            "tables_from": ("the last warm-up step" if args.warmup else "the timed steps") +
                           " with an event pair on every launch (event-instrumented step: per-launch times include the"
                           " events' overhead; the timed step's kernel times are the rocprofv3 trace)",
            "kernels": {p["kernel"]: {"share": round(p["ms"] / total_kernel_ms, 4),
                                      "avg_us": round(p["ms"] / p["launches"] * 1e3, 2),
                                      "per_step": p["launches"] // table_steps,
                                      "tflops": round(p["flop"] / (p["ms"] * 1e-3) / 1e12, 1) if p["flop"] else None,
                                      "gbps": round(p["bytes"] / (p["ms"] * 1e-3) / 1e9, 0) if p["bytes"] else None}
                        for p in sorted(prof, key=lambda p: -p["ms"])[:14]},
            "shapes": {e["kernel"]: {"avg_us": round(e["ms"] / e["launches"] * 1e3, 2),
                                     "per_step": e["launches"] // table_steps,
                                     "tflops": round(e["flop"] / (e["ms"] * 1e-3) / 1e12, 1)}
                       for e in sorted(shapes, key=lambda e: -e["ms"]) if "@" in e["kernel"]},
        }
        if SHARED_DEVICE:
            out["shared_device"] = "all ranks on cuda:0 over gloo: launch rehearsal, not a scaling measurement"
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, sd)
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
