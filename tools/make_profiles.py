"""Turn a gpurun profile directory (tools/gpu_profile.sh) into the committed artifacts:

    profiles/<tag>/kernel_stats.csv      rocprofv3 --kernel-trace --stats summary of the bench command
    profiles/<tag>/pmc_*.csv             per-kernel sums of each PMC pass (counter totals, dispatch counts)
    profiles/<tag>/bench.json            the bench line of the same box
    profiles/pmc_traffic.json            HBM bytes per launch per kernel instantiation, read by bench.py

HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB -> bytes): on gfx950 FETCH_SIZE reports half the bytes of
16-B-per-lane streaming reads (MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for 16-B stores.
Kernel names are normalised to the bench's "conv_kernel<bf16,KIND,IN,OUT,NT>" style.
usage: python tools/make_profiles.py gpurun_out/prof_<tag> <tag>
"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _demangle(name: str) -> str:
    """Itanium names of this library's kernels (_ZN2gt<len><name>[I<template args>E]...) -> "gt::name<args>(";
    template args DF16b (__bf16), f (float), Li<n>E (int), Lb<0|1>E (bool). Other names are returned as they are."""
    m = re.match(r"_ZN2gt(\d+)(\w+)", name)
    if not m:
        return name
    n = int(m.group(1))
    base, rest = m.group(2)[:n], m.group(2)[n:]
    args = []
    if rest.startswith("I"):
        for t in re.finditer(r"DF16b|f|Li(-?\d+)E|Lb([01])E", rest[1:]):
            tok = t.group(0)
            args.append("__bf16" if tok == "DF16b" else "float" if tok == "f" else
                        t.group(1) if t.group(1) is not None else ("true" if t.group(2) == "1" else "false"))
            if rest[1:].startswith("E", t.end()):
                break
    return f"void gt::{base}" + (f"<{', '.join(args)}>" if args else "") + "("


def norm(name: str) -> str:
    """rocprofv3 kernel name (mangled or demangled) -> the name decoder.cpp / bench.py use for the same kernel
    instantiation ("conv_kernel<bf16,KIND,IN,OUT,NT[,w8][,tf5]>", "conv64_kernel<IN>", "attn_kv_kernel<bf16>",
    "rbout_identity_kernel<bf16>", "rbout_input_kernel<bf16>", ...). Kernels outside namespace gt (the runtime's
    copies / fills, torch's elementwise kernels) keep their base name; a gt:: kernel that does not parse raises."""
    d = _demangle(name)
    m = re.match(r"(?:void )?gt::(\w+)(?:<([^()]*)>)?\(", d)
    if not m:
        return d.split("(")[0]
    base, args = m.group(1), [a.strip() for a in (m.group(2) or "").split(",") if a.strip()]
    ty = lambda a: {"__bf16": "bf16", "bf16": "bf16", "float": "float"}[a]
    try:
        if base == "conv_kernel":            # <A, KIND, IN, OUT, NT, W8, TF>
            A, kind, im, om, nt, w8, tf = args
            return (f"conv_kernel<{ty(A)},{kind},{im},{om},{nt}" + (",w8" if w8 in ("1", "true") else "") +
                    ("" if tf == "4" else ",tf" + tf) + ">")
        if base == "conv1s_kernel":          # <IN, OUT, NT, CIN>: the bench names it without CIN (in its shape)
            return f"{base}<{args[0]},{args[1]},{args[2]}>"
        if base == "conv64_kernel":          # <IN>
            return f"conv64_kernel<{args[0]}>"
        if base in ("conv3w_kernel", "conv3w_a8_kernel"):   # <IN, COUT, CB>
            return f"{base}<{','.join(args)}>"
        if base == "attn_down_kernel":       # <C, W8>
            return f"{base}<{args[0]}" + (",w8" if args[1] in ("true", "1") else "") + ">"
        if base == "attn_up_kernel":         # <W8>
            return base + ("<w8>" if args[0] in ("true", "1") else "")
        if base == "gn_mish_kernel":         # <A, RES>: the ResnetBlock output, residual res_conv(input) or identity
            return ("rbout_input_kernel" if args[1] in ("true", "1") else "rbout_identity_kernel") + f"<{ty(args[0])}>"
        if base in ("attn_kv_kernel", "final_kernel", "to_nchw_kernel"):
            return f"{base}<{ty(args[0])}>"
        if base == "attn_merge_kernel" and args:   # <DR>: rows per workgroup
            return f"{base}<{args[0]}>"
        if base == "attn_fold_kernel" and args:
            return f"{base}<{ty(args[0])}>"
        if not args:
            return base
    except (KeyError, ValueError, IndexError):
        pass
    raise ValueError(f"unparsed gt:: kernel name: {d}")


def pmc_sums(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = norm(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return agg, {k: len(v) for k, v in disp.items()}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    dst = os.path.join(REPO, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    for f in glob.glob(os.path.join(src, "kt", "**", "*kernel_stats.csv"), recursive=True):
        # rocprofv3 -M (mangled names: its demangler garbles __bf16 template arguments); add the bench's name
        rows = list(csv.DictReader(open(f)))
        with open(os.path.join(dst, "kernel_stats.csv"), "w", newline="") as out:
            w = csv.DictWriter(out, fieldnames=["Kernel"] + list(rows[0].keys()) if rows else ["Kernel"])
            w.writeheader()
            for r in rows:
                w.writerow({"Kernel": norm(r["Name"]), **r})
    if os.path.exists(os.path.join(src, "bench.json")):   # the JSON line (stderr may be interleaved)
        lines = [l for l in open(os.path.join(src, "bench.json")) if l.startswith("{")]
        if lines:
            with open(os.path.join(dst, "bench.json"), "w") as f:
                f.write(lines[-1])
    traffic = {}
    for p in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_sq2"):
        d = os.path.join(src, p)
        if not os.path.isdir(d):
            continue
        agg, n = pmc_sums(d)
        cols = sorted({c for v in agg.values() for c in v})
        with open(os.path.join(dst, p + ".csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "dispatches"] + cols)
            for k in sorted(agg, key=lambda k: -sum(agg[k].values())):
                w.writerow([k, n[k]] + [f"{agg[k].get(c, 0):.6g}" for c in cols])
        for k, v in agg.items():
            t = traffic.setdefault(k, {"dispatches": n[k]})
            if "FETCH_SIZE" in v:
                t["fetch_kb_per_launch_raw"] = v["FETCH_SIZE"] / n[k]
            if "WRITE_SIZE" in v:
                t["write_kb_per_launch"] = v["WRITE_SIZE"] / n[k]
    for k, t in traffic.items():
        if "fetch_kb_per_launch_raw" in t and "write_kb_per_launch" in t:
            t["hbm_bytes_per_launch"] = (2 * t["fetch_kb_per_launch_raw"] + t["write_kb_per_launch"]) * 1024
    traffic = {k: v for k, v in traffic.items() if "hbm_bytes_per_launch" in v}
    # the configuration the PMC passes ran (bench.py reads these bytes only for the same workload: the per-launch
    # average of an instantiation depends on its shape mix, which depends on batch, frames, dtype and speakers)
    cfg = json.load(open(os.path.join(dst, "bench.json")))["config"]
    config = {k: cfg[k] for k in ("global_batch", "seq_len", "n_spks")}
    config["dtype"] = json.load(open(os.path.join(dst, "bench.json")))["dtype"]
    with open(os.path.join(REPO, "profiles", "pmc_traffic.json"), "w") as f:
        json.dump({"source": f"profiles/{tag} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)",
                   "formula": "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per launch (gfx950 FETCH_SIZE halving)",
                   "config": config, "kernels": traffic}, f, indent=1, sort_keys=True)
    print(f"wrote {dst} and profiles/pmc_traffic.json ({len(traffic)} kernels)")


if __name__ == "__main__":
    main()
