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
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def norm(name: str) -> str:
    m = re.match(r"_ZN2gt(\d+)(\w+?)I(DF16b|f)((?:Li-?\d+E)*)E", name)
    if m:
        base = m.group(2)[: int(m.group(1))]
        ty = "bf16" if m.group(3) == "DF16b" else "float"
        ints = re.findall(r"Li(-?\d+)E", m.group(4))
        if base == "conv_kernel" and len(ints) == 6:   # trailing W8 flag and tile rows: "...,w8,tf5>" / nothing
            ints = ints[:4] + (["w8"] if ints[4] == "1" else []) + (["tf5"] if ints[5] == "5" else [])
        return f"{base}<{','.join([ty] + ints)}>"
    m = re.match(r"(?:void )?gt::(\w+)(<[^(]*>)?\(", name)
    if m:
        return m.group(1) + (m.group(2) or "").replace(" ", "")
    return name.split("(")[0]


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
        shutil.copy(f, os.path.join(dst, "kernel_stats.csv"))
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
    with open(os.path.join(REPO, "profiles", "pmc_traffic.json"), "w") as f:
        json.dump({"source": f"profiles/{tag} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)",
                   "formula": "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per launch (gfx950 FETCH_SIZE halving)",
                   **traffic}, f, indent=1, sort_keys=True)
    print(f"wrote {dst} and profiles/pmc_traffic.json ({len(traffic)} kernels)")


if __name__ == "__main__":
    main()
