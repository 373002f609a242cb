#!/bin/bash
# Time experiment builds (ab/<name>/libgradtts.so) with the bench on one box; usage: tools/ab_variants.sh name...
mkdir -p gpurun_out/var
for v in "$@"; do
  if [ "$v" = "tree" ]; then unset GRADTTS_LIB; else export GRADTTS_LIB=$PWD/ab/$v/libgradtts.so; fi
  GRADTTS_BENCH_NO_FINITE_CHECK=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 3 --warmup 2 --n-timesteps 10 $BENCH_ARGS > gpurun_out/var/$v.json 2> gpurun_out/var/$v.err
  rc=$?; echo "$v rc=$rc"
  case $rc in 0) ;; *) tail -3 gpurun_out/var/$v.err; exit $rc;; esac
done
python3 - "$@" <<'PY'
import json, sys
vs = sys.argv[1:]
d = {v: json.load(open(f"gpurun_out/var/{v}.json")) for v in vs}
print("variant".ljust(12), " ".join(v[:9].rjust(9) for v in vs))
print("ms/step".ljust(12), " ".join(f"{d[v]['ms_per_step']:9.2f}" for v in vs))
keys = list(d[vs[0]]["shapes"].keys())[:int(__import__("os").environ.get("AB_ROWS", "14"))]
for k in keys:
    print(k.replace("conv_kernel<bf16,", "c<")[:38].ljust(38), " ".join(f"{d[v]['shapes'].get(k, {}).get('avg_us', 0):9.1f}" for v in vs))
PY
