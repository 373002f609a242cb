#!/bin/bash
# Same-box A/B of env-var variants of the in-tree library (bench at N=10) plus ab/<name> builds.
# usage: tools/ab_env.sh "label:ENV=VAL ENV2=VAL" "label2:" "lib:prev" ...
mkdir -p gpurun_out/var
for spec in "$@"; do
  label=${spec%%:*}; rest=${spec#*:}
  if [[ $label == lib ]]; then label=$rest; envs="GRADTTS_LIB=$PWD/ab/$rest/libgradtts.so"; else envs=$rest; fi
  env $envs GRADTTS_BENCH_NO_FINITE_CHECK=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 3 --warmup 2 --n-timesteps 10 > gpurun_out/var/$label.json 2> gpurun_out/var/$label.err
  rc=$?; echo "$label rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/var/$label.err; exit $rc; }
done
python3 - "$@" <<'PY'
import json, sys
labels = [(s.split(":")[1] if s.startswith("lib:") else s.split(":")[0]) for s in sys.argv[1:]]
d = {l: json.load(open(f"gpurun_out/var/{l}.json")) for l in labels}
print("variant".ljust(40), " ".join(l[:9].rjust(9) for l in labels))
print("ms/step".ljust(40), " ".join(f"{d[l]['ms_per_step']:9.2f}" for l in labels))
keys = []
for l in labels:
    for k in list(d[l]["shapes"].keys())[:16]:
        if k not in keys: keys.append(k)
for k in keys:
    print(k.replace("conv_kernel<bf16,", "c<")[:40].ljust(40), " ".join(f"{d[l]['shapes'].get(k, {}).get('avg_us', 0):9.1f}" for l in labels))
PY
