#!/bin/bash
# same-box A/B of several builds: the in-tree library ("tree") and ab/<name>/libgradtts.so for each name given.
# Decoder parity tests on every variant first, then R rounds of alternating default-config bench runs; one summary line
# per run (value, ms/step, the shapes matching $SHAPES).   usage: R=2 SHAPES=conv64 tools/ab_multi.sh name1 name2 ...
mkdir -p gpurun_out/abm
R=${R:-2}; SHAPES=${SHAPES:-conv64}
for v in "$@"; do
  GRADTTS_LIB=$PWD/ab/$v/libgradtts.so timeout -k 10 300 python -u -m pytest tests/test_decoder_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/abm/pt_$v.log 2>&1; rc=$?
  echo "$v tests: $(tail -1 gpurun_out/abm/pt_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in $(seq 1 $R); do
  for v in tree "$@"; do
    if [ $v = tree ]; then unset GRADTTS_LIB; else export GRADTTS_LIB=$PWD/ab/$v/libgradtts.so; fi
    timeout -k 10 200 python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abm/b_${v}_${r}.json 2>/dev/null || exit 1
    python3 - gpurun_out/abm/b_${v}_${r}.json $v "$SHAPES" <<'PY' || exit 1
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
pat = sys.argv[3].split(",")
sh = {k.split("_kernel")[0] + k[k.index("<"):]: v["avg_us"] for k, v in d["shapes"].items() if any(p in k for p in pat)}
print(sys.argv[2], round(d["value"]), round(d["ms_per_step"], 2), sh)
PY
  done
done
