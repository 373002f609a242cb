#!/bin/bash
# conv3w bring-up on one GPU box: its parity tests, the throughput-plan / bench-shape decoder tests, then the default
# bench with conv3w on and off (same box). Each GPU step has its own limit; a failing step stops the script.
set -u
OUT=gpurun_out/${1:-c3w}
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_conv3w_gpu.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_c3w.log 2>&1
rc=$?; echo "c3w tests rc=$rc"; grep -E "PARITY|passed|failed|Error" $OUT/pytest_c3w.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u -m pytest tests/test_small_batch_gpu.py tests/test_decoder_gpu.py -x -q --timeout 300 --timeout-method thread -k "throughput or bench_shape or plans_agree" > $OUT/pytest_tp.log 2>&1
rc=$?; echo "throughput tests rc=$rc"; tail -3 $OUT/pytest_tp.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $OUT/bench_on.json 2> $OUT/bench_on.err || { echo "bench on failed"; tail $OUT/bench_on.err; exit 1; }
GT_CONV3W=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline > $OUT/bench_off.json 2> $OUT/bench_off.err || { echo "bench off failed"; exit 1; }
python3 - $OUT <<'PY'
import json, sys
for k in ("on", "off"):
    d = json.load(open(f"{sys.argv[1]}/bench_{k}.json"))
    print(k, round(d["value"]), "mel-frames/s", round(d["ms_per_step"], 2), "ms", d["roofline"]["kernel"], round(d["roofline"]["frac"], 3))
    for n, v in list(d["shapes"].items())[:14]: print("   ", n, v)
PY
# profile: rocprofv3 kernel trace of a short bench, then the SQ counter passes of the conv3w kernels
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 -M --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/kt.log 2>&1 || { echo "ktrace failed"; exit 1; }
f=$(find $OUT/kt -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv
python3 - $OUT/kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f"{r['Name'][:64]:64s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:8.1f} us {float(r['Percentage']):6.2f} %")
print("total ms", tot / 1e6)
PY
bash tools/pmc_kernels.sh conv3w $OUT/pmc > $OUT/pmc.log 2>&1; echo "pmc rc=$?"; tail -20 $OUT/pmc.log
