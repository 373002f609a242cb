#!/bin/bash
# Latency regime (B = 1, T = 512): bench lines for bf16, bf16_w8 and fp8 at N = 50 and a rocprofv3 kernel-trace summary
# of the bf16 decode.   usage (through gpurun): bash tools/b1_profile.sh [tag]  -> gpurun_out/<tag>/
set -u
OUT=gpurun_out/${1:-b1}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for dt in bf16 bf16_w8 fp8; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --batch 1 --dtype $dt --steps 5 > $OUT/bench_$dt.json 2> $OUT/bench_$dt.err || { echo "bench $dt failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_$dt.json').read().strip().splitlines()[-1]); print('$dt B=1', round(d['value']), 'mel-frames/s', round(d['ms_per_step'],2), 'ms per decode')"
done
timeout -k 10 300 rocprofv3 -M --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --no-cpu-baseline --batch 1 --steps 2 --warmup 1 > $OUT/kt.log 2>&1 || { echo "rocprof failed"; exit 1; }
cp $(find $OUT/kt -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv && rm -rf $OUT/kt
echo done
