#!/bin/bash
# A/B of the elementwise first-block ResnetBlock output (GT_RB_INPUT=1, default) against the 1x1 conv_kernel path
# (GT_RB_INPUT=0) on one box: decoder parity tests, then alternating bench runs.
set -u
OUT=gpurun_out/ab_rbinput
mkdir -p $OUT
GRADTTS_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 600 python3 -u -m pytest tests/test_decoder_gpu.py tests/test_small_batch_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  for v in 0 1; do
    GT_RB_INPUT=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || { echo "bench failed"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$OUT/bench_${v}_$i.json').read().strip().splitlines()[-1]); k=[s for s in d['shapes'] if 'rbout_input' in s or '2,0,2,64' in s]; print('GT_RB_INPUT=$v run $i', round(d['value']), [(s, d['shapes'][s]['avg_us']) for s in k])"
  done
done
