#!/bin/bash
# Split-K of the small-batch plan: small-batch / decoder parity tests, then same-box B = 1 and B = 4 decodes with
# GT_KSPLIT=0 / 1 (bf16, T = 512, N = 50).
set -u
OUT=gpurun_out/ab_ksplit
mkdir -p $OUT
GRADTTS_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 600 python3 -u -m pytest tests/test_small_batch_gpu.py tests/test_decoder_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "Error|error|assert|FAILED" $OUT/pytest.log | head -8; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  for bb in 1 4; do
    for v in 0 1; do
      GT_KSPLIT=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --batch $bb --steps 5 > $OUT/bench_b${bb}_${v}_$i.json 2> $OUT/bench_b${bb}_${v}_$i.err || { echo "bench failed"; tail -3 $OUT/bench_b${bb}_${v}_$i.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/bench_b${bb}_${v}_$i.json').read().strip().splitlines()[-1]); print('B=$bb GT_KSPLIT=$v run $i', round(d['value']), 'mel-frames/s', round(d['ms_per_step'], 2), 'ms')"
    done
  done
done
