#!/bin/bash
# scratch: small-plan tests, then B = 1 decodes with split-K off / on for the fp8-weight mode
set -u
OUT=gpurun_out/tmp; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_small_batch_gpu.py tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -15 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for cfg in 0 256 0 256; do
  GT_SK_TARGET=$cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline --batch 1 --dtype bf16_w8 --steps 3 --warmup 1 > $OUT/w8_$cfg.json 2> $OUT/w8_$cfg.err || { echo "bench failed"; tail -3 $OUT/w8_$cfg.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/w8_$cfg.json').read().strip().splitlines()[-1]); print('w8 B=1 sk=$cfg', round(d['ms_per_step'],2), 'ms')"
done
