#!/bin/bash
# scratch A/B: B = 1 decode under split-K targets
set -u
OUT=gpurun_out/tmp; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_small_batch_gpu.py tests/test_attn_mf_gpu.py tests/test_decoder_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -15 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log; grep -h "split-K\|small vs" $OUT/pytest.log | head
for cfg in 0 256 384 512 0 256; do
  GT_SK_TARGET=$cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline --batch 1 --steps 3 --warmup 1 > $OUT/b_$cfg.json 2> $OUT/b_$cfg.err || { echo "bench failed"; tail -3 $OUT/b_$cfg.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/b_$cfg.json').read().strip().splitlines()[-1])
k=[s for s in d['shapes'] if 'tf1' in s and ',0,' in s]
print('sk=$cfg', round(d['ms_per_step'],2), 'ms', [(s.split('@')[0][-14:]+'@'+s.split('@')[1], round(d['shapes'][s]['avg_us'],1)) for s in k])"
done
for B in 2 4; do for cfg in 0 256; do
  GT_SK_TARGET=$cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline --batch $B --steps 3 --warmup 1 > $OUT/b${B}_$cfg.json 2> $OUT/b${B}_$cfg.err || { echo "bench failed"; tail -3 $OUT/b${B}_$cfg.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/b${B}_$cfg.json').read().strip().splitlines()[-1]); print('B=$B sk=$cfg', round(d['ms_per_step'],2), 'ms')"
done; done
