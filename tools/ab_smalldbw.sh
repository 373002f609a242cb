#!/bin/bash
# Small-plan double-buffered weight slabs (tree, GT_SMALL_DBW=1) against the split half-slab pipeline
# (ab/nodbw): small-batch / decoder parity tests on the tree build, then alternating B = 1 and B = 4 decodes.
set -u
OUT=gpurun_out/ab_sdbw
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_small_batch_gpu.py tests/test_decoder_gpu.py tests/test_fp8_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "Error|error|assert|FAILED" $OUT/pytest.log | head -8; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  for bb in 1 4; do
    for v in tree nodbw; do
      if [ $v = tree ]; then unset GRADTTS_LIB; else export GRADTTS_LIB=$PWD/ab/nodbw/libgradtts.so; fi
      timeout -k 10 300 python3 bench.py --no-cpu-baseline --batch $bb --steps 5 > $OUT/b_${v}_${bb}_$i.json 2> $OUT/b_${v}_${bb}_$i.err || { echo "bench failed"; tail -3 $OUT/b_${v}_${bb}_$i.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/b_${v}_${bb}_$i.json').read().strip().splitlines()[-1]); print('$v B=$bb run $i', round(d['value']), 'mel-frames/s', round(d['ms_per_step'], 2), 'ms', [(k, v['avg_us']) for k, v in list(d['shapes'].items())[:3]])"
    done
  done
done
