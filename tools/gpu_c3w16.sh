#!/bin/bash
# conv3w on v_mfma_f32_16x16x32_bf16: its parity tests and the decoder tests, then the default bench line.
set -u
OUT=gpurun_out/c3w16; mkdir -p $OUT
GRADTTS_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 600 python3 -u -m pytest tests/test_conv3w_gpu.py tests/test_decoder_gpu.py tests/test_fp8_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
python3 tools/ab_summary.py $OUT/bench.json c3w16 || exit 1
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['roofline'])"
# same box: the previous commit (ab/head) against the tree, twice each, short decodes
AB_ROWS=10 bash tools/ab_variants.sh head tree head tree || exit 1
