#!/bin/bash
# Same-box A/B of one on/off environment knob of the library: the decoder parity tests with the default (on), then
# alternating default-config bench runs with KNOB=0 / KNOB=1 (two each); prints the bench value and the shapes whose
# name matches PATTERN.   usage: tools/ab_knob.sh KNOB PATTERN
set -u
KNOB=$1; PAT=$2
OUT=gpurun_out/ab_$KNOB
mkdir -p $OUT
GRADTTS_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 600 python3 -u -m pytest tests/test_decoder_gpu.py tests/test_small_batch_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  for v in 0 1; do
    env $KNOB=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || { echo "bench failed"; exit 1; }
    python3 -c "import json,re; d=json.loads(open('$OUT/bench_${v}_$i.json').read().strip().splitlines()[-1]); k=[s for s in d['shapes'] if re.search('$PAT', s)]; print('$KNOB=$v run $i', round(d['value']), [(s, d['shapes'][s]['avg_us']) for s in k])"
  done
done
