#!/bin/bash
# Development round trip on one GPU box: smoke(), the GPU suite (parity errors to parity.jsonl), the default bench line
# and the B = 1 latency lines (bf16, fp8 at N = 50). Each GPU step has its own time limit; a failing step ends the script.
# usage: tools/gpu_dev.sh <tag> [pytest selection]   -> gpurun_out/dev_<tag>/
set -u
TAG=${1:-dev}
SEL=${2:-tests}
OUT=gpurun_out/dev_$TAG
mkdir -p $OUT
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
GRADTTS_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 900 python3 -u -m pytest $SEL -m gpu -v --timeout 300 \
  --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
python3 tools/ab_summary.py $OUT/bench.json default || exit 1
for dt in bf16 fp8; do
  timeout -k 10 200 python3 bench.py --batch 1 --dtype $dt --no-cpu-baseline > $OUT/b1_$dt.json 2> $OUT/b1_$dt.err || { echo "b1 $dt failed"; tail -5 $OUT/b1_$dt.err; exit 1; }
  python3 tools/ab_summary.py $OUT/b1_$dt.json b1_$dt || exit 1
done
