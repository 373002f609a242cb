#!/bin/bash
# Quick health check of the current tree on one GPU box: smoke(), the GPU suite, the default bench line.
# usage: tools/gpu_check_head.sh <tag>   -> gpurun_out/check_<tag>/
set -u
TAG=${1:-head}
OUT=gpurun_out/check_$TAG
mkdir -p $OUT
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
GRADTTS_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
cat $OUT/bench.json | cut -c1-400
