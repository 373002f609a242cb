#!/bin/bash
# End-of-round evidence on one GPU box (run through gpurun): smoke(), the full GPU suite, then the profile of the
# default bench (tools/gpu_profile.sh). Each GPU step has its own time limit; a failing step stops the script.
# usage: tools/gpu_final.sh <tag>     -> gpurun_out/final_<tag>/ and gpurun_out/prof_<tag>/
set -u
TAG=${1:-r03}
OUT=gpurun_out/final_$TAG
mkdir -p $OUT
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
GRADTTS_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_profile.sh $TAG
