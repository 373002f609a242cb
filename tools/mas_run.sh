#!/bin/bash
# MAS: GPU tests, then the a18 / ragged bench lines; extra args = A/B variant names (ab/<name>/libgradtts.so)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mas
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mas_gpu.py > gpurun_out/mas/test.log 2>&1 || { tail -30 gpurun_out/mas/test.log; exit 1; }
tail -2 gpurun_out/mas/test.log
bash tools/mas_ab.sh tree "$@"
