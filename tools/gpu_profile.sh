#!/bin/bash
# Profiling pass on the GPU box (run through gpurun). Every GPU step has its own time limit; a crash,
# abort or timeout exit code stops the script (no further GPU work in that call).
# usage: tools/gpu_profile.sh <tag> [bench args...]
set -u
TAG=${1:-r01}; shift || true
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() {  # run <limit_s> <log> cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > $log 2>&1
  local rc=$?
  echo "[$rc] $*" | cut -c1-200
  case $rc in 124|134|137|139) echo "fatal exit $rc -- stopping"; exit $rc;; esac
  return 0
}
BENCH="python3 bench.py --no-cpu-baseline $*"
run 300 $OUT/bench.log $BENCH --steps 3 --warmup 1
run 400 $OUT/ktrace.log rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $BENCH --steps 2 --warmup 1
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
run 300 $OUT/pmc_fetch.log rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- $BENCH --steps 1 --warmup 0 --n-timesteps 2
run 300 $OUT/pmc_write.log rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pmc -- $BENCH --steps 1 --warmup 0 --n-timesteps 2
run 300 $OUT/pmc_sq.log rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_sq -o pmc -- $BENCH --steps 1 --warmup 0 --n-timesteps 2
run 300 $OUT/pmc_sq2.log rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc_sq2 -o pmc -- $BENCH --steps 1 --warmup 0 --n-timesteps 2
find $OUT -name "*.csv" | head -50
echo done
