#!/bin/bash
# Round profile on the GPU box (run through gpurun). Each GPU step has its own time limit; any failing
# step stops the script (no further GPU work in that call).
# usage: tools/gpu_profile.sh <tag> [bench args...]     -> gpurun_out/prof_<tag>/
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
  [ $rc -eq 0 ] || { echo "step failed ($rc) -- stopping"; exit $rc; }
}
BENCH="python3 bench.py $*"
run 300 $OUT/bench.json $BENCH   # (stderr interleaved; make_profiles.py keeps the JSON line)
run 400 $OUT/ktrace.log rocprofv3 -M --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $*
run 300 $OUT/pmc_fetch.log rocprofv3 -M --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --n-timesteps 2 $*
run 300 $OUT/pmc_write.log rocprofv3 -M --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pmc -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --n-timesteps 2 $*
run 300 $OUT/pmc_sq.log rocprofv3 -M --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_sq -o pmc -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --n-timesteps 2 $*
run 300 $OUT/pmc_sq2.log rocprofv3 -M --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES --output-format csv -d $OUT/pmc_sq2 -o pmc -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --n-timesteps 2 $*
echo done
