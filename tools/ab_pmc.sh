#!/bin/bash
# A/B counter pass: bench (N=2 timesteps) under rocprofv3 PMC sets, for the in-tree library and an
# alternative one (GRADTTS_LIB). usage: tools/ab_pmc.sh <tag> <libpath|default>
set -u
TAG=$1; LIBP=$2
OUT=gpurun_out/ab_$TAG; mkdir -p $OUT
if [ "$LIBP" != "default" ]; then export GRADTTS_LIB=$PWD/$LIBP; fi
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() { local lim=$1 log=$2; shift 2; timeout -k 10 $lim "$@" > $log 2>&1; local rc=$?; echo "[$rc] $*" | cut -c1-160
  case $rc in 0) ;; *) echo "exit $rc -- stopping"; exit $rc;; esac; }
B="python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --n-timesteps 2"
run 200 $OUT/bench.log python3 bench.py --no-cpu-baseline --steps 3 --warmup 1
run 300 $OUT/pa.log rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pa -o pmc -- $B
run 300 $OUT/pb.log rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU --output-format csv -d $OUT/pb -o pmc -- $B
run 300 $OUT/pc.log rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_BUSY_CU_CYCLES SQ_INST_LEVEL_LDS --output-format csv -d $OUT/pc -o pmc -- $B
echo done
