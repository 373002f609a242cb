#!/bin/bash
# SQ counters of the training step's kernels (one pass; tools/kstats_db.py-style summary by kernel).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 -M --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_train -o pmc -- python3 tools/train_step.py --steps 1 > gpurun_out/pmc_train.log 2>&1
