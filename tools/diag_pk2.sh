#!/bin/bash
# packed-fp32 build (ab/pk): per-stage determinism at the bench shape (bf16, fp32), then same-box bench A/B
mkdir -p gpurun_out/pk
export GRADTTS_LIB=$PWD/ab/pk/libgradtts.so
timeout -k 10 300 python tools/diag_determinism.py bf16 > gpurun_out/pk/det_bf16.log 2>&1; echo "det bf16 rc=$?"; grep -c "identical=True" gpurun_out/pk/det_bf16.log; grep "identical=False" gpurun_out/pk/det_bf16.log | head -5
timeout -k 10 300 python -m pytest tests/test_configs_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pk/cfg.log 2>&1; echo "configs rc=$?"; tail -2 gpurun_out/pk/cfg.log
unset GRADTTS_LIB
bash tools/ab_variants_full.sh pk
