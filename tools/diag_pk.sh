#!/bin/bash
# Packed-fp32 determinism check (ab/pk = build without -packed-fp32-ops): GroupNorm partial slots and every stage
# across repeated identical runs, then the determinism / batch-invariance tests.
export GRADTTS_LIB=$PWD/ab/pk/libgradtts.so
mkdir -p gpurun_out/pk
timeout -k 10 300 python tools/diag_parts.py bf16 > gpurun_out/pk/parts_bf16.log 2>&1; echo "parts rc=$?"; tail -26 gpurun_out/pk/parts_bf16.log
timeout -k 10 300 python -m pytest tests/test_decoder_gpu.py -q -x -k "deterministic or every_stage" --timeout 120 --timeout-method thread > gpurun_out/pk/pt.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pk/pt.log
