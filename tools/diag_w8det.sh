#!/bin/bash
# W8 (fp8-weight) run-to-run determinism with the packed-fp32 build (ab/pk): per GroupNorm partial slot (which
# producer's statistics differ), then per U-Net stage.
mkdir -p gpurun_out/w8det
export GRADTTS_LIB=$PWD/ab/pk/libgradtts.so
B=${B:-32} T=${T:-512} SLOTS=${SLOTS:-24} timeout -k 10 300 python tools/diag_parts.py w8 > gpurun_out/w8det/parts_pk.log 2>&1
rc=$?; echo "parts rc=$rc"; grep -c "differing per rep \[0, 0, 0\]" gpurun_out/w8det/parts_pk.log; grep -v "\[0, 0, 0\]" gpurun_out/w8det/parts_pk.log | head -5; [ $rc -eq 0 ] || exit $rc
B=32 T=512 timeout -k 10 300 python tools/diag_determinism.py w8 > gpurun_out/w8det/stages_pk.log 2>&1
rc=$?; echo "stages rc=$rc"; echo "identical stages: $(grep -c 'identical=True' gpurun_out/w8det/stages_pk.log) of $(grep -c identical gpurun_out/w8det/stages_pk.log)"
exit $rc
