#!/bin/bash
# same-box A/B of ab/<variant>/libgradtts.so against the in-tree build: decoder parity tests on the variant
# (GRADTTS_LIB), then alternating default-config bench runs. usage: tools/ab_variant.sh <variant>
V=$1
mkdir -p gpurun_out/abv
GRADTTS_LIB=$PWD/ab/$V/libgradtts.so timeout -k 10 300 python -u -m pytest tests/test_decoder_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/abv/pt_$V.log 2>&1; rc=$?
tail -2 gpurun_out/abv/pt_$V.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in tree $V; do
    if [ $v = tree ]; then unset GRADTTS_LIB; else export GRADTTS_LIB=$PWD/ab/$V/libgradtts.so; fi
    timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/abv/b_${v}_${r}.json 2>/dev/null || exit 1
    python3 tools/ab_summary.py gpurun_out/abv/b_${v}_${r}.json $v || exit 1
  done
done
