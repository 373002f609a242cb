#!/bin/bash
# Same-box comparison of the in-tree build ("tree") and ab/<name> builds at the default bench config,
# alternating twice. usage: tools/ab_variants_full.sh name...
mkdir -p gpurun_out/abf
for r in 1 2; do
  for v in tree "$@"; do
    if [ "$v" = tree ]; then unset GRADTTS_LIB; else export GRADTTS_LIB=$PWD/ab/$v/libgradtts.so; fi
    timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/abf/b_${v}_${r}.json 2>/dev/null || exit 1
    python3 tools/ab_summary.py gpurun_out/abf/b_${v}_${r}.json $v || exit 1
  done
done
