#!/bin/bash
# MAS timing variants (ab/<name>/libgradtts.so) and the kernel trace of the a18 case; usage: tools/mas_ab.sh name...
set -e
mkdir -p gpurun_out/masab
for v in "$@"; do
  if [ "$v" = "tree" ]; then unset GRADTTS_LIB; else export GRADTTS_LIB=$PWD/ab/$v/libgradtts.so; fi
  timeout -k 10 120 python bench_mas.py --no-cpu-baseline > gpurun_out/masab/$v.json 2>/dev/null
  timeout -k 10 120 python bench_mas.py --ragged --no-cpu-baseline > gpurun_out/masab/${v}_rag.json 2>/dev/null
  python3 -c "import json;a=json.load(open('gpurun_out/masab/$v.json'));b=json.load(open('gpurun_out/masab/${v}_rag.json'));print('$v', round(a['ms_per_step']*1e3,1), round(b['ms_per_step']*1e3,1))"
done
unset GRADTTS_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/masab/prof -o mas --output-format csv -- python3 $GRAFT_REPO_ROOT/bench_mas.py --no-cpu-baseline > /dev/null 2>&1
cd $GRAFT_REPO_ROOT; find gpurun_out/masab/prof -name "*stats.csv" | head -3; cat $(find gpurun_out/masab/prof -name "*kernel_stats.csv" | head -1) | cut -c1-200
