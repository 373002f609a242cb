#!/bin/bash
# Every BASELINE config on the current tree, one box: bench lines (roofline + CPU baseline of each workload) and the
# rocprofv3 kernel-trace summary of each. Each GPU step under its own limit; a failing step ends the script.
#   usage (through gpurun): bash tools/gpu_configs.sh <outdir-tag>     -> gpurun_out/<tag>/{c*.json, c*_kernel_stats.csv}
set -u
OUT=gpurun_out/${1:-configs}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() {   # run <name> <limit> <bench args...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -3 $OUT/$name.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', round(d['value'],1), d['unit'], round(d['ms_per_step'],2), 'ms/step', d['roofline']['kernel'], round(d['roofline']['frac'],3), 'cpu', round(d.get('cpu_baseline',{}).get('value',0),2))"
  timeout -k 10 $lim rocprofv3 -M --kernel-trace --stats --output-format csv -d $OUT/kt_$name -o kt -- python3 bench.py --no-cpu-baseline "$@" > $OUT/kt_$name.log 2>&1 || { echo "$name ktrace failed"; exit 1; }
  cp $(find $OUT/kt_$name -name "*kernel_stats.csv" | head -1) $OUT/${name}_kernel_stats.csv && rm -rf $OUT/kt_$name
}
run c2_bf16 300 --steps 5 --warmup 2
run c2_fp32 300 --steps 2 --warmup 1 --dtype fp32
run c3 400 --steps 2 --warmup 1 --batch 64 --n-spks 247 --n-timesteps 100
run c5_bf16_b32 400 --steps 1 --warmup 1 --n-timesteps 1000
run c5_w8_b32 400 --steps 1 --warmup 1 --n-timesteps 1000 --dtype bf16_w8
run c5_fp8_b32 400 --steps 1 --warmup 1 --n-timesteps 1000 --dtype fp8
run c5_w8_b1 300 --steps 1 --warmup 1 --n-timesteps 1000 --dtype bf16_w8 --batch 1
run c5_fp8_b1 300 --steps 1 --warmup 1 --n-timesteps 1000 --dtype fp8 --batch 1
run c5_bf16_b1 300 --steps 1 --warmup 1 --n-timesteps 1000 --batch 1
run c2_b1 300 --steps 5 --warmup 2 --batch 1
echo done
