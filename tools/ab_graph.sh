mkdir -p gpurun_out/ab
for cfg in "--batch 32" "--batch 1 --n-timesteps 1000 --dtype bf16_w8 --steps 1 --warmup 1" "--batch 4 --n-timesteps 100 --steps 2 --warmup 1"; do
  for g in 1 0; do
    GT_GRAPHS=$g GRADTTS_BENCH_TIMED_EVENTS=0 timeout -k 10 300 python bench.py --no-cpu-baseline $cfg > gpurun_out/ab/b.json 2>gpurun_out/ab/err || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/b.json')); print(sys.argv[1], 'graphs', sys.argv[2], round(d['value']), 'mel-frames/s', round(d['ms_per_step'],2), 'ms')" "$cfg" $g
  done
done
