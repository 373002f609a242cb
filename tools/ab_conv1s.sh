# conv1s (csrc/conv1s.hip) on the GPU box: its parity tests, then bench A/B against conv_kernel (GT_CONV1S=0) on the
# same box, two rounds; per-shape times of the 1x1 convs from each bench line.  usage: bash tools/ab_conv1s.sh
mkdir -p gpurun_out/c1s
timeout -k 10 400 python3 -u -m pytest tests/test_conv1s_gpu.py -v -rA --timeout 120 --timeout-method thread > gpurun_out/c1s/pytest.log 2>&1; rc=$?
grep -E "PARITY|PASSED|FAILED" gpurun_out/c1s/pytest.log | cut -c1-180 | head -80
[ $rc -eq 0 ] || { echo pytest failed; exit 1; }
for i in 1 2; do for v in 1 0; do
  GT_CONV1S=$v timeout -k 10 240 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c1s/bench_${v}_${i}.json 2>gpurun_out/c1s/bench_${v}_${i}.err || { echo bench failed; exit 1; }
  python3 -c "
import json,sys;d=json.loads(open('gpurun_out/c1s/bench_${v}_${i}.json').read().strip().splitlines()[-1])
print('c1s=$v', round(d['value']), round(d['ms_per_step'],2))
for k,x in d['shapes'].items():
  if 'conv1s' in k or 'conv_kernel<bf16,2,' in k: print('   ',k,x['avg_us'])
"
done; done
