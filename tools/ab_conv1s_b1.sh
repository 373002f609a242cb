mkdir -p gpurun_out/c1s
timeout -k 10 400 python3 -u -m pytest tests/test_conv1s_gpu.py -v -rA --timeout 120 --timeout-method thread > gpurun_out/c1s/pytest_small.log 2>&1; rc=$?
grep -E "PASSED|FAILED" gpurun_out/c1s/pytest_small.log | cut -c1-150
[ $rc -eq 0 ] || { tail -30 gpurun_out/c1s/pytest_small.log; exit 1; }
for i in 1 2; do for v in 1 0; do
  GT_CONV1S=$v timeout -k 10 240 python3 bench.py --steps 5 --warmup 2 --batch 1 --no-cpu-baseline > gpurun_out/c1s/b1_${v}_${i}.json 2>gpurun_out/c1s/b1_${v}_${i}.err || { echo bench failed; tail -3 gpurun_out/c1s/b1_${v}_${i}.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/c1s/b1_${v}_${i}.json').read().strip().splitlines()[-1])
print('B=1 c1s=$v', round(d['value']), round(d['ms_per_step'],2))
for k,x in d['shapes'].items():
  if 'conv1s' in k or 'conv_kernel<bf16,2,' in k: print('   ',k,x['avg_us'], x['per_step'])
"
done; done
