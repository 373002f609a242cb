timeout -k 10 900 python3 -u -m pytest tests/test_attn_down_gpu.py tests/test_conv3w_gpu.py tests/test_fp8_gpu.py tests/test_decoder_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
AB_ROWS=12 bash tools/ab_variants.sh bar1 tree bar1 tree || exit 1
for v in "0 0" "0 1" "1 1"; do set -- $v; GT_ATTN_MF=$1 GT_ATTN_DS=$2 GRADTTS_BENCH_NO_FINITE_CHECK=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 3 --warmup 2 --n-timesteps 10 > gpurun_out/ab_$1$2.json 2>/dev/null || exit 1; python3 -c "
import json; d=json.load(open('gpurun_out/ab_$1$2.json')); print('MF=$1 DS=$2', round(d['ms_per_step'],2), 'ms/step', round(d['value']), {k[:24]:v['avg_us'] for k,v in d['shapes'].items() if 'attn_' in k and 'kv' not in k})"; done
for v in 0 1; do GT_ATTN_MF=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --batch 1 > gpurun_out/b1_$v.json 2>/dev/null || exit 1; python3 -c "
import json; d=json.load(open('gpurun_out/b1_$v.json')); print('B=1 MF=$v', round(d['ms_per_step'],2), 'ms/decode', round(d['value']))"; done
