bash tools/diag_w8det.sh || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_decoder_gpu.py tests/test_small_batch_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_c64.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pt_c64.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_c64.json 2> gpurun_out/bench_c64.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('gpurun_out/bench_c64.json')); print(round(d['value']), round(d['ms_per_step'],2)); [print(k, v) for k, v in d['shapes'].items() if 'conv64' in k]"
