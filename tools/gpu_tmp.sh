timeout -k 10 900 python3 -u -m pytest tests/test_decoder_gpu.py tests/test_fp8_gpu.py tests/test_small_batch_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
AB_ROWS=8 bash tools/ab_variants.sh nopair tree nopair tree
