OUT=gpurun_out/c3w2; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_conv3w_gpu.py -x -q -s --timeout 200 --timeout-method thread > $OUT/pytest_c3w.log 2>&1; rc=$?
grep -E "PARITY|passed|failed" $OUT/pytest_c3w.log | tail -80; [ $rc -eq 0 ] || exit $rc
