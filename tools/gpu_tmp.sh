timeout -k 10 600 python -u -m pytest tests/test_decoder_gpu.py tests/test_small_batch_gpu.py tests/test_configs_gpu.py tests/test_torch_ops_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_tree.log 2>&1; rc=$?; echo "tree tests rc=$rc: $(tail -1 gpurun_out/pt_tree.log)"; [ $rc -eq 0 ] || exit $rc
R=2 SHAPES=conv64,conv_kernel bash tools/ab_multi.sh base
