# packed-fp32 build with the statistics accumulation kept out of packed ops (ab/pk2): every W8 stage identical
# across reps, and the W8 / bf16 / fp32 determinism and batch-invariance tests
mkdir -p gpurun_out/w8det
export GRADTTS_LIB=$PWD/ab/pk2/libgradtts.so
B=32 T=512 SLOTS=24 timeout -k 10 300 python tools/diag_parts.py w8 > gpurun_out/w8det/pk2_parts.log 2>&1 || exit 1
echo "pk2 slots identical: $(grep -c 'differing per rep \[0, 0, 0\]' gpurun_out/w8det/pk2_parts.log) of $(grep -c 'slot' gpurun_out/w8det/pk2_parts.log)"
B=32 T=512 timeout -k 10 300 python tools/diag_determinism.py w8 > gpurun_out/w8det/pk2_stages.log 2>&1 || exit 1
echo "pk2 identical stages: $(grep -c 'identical=True' gpurun_out/w8det/pk2_stages.log) of $(grep -c identical gpurun_out/w8det/pk2_stages.log)"
timeout -k 10 600 python -u -m pytest tests/test_decoder_gpu.py tests/test_small_batch_gpu.py tests/test_configs_gpu.py -q -k "determin or invariant or c5" --timeout 300 --timeout-method thread > gpurun_out/w8det/pk2_pytest.log 2>&1; rc=$?; echo "pk2 pytest rc=$rc"; tail -2 gpurun_out/w8det/pk2_pytest.log
