for lib in ab/head/libgradtts.so grad-tts_amd/gradtts_amd/libgradtts.so; do
  for f in estimator_s247.npz estimator_s1.npz; do
    for dt in w8 bf16; do
      GRADTTS_LIB=$PWD/$lib timeout -k 10 120 python tools/diag_w8.py $f $dt 2>&1 | tail -1 || exit 1
    done
  done
done
