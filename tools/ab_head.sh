# same-box A/B: full GPU tests on the new lib, then alternating bench runs (head vs new)
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pt.log 2>&1; rc=$?
tail -2 gpurun_out/ab/pt.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in head new; do
    if [ $v = head ]; then export GRADTTS_LIB=$PWD/ab/head/libgradtts.so; else unset GRADTTS_LIB; fi
    timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/ab/b_${v}_${r}.json 2>/dev/null || exit 1
    python3 tools/ab_summary.py gpurun_out/ab/b_${v}_${r}.json $v || exit 1
  done
done
