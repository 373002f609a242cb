# Small-batch tile plan: parity tests and a batch-size sweep of both plans (GT_SMALL_B=0: throughput plan only)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/sb_tests.log 2>&1 || exit 1
for B in 1 2 4; do
  for SB in 0 4; do
    GT_SMALL_B=$SB timeout -k 10 200 python bench.py --batch $B --n-timesteps 50 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/sb_b${B}_s${SB}.json 2>/dev/null || exit 1
  done
done
GT_GRAPHS=1 timeout -k 10 200 python bench.py --batch 1 --n-timesteps 50 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/sb_b1_graphs.json 2>/dev/null
