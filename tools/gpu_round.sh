#!/bin/bash
# Round-3 GPU check: the -m gpu suite (parity errors to gpurun_out/parity.jsonl), the default bench, and a 2-rank
# launch rehearsal of bench.py on the one GPU (gloo, shared device). Each step under its own time limit; a failing
# step ends the script.   usage (through gpurun): bash tools/gpu_round.sh [pytest -k expression]
mkdir -p gpurun_out
export GRADTTS_PARITY_LOG=gpurun_out/parity.jsonl
rm -f $GRADTTS_PARITY_LOG
K=${1:+-k "$1"}
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread $K > gpurun_out/pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print(round(d['value']), 'mel-frames/s', round(d['ms_per_step'],2), 'ms', d['roofline']['kernel'], round(d['roofline']['frac'],4), d.get('cpu_baseline',{}).get('value'))"
GRADTTS_BENCH_SHARED_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err
rc=$?; echo "2-rank rehearsal rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_2rank.err; exit $rc; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_2rank.json').read().strip().splitlines()[-1]); print('2-rank', d['n_gpus'], d['config']['global_batch'], round(d['value']))"
