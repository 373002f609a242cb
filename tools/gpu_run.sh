#!/bin/bash
# GPU round trip used during development: the -m gpu suite (achieved parity errors appended to
# gpurun_out/parity.jsonl), then the default bench. Each GPU step has its own time limit; a failing step
# ends the script.   usage (through gpurun): bash tools/gpu_run.sh [pytest -k expression]
mkdir -p gpurun_out
export GRADTTS_PARITY_LOG=gpurun_out/parity.jsonl
rm -f $GRADTTS_PARITY_LOG
K=${1:+-k "$1"}
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread $K > gpurun_out/pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print(round(d['value']), 'mel-frames/s', round(d['ms_per_step'],2), 'ms', d['roofline']['kernel'], round(d['roofline']['frac'],4))"
