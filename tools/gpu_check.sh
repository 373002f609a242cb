#!/bin/bash
# GPU round trip used during development: parity tests, then the default bench with per-kernel table.
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pt.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench.json"))
print(round(d["value"]), "mel-frames/s", round(d["ms_per_step"], 2), "ms/step", d["roofline"]["kernel"], round(d["roofline"]["frac"], 4))
for k, v in d["kernels"].items(): print(" ", k, v)
for k, v in list(d["shapes"].items())[:24]: print("   ", k, v)
PY
