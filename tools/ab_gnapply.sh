timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pt.log 2>&1; echo pytest=$?; tail -2 gpurun_out/pt.log
mkdir -p gpurun_out/var
for v in 100000 256 128 64; do
  GT_GN_APPLY_MIN_C=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --n-timesteps 10 > gpurun_out/var/gn$v.json 2>/dev/null || exit 1
done
python3 - <<'PY'
import json
for v in [100000, 256, 128, 64]:
    d = json.load(open(f"gpurun_out/var/gn{v}.json"))
    sh = {k: x["avg_us"] for k, x in d["shapes"].items() if ("0,2,0" in k or "0,3,0" in k or "gn_apply" in k)}
    print(v, round(d["ms_per_step"], 2), sh)
PY
