"""One-line summary of a bench.py output file (same-box A/B runs): value, ms/step, the top kernels' avg µs."""
import json
import sys

d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
top = sorted(d["kernels"].items(), key=lambda kv: -kv[1]["share"])[:8]
print(sys.argv[2] if len(sys.argv) > 2 else "", round(d["value"]), round(d["ms_per_step"], 2),
      {k.replace("conv_kernel", "ck").replace("<bf16,", "<"): v["avg_us"] for k, v in top})
