#!/bin/bash
# Same-box A/B of the tree against ab/head: interleaved bench runs (tools/ab_variants.sh), the attention / attn_down
# tests, and one counter pass (LDS instructions and bank conflicts) per library. usage: tools/ab_lds.sh <tag>
set -u
TAG=${1:-lds}
OUT=gpurun_out/ab_$TAG; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_attn_down_gpu.py tests/test_decoder_gpu.py > $OUT/test.log 2>&1 || { tail -20 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
AB_ROWS=40 bash tools/ab_variants.sh tree head > $OUT/ab.txt 2>&1 || { cat $OUT/ab.txt; exit 1; }
grep -i "ms/step\|attn_fold\|attn_down\|attn_merge" $OUT/ab.txt
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in tree head; do
  if [ $v = tree ]; then unset GRADTTS_LIB; else export GRADTTS_LIB=$PWD/ab/head/libgradtts.so; fi
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_VALU --output-format csv -d $OUT/pmc_$v -o pmc -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --n-timesteps 2 > $OUT/pmc_$v.log 2>&1 || { echo pmc failed; exit 1; }
done
unset GRADTTS_LIB
python3 - $OUT <<'PY'
import csv, glob, collections, sys
for v in ("tree", "head"):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{sys.argv[1]}/pmc_{v}/**/pmc_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void gt::", "")
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, c in sorted(agg.items()):
        if "attn" in k:
            print(v, k[:50], "conflicts/LDS instr %.3f" % (c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_INSTS_LDS"], 1)))
PY
