#!/bin/bash
# PMC counters for the kernels matching a regex, from a short bench (2 U-Net evaluations). Separate passes (one
# rocprofv3 run each, within the per-block slot limits).   usage: tools/pmc_kernels.sh <regex> <outdir> [bench args]
RE=$1; OUT=$2; shift 2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
B="python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --n-timesteps 2 $*"
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA" \
            "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 -M --kernel-include-regex "$RE" --pmc $pass --output-format csv -d $OUT/p$i -o pmc -- $B > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/p$i.log; exit $rc; }
done
python3 - $OUT <<'PY'
import csv, glob, collections, sys, re
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/p*/**/pmc_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void gt::", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":   # effective clock: GUI_ACTIVE is summed over the 8 XCDs
            agg[k]["_ns"] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
for k, c in agg.items():
    mf = c.get("SQ_INSTS_MFMA", 0) or 1; wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(k[:70])
    print("  " + " ".join(f"{x}={c[x]:.4g}" for x in sorted(c)))
    print(f"  valu/mfma={c['SQ_INSTS_VALU']/mf:.2f} lds/mfma={c['SQ_INSTS_LDS']/mf:.2f} salu/mfma={c['SQ_INSTS_SALU']/mf:.2f} "
          f"wait_any={c['SQ_WAIT_ANY']/wc:.2f} wait_inst={c['SQ_WAIT_INST_ANY']/wc:.2f} active={c['SQ_ACTIVE_INST_ANY']/wc:.2f} "
          f"valu_act={c['SQ_ACTIVE_INST_VALU']/wc:.2f} lds_act={c['SQ_ACTIVE_INST_LDS']/wc:.2f} vmem_act={c.get('SQ_ACTIVE_INST_VMEM',0)/wc:.2f} "
          f"mfma_busy/busy_cu={c['SQ_VALU_MFMA_BUSY_CYCLES']/max(c['SQ_BUSY_CU_CYCLES'],1):.3f} hbm_MB={(2*c.get('FETCH_SIZE',0)+c.get('WRITE_SIZE',0))/1024:.1f} "
          f"clock_GHz={c.get('GRBM_GUI_ACTIVE',0)/8/max(c.get('_ns',1),1):.3f} kernel_us={c.get('_ns',0)/1e3:.1f} "
          f"mfma_pipe_util={c['SQ_VALU_MFMA_BUSY_CYCLES']/1024/max(c.get('GRBM_GUI_ACTIVE',0)/8,1):.3f}")
PY
