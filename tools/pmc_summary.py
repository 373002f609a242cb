"""Summarise rocprofv3 --pmc csv passes per kernel instantiation (sum over dispatches)."""
import csv, sys, glob, collections, re

def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for f in glob.glob(d + "/**/pmc_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            m = re.search(r"conv_kernel<([^>]*)>", k)
            k = ("conv<" + m.group(1) + ">") if m else k.split("(")[0].replace("void gt::", "")
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Counter_Name"] in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU"):
                n[(k, r["Counter_Name"])] += 1
    return agg

if __name__ == "__main__":
    root = sys.argv[1]
    a = load(root)
    keys = sorted(a, key=lambda k: -a[k].get("SQ_BUSY_CYCLES", 0))
    for k in keys[:12]:
        c = a[k]
        mf = c.get("SQ_INSTS_MFMA", 0) or 1
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        print(f"{k[:60]:60s} busy={c.get('SQ_BUSY_CYCLES',0):.3g} mfma_busy/busy_cu={c.get('SQ_VALU_MFMA_BUSY_CYCLES',0)/max(c.get('SQ_BUSY_CU_CYCLES',1),1):.3f} "
              f"valu/mfma={c.get('SQ_INSTS_VALU',0)/mf:.2f} lds/mfma={c.get('SQ_INSTS_LDS',0)/mf:.2f} bankconf/lds={c.get('SQ_LDS_BANK_CONFLICT',0)/max(c.get('SQ_INSTS_LDS',1),1):.2f} "
              f"wait_any/wave={c.get('SQ_WAIT_ANY',0)/wc:.2f} wait_inst/wave={c.get('SQ_WAIT_INST_ANY',0)/wc:.2f} active/wave={c.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} "
              f"waitlds/wave={c.get('SQ_WAIT_INST_LDS',0)/wc:.2f} vmem_act/wave={c.get('SQ_ACTIVE_INST_VMEM',0)/wc:.2f} valu_act/wave={c.get('SQ_ACTIVE_INST_VALU',0)/wc:.2f} lds_act/wave={c.get('SQ_ACTIVE_INST_LDS',0)/wc:.2f} salu/mfma={c.get('SQ_INSTS_SALU',0)/mf:.2f}")
