"""Aggregate rocprofv3 --pmc passes per kernel name (sum over dispatches).
Usage: python tools/pmc_agg.py DIR PATTERN [PATTERN...]"""
import csv, glob, os, sys
from collections import defaultdict
root, pats = sys.argv[1], sys.argv[2:]
agg = defaultdict(lambda: defaultdict(float))
for p in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(p)):
        nm = r["Kernel_Name"]
        for pt in pats:
            if pt in nm:
                agg[pt][r["Counter_Name"]] += float(r["Counter_Value"])
for pt in pats:
    a = agg[pt]
    wc = a.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"== {pt}")
    print("  " + "  ".join(f"{k}={v:.3g}" for k, v in sorted(a.items())))
    print(f"  wait_any/wave_cyc={a.get('SQ_WAIT_ANY', 0) / wc:.2f} wait_inst/wave_cyc={a.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} "
          f"active/wave_cyc={a.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} "
          f"tcc_hit={a.get('TCC_HIT_sum', 0) / max(1, a.get('TCC_HIT_sum', 0) + a.get('TCC_MISS_sum', 0)):.2f} "
          f"valu/vmem={a.get('SQ_INSTS_VALU', 0) / max(1, a.get('SQ_INSTS_VMEM', 0)):.1f}")
