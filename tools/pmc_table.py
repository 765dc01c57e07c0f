"""Join rocprofv3 --pmc passes into one per-dispatch table for one kernel name pattern.
Usage: python tools/pmc_table.py DIR_WITH_pN PATTERN [last_n_dispatches]"""
import csv, glob, os, sys
from collections import defaultdict
root, pat = sys.argv[1], sys.argv[2]
last = int(sys.argv[3]) if len(sys.argv) > 3 else 12
rows = defaultdict(dict)  # (pass, dispatch idx within pattern) -> counters
for p in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    d = defaultdict(dict)
    order = []
    for r in csv.DictReader(open(p)):
        if pat not in r["Kernel_Name"]:
            continue
        did = int(r["Dispatch_Id"])
        if did not in d:
            order.append(did)
        d[did][r["Counter_Name"]] = float(r["Counter_Value"])
    for i, did in enumerate(order[-last:]):
        rows[i].update(d[did])
keys = sorted({k for v in rows.values() for k in v})
print("idx " + " ".join(f"{k[:18]:>18s}" for k in keys))
for i in sorted(rows):
    print(f"{i:3d} " + " ".join(f"{rows[i].get(k, float('nan')):18.0f}" for k in keys))
