"""Sum rocprofv3 --pmc counters over the dispatches of kernels matching any PATTERN, per solve.
Usage: python tools/traffic_sum.py OUTDIR SOLVES PATTERN [PATTERN...] > json
OUTDIR holds one sub-directory per pass (each with *counter_collection.csv).
A PATTERN starting with '!' excludes matching kernels (one-off workspace builds)."""
import csv, glob, json, os, sys
from collections import defaultdict
root, solves, args = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
pats = [a for a in args if not a.startswith("!")]
excl = [a[1:] for a in args if a.startswith("!")]
tot = defaultdict(float)
disp = defaultdict(set)
for p in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(p)):
        if not any(pt in r["Kernel_Name"] for pt in pats) or any(x in r["Kernel_Name"] for x in excl):
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add(r["Dispatch_Id"])
res = {k: v / solves for k, v in tot.items()}
res["dispatches_per_solve"] = {k: len(v) / solves for k, v in disp.items()}
res["patterns"] = pats
res["excluded"] = excl
# MI355X_MICROARCH.md §HBM: FETCH_SIZE (kB) reports 1/2 of wide streaming reads on gfx950 -> x2;
# WRITE_SIZE (kB) is exact for streaming stores. Random 4-byte gathers are uncalibrated: the
# uncorrected sum is kept beside the corrected one.
if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
    res["hbm_bytes_per_sssp"] = 1024.0 * (2.0 * res["FETCH_SIZE"] + res["WRITE_SIZE"])
    res["hbm_bytes_per_sssp_uncorrected"] = 1024.0 * (res["FETCH_SIZE"] + res["WRITE_SIZE"])
print(json.dumps(res, indent=1))
