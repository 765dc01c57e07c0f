"""Per-kernel bytes and bandwidth from tools/pmc_kernels.sh output: 2*FETCH_SIZE + WRITE_SIZE
(KB units, MI355X_MICROARCH.md HBM section) against the kernel-trace durations.
Usage: python tools/pmc_kernel_table.py gpurun_out/TAG"""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
def short(n):
    return n.replace("pj::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:44]
dur = defaultdict(float); calls = defaultdict(int)
for r in csv.DictReader(open(glob.glob(os.path.join(root, "kt", "*kernel_trace.csv"))[0])):
    k = short(r["Kernel_Name"]); dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9; calls[k] += 1
cnt = defaultdict(lambda: defaultdict(float))
for p in glob.glob(os.path.join(root, "p*", "*counter_collection.csv")):
    for r in csv.DictReader(open(p)):
        cnt[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
rows = []
for k, c in cnt.items():
    b = (2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024
    rows.append((dur.get(k, 0), k, b))
print(f"{'kernel':44s} {'calls':>6s} {'time_ms':>9s} {'GB':>8s} {'GB/s':>8s}")
for t, k, b in sorted(rows, reverse=True)[:20]:
    print(f"{k:44s} {calls.get(k, 0):6d} {t * 1e3:9.2f} {b / 1e9:8.2f} {b / 1e9 / t if t else 0:8.0f}")
