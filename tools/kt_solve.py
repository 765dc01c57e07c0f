"""Per-kernel timeline of the last solve in a rocprofv3 kernel trace.
Usage: python tools/kt_solve.py run_kernel_trace.csv START_KERNEL END_KERNEL [max_lines]"""
import csv, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
start, end = sys.argv[2], sys.argv[3]
mx = int(sys.argv[4]) if len(sys.argv) > 4 else 60
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if start in r["Kernel_Name"]]
j = idx[-1]
t0 = int(rows[j]["Start_Timestamp"])
tot = defaultdict(float)
n = 0
while j < len(rows) and end not in rows[j]["Kernel_Name"]:
    r = rows[j]
    nm = r["Kernel_Name"].replace("pj::(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot[nm] += d
    if n < mx:
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {d:8.1f} {nm}")
    n += 1
    j += 1
print("span", (int(rows[j - 1]["End_Timestamp"]) - t0) / 1e3, "us")
for k, v in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"  {k:50s} {v:9.1f} us")
