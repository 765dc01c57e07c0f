"""Summarise a rocprofv3 kernel trace: per-kernel stats and the timeline of the last dispatches."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
tail = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
agg = defaultdict(lambda: [0, 0])
def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0][:60]


for r in rows:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    k = short(r["Kernel_Name"])
    agg[k][0] += 1
    agg[k][1] += d
for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k:50s} calls {c:6d} total_us {t / 1e3:10.1f} avg_us {t / c / 1e3:9.2f}")
print("--- timeline (us from first shown, duration us)")
t0 = int(rows[-tail]["Start_Timestamp"])
for r in rows[-tail:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{short(r['Kernel_Name'])[:42]:42s} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} "
          f"vgpr {r['VGPR_Count']} sgpr {r['SGPR_Count']} grid {r['Grid_Size_X']}")
