"""Summarise a rocprofv3 kernel_stats.csv: per-kernel total/avg (optionally divided by a solve count).
Usage: python tools/kt_summary.py path/run_kernel_stats.csv [solves] [top]"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
div = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 14
for r in rows[:top]:
    name = r["Name"].replace("pj::(anonymous namespace)::", "").replace("void ", "")[:70]
    print(f"{name:70s} {int(r['Calls']) / div:8.1f} calls {float(r['TotalDurationNs']) / 1e6 / div:9.3f} ms "
          f"avg {float(r['AverageNs']) / 1e3:9.1f} us")
