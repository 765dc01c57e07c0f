"""Group one solve's kernels between host syncs (copyBuffer = D2H of the control block).
Usage: python tools/trace_bands.py run_kernel_trace.csv [solve_index=-2] [marker=v2_source_k]"""
import csv, re, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
k = int(sys.argv[2]) if len(sys.argv) > 2 else -2
marker = sys.argv[3] if len(sys.argv) > 3 else "v2_source_k"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
i0 = idx[k]; i1 = idx[k + 1] if k + 1 < len(idx) and k != -1 else len(rows)
t0 = int(rows[i0]["Start_Timestamp"])
seg = defaultdict(float); segs = []; start = t0; n = 0
def short(nm):
    nm = nm.replace("pj::(anonymous namespace)::", "").replace("void ", "")
    nm = re.sub(r"<unsigned int>|<unsigned int, true>", "", re.sub(r"\(.*", "", nm))
    return nm.replace("__amd_rocclr_", "")
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    nm = short(r["Kernel_Name"])
    seg[nm] += (e - s) / 1e3; n += 1
    if nm == "copyBuffer":
        segs.append((start, e, n, dict(seg))); seg = defaultdict(float); start = e; n = 0
segs.append((start, int(rows[i1 - 1]["End_Timestamp"]), n, dict(seg)))
for s, e, n, d in segs:
    top = sorted(d.items(), key=lambda x: -x[1])[:4]
    print(f"{(s - t0) / 1e3:8.1f} span {(e - s) / 1e3:7.1f} n {n:3d} | " + " ".join(f"{a}={b:.0f}" for a, b in top))
