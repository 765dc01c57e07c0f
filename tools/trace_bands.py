"""Group one solve's kernels between host syncs (v2_publish_k / copyBuffer: the control block to the host);
per segment: start, span, kernels, busy time, the idle gap before it, the top kernels.
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
seg = defaultdict(float); segs = []; start = t0; n = 0; busy = 0.0; prev_end = t0; gap = 0.0
def short(nm):
    nm = nm.replace("pj::(anonymous namespace)::", "").replace("void ", "")
    nm = re.sub(r"<unsigned int>|<unsigned int, true>", "", re.sub(r"\(.*", "", nm))
    return nm.replace("__amd_rocclr_", "")
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    nm = short(r["Kernel_Name"])
    if n == 0:
        gap = max(0.0, (s - prev_end) / 1e3)
    seg[nm] += (e - s) / 1e3; n += 1; busy += (e - s) / 1e3; prev_end = e
    if nm in ("copyBuffer", "v2_publish_k"):
        segs.append((start, e, n, busy, gap, dict(seg))); seg = defaultdict(float); start = e; n = 0; busy = 0.0
segs.append((start, int(rows[i1 - 1]["End_Timestamp"]), n, busy, gap, dict(seg)))
tot_gap = 0.0
for s, e, n, b, gp, d in segs:
    top = sorted(d.items(), key=lambda x: -x[1])[:4]
    tot_gap += gp
    print(f"{(s - t0) / 1e3:8.1f} span {(e - s) / 1e3:7.1f} n {n:3d} busy {b:7.1f} gap {gp:5.1f} | " +
          " ".join(f"{a}={c:.0f}" for a, c in top))
print(f"segments {len(segs)}, idle before segments {tot_gap:.1f} us, solve span {(prev_end - t0) / 1e3:.1f} us")
