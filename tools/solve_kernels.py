"""Per-solve kernel time by kernel from a rocprofv3 kernel trace of consecutive solves.
Usage: python tools/solve_kernels.py run_kernel_trace.csv [marker=v2_init_k] [names=pull_round,hub_k<true>,...]
One line per solve (a solve starts at each launch of the marker kernel): span, busy time and the
summed duration (us) of each named kernel (substring match)."""
import csv, re, sys

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else "v2_init_k"
names = (sys.argv[3] if len(sys.argv) > 3 else
         "v2_pull_round_k,v2_hub_k<true>,v2_hub_k<false>,v2_pull_k,v2_heavy_push_k,v2_select_k,unlabel_k").split(",")
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
print("solve  span_us  busy_us " + " ".join(f"{re.sub(r'^v2_', '', n)[:14]:>14}" for n in names))
for j, i0 in enumerate(idx):
    i1 = idx[j + 1] if j + 1 < len(idx) else len(rows)
    seg = rows[i0:i1]
    # the solve ends at its unlabel launch (later rows belong to the host's next steps)
    end = next((k for k, r in enumerate(seg) if "unlabel_k" in r["Kernel_Name"]), len(seg) - 1)
    seg = seg[:end + 1]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    per = []
    for n in names:
        per.append(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg if n in r["Kernel_Name"]))
    print(f"{j:5d} {(t1 - t0) / 1e3:8.1f} {busy / 1e3:8.1f} " + " ".join(f"{p / 1e3:14.1f}" for p in per))
