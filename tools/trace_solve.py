"""Print the kernel timeline of one solve from a rocprofv3 kernel trace.
Usage: python tools/trace_solve.py run_kernel_trace.csv [solve_index=-2] [marker=v2_source_k] [max_rows]"""
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
k = int(sys.argv[2]) if len(sys.argv) > 2 else -2
marker = sys.argv[3] if len(sys.argv) > 3 else "v2_source_k"
mx = int(sys.argv[4]) if len(sys.argv) > 4 else 10**9
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
i0 = idx[k]
i1 = idx[k + 1] if k + 1 < len(idx) and k != -1 else len(rows)
t0 = prev = int(rows[i0]["Start_Timestamp"])
busy = 0
for n, r in enumerate(rows[i0:i1]):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    nm = r["Kernel_Name"].replace("pj::(anonymous namespace)::", "").replace("void ", "")
    nm = re.sub(r"\(.*", "", nm)
    busy += e - s
    if n < mx:
        print(f"{(s - t0) / 1e3:9.1f} gap {(s - prev) / 1e3:6.1f} dur {(e - s) / 1e3:7.1f} {nm[:60]}")
    prev = e
print(f"solve span {(prev - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, launches {i1 - i0}")
