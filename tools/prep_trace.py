"""Timeline of the k26w solver preparation from a rocprofv3 --kernel-trace --hip-trace run of
tools/stats_probe.py: kernels from the relabel's degree_k through the first v2_init_k, with the
HIP API calls longer than a threshold that fall in the same window (host-side gaps: allocations,
frees, synchronizations). Usage: python tools/prep_trace.py DIR [min_us=50]"""
import csv, glob, os, sys

d = sys.argv[1]
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 50.0
kt = list(csv.DictReader(open(glob.glob(os.path.join(d, "*kernel_trace.csv"))[0])))
ht = list(csv.DictReader(open(glob.glob(os.path.join(d, "*hip_api_trace.csv"))[0])))
kt.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    return n.replace("pj::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:44]


i0 = next(i for i, r in enumerate(kt) if "degree_k" in r["Kernel_Name"])
i1 = next(i for i, r in enumerate(kt) if i > i0 and "v2_init_k" in r["Kernel_Name"])
t0, t1 = int(kt[i0]["Start_Timestamp"]), int(kt[i1]["End_Timestamp"])
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", short(r["Kernel_Name"])) for r in kt[i0:i1 + 1]]
for r in ht:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e >= t0 and s <= t1 and (e - s) / 1e3 >= min_us:
        ev.append((s, e, "H", r["Function"]))
ev.sort()
busy = sum(e - s for s, e, k, _ in ev if k == "K")
print(f"# prep window {((t1 - t0) / 1e6):.2f} ms (degree_k start -> first v2_init_k end), kernels busy {busy / 1e6:.2f} ms; "
      f"HIP calls >= {min_us:.0f} us listed (H)")
for s, e, k, n in ev:
    print(f"{(s - t0) / 1e3:10.1f} us  {k}  {(e - s) / 1e3:9.1f} us  {n}")
