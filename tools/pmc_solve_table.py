"""Per-kernel time and PMC bytes per k26w SSSP from one round cycle (tools/cycle.sh kt + pmc layout):
launches and time per solve from the bench's kernel trace (TAG/kt, solves = v2_init_k launches),
2*FETCH_SIZE + WRITE_SIZE per solve from the traffic_probe passes (TAG/pmc_FETCH_SIZE,
TAG/pmc_WRITE_SIZE, solves = v2_init_k dispatches). Usage: python tools/pmc_solve_table.py gpurun_out/TAG"""
import csv, glob, os, sys
from collections import defaultdict

root = sys.argv[1]


def short(n):
    return n.replace("pj::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40]


dur, calls, solves_t = defaultdict(float), defaultdict(int), 0
for r in csv.DictReader(open(glob.glob(os.path.join(root, "kt", "*kernel_trace.csv"))[0])):
    k = short(r["Kernel_Name"])
    dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    calls[k] += 1
    solves_t += k == "v2_init_k"
byt, solves_p = defaultdict(float), {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    n = 0
    for p in glob.glob(os.path.join(root, f"pmc_{c}", "*counter_collection.csv")):
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"])
            n += k == "v2_init_k"
            byt[(k, c)] += float(r["Counter_Value"])
    solves_p[c] = max(n, 1)
solve_kernels = [k for k in dur if k.startswith("v2_") or k == "unlabel_k"]
solve_kernels = [k for k in solve_kernels if not any(x in k for x in ("interleave", "light_csr", "long_", "wmax",
                                                                          "haslight", "w8", "bin_r2"))]
print(f"# per k26w SSSP: {solves_t} solves in the kernel trace, {solves_p['FETCH_SIZE']} in the PMC passes")
print(f"{'kernel':40s} {'launches':>8s} {'ms':>7s} {'GB':>7s} {'GB/s':>7s} {'of 8TB/s':>8s}")
tt, tb = 0.0, 0.0
for k in sorted(solve_kernels, key=lambda k: -dur[k]):
    t = dur[k] / max(solves_t, 1)
    b = (2 * byt[(k, "FETCH_SIZE")] / solves_p["FETCH_SIZE"] + byt[(k, "WRITE_SIZE")] / solves_p["WRITE_SIZE"]) * 1024
    tt, tb = tt + t, tb + b
    print(f"{k:40s} {calls[k] / max(solves_t, 1):8.1f} {t * 1e3:7.3f} {b / 1e9:7.2f} {b / 1e9 / t if t else 0:7.0f}"
          f" {b / t / 8e12 if t else 0:8.2f}")
print(f"{'all solve kernels':40s} {'':8s} {tt * 1e3:7.3f} {tb / 1e9:7.2f} {tb / 1e9 / tt:7.0f} {tb / tt / 8e12:8.2f}")
