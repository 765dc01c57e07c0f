"""Per-kernel time, DRAM-side bytes and counted work per k26w SSSP from one round cycle
(tools/cycle.sh `wtable` layout), all three over the same command, tools/traffic_probe.py:
  TAG/wkt                   rocprofv3 kernel trace (time per kernel; solves = v2_init_k launches)
  TAG/wpmc_<group>          rocprofv3 --pmc passes: TCC_EA0_RDREQ_sum + TCC_EA0_RDREQ_32B_sum,
                            FETCH_SIZE, WRITE_SIZE (one group per run)
  TAG/probe_work.json       the probe's per-solve pj_stats: the device work counters per kernel
                            class and pj_build_id()
and the FETCH_SIZE calibration (tools/calib_table.py; default profiles/r06/gather_calib.json):
DRAM-side read bytes = (RDREQ - RDREQ_32B) x bytes_per_request + RDREQ_32B x 32.
Prints the table and writes TAG/traffic_k26w.json, the file bench.py reads for
roofline.traffic (stamped with the build id: bench.py reports traffic only for that build).
Usage: python tools/pmc_solve_table.py gpurun_out/TAG [calibration.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]
cal_path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))), "profiles", "r06", "gather_calib.json")
cal = json.load(open(cal_path))
bpr = cal["bytes_per_request"]
PEAK = 8e12
PREP = ("interleave", "light_csr", "light_tiles", "long_", "v2_w1_k", "v2_hw_k", "haslight")
WORK = {"v2_pull_round_k": "light_round", "v2_hub_k<true>": "light_hub", "v2_pull_k": "heavy_pull",
        "v2_heavy_push_k": "heavy_push"}  # (heavy_push includes v2_hub_k<false>, the push's hub segments)


def short(n):
    n = n.replace("pj::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    return n.replace("<unsigned int>", "").replace("<unsigned long long>", "")[:40]


def solve_kernel(k):
    return k.startswith("v2_") and not any(x in k for x in PREP)


dur, calls, solves_t = defaultdict(float), defaultdict(int), 0
for r in csv.DictReader(open(glob.glob(os.path.join(root, "wkt", "**", "*kernel_trace.csv"), recursive=True)[0])):
    k = short(r["Kernel_Name"])
    dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    calls[k] += 1
    solves_t += k == "v2_init_k"
ctr, solves_p = defaultdict(float), {}
for p in glob.glob(os.path.join(root, "wpmc_*", "**", "*counter_collection.csv"), recursive=True):
    grp = os.path.relpath(p, root).split(os.sep)[0]
    inits = set()
    for r in csv.DictReader(open(p)):
        k = short(r["Kernel_Name"])
        if k == "v2_init_k":
            inits.add(r.get("Dispatch_Id", len(inits)))
        ctr[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        solves_p[r["Counter_Name"]] = grp
    solves_p[grp] = max(len(inits), 1)
ns = {c: solves_p[g] for c, g in list(solves_p.items()) if isinstance(g, str)}
work = json.load(open(os.path.join(root, "probe_work.json")))
sol = work["solves"]
wk = {name: [sum(s["work_by_kernel"][name][j] for s in sol) / len(sol) for j in range(3)]
      for name in ("light_round", "light_hub", "heavy_pull", "heavy_push")}


def per_solve(k, c):
    return ctr[(k, c)] / ns[c] if c in ns else 0.0


rows, tot = [], defaultdict(float)
for k in sorted([k for k in dur if solve_kernel(k)], key=lambda k: -dur[k]):
    t = dur[k] / max(solves_t, 1)
    rq, r32 = per_solve(k, "TCC_EA0_RDREQ_sum"), per_solve(k, "TCC_EA0_RDREQ_32B_sum")
    rd = (rq - r32) * bpr + r32 * 32
    wr = per_solve(k, "WRITE_SIZE") * 1024
    fx2 = 2 * per_solve(k, "FETCH_SIZE") * 1024 + wr
    w = wk.get(WORK.get(k, ""), [0, 0, 0])
    if k == "v2_hub_k<false>":
        w = [0, 0, 0]  # (counted with v2_heavy_push_k)
    row = {"kernel": k, "launches": calls[k] / max(solves_t, 1), "ms": t * 1e3, "dram_bytes": rd + wr,
           "fetch_x2_bytes": fx2, "records": w[0], "probes": w[1], "work_bytes": w[2]}
    rows.append(row)
    for key in ("ms", "dram_bytes", "fetch_x2_bytes", "records", "probes", "work_bytes"):
        tot[key] += row[key]
n, nnz = work["n"], work["nnz"]
o = 4 if nnz < 2**31 else 8
fixed = sum(4 * n + s["reached"] * (12 + 2 * o) for s in sol) / len(sol)
model8d = sum(4 * n + s["reached"] * (12 + 2 * o) + s["reached_edges"] * 12 for s in sol) / len(sol)
t = tot["ms"] / 1e3
print(f"# per k26w SSSP ({solves_t} solves in the kernel trace, PMC passes {dict(sorted(ns.items()))} solves), "
      f"build {work['build_id']}; DRAM bytes = (RDREQ - RDREQ_32B) x {bpr:.1f} + RDREQ_32B x 32 + WRITE_SIZE; "
      f"work = device counters (records as stored + probes)")
print(f"{'kernel':32s} {'launch':>6s} {'ms':>7s} {'DRAM GB':>8s} {'of 8TB/s':>8s} {'records M':>9s} {'probes M':>8s} "
      f"{'work GB':>8s} {'work/8TB/s':>10s}")
for r in rows:
    tt = r["ms"] / 1e3
    print(f"{r['kernel']:32s} {r['launches']:6.1f} {r['ms']:7.3f} {r['dram_bytes'] / 1e9:8.2f} "
          f"{r['dram_bytes'] / tt / PEAK if tt else 0:8.2f} {r['records'] / 1e6:9.1f} {r['probes'] / 1e6:8.1f} "
          f"{r['work_bytes'] / 1e9:8.3f} {r['work_bytes'] / tt / PEAK if tt else 0:10.3f}")
print(f"{'all solve kernels':32s} {'':6s} {tot['ms']:7.3f} {tot['dram_bytes'] / 1e9:8.2f} "
      f"{tot['dram_bytes'] / t / PEAK:8.2f} {tot['records'] / 1e6:9.1f} {tot['probes'] / 1e6:8.1f} "
      f"{tot['work_bytes'] / 1e9:8.3f} {tot['work_bytes'] / t / PEAK:10.3f}")
print(f"# scanned-work model per solve: 4N + n_r(12 + 2*{o}) = {fixed / 1e9:.3f} GB, + work {tot['work_bytes'] / 1e9:.3f} "
      f"GB = {(fixed + tot['work_bytes']) / 1e9:.3f} GB over {tot['ms']:.3f} ms: frac "
      f"{(fixed + tot['work_bytes']) / t / PEAK:.4f}; SURVEY §8d model {model8d / 1e9:.2f} GB (frac_model "
      f"{model8d / t / PEAK:.4f}); DRAM-side {tot['dram_bytes'] / 1e9:.2f} GB (traffic_frac "
      f"{tot['dram_bytes'] / t / PEAK:.4f}); 2 x FETCH_SIZE + WRITE_SIZE {tot['fetch_x2_bytes'] / 1e9:.2f} GB")
out = {"build_id": work["build_id"], "calibration": os.path.relpath(cal_path, os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "bytes_per_request": bpr, "solves_kernel_trace": solves_t, "solves_pmc": ns,
    "ms_per_sssp_kernels": tot["ms"], "hbm_bytes_per_sssp": tot["dram_bytes"],
    "hbm_bytes_per_sssp_fetch_x2": tot["fetch_x2_bytes"], "work_bytes_per_sssp": tot["work_bytes"],
    "fixed_bytes_per_sssp": fixed, "model_8d_bytes_per_sssp": model8d, "scanned_edges_per_sssp": tot["records"],
    "probes_per_sssp": tot["probes"], "kernels": rows}
with open(os.path.join(root, "traffic_k26w.json"), "w") as f:
    json.dump(out, f, indent=1)
