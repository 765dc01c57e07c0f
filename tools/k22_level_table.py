"""The per-level table of configs[1] from tools/cycle.sh `klevels` (tools/k22_levels.py under a
kernel trace and --pmc passes): each logged bfs_level_k launch (level, push / pull, frontier,
edges scanned) beside its kernel time and its DRAM-side bytes (calibrated as
tools/pmc_solve_table.py: (RDREQ - RDREQ_32B) x bytes_per_request + RDREQ_32B x 32 + WRITE_SIZE;
2 x FETCH_SIZE + WRITE_SIZE beside it). Launches are matched in dispatch order: the workspace
solve's launches come first and are skipped (the log names every launch of the logged solves).
Usage: python tools/k22_level_table.py gpurun_out/TAG [calibration.json]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

root = sys.argv[1]
cal = json.load(open(sys.argv[2] if len(sys.argv) > 2 else os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r06", "gather_calib.json")))
bpr = cal["bytes_per_request"]

solves, cur = [], None
for ln in open(os.path.join(root, "klevels.log")):
    if ln.startswith("solve root"):
        cur = {"root": int(ln.split()[2]), "launches": []}
        solves.append(cur)
    elif ln.startswith("level_launch") and cur is not None:
        f = ln.split()
        kv = dict(zip(f[2::2], f[3::2]))
        cur["launches"].append(kv)
    elif ln.startswith("solve_done") and cur is not None:
        f = ln.split()
        cur.update(dict(zip(f[3::2], f[4::2])))


def dispatches(path, name="bfs_level_k"):
    rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
    return rows


kt = dispatches(glob.glob(os.path.join(root, "klkt", "**", "*kernel_trace.csv"), recursive=True)[0])
kt.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3 for r in kt]
ctr = defaultdict(dict)  # counter -> dispatch index -> value
for p in glob.glob(os.path.join(root, "klpmc_*", "**", "*counter_collection.csv"), recursive=True):
    rows = [r for r in csv.DictReader(open(p)) if "bfs_level_k" in r["Kernel_Name"]]
    byc = defaultdict(list)
    for r in rows:
        byc[r["Counter_Name"]].append((int(r.get("Dispatch_Id", 0)), float(r["Counter_Value"])))
    for c, v in byc.items():
        v.sort()
        ctr[c] = [x for _, x in v]
total_logged = sum(len(s["launches"]) for s in solves)
skip = len(dur) - total_logged  # the workspace solve's launches
print(f"# configs[1] Kronecker s22 unit-weight BFS, per level launch ({len(solves)} roots; "
      f"{skip} unlogged launches of the workspace solve skipped); DRAM bytes = (RDREQ - RDREQ_32B) x {bpr:.0f} + "
      f"RDREQ_32B x 32 + WRITE_SIZE; scanned = push: frontier out-edges, pull: in-edge probes")
print(f"{'root':>9s} {'lvl':>3s} {'kind':>6s} {'from':>6s} {'frontier':>9s} {'f_edges':>10s} {'scanned':>10s} "
      f"{'us':>7s} {'DRAM MB':>8s} {'2F+W MB':>8s} {'GB/s':>6s}")
i = skip
agg = defaultdict(lambda: [0, 0.0, 0.0, 0.0])
for s in solves:
    L = s["launches"]
    for j, e in enumerate(L):
        # a pull level's probes are logged by the next launch (prev_scanned); a push level scans its frontier edges
        kind = e["mode"] if e["frontier_from"] not in ("end", "idle") else e["frontier_from"]
        scanned = int(e["frontier_edges"]) if kind == "push" else (int(L[j + 1]["prev_scanned"]) if j + 1 < len(L) else 0)
        if e["frontier_from"] == "small":
            kind, scanned = "small", int(e["frontier_edges"])
        t = dur[i] if i < len(dur) else float("nan")
        rq = ctr.get("TCC_EA0_RDREQ_sum", [])
        r32 = ctr.get("TCC_EA0_RDREQ_32B_sum", [])
        wr = ctr.get("WRITE_SIZE", [])
        fs = ctr.get("FETCH_SIZE", [])
        dram = ((rq[i] - r32[i]) * bpr + r32[i] * 32 + wr[i] * 1024) if i < min(len(rq), len(r32), len(wr)) else float("nan")
        f2w = (2 * fs[i] + wr[i]) * 1024 if i < min(len(fs), len(wr)) else float("nan")
        print(f"{s['root']:9d} {e['level']:>3s} {kind:>6s} {e['frontier_from']:>6s} {int(e['frontier']):9d} "
              f"{int(e['frontier_edges']):10d} {scanned:10d} {t:7.1f} {dram / 1e6:8.2f} {f2w / 1e6:8.2f} "
              f"{dram / 1e3 / t if t else 0:6.0f}")
        a = agg[kind]
        a[0] += 1
        a[1] += t
        a[2] += dram
        a[3] += scanned
        i += 1
    print(f"{'':9s} solve: kernel_ms {s.get('kernel_ms')} levels {s.get('levels')} push {s.get('push')} pull "
          f"{s.get('pull')} scanned_edges {s.get('scanned_edges')} reached_edges {s.get('reached_edges')}")
print("# per kind over all roots: launches, us, DRAM MB, scanned M")
for k, (c, t, b, sc) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k:>6s} {c:4d} {t:9.1f} {b / 1e6:9.1f} {sc / 1e6:9.2f}")
