"""Time per light-round kind of k26w solves: the stats_probe.py log with round_log=1 (one stderr
line per v2_pull_round_k launch: kind push / dense / pull / empty, frontier, its light edges)
matched launch by launch with a rocprofv3 kernel trace of the same run (v2_pull_round_k and the
v2_hub_k<true> launch after it). Usage: python tools/round_kinds.py probe.log run_kernel_trace.csv"""
import csv
import re
import sys
from collections import defaultdict

solves, cur = [], []
for ln in open(sys.argv[1]):
    m = re.match(r"round (\d+) lo (\d+) (\w+) frontier (\d+) light_edges (\d+)", ln)
    if m:
        cur.append((m.group(3), int(m.group(2)), int(m.group(4)), int(m.group(5))))
    elif ln.startswith("== solve root"):
        solves.append(cur)
        cur = []
rows = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
runs, hubs, run = [], [], None
for r in rows:
    nm = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "v2_init_k" in nm:
        run = []
        runs.append(run)
    elif "v2_pull_round_k" in nm and run is not None:
        run.append([d, 0.0])
    elif "v2_hub_k<true>" in nm and run:
        run[-1][1] = d
runs = runs[-len(solves):]
tot = defaultdict(lambda: [0, 0.0, 0.0, 0])
for sv, rn in zip(solves, runs):
    if len(sv) != len(rn):
        print(f"mismatch: {len(sv)} logged rounds, {len(rn)} launches")
        continue
    print(f"solve: {len(rn)} round launches, round kernels {sum(x[0] for x in rn):.1f} us, hub {sum(x[1] for x in rn):.1f} us")
    for (kind, lo, fr, le), (d, h) in zip(sv, rn):
        t = tot[kind]
        t[0] += 1
        t[1] += d
        t[2] += h
        t[3] += le
        if d + h > 40:
            print(f"  lo {lo:5d} {kind:5s} frontier {fr:9d} light_edges {le:10d}: round {d:8.1f} us, hub {h:7.1f} us")
n = max(1, len(solves))
print("per solve, by kind: launches, round kernel us, hub us, frontier light edges")
for k, t in sorted(tot.items()):
    print(f"  {k:5s} {t[0] / n:6.1f} {t[1] / n:9.1f} {t[2] / n:8.1f} {t[3] / n:12.0f}")
