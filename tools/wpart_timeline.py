"""GPU busy time against wall span of the weighted partition's solves, from a rocprofv3
kernel trace of tools/probe_wpart.py: per solve (split at the wp_seed_k launches) the span
from the first seed to the last kernel before the next solve, each stream's summed kernel
time, the union of all streams' busy intervals, and the kernels by name. Idle span (span -
union) is host-side time: waits, transport steps, launch gaps.
Usage: python tools/wpart_timeline.py <run_kernel_trace.csv> [world=2]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
world = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def name(r):
    n = re.sub(r"^void ", "", r["Kernel_Name"]).replace("pj::(anonymous namespace)::", "")
    return n.split("(")[0]


names = [name(r) for r in rows]
gen = [i for i, n in enumerate(names) if n == "wp_kron_count_k"]
# world 1 generates one block, world 2 two: the segment of this world starts at its first block
start = gen[1] if world > 1 and len(gen) > 1 else (gen[0] if gen else 0)
seg = rows[start:]
segn = names[start:]
seeds = [i for i, n in enumerate(segn) if n == "wp_seed_k"]
solves = [seeds[i:i + world] for i in range(0, len(seeds), world)]
print(f"world {world}: {len(solves)} solves")
tot = collections.defaultdict(float)
for si, grp in enumerate(solves):
    a = grp[0]
    b = solves[si + 1][0] if si + 1 < len(solves) else len(seg)
    part = seg[a:b]
    # the solve's kernels end with wp_reach_k (one per rank): drop what follows (unlabel, copies)
    reach = [j for j, r in enumerate(part) if name(r) == "wp_reach_k"]
    if len(reach) >= world:
        part = part[:reach[world - 1] + 1]
    t0 = min(int(r["Start_Timestamp"]) for r in part)
    t1 = max(int(r["End_Timestamp"]) for r in part)
    per_stream = collections.defaultdict(float)
    by_name = collections.defaultdict(lambda: [0, 0.0])
    iv = []
    for r in part:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        per_stream[r["Stream_Id"]] += (e - s) / 1e6
        by_name[name(r)][0] += 1
        by_name[name(r)][1] += (e - s) / 1e6
        iv.append((s, e))
    iv.sort()
    union, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                union += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        union += ce - cs
    span = (t1 - t0) / 1e6
    print(f"solve {si}: span {span:.3f} ms, busy union {union / 1e6:.3f} ms, idle {span - union / 1e6:.3f} ms, "
          f"launches {len(part)}, per stream {{{', '.join(f'{k}: {v:.3f}' for k, v in sorted(per_stream.items()))}}}")
    for k, (c, d) in by_name.items():
        tot[k] += d
for k, d in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"  {k:40s} {d / max(1, len(solves)):8.3f} ms per solve (both ranks)")
