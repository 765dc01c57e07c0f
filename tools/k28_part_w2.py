"""configs[3]'s exchange path on one GPU (as bench.py's k28_partitioned_host_w2): the s28 unit-weight
partition at world 2, both ranks in this process over the host transport, the bench's roots; ms per BFS
under part option sets, interleaved. Usage: python tools/k28_part_w2.py [scale=28] [passes=2]
[sets=pull_first=1+pull_first=0]  (a set: k=v/k=v...)"""
import os
import sys
import time

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import paralleljohnson_amd as pj  # noqa: E402
from paralleljohnson_amd.partition import Comm, bfs_group, load_kronecker  # noqa: E402

opts = dict(kv.split("=", 1) for kv in sys.argv[1:])
scale = int(opts.get("scale", "28"))
passes = int(opts.get("passes", "2"))
sets = [dict(kv.split("=") for kv in x.split("/")) for x in opts.get("sets", "pull_first=1+pull_first=0").split("+")]
ctxs = [pj.Context(0) for _ in range(2)]
comms = Comm.group(ctxs, "host")
parts = [load_kronecker(ctxs[r], scale, 16, 1, r, 2) for r in range(2)]
rng = np.random.default_rng(1 + 7)
roots = []
for c in rng.integers(0, 1 << scale, 64):
    st = bfs_group(parts, comms, int(c))
    if st[0]["reached"] > 1:
        roots.append(int(c))
    if len(roots) == 4:
        break
print("roots", roots, flush=True)
for ps in range(passes):
    for o in sets:
        for p in parts:
            for k, v in o.items():
                p.set_option(k, float(v))
        for r in roots:
            bfs_group(parts, comms, r)  # (warm)
        t = time.perf_counter()
        for r in roots:
            bfs_group(parts, comms, r)
        ms = 1e3 * (time.perf_counter() - t) / len(roots)
        print(f"pass {ps} {o} ms per BFS {ms:.3f}", flush=True)
for p in parts:
    p.close()
for c in comms:
    c.close()
