"""The single-GPU BFS (bfs.hip) on configs[3]'s graph (Kronecker s28 ef16, unit weights, 2^33 entries),
for comparison with the world-1 partitioned leg (part.hip, secondary.k28_partitioned): the bench's roots
(sample_roots seed 4, 4 roots), mean / median kernel ms and GTEPS by the reached edges.
Usage: python tools/k28_bfs_time.py [scale=28] [rootlist=a/b/..] [key=value ...]  (libpj graph options;
rootlist: these roots instead)"""
import os
import sys
import time

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import paralleljohnson_amd as pj  # noqa: E402

opts = dict(kv.split("=") for kv in sys.argv[1:])
scale = int(opts.pop("scale", "28"))
rootlist = opts.pop("rootlist", "")
ctx = pj.Context(0)
t0 = time.time()
g = ctx.generate_kronecker(scale, 16, 1)
print(f"s{scale}: n {g.n} nnz {g.nnz} built in {time.time() - t0:.2f} s", flush=True)
for k, v in opts.items():
    g.set_option(k, float(v))
roots = [int(x) for x in rootlist.split("/")] if rootlist else [int(r) for r in g.sample_roots(4, 4)]
g.sssp(roots[0], copy=False)  # (workspace)
ts, te = [], []
for rep in range(3):
    for r in roots:
        g.sssp(r, copy=False)
        st = g.stats()
        ts.append(st["kernel_ms"])
        rs = g.reach_stats()
        te.append(rs["reached_edges"])
        if rep == 0:
            print(f"root {r} kernel_ms {st['kernel_ms']:.3f} levels {st['levels']} td/bu {st['td_levels']}/{st['bu_levels']} "
                  f"reached {rs['reached']} m_r {rs['reached_edges']}", flush=True)
ts = np.array(ts)
print(f"s{scale} bfs.hip: mean kernel_ms {ts.mean():.3f} median {np.median(ts):.3f} "
      f"GTEPS(m_r) {np.mean(te) / ts.mean() / 1e6:.1f}", flush=True)
g.close()
