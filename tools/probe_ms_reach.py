"""How much of a multi-source pass's pull work goes to vertices that no source of the pass reaches:
per 512-source pass of configs[4] (the 1024 smallest ids with out-degree >= 1), the vertices
reached by none / some / all of the pass's sources and their in-edges.
Usage: python tools/probe_ms_reach.py"""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import paralleljohnson_amd as pj

INF = 100000  # PJ_INT_INF
ctx = pj.Context(0)
g = ctx.generate_webgraph(916428, 5105039, 1)
row, col = g.get_csr()[:2]
n = g.n
deg = np.diff(row)
src = np.nonzero(deg > 0)[0][:1024]
indeg = np.bincount(col, minlength=n)
print(f"n {n} m {col.size}", flush=True)
for p in range(2):
    s = src[512 * p: 512 * (p + 1)]
    d = g.sssp_batch(s)
    reached = (d < INF)
    cnt = reached.sum(axis=0)
    none, all_ = cnt == 0, cnt == len(s)
    some = ~none & ~all_
    levels = int(d[reached].max())
    for tag, m in (("none", none), ("some", some), ("all", all_)):
        print(f"pass {p}: reached by {tag}: {int(m.sum())} vertices, {int(indeg[m].sum())} in-edges "
              f"({indeg[m].sum() / col.size:.3f} of m)", flush=True)
    # unit pull work bound: per vertex, the levels it holds a need bit (from level 1 to the last
    # level at which some source of the pass reaches it, or to the end if some never does)
    last = np.where(reached, d, -1).max(axis=0)
    hold = np.where(cnt < len(s), levels, last)
    print(f"pass {p}: levels {levels}; sum over vertices of in-degree x levels with a need bit: "
          f"{int((indeg * hold).sum())}, of which unreached-by-all vertices {int((indeg * hold)[none].sum())}",
          flush=True)
