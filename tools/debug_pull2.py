import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (R, os.path.join(R, "oracle"), os.path.join(R, "tests")):
    sys.path.insert(0, p)
import numpy as np
import oracle as O
import paralleljohnson_amd as pj
from helpers import random_graph

ctx = pj.Context(0)
direction, kind = 2, "uniform"
rng = np.random.default_rng(100 + 7 * direction + len(kind))
for trial in range(4):
    n = int(rng.integers(2, 60000))
    src, dst = random_graph(rng, kind, n)
    roots = [int(src[0]) if len(src) else 0, int(rng.integers(0, n)), n, -5]
g = ctx.load_coo(src, dst, n=n)
row, col, _ = O.coo2csr(src.astype(np.uint32), dst.astype(np.uint32), n)
crow, ccol, _ = O.coo2csr(dst.astype(np.uint32), src.astype(np.uint32), n)
r = 7305
exp = O.bfs(row, col, r)
g.set_option("direction", 2)
for L in range(1, 15):
    g.set_option("max_levels", L)
    d = g.sssp(r)
    e = np.where(exp <= L, exp, 100000)
    bad = np.nonzero(d != e)[0]
    print(f"L={L} levels {g.stats()['levels']} mismatches {len(bad)}", flush=True)
    if len(bad):
        for v in bad[:6]:
            ins = ccol[crow[v]:crow[v + 1]]
            print(f"  v {v} got {d[v]} exp {e[v]} indeg {len(ins)} in-nbr dists(gpu) {d[ins][:20].tolist()} word {v >> 6} bit {v & 63}")
        break
