"""Reproduce a pull-level parity failure and describe the mismatching vertices."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
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
    for r in roots:
        exp = O.bfs(row, col, r)
        for rep in range(3):
            g.set_option("direction", direction)
            d = g.sssp(r)
            bad = np.nonzero(d != exp)[0]
            st = g.stats()
            print(f"trial {trial} n {n} m {len(src)} root {r} rep {rep}: mismatches {len(bad)} levels {st['levels']} "
                  f"td/bu {st['td_levels']}/{st['bu_levels']}", flush=True)
            if len(bad):
                print("   sample idx", bad[:8], "got", d[bad[:8]], "exp", exp[bad[:8]])
                print("   got-exp histogram", np.unique(d[bad].astype(np.int64) - exp[bad], return_counts=True))
                print("   isolated?", [(row[v+1]-row[v]) for v in bad[:8]])
    g.close()
