"""Level profile of the web-Google-shaped graph (configs[0]) from source 0: per level the
frontier size, its out-edges, the unvisited vertices and their in-edges (what push and pull
levels would scan), the direction the solver chose, and kernel time by forced direction."""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import paralleljohnson_amd as pj

ctx = pj.Context(0)
g = ctx.generate_webgraph()
row, col, _ = g.get_csr()
n = g.n
d = g.sssp(0)
outdeg = np.diff(row)
indeg = np.bincount(col, minlength=n)
L = int(d[d < 100000].max())
unv_in = int(indeg.sum())
modes = []
prev = (0, 0)
for k in range(1, L + 3):
    g.set_option("max_levels", k)
    g.sssp(0, copy=False)
    st = g.stats()
    cur = (st["td_levels"], st["bu_levels"])
    modes.append("push" if cur[0] > prev[0] else ("pull" if cur[1] > prev[1] else "-"))
    prev = cur
g.set_option("max_levels", 0)
print("level  frontier  out_edges   unvisited  unv_in_edges  mode")
unvisited = n
unv_in = int(indeg.sum())
for l in range(L + 1):
    f = d == l
    print(f"{l:5d} {int(f.sum()):9d} {int(outdeg[f].sum()):10d} {unvisited:11d} {unv_in:13d}  {modes[l] if l < len(modes) else '?'}")
    unvisited -= int(f.sum())
    unv_in -= int(indeg[f].sum())
for name, kv in (("auto", {}), ("push", {"direction": 1}), ("pull", {"direction": 2})):
    for k, v in kv.items():
        g.set_option(k, v)
    ts = []
    for _ in range(6):
        g.sssp(0, copy=False)
        ts.append(g.stats()["kernel_ms"])
    print(name, "kernel_ms", np.round(ts, 4).tolist(), g.stats())
    g.set_option("direction", 0)
