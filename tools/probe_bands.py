"""Per-band workload of a weighted solve: vertices settled, out-edges, light edges (w < delta).
Usage: python tools/probe_bands.py SCALE [delta=24] [nroots=2]"""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import numpy as np
import paralleljohnson_amd as pj
scale = int(sys.argv[1]); delta = int(sys.argv[2]) if len(sys.argv) > 2 else 24
nroots = int(sys.argv[3]) if len(sys.argv) > 3 else 2
ctx = pj.Context(0)
g = ctx.generate_kronecker(scale, 16, 1, weighted=True)
t = time.time()
row, col, w = g.get_csr()
deg = np.diff(row)
light = np.zeros(g.n, np.int64)
nz = deg > 0
lc = np.add.reduceat((w < delta).astype(np.int64), row[:-1][nz])
light[nz] = lc
del col
print(f"csr on host {time.time() - t:.1f}s n {g.n} nnz {g.nnz} light frac {light.sum() / g.nnz:.3f}", flush=True)
for r in [int(x) for x in g.sample_roots(2, nroots)]:
    d = g.sssp(r)
    s = g.stats()
    reach = d < 100000
    b = d[reach] // delta
    nb = int(b.max()) + 1
    cnt = np.bincount(b, minlength=nb)
    de = np.bincount(b, weights=deg[reach], minlength=nb)
    le = np.bincount(b, weights=light[reach], minlength=nb)
    print(f"root {r} deg {deg[r]} ms {s['kernel_ms']:.2f} reached {reach.sum()} max dist {d[reach].max()} bands {nb}")
    for i in range(nb):
        if cnt[i]:
            print(f"  band {i:3d} [{i * delta:5d},{(i + 1) * delta:5d}) verts {cnt[i]:10d} edges {int(de[i]):12d} light {int(le[i]):11d} maxdeg {int(deg[reach][b == i].max()):9d}")
    h = np.bincount(d[reach & (d < delta)], minlength=delta)
    print("  band0 dist histogram", h.tolist(), flush=True)
