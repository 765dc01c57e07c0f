"""Grid sweep of libpj graph options on weighted Kronecker (bench roots):
python tools/probe_grid.py SCALE key1=v1,v2 key2=v3,v4 ..."""
import itertools, os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import numpy as np
import paralleljohnson_amd as pj
ctx = pj.Context(0)
scale = int(sys.argv[1])
axes = [(a.split("=")[0], [float(x) for x in a.split("=")[1].split(",")]) for a in sys.argv[2:]]
g = ctx.generate_kronecker(scale, 16, 1, weighted=True)
roots = [int(r) for r in g.sample_roots(2, 6)]
g.sssp(roots[0], copy=False)
ref = None
for combo in itertools.product(*[v for _, v in axes]):
    for (k, _), v in zip(axes, combo):
        g.set_option(k, v)
    ms = []
    for r in roots:
        g.sssp(r, copy=False)
        s = g.stats()
        ms.append(s["kernel_ms"])
    d = g.copy_dist()
    chk = int(np.sum(d[d < 100000].astype(np.int64)))
    if ref is None:
        ref = chk
    tag = " ".join(f"{k}={v:g}" for (k, _), v in zip(axes, combo))
    print(f"{tag}: mean {np.mean(ms):.2f} ms {[round(x, 2) for x in ms]} bands {s['levels']} rounds {s['relax_rounds']} "
          f"push/pull {s['td_levels']}/{s['bu_levels']} chk {'ok' if chk == ref else 'MISMATCH'}", flush=True)
