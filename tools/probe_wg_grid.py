"""Grid sweep of BFS options on the web-Google-shaped graph (source 0): python tools/probe_wg_grid.py key=v1,v2 ..."""
import itertools, os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import numpy as np
import paralleljohnson_amd as pj
ctx = pj.Context(0)
g = ctx.generate_webgraph()
axes = [(a.split("=")[0], [float(x) for x in a.split("=")[1].split(",")]) for a in sys.argv[1:]]
g.sssp(0, copy=False)
ref = g.copy_dist()
for combo in itertools.product(*[v for _, v in axes]):
    for (k, _), v in zip(axes, combo):
        g.set_option(k, v)
    ms = []
    for _ in range(7):
        g.sssp(0, copy=False)
        ms.append(g.stats()["kernel_ms"])
    s = g.stats()
    ok = (g.copy_dist() == ref).all()
    tag = " ".join(f"{k}={v:g}" for (k, _), v in zip(axes, combo))
    print(f"{tag}: median {np.median(ms) * 1e3:.0f} us levels {s['levels']} td/bu {s['td_levels']}/{s['bu_levels']} {'ok' if ok else 'MISMATCH'}", flush=True)
