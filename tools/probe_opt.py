"""Sweep one libpj graph option on weighted Kronecker: python tools/probe_opt.py SCALE KEY v1 v2 ..."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import numpy as np
import paralleljohnson_amd as pj
ctx = pj.Context(0)
scale, key = int(sys.argv[1]), sys.argv[2]
g = ctx.generate_kronecker(scale, 16, 1, weighted=True)
roots = [int(r) for r in g.sample_roots(2, 4)]
g.sssp(roots[0], copy=False)
for v in [float(x) for x in sys.argv[3:]]:
    g.set_option(key, v)
    ms = []
    for r in roots:
        g.sssp(r, copy=False)
        s = g.stats()
        ms.append(s["kernel_ms"])
    print(f"{key}={v}: mean {np.mean(ms):.2f} ms  {[round(x, 2) for x in ms]} bands {s['levels']} push/pull {s['td_levels']}/{s['bu_levels']}", flush=True)
