"""Unit-weight solve times: web-Google-shaped synthetic (configs[0], source 0) and Kronecker s22
(configs[1], 8 sampled roots), median kernel ms per direction policy.
Usage: python tools/bfs_time.py [key=value ...]   (libpj graph options)"""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import paralleljohnson_amd as pj

ctx = pj.Context(0)
opts = [kv.split("=") for kv in sys.argv[1:]]
for name, g, roots in (("wg", ctx.generate_webgraph(), [0]), ("k22", None, None)):
    if g is None:
        g = ctx.generate_kronecker(22, 16, 1)
        roots = [int(r) for r in g.sample_roots(7, 8)]
    for k, v in opts:
        g.set_option(k, float(v))
    for mode in (0, 1, 2):
        g.set_option("direction", mode)
        ts = []
        for _ in range(4):
            for r in roots:
                g.sssp(r, copy=False)
                ts.append(g.stats()["kernel_ms"])
        print(f"{name} direction={mode} median kernel_ms {np.median(ts):.4f} min {np.min(ts):.4f}", flush=True)
    g.close()
