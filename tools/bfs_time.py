"""Unit-weight solve times: web-Google-shaped synthetic (configs[0]: source 0 and 7 sampled roots) and
Kronecker s22 (configs[1], 8 sampled roots), median kernel ms per direction policy, with and without
the one-workgroup small-frontier levels (option bfs_small). Distances of every variant are checked
against the first variant of the same root (bit-exact).
Usage: python tools/bfs_time.py [graphs=wg,k22] [dirs=0,1,2] [smalls=0,1] [seed=7] [key=value ...]  (libpj graph
options; seed=2 gives the bench's k22 roots)"""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import paralleljohnson_amd as pj

ctx = pj.Context(0)
opts = dict(kv.split("=") for kv in sys.argv[1:])
graphs = opts.pop("graphs", "wg,k22").split(",")
dirs = [int(x) for x in opts.pop("dirs", "0,1,2").split(",")]
smalls = [int(x) for x in opts.pop("smalls", "0,1").split(",")]
seed = int(opts.pop("seed", "7"))
tag = " ".join(f"{k}={v}" for k, v in opts.items())
for name in graphs:
    if name == "wg":
        g = ctx.generate_webgraph()
        roots = [0] + [int(r) for r in g.sample_roots(seed, 3)]
    else:
        g = ctx.generate_kronecker(22, 16, 1)
        roots = [int(r) for r in g.sample_roots(seed, 8)]
    for k, v in opts.items():
        g.set_option(k, float(v))
    ref = {}
    for mode in dirs:
        g.set_option("direction", mode)
        for small in smalls:
            g.set_option("bfs_small", small)
            ts, t0, lv = [], [], []
            for rep in range(4):
                for r in roots:
                    d = g.sssp(r, copy=(rep == 0))
                    st = g.stats()
                    ts.append(st["kernel_ms"])
                    if r == roots[0]:
                        t0.append(st["kernel_ms"])
                    if rep == 0:
                        lv.append(st["levels"])
                        if r in ref:
                            assert np.array_equal(d, ref[r]), (name, mode, small, r)
                        else:
                            ref[r] = d
            print(f"{name} {tag} direction={mode} small={small} median kernel_ms {np.median(ts):.4f} mean {np.mean(ts):.4f} "
                  f"min {np.min(ts):.4f} root0 {np.median(t0):.4f} levels {lv}", flush=True)
    g.close()
print("bfs_time: all variants bit-identical", flush=True)
