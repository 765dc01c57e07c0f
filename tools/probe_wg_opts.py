"""web-Google-shaped synthetic (configs[0]), source 0: median kernel time per option set,
interleaved over repetitions so drift hits every set alike.
usage: probe_wg_opts.py "alpha=7" "beta=48,grid_per_cu=3" ...  (the base set is always run)"""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import paralleljohnson_amd as pj

DEFAULTS = {"alpha": 14.0, "beta": 24.0, "grid_per_cu": 0.0, "bfs_small": 1.0}
sets = [""] + sys.argv[1:]
ctx = pj.Context(0)
g = ctx.generate_webgraph()
ref = g.sssp(0)
times = {s: [] for s in sets}
lv = {}
for rep in range(6):
    for s in sets:
        opts = dict(DEFAULTS)
        for kv in filter(None, s.split(",")):
            k, v = kv.split("=")
            opts[k] = float(v)
        for k, v in opts.items():
            g.set_option(k, v)
        for _ in range(3):
            g.sssp(0, copy=False)
        for _ in range(20):
            g.sssp(0, copy=False)
            times[s].append(g.stats()["kernel_ms"])
        st = g.stats()
        lv[s] = (st["levels"], st["td_levels"], st["bu_levels"])
        if rep == 0:
            assert np.array_equal(g.sssp(0), ref), s
for s in sets:
    t = np.array(times[s])
    print(f"{s or 'base':40s} median {np.median(t) * 1000:7.1f} us  p10 {np.percentile(t, 10) * 1000:7.1f}"
          f"  levels/td/bu {lv[s]}", flush=True)
