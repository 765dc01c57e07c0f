import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np
import paralleljohnson_amd as pj
ctx = pj.Context(0)
g = ctx.generate_webgraph(seed=1)
row, _, _ = g.get_csr()
src = np.nonzero(np.diff(row) >= 1)[0][:1024]
for rep in range(2):
    for wd in (8, 16):
        g.set_option("ms_width", wd)
        g.sssp_batch(src[:64], copy=False)
        ts = []
        for _ in range(3):
            t = time.perf_counter(); g.sssp_batch(src, copy=False); ts.append(time.perf_counter() - t)
        print(f"width {wd}: wall min {1e3 * min(ts):.2f} med {1e3 * sorted(ts)[1]:.2f} ms kernel {g.stats()['kernel_ms']:.2f} ms", flush=True)
# parity of width 8 vs width 4 rows on a few sources
g.set_option("ms_width", 16); a = g.sssp_batch(src[:1000])
g.set_option("ms_width", 4); b = g.sssp_batch(src[:1000])
print("rows equal", bool((a == b).all()))
