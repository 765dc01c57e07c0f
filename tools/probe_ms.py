"""MS1024 on the web-Google-shaped graph: batched multi-source wall/kernel time per pass width."""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import numpy as np
import paralleljohnson_amd as pj
ctx = pj.Context(0)
g = ctx.generate_webgraph()
row, _, _ = g.get_csr()
src = [int(x) for x in np.nonzero(np.diff(row) > 0)[0][:1024]]
import itertools
for wd, al in itertools.product((1, 4), (0, 4, 16, 64)):
    g.set_option("ms_width", wd)
    g.set_option("ms_alpha", al)
    g.sssp_batch(src[:64], copy=False)
    ts = []
    for _ in range(3):
        t = time.perf_counter(); g.sssp_batch(src, copy=False); ts.append(time.perf_counter() - t)
    print(f"width {wd} alpha {al}: wall {1e3 * min(ts):.2f} ms kernel {g.stats()['kernel_ms']:.2f} ms levels {g.stats()['levels']}", flush=True)
