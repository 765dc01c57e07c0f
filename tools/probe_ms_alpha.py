"""MS1024 (web-Google-shaped, 1024 sources) wall / kernel time under ms_alpha (push threshold) values."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import paralleljohnson_amd as pj
ctx = pj.Context(0)
g = ctx.generate_webgraph(seed=1)
row, _, _ = g.get_csr()
src = np.nonzero(np.diff(row) >= 1)[0][:1024]
for rep in range(2):
    for al in [float(x) for x in sys.argv[1:]] or [0.0, 4.0, 16.0, 64.0]:
        g.set_option("ms_alpha", al)
        g.sssp_batch(src[:64], copy=False)
        ts = []
        for _ in range(3):
            t = time.perf_counter(); g.sssp_batch(src, copy=False); ts.append(time.perf_counter() - t)
        print(f"alpha {al}: wall min {1e3 * min(ts):.2f} ms kernel {g.stats()['kernel_ms']:.2f} ms", flush=True)
