"""MS1024 on the web-Google-shaped graph at the default pass width (for kernel traces)."""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import numpy as np
import paralleljohnson_amd as pj
ctx = pj.Context(0)
g = ctx.generate_webgraph()
row, _, _ = g.get_csr()
src = [int(x) for x in np.nonzero(np.diff(row) > 0)[0][:1024]]
g.sssp_batch(src[:64], copy=False)
for _ in range(int(os.environ.get("PJ_REPS", "3"))):
    t = time.perf_counter(); g.sssp_batch(src, copy=False)
    print(f"wall {1e3 * (time.perf_counter() - t):.2f} ms", g.stats(), flush=True)
