"""Fixed MS1024 workload for rocprofv3 passes: the bench's 1024 sources on the web-Google-shaped
graph, batched with the default pass width, run REPS times after one warmup batch.
Usage: python tools/ms_pmc_probe.py [reps=2] [ms_streams] (ms_streams 1: one pass at a time, so the
kernel durations of a trace are not inflated by the other slot's kernels)"""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import numpy as np
import paralleljohnson_amd as pj
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
ctx = pj.Context(0)
g = ctx.generate_webgraph()
if len(sys.argv) > 2:
    g.set_option("ms_streams", float(sys.argv[2]))
row, _, _ = g.get_csr()
src = np.nonzero(np.diff(row) >= 1)[0][:1024]
g.sssp_batch(src[:64], copy=False)
for _ in range(reps):
    g.sssp_batch(src, copy=False)
print(f"ms_pmc_probe: {reps} batches of {len(src)} sources, kernel_ms {g.stats()['kernel_ms']:.3f}", flush=True)
