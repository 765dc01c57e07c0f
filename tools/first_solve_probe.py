import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import paralleljohnson_amd as pj
ctx = pj.Context(0)
g = ctx.generate_webgraph()
for i in range(3):
    t = time.perf_counter(); d = g.sssp(0, copy=False); t1 = time.perf_counter(); out = g.copy_dist(); t2 = time.perf_counter()
    print(f"solve {i}: sssp {1e3*(t1-t):.2f} ms (kernel {g.stats()['kernel_ms']:.3f}) copy_dist {1e3*(t2-t1):.2f} ms", flush=True)
g2 = ctx.generate_kronecker(20, 16, 1)
for i in range(2):
    t = time.perf_counter(); g2.sssp(1, copy=False); t1 = time.perf_counter()
    print(f"k20 solve {i}: {1e3*(t1-t):.2f} ms", flush=True)
