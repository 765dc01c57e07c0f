"""Radix-sort probe: builds Kronecker graphs on the device (unit: one sort of u32 pairs;
weighted: the record sorts), a few times each; run under rocprofv3 for per-kernel times.
Usage: python tools/sort_probe.py [scale] [reps]"""
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import paralleljohnson_amd as pj  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ctx = pj.Context(0)
for weighted in (False, True):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        g = ctx.generate_kronecker(scale, 16, 1, weighted=weighted)
        ts.append(time.perf_counter() - t)
        g.close()
    print(f"s{scale} weighted={weighted}: build {min(ts) * 1000:.1f} ms (min of {reps})", flush=True)
