"""Weighted delta-stepping over the 1D partition at world 1 (no exchange) vs the
single-GPU solver, Kronecker weighted: python tools/probe_wpart.py SCALE [roots]"""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R)
import numpy as np
import torch
import paralleljohnson_amd as pj
from paralleljohnson_amd.partition import PartitionedDelta, gather_dist, load_weighted
scale = int(sys.argv[1]); nroots = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ctx = pj.Context(0)
g = ctx.generate_kronecker(scale, 16, 1, weighted=True)
roots = [int(r) for r in g.sample_roots(2, nroots)]
single = {}
for r in roots:
    g.sssp(r, copy=False); g.sssp(r)
    single[r] = (g.copy_dist(), g.stats()["kernel_ms"])
ops = load_weighted(ctx, g, 0, 1)
g.close()
sp = PartitionedDelta(ops, None)
for r in roots:
    sp.solve(r)
    torch.cuda.synchronize(); t = time.perf_counter(); st = sp.solve(r); torch.cuda.synchronize()
    el = time.perf_counter() - t
    ok = np.array_equal(gather_dist(ops, None), single[r][0])
    print(f"s{scale} root {r}: partitioned(world 1) {1e3 * el:.1f} ms, {st['reached_edges'] / el / 1e9:.1f} GTEPS, "
          f"bands {st['bands']} rounds {st['rounds']}; single-GPU {single[r][1]:.2f} ms; equal {ok}", flush=True)
