"""configs[3] at world 1: the unit-weight partition (part.hip) solved by bfs.hip on its borrowed rows
(option single_gpu 1) against its own level loop (single_gpu 0), on the bench's roots (bench.py
run_partitioned: rng(seed + 7) candidates with reached > 1) -- host wall per pj_part_bfs and the
solve_ms it reports, then the same roots on a pj.Graph of the same graph (kernel_ms).
Usage: python tools/k28_part_single.py [scale=28] [graph=1]"""
import os
import sys
import time

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import paralleljohnson_amd as pj  # noqa: E402
from paralleljohnson_amd.partition import Comm, load_kronecker  # noqa: E402

opts = dict(kv.split("=") for kv in sys.argv[1:])
scale = int(opts.get("scale", "28"))
ctx = pj.Context(0)
comm = Comm.for_rank(ctx, 1, 0)
ops = load_kronecker(ctx, scale, 16, 1, 0, 1)
rng = np.random.default_rng(1 + 7)
roots = []
for c in rng.integers(0, 1 << scale, 64):
    st = ops.bfs(comm, int(c))
    if st["reached"] > 1:
        roots.append(int(c))
    if len(roots) == 4:
        break
print("roots", roots, flush=True)
for single in (1, 0, 1, 0):
    ops.set_option("single_gpu", single)
    for r in roots:
        ops.bfs(comm, r)  # (warm)
    walls, sms = [], []
    for r in roots:
        t = time.perf_counter()
        st = ops.bfs(comm, r)
        walls.append(1e3 * (time.perf_counter() - t))
        sms.append(st["solve_ms"])
    print(f"single_gpu={single} wall ms {np.round(walls, 3).tolist()} mean {np.mean(walls):.3f}  solve_ms mean "
          f"{np.mean(sms):.3f} levels td/bu {st['td_levels']}/{st['bu_levels']}", flush=True)
ops.close()
if opts.get("graph", "1") == "1":
    g = ctx.generate_kronecker(scale, 16, 1)
    for rep in range(2):
        ks = []
        for r in roots:
            t = time.perf_counter()
            g.sssp(r, copy=False)
            ks.append((g.stats()["kernel_ms"], 1e3 * (time.perf_counter() - t)))
        print("pj.Graph kernel_ms / wall ms", [(round(a, 3), round(b, 3)) for a, b in ks], flush=True)
    g.close()
comm.close()
