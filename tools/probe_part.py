"""Timing probe of the partitioned BFS at world 1 (or under torchrun): Kronecker
s{scale}, a few roots, per-solve wall time and level mix, next to the single-GPU
solver on the same graph (world 1 only).
Usage: python tools/probe_part.py [scale] [roots] [--single]"""
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import torch  # noqa: E402

import paralleljohnson_amd as pj  # noqa: E402
from paralleljohnson_amd.partition import Exchange, PartitionedBFS, load_kronecker  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
nroots = int(sys.argv[2]) if len(sys.argv) > 2 else 4
single = "--single" in sys.argv
world = int(os.environ.get("WORLD_SIZE", "1"))
rank = int(os.environ.get("RANK", "0"))
ex = None
if world > 1:
    import torch.distributed as dist
    dist.init_process_group("nccl")
    ex = Exchange()
local = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(local)
ctx = pj.Context(local)
t0 = time.perf_counter()
ops = load_kronecker(ctx, scale, 16, 1, rank, world)
torch.cuda.synchronize()
print(f"rank {rank}: s{scale} block [{ops.lo},{ops.hi}) nnz_local {ops.nnz_local} build {time.perf_counter() - t0:.2f} s",
      flush=True)
bfs = PartitionedBFS(ops, ex)
roots = [1, 777, 12345, 99991, 4242, 31337, 2**scale - 5, 65536][:nroots]
for r in roots:
    bfs.solve(r)  # warm
    torch.cuda.synchronize()
    t = time.perf_counter()
    st = bfs.solve(r)
    torch.cuda.synchronize()
    ms = 1000 * (time.perf_counter() - t)
    if rank == 0:
        print(f"root {r}: {ms:.3f} ms levels {st['levels']} td {st['td_levels']} bu {st['bu_levels']} "
              f"n_r {st['reached']} m_r {st['reached_edges']} sent {st['ids_sent']} "
              f"-> {st['reached_edges'] / ms / 1e6:.1f} GTEPS", flush=True)
ops.close()
if single and world == 1:
    g = ctx.generate_kronecker(scale, 16, 1)
    for r in roots:
        g.sssp(r, copy=False)
        t = time.perf_counter()
        g.sssp(r, copy=False)
        ms = 1000 * (time.perf_counter() - t)
        print(f"single-GPU root {r}: {ms:.3f} ms kernel {g.stats()['kernel_ms']:.3f} ms", flush=True)
    g.close()
