"""`parallel_johnson webfile source_node sol_file` across several GPUs.

    python -m torch.distributed.run --nproc-per-node P --master-addr 127.0.0.1 \\
        -m paralleljohnson_amd.run webfile source_node sol_file

is the multi-GPU form of the reference's `mpirun -np P parallel_johnson ...`
(README:9, ParallelJohnson.cpp:286-676): one process per GPU, the vertex set
split in contiguous blocks (nn2rank :169-200), the exchange over RCCL
(paralleljohnson_amd/partition.py). Arguments, stderr progress lines, the
stdout `Time:` line and the sol_file bytes follow the reference (see the
single-GPU CLI, paralleljohnson_amd/csrc/cli.cpp); with one process and no
launcher it runs alone on one GPU. Unit weights only (the reference's w = 1,
:147) unless PJ_WEIGHTED=1: then the third column is an integer weight (as in
the single-GPU CLI) and the solve is delta-stepping over the partition
(PartitionedDelta, wpart.hip). Environment: PJ_DEVICE overrides the GPU ordinal (default LOCAL_RANK),
PJ_BACKEND overrides the torch.distributed backend (default nccl = RCCL; gloo
stages the exchange through host memory, for rehearsals with several ranks
on one GPU).
"""
import ctypes
import os
import sys
import time


def _atoi(s: str) -> int:
    """C atoi (:448): leading blanks, optional sign, digits; 0 when none."""
    return ctypes.CDLL(None).atoi(s.encode())


def main(argv=None) -> int:
    argv = sys.argv if argv is None else argv
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if len(argv) != 4:  # :294-303
        if rank == 0:
            print("to run this program must supply the following command line arguments (in order)",
                  file=sys.stderr)
            print("argv[1]---web graph file.", file=sys.stderr)
            print("argv[2]---source node number.", file=sys.stderr)
            print("argv[3]---file to save the solution.", file=sys.stderr)
        return 255
    import torch
    import paralleljohnson_amd as pj
    from paralleljohnson_amd.partition import (Exchange, PartitionedBFS, PartitionedDelta, gather_dist,
                                               load_snap, load_weighted)

    local = int(os.environ.get("PJ_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(local)
    ex = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("PJ_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        ex = Exchange()

    def msg(s):  # print_msg :49-53
        if rank == 0:
            print(s, file=sys.stderr, flush=True)

    msg("process 0 reads in the web graph data......")
    ctx = pj.Context(local)
    weighted = os.environ.get("PJ_WEIGHTED", "0") not in ("", "0")
    if weighted:  # every rank parses the file on its GPU and cuts its weighted block
        g = ctx.load_snap(argv[1], weighted=True)
        ops = load_weighted(ctx, g, rank, world)
        g.close()
    else:
        ops = load_snap(ctx, argv[1], rank, world)
    msg(f"N = {ops.n}")  # :320
    msg("read in the webgraph is done.")
    msg("distribute sparse matrix is done.")
    source = _atoi(argv[2])
    msg(f"compute shortest paths from source node: {source}")
    msg("parallel Johnson's algorithm starts......")
    bfs = PartitionedDelta(ops, ex) if weighted else PartitionedBFS(ops, ex)
    torch.cuda.synchronize()
    if ex is not None:
        ex.dist.barrier()
    t0 = time.perf_counter()
    bfs.solve(source)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if ex is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        ex.dist.all_reduce(t, op=ex.dist.ReduceOp.MAX)
        elapsed = float(t[0])
    dist_all = gather_dist(ops, ex)
    msg("parallel Johnson's algorithm completes.")
    if rank == 0:
        print(f"Time: {elapsed:g} seconds when using {world} processes.", flush=True)  # :603
        pj.write_sol(dist_all, argv[3])  # :615-618
        msg(f"the shortest path distance vector has been saved in file {argv[3]}")
    ops.close()
    if ex is not None:
        ex.dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
