#!/usr/bin/env python3
"""Benchmark: unit-weight SSSP on Graph500 Kronecker s22/ef16 (BASELINE.json configs[1]).

One step = one SSSP (dist init -> distances final on the device) from one root
over the HBM-resident graph. Multi-GPU (torchrun, one process per GPU): the
graph is replicated and the roots are sharded across ranks (Graph500-style
source sharding, no data-path collective) -> weak scaling.

Prints ONE JSON line (rank 0):
  value    = GTEPS = sum over ranks of m_r (edges of the reached component,
             Graph500 TEPS convention over directed CSR entries) / max-over-ranks time
  roofline = algorithmic bytes per SSSP (SURVEY.md §8d:
             B = 4N + n_r(12 + 2*O) + m_r(8 + 4*weighted)) / the solve's device
             time measured with HIP events on libpj's stream
  cpu_baseline = the reference's BSP heap algorithm (oracle port, host threads)
             on a bounded sample of the same roots, rank 0 at N=1 only
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GTEPS + time-to-solution, SSSP web-Google & Graph500 s26, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def algorithmic_bytes(n, n_r, m_r, nnz, weighted=False):
    o = 4 if nnz < 2**31 else 8
    return 4 * n + n_r * (12 + 2 * o) + m_r * (8 + 4 * int(weighted))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--edgefactor", type=int, default=16)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_s22.json"))
    ap.add_argument("--opt", action="append", default=[], help="libpj graph option key=value (tuning)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))

    import paralleljohnson_amd as pj

    ctx = pj.Context(local)
    g = ctx.generate_kronecker(args.scale, args.edgefactor, args.seed)
    for kv in args.opt:
        k, v = kv.split("=")
        g.set_option(k, float(v))
    n_roots = 64
    roots = g.sample_roots(args.seed + 1, n_roots)
    # weak scaling: rank r takes roots r, r+world, ... (distinct roots per rank)
    my_roots = [int(roots[(rank + world * k) % len(roots)]) for k in range(args.steps)]

    for k in range(args.warmup):
        g.sssp(my_roots[k % len(my_roots)], copy=False)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    kernel_ms = []
    barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        g.sssp(my_roots[k], copy=False)
        kernel_ms.append(g.stats()["kernel_ms"])
    barrier()
    elapsed = time.perf_counter() - t0

    # untimed: reached-component statistics per root (m_r, n_r)
    reach = {}
    levels = {}
    for r in set(my_roots):
        g.sssp(r, copy=False)
        st = g.reach_stats()
        reach[r] = (st["reached"], st["reached_edges"])
        levels[r] = (st["td_levels"], st["bu_levels"])
    m_sum = float(sum(reach[r][1] for r in my_roots))
    b_sum = float(sum(algorithmic_bytes(g.n, reach[r][0], reach[r][1], g.nnz) for r in my_roots))
    t_kernel_sum = sum(kernel_ms) / 1000.0

    if dist is not None:
        t = torch.tensor([elapsed, m_sum, b_sum, t_kernel_sum], dtype=torch.float64, device="cuda")
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed = float(tmax[0])
        m_sum, b_sum, t_kernel_sum = float(t[1]), float(t[2]), float(t[3])

    value = m_sum / elapsed / 1e9
    achieved = b_sum / t_kernel_sum / 1e9  # GB/s, per-solve algorithmic bytes / device time

    traffic = None
    if os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            tj = json.load(f)
        if tj.get("scale") == args.scale and tj.get("edgefactor") == args.edgefactor:
            traffic = tj.get("hbm_bytes_per_sssp")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(g, my_roots, reach, args)

    if rank == 0:
        mean_ms = 1000.0 * elapsed / args.steps
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GTEPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(mean_ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": f"synthetic: Graph500 Kronecker (A,B,C=0.57,0.19,0.19) scale {args.scale} edgefactor "
                    f"{args.edgefactor}, both directions, on-GPU generator seed {args.seed}",
            "config": {
                "workload": f"graph500-kronecker-s{args.scale}-ef{args.edgefactor}-unit-sssp",
                "n_vertices": g.n, "nnz": g.nnz, "roots_per_rank": args.steps,
                "parallelism": f"source-sharded x{world} (graph replicated, no data-path collective)",
            },
            "gteps_graph500": round(value / 2, 3),
            "time_to_solution_ms": round(mean_ms, 4),
            "kernel_ms_mean": round(1000.0 * t_kernel_sum / (args.steps * world), 4),
            "levels_td_bu": levels[my_roots[0]],
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "scope": "whole SSSP solve (all frontier kernels of one root); "
                         "bytes = SURVEY.md §8d algorithmic bytes",
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(g, my_roots, reach, args):
    """The reference algorithm (oracle port of :466-594) on host threads, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # cpu_baseline leg only

    O.build()
    row, col, _ = g.get_csr()
    col = col.view(np.uint32)
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    t_sum, m_sum, done = 0.0, 0, []
    t_start = time.perf_counter()
    for r in dict.fromkeys(my_roots):
        dist, st = O.reference_sssp(row, col, r, threads)
        t_sum += st.solve_s
        m_sum += reach[r][1]
        done.append(r)
        if time.perf_counter() - t_start > args.cpu_seconds:
            break
    return {
        "value": round(m_sum / t_sum / 1e9, 4),
        "unit": "GTEPS",
        "cores": threads,
        "kind": "port",
        "sample": f"{len(done)} root(s) of the same s{args.scale} graph, reference BSP heap algorithm "
                  f"(30 pops/round, {threads} partitions on {threads} host threads), solve time only "
                  f"({t_sum:.2f} s)",
        "ms_per_sssp": round(1000.0 * t_sum / len(done), 2),
    }


if __name__ == "__main__":
    main()
