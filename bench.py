#!/usr/bin/env python3
"""Benchmark of the relaxation hot path (BASELINE.json metric: "GTEPS + time-to-solution,
SSSP web-Google & Graph500 s26, 1/2/4/8 GPUs").

Main workload (the `value` of the JSON line): BASELINE.json configs[2], Graph500
Kronecker scale 26, edgefactor 16 (2^31 directed CSR entries, both directions),
integer weights 1..255, SSSP by delta-stepping, single GPU resident. One step =
one SSSP (dist init -> distances final in input ids on the device) from one root.
Multi-GPU (torchrun, one process per GPU): the graph is replicated and the roots
are sharded across ranks (Graph500-style source sharding, no data-path
collective) -> weak scaling.

At N=1 the same line also carries `secondary` results: configs[1] (Kronecker s22
unit weights, direction-optimizing BFS) and configs[0] (web-Google-shaped
synthetic, source 0). Inputs are generated on the device (no dataset access).

  value        = GTEPS = sum over ranks of m_r / max-over-ranks wall time of the
                 timed steps; m_r = CSR entries of the reached vertices
                 (Graph500 TEPS over directed entries; gteps_graph500 = value / 2)
  roofline     = scanned-work bytes per SSSP, B = 4N + n_r(12 + 2*O) + the edge
                 records the solve read (as stored) + the probes of their other
                 ends, both counted on the device in every timed solve, divided by
                 the solve's device time (HIP events on libpj's stream); traffic =
                 the calibrated DRAM-side bytes of the per-kernel table measured on
                 this build (profiles/traffic_k26w.json, else null); frac_model_8d
                 keeps SURVEY.md §8d's every-reached-edge model
  cpu_baseline = the reference's BSP heap algorithm (oracle port of :466-594,
                 weights honoured) on host threads, rank 0 at N=1 only, on a
                 bounded sample of one solve of the same graph
"""
import argparse
import json
import os
import sys
import tempfile
import time


import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GTEPS + time-to-solution, SSSP web-Google & Graph500 s26, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

WORKLOADS = {
    "k26w": dict(kind="kronecker", scale=26, weighted=True,
                 name="graph500-kronecker-s26-ef16-w1..255-delta-stepping-sssp"),
    "k22": dict(kind="kronecker", scale=22, weighted=False, name="graph500-kronecker-s22-ef16-unit-sssp"),
    "wg": dict(kind="webgraph", weighted=False, name="web-google-shaped-synthetic-unit-sssp-source0"),
}


def host_cpu():
    """Host CPU model and logical core count (report nproc and the CPU model)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "host_nproc": os.cpu_count()}


def cpu_share():
    """Host threads this job may use: the box's CPU share (OMP_NUM_THREADS is set to it on the
    GPU box; os.cpu_count() shows the whole machine there), else the affinity set."""
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        return int(omp)
    return len(os.sched_getaffinity(0))


def algorithmic_bytes(n, n_r, m_r, nnz, weighted=False):
    o = 4 if nnz < 2**31 else 8
    return 4 * n + n_r * (12 + 2 * o) + m_r * (8 + 4 * int(weighted))


def make_graph(ctx, wl, args):
    if wl["kind"] == "webgraph":
        return ctx.generate_webgraph(seed=args.seed)
    scale = args.scale if args.scale else wl["scale"]
    return ctx.generate_kronecker(scale, args.edgefactor, args.seed, weighted=wl["weighted"])


def run_workload(ctx, key, args, rank, world, barrier, steps, warmup):
    """Timed SSSPs of one workload on this rank; returns per-rank sums."""
    import paralleljohnson_amd as pj
    wl = WORKLOADS[key]
    t_gen = time.perf_counter()
    g = make_graph(ctx, wl, args)
    build_s = time.perf_counter() - t_gen  # generation on the device + radix sort + CSR
    for kv in args.opt:
        k, v = kv.split("=")
        g.set_option(k, float(v))
    if wl["kind"] == "webgraph":
        roots = [0]  # configs[0]: source 0
    else:
        roots = [int(r) for r in g.sample_roots(args.seed + 1, 64)]
    my_roots = [roots[(rank + world * k) % len(roots)] for k in range(max(steps, 1))]
    t_prep = time.perf_counter()
    g.sssp(my_roots[0], copy=False)  # first solve builds the solver workspace (untimed)
    prep_s = time.perf_counter() - t_prep  # weighted: degree-ordered relabel + light CSR + workspace
    gen_s = time.perf_counter() - t_gen
    for k in range(warmup):
        g.sssp(my_roots[k % len(my_roots)], copy=False)
    sts = [pj.Stats() for _ in range(steps)]  # (filled in the loop, read after it: no dicts in the timed region)
    barrier()
    t0 = time.perf_counter()
    for k in range(steps):
        g.sssp(my_roots[k], copy=False)
        g.stats_into(sts[k])
    barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = [st.kernel_ms for st in sts]
    work = [(st.scanned_edges, st.probes, st.work_bytes) for st in sts]
    reach, levels = {}, {}
    for r in set(my_roots):  # untimed: reached-component statistics per root
        g.sssp(r, copy=False)
        st = g.reach_stats()
        reach[r] = (st["reached"], st["reached_edges"])
        levels[r] = (st["levels"], st["td_levels"], st["bu_levels"], st["relax_rounds"])
    m_sum = float(sum(reach[r][1] for r in my_roots[:steps]))
    b_sum = float(sum(algorithmic_bytes(g.n, reach[r][0], reach[r][1], g.nnz, wl["weighted"])
                      for r in my_roots[:steps]))
    # the scanned-work model (weighted solves count their work on the device, every solve):
    # 4N + n_r(12 + 2*O) + the records read as stored + the probes of their other ends
    o = 4 if g.nnz < 2**31 else 8
    w_sum = float(sum(4 * g.n + reach[r][0] * (12 + 2 * o) for r in my_roots[:steps]) + sum(x[2] for x in work))
    return dict(g=g, wl=wl, elapsed=elapsed, m_sum=m_sum, b_sum=b_sum, w_sum=w_sum, t_kernel=sum(kernel_ms) / 1000.0,
                scanned=float(sum(x[0] for x in work)), probes=float(sum(x[1] for x in work)),
                roots=my_roots[:steps], reach=reach, levels=levels, gen_s=gen_s, build_s=build_s, prep_s=prep_s)


def tts_process(args, wl, td):
    """SURVEY.md §8d time-to-solution (process start -> sol_file closed) as ONE wall clock:
    bin/pj_kron_tts, a fresh process through the C-ABI (pj_create, on-device Kronecker
    generation + radix sort + CSR, the first solve with the solver's preparation, D2H,
    pj_write_sol), timed by this process from launch to exit, for the bench's first root
    (picked inside the tool). Run before this process builds anything, so the tool has
    the GPU to itself, as a user's run would. The reference cannot read a 2^31-line text
    file (:66/:117), so the graph comes from the generator."""
    import subprocess
    tool = os.path.join(ROOT, "paralleljohnson_amd", "bin", "pj_kron_tts")
    scale = args.scale if args.scale else wl["scale"]
    out = os.path.join(td, "sol_tts.txt")
    env = dict(os.environ)
    env["PJ_TTS_LAUNCH_NS"] = str(time.monotonic_ns())  # (CLOCK_MONOTONIC, as the tool's steady_clock)
    t3 = time.perf_counter()
    p = subprocess.run([tool, str(scale), str(args.edgefactor), str(args.seed), str(int(wl["weighted"])),
                        f"sample:{args.seed + 1}", out], capture_output=True, text=True, timeout=300, env=env)
    wall = time.perf_counter() - t3
    t_end = time.monotonic_ns()
    if p.returncode != 0:
        raise RuntimeError(f"pj_kron_tts failed: {p.stderr[-400:]}")
    f = p.stdout.split()
    phases = dict(zip(("create_s", "build_s", "solve_prep_s", "d2h_s", "write_s", "launch_s", "teardown_s"),
                      (float(x) for x in f[1:8])))
    phases["exit_s"] = round((t_end - int(f[11])) * 1e-9, 4)
    phases["unaccounted_s"] = round(wall - sum(v for v in phases.values() if v > 0), 4)
    return {"wall": round(wall, 4), "phases": phases, "root": int(f[9]), "sol": out}


def time_to_solution(ctx_s, res, tts, td):
    """The tool's wall clock (tts_process) with this process's phases as a breakdown, and
    whether the tool's sol_file equals this process's for the same root."""
    import paralleljohnson_amd as pj
    g = res["g"]
    t0 = time.perf_counter()
    d = g.sssp(tts["root"])
    t1 = time.perf_counter()
    pj.write_sol(d, os.path.join(td, "sol.txt"))
    t2 = time.perf_counter()
    phases = {"hip_context_s": round(ctx_s, 4), "graph_build_s": round(res["build_s"], 4),
              "solver_prep_s": round(res["prep_s"], 4), "solve_and_d2h_s": round(t1 - t0, 4),
              "write_sol_s": round(t2 - t1, 4)}
    same = open(tts["sol"], "rb").read() == open(os.path.join(td, "sol.txt"), "rb").read()
    return tts["wall"], {"wall_clock": "bin/pj_kron_tts, process launch -> exit (sol_file closed), run before "
                                       "this process built its graph",
                         "process_phases": tts["phases"], "root": tts["root"], "sol_identical_to_bench_process": same,
                         "in_process_breakdown": phases}


def partition_transport(ctx, rank, world, backend):
    """The partitioned leg's pj_comm: one rank without a transport at world 1; at world > 1
    libpj's RCCL group (one process per GPU, the group id handed out by rank 0 over
    torch.distributed), or under a gloo rehearsal (PJ_BENCH_BACKEND=gloo) the host-buffer
    callbacks over torch.distributed, which transport_guard rejects before any GPU work."""
    from paralleljohnson_amd.partition import Comm, TorchDistTransport
    if world == 1:
        return Comm.for_rank(ctx, 1, 0)
    if backend != "nccl":
        return Comm.from_callbacks(TorchDistTransport(), rank, world)
    import torch.distributed as dist
    box = [Comm.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)  # bootstrap only: the solve's collectives are libpj's RCCL calls
    return Comm.for_rank(ctx, world, rank, box[0])


def transport_guard(comm, world):
    """The group the partitioned leg runs on, as the transport itself reports it (RCCL:
    ncclCommCount / ncclCommUserRank, the reference's MPI_Comm_size / rank at :291-292). At
    world > 1 anything but an RCCL communicator of exactly `world` ranks fails the leg, so an
    N-GPU line cannot report a partitioned solve that did not run over N GPUs."""
    count, index = comm.transport_ranks()
    info = {"transport": comm.kind, "transport_ranks": count, "transport_rank": index}
    if world > 1 and (comm.kind != "rccl" or count != world):
        raise RuntimeError(f"partitioned leg at world {world} needs an RCCL communicator of {world} ranks; the "
                           f"transport is {comm.kind!r} reporting {count} rank(s)")
    return info


def run_partitioned(ctx, args, rank, world, barrier, backend="nccl", nroots=4):
    """configs[3]: Kronecker s{part_scale} unit-weight BFS, 1D vertex partition over the
    `world` ranks (libpj's level loop, pj_part_bfs, over RCCL: one process per GPU); strong
    scaling. The transport is formed and checked (transport_guard) before the graph is built."""
    from paralleljohnson_amd.partition import load_kronecker
    t0 = time.perf_counter()
    comm = partition_transport(ctx, rank, world, backend)
    try:
        tinfo = transport_guard(comm, world)
    except Exception:
        comm.close()
        raise
    ops = load_kronecker(ctx, args.part_scale, args.edgefactor, args.seed, rank, world)
    build_s = time.perf_counter() - t0
    rng = np.random.default_rng(args.seed + 7)
    roots = []
    for c in rng.integers(0, 1 << args.part_scale, 64):  # same candidates on every rank
        st = ops.bfs(comm, int(c))  # untimed: keep roots in the giant component (degree >= 1)
        if st["reached"] > 1:
            roots.append((int(c), dict(st)))
        if len(roots) == nroots:
            break
    barrier()
    t = time.perf_counter()
    for r, _ in roots:
        ops.bfs(comm, r)
    barrier()
    elapsed = time.perf_counter() - t
    m = float(sum(st["reached_edges"] for _, st in roots))
    b = float(sum(algorithmic_bytes(ops.n, st["reached"], st["reached_edges"], 2 * (args.edgefactor << args.part_scale))
                  for _, st in roots))
    st0 = roots[0][1]
    res = dict(elapsed=elapsed, m=m, b=b, n=ops.n, nnz_local=ops.nnz_local, build_s=build_s, roots=len(roots),
               st0=st0, transport=tinfo, build_phases=ops.build_phases())
    ops.close()
    comm.close()
    return res


def run_partitioned_host(args, world_h=2, nroots=4):
    """configs[3]'s exchange path on ONE GPU: the s{part_scale} 1D partition at world 2 with
    both ranks in this process sharing the GPU over the host transport (device copies
    between the ranks' buffers, host barriers; NOT xGMI/RCCL). Puts the per-level owner
    exchange (:522-554) and termination allreduce (:589-590) cost on record at full size."""
    import paralleljohnson_amd as pj
    from paralleljohnson_amd.partition import Comm, bfs_group, load_kronecker
    ctxs = [pj.Context(0) for _ in range(world_h)]
    comms = Comm.group(ctxs, "host")
    t0 = time.perf_counter()
    parts, build_rank_s = [], []
    for r in range(world_h):  # (the ranks build one after the other, each with the whole GPU)
        t1 = time.perf_counter()
        parts.append(load_kronecker(ctxs[r], args.part_scale, args.edgefactor, args.seed, r, world_h))
        build_rank_s.append(round(time.perf_counter() - t1, 3))
    build_s = time.perf_counter() - t0
    try:
        rng = np.random.default_rng(args.seed + 7)  # run_partitioned's candidates
        roots = []
        for c in rng.integers(0, 1 << args.part_scale, 64):
            st = bfs_group(parts, comms, int(c))
            if st[0]["reached"] > 1:
                roots.append((int(c), st))
            if len(roots) == nroots:
                break
        t = time.perf_counter()
        for r, _ in roots:
            bfs_group(parts, comms, r)
        elapsed = time.perf_counter() - t
        m = float(sum(st[0]["reached_edges"] for _, st in roots))
        st0 = roots[0][1]
        return {
            "workload": f"graph500-kronecker-s{args.part_scale}-ef{args.edgefactor}-unit-bfs, 1D vertex partition at "
                        f"world {world_h}, both ranks on ONE GPU over the host transport (device copies + host "
                        f"barriers; not xGMI/RCCL)",
            "roots": len(roots), "ms_per_bfs": round(1000.0 * elapsed / len(roots), 3),
            "gteps": round(m / elapsed / 1e9, 3),
            "levels_td_bu": [st0[0]["td_levels"], st0[0]["bu_levels"]],
            "ids_sent_per_bfs_by_rank": [x["sent"] for x in st0],
            "nnz_local_by_rank": [p.nnz_local for p in parts],
            "device_bytes_by_rank": [p.device_bytes() for p in parts],
            "build_s": round(build_s, 2), "build_s_by_rank": build_rank_s,
            "build_phases_by_rank": [p.build_phases() for p in parts],
        }
    finally:
        for p in parts:
            p.close()
        for c in comms:
            c.close()
        for c in ctxs:
            c.close()


def run_multisource(ctx, args, rank, world, barrier, n_src=1024):
    """configs[4]: 1024 sources on the web-Google-shaped graph, batched (up to 512 per pass),
    source batches sharded over the ranks (no data-path collective)."""
    g = ctx.generate_webgraph(seed=args.seed)
    row, _, _ = g.get_csr()
    deg = np.diff(row)
    sources = np.nonzero(deg >= 1)[0][:n_src]  # the smallest ids with out-degree >= 1
    mine = sources[rank::world]
    g.sssp_batch(mine[:64], copy=False)  # untimed warmup (workspace)
    g.sssp_batch(mine, copy=False)  # untimed: the pass level counts that size the launch batches
    reps = []
    for _ in range(args.ms_reps):  # every rep is the whole batch of this rank's sources
        barrier()
        t = time.perf_counter()
        g.sssp_batch(mine, copy=False)
        barrier()
        reps.append(time.perf_counter() - t)
    elapsed = float(np.median(reps))
    # m_r and n_r per source (untimed): every source's reached out-edge sum and reached count
    m, b = 0.0, 0.0
    for s0 in range(0, len(mine), 64):
        d = g.sssp_batch(mine[s0:s0 + 64])
        reached = d < 100000
        m_rows = (reached * deg[None, :]).sum(axis=1).astype(np.float64)
        n_rows = reached.sum(axis=1)
        m += float(m_rows.sum())
        b += float(sum(algorithmic_bytes(g.n, int(nr), float(mr), g.nnz, False) for nr, mr in zip(n_rows, m_rows)))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the reference takes one source per run, so 1024 single-source runs;
        # time the first 16 sources and scale to 1024 (labelled extrapolated)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # cpu_baseline leg only
        O.build()
        col = g.get_csr()[1].view(np.uint32)
        threads = max(1, min(args.cpu_threads, cpu_share()))
        k, solve_s = 16, 0.0
        for s in sources[:k]:
            _, st = O.reference_sssp(row, col, int(s), threads)
            solve_s += st.solve_s
        cpu = {"value_s_extrapolated": round(solve_s * len(sources) / k, 3), "sample": f"{k} of {len(sources)} "
               f"single-source solves timed ({solve_s:.3f} s), scaled to {len(sources)}", "cores": threads,
               "kind": "port"}
    g.close()
    return dict(elapsed=elapsed, m=m, b=b, n_src=len(mine), cpu=cpu, reps=reps)


def run_weighted_batch(g, args, n_roots=16, reps=3):
    """Johnson-style weighted rows on configs[2]'s graph: pj_sssp_batch over n_roots roots with
    1 (the serial loop), 2 and 3 delta-stepping solves in flight (delta.hip delta_batch: one
    stream, frontier ring and counter block per slot, the graph and light CSR shared); rows
    stay on the device (copy=False), median of `reps` timed batches each."""
    roots = [int(x) for x in g.sample_roots(args.seed + 7, n_roots)]
    out = {"workload": f"{n_roots} roots of configs[2]'s graph (sample_roots seed {args.seed + 7}), "
                       "one pj_sssp_batch call, rows left in HBM", "ms_per_root_by_streams": {}}
    for slots in (1, 2, 3):
        g.set_option("batch_streams", slots)
        g.sssp_batch(roots[:slots], copy=False)  # untimed: the slots' workspaces
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            g.sssp_batch(roots, copy=False)
            ts.append(time.perf_counter() - t)
        out["ms_per_root_by_streams"][str(slots)] = round(1000.0 * float(np.median(ts)) / n_roots, 4)
    g.set_option("batch_streams", 2)
    by = out["ms_per_root_by_streams"]
    out["default_streams"] = 2
    out["speedup_default_vs_serial"] = round(by["1"] / by["2"], 3)
    out["speedup_best_vs_serial"] = round(by["1"] / min(by.values()), 3)
    return out


def run_wpartitioned_host(args, world_h=2, nroots=3, scale=26):
    """The weighted 1D partition (wpart.hip + libpj's band loop: tail switch, heavy and light
    pulls through all-gathered byte maps) on configs[2]'s graph (Kronecker s26, weights
    1..255) at world 2, both ranks in this process on ONE GPU over the host transport (device
    copies + host barriers; not xGMI/RCCL): the reference's only mode (:344-594) for a graph
    split over ranks, timed per solve."""
    import paralleljohnson_amd as pj
    from paralleljohnson_amd.partition import Comm, delta_group, load_weighted_kronecker
    ctxs = [pj.Context(0) for _ in range(world_h)]
    comms = Comm.group(ctxs, "host")
    parts, roots = [], None
    try:
        g = ctxs[0].generate_kronecker(scale, args.edgefactor, args.seed, weighted=True)  # (the bench's roots)
        roots = [int(x) for x in g.sample_roots(args.seed + 1, nroots)]
        g.close()
        t0 = time.perf_counter()
        for r in range(world_h):  # each rank generates only its block's rows (pj_wpart_generate_kronecker)
            parts.append(load_weighted_kronecker(ctxs[r], scale, args.edgefactor, args.seed, r, world_h))
        build_s = time.perf_counter() - t0
        delta_group(parts, comms, roots[0])  # warm-up (workspace)
        sts = []
        t = time.perf_counter()
        for r in roots:
            sts.append(delta_group(parts, comms, r))
        elapsed = time.perf_counter() - t
        m = float(sum(st[0]["reached_edges"] for st in sts))
        st0 = sts[0]
        return {
            "workload": f"graph500-kronecker-s{scale}-ef{args.edgefactor}-w1..255-delta-stepping, 1D vertex partition "
                        f"at world {world_h}, both ranks on ONE GPU over the host transport (not xGMI/RCCL)",
            "roots": len(roots), "ms_per_sssp": round(1000.0 * elapsed / len(roots), 3),
            "gteps": round(m / elapsed / 1e9, 3), "bands": st0[0]["bands"], "light_rounds": st0[0]["rounds"],
            "heavy_pulls": st0[0]["heavy_pulls"], "light_pulls": st0[0]["bu_levels"],
            "solve_ms_max_rank": [round(max(x["solve_ms"] for x in st), 2) for st in sts],
            "pairs_sent_per_sssp_by_rank": [x["sent"] for x in st0],
            "build_s": round(build_s, 2), "build": "per block (pj_wpart_generate_kronecker)",
            "device_bytes_by_rank": [p.device_bytes() for p in parts],
        }
    finally:
        for p in parts:
            p.close()
        for c in comms:
            c.close()
        for c in ctxs:
            c.close()


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n):
    """`bench.py --gpus N` without a launcher: N rank processes of this script under torch's
    launcher on 127.0.0.1 (one per GPU, LOCAL_RANK = its GPU), started as a child process from
    a parent that never touches the GPU; rank 0's line goes straight to stdout. Returns the
    launcher's exit status."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def launch_check(rank, world, backend):
    """--launch-check: the rank bookkeeping of a run without the GPU legs -- the process group,
    the timed-region barriers and the max-over-ranks / sum-over-ranks reductions the line
    uses -- so that the N-rank launch is testable on the CPU (gloo)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group(backend="gloo" if backend != "nccl" else backend)
    el, m = 0.5 + rank, float(10 * (rank + 1))  # per-rank stand-ins for (elapsed, units processed)
    if world > 1:
        dist.barrier()
        t = torch.tensor([el, m], dtype=torch.float64)
        tm = t[:1].clone()
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        el, m = float(tm[0]), float(t[1])
    line = {"launch_check": True, "n_gpus": world, "elapsed_max": el, "units_sum": m}
    if os.environ.get("PJ_BENCH_FORCE_PART") == "1" and world > 1:
        # the partitioned leg's transport and its guard (no GPU: the gloo rehearsal's
        # host-buffer transport is rejected before any device work)
        try:
            comm = partition_transport(None, rank, world, backend)
            try:
                line["k28_partitioned"] = transport_guard(comm, world)
            finally:
                comm.close()
        except Exception as e:  # noqa: BLE001 (reported as the bench line reports it)
            line["k28_partitioned"] = {"error": f"rank {rank}: {type(e).__name__}: {e}"[:300]}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="k26w", choices=sorted(WORKLOADS))
    ap.add_argument("--scale", type=int, default=0, help="override the Kronecker scale (testing only)")
    ap.add_argument("--edgefactor", type=int, default=16)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=64, help="cap of the CPU legs' thread count")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--part-scale", type=int, default=28, help="Kronecker scale of the partitioned run (configs[3])")
    ap.add_argument("--no-partitioned", action="store_true")
    ap.add_argument("--part-timeout", type=float, default=240.0,
                    help="watchdog of the partitioned leg (s): past it the line is emitted without that leg")
    ap.add_argument("--ms-reps", type=int, default=7, help="timed MS1024 batches (median reported)")
    ap.add_argument("--no-part-host", action="store_true", help="skip the world-2 host-transport partitioned leg")
    ap.add_argument("--no-tts", action="store_true", help="skip the time-to-solution process (tuning runs)")
    ap.add_argument("--opt", action="append", default=[], help="libpj graph option key=value (tuning)")
    ap.add_argument("--launch-check", action="store_true",
                    help="test only: start the ranks, rendezvous, barrier and the max/sum reductions of the line, "
                         "no GPU work (the CPU test of the --gpus launch path)")
    args = ap.parse_args()

    # --gpus N means N ranks, one process per GPU (the reference's `mpirun -np P`, README:9).
    # Without a launcher (no WORLD_SIZE) this process starts them itself, before anything here
    # touches torch or the GPU, and only relays rank 0's line and the exit status.
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s); refusing to report a "
              f"{world}-rank run as {args.gpus} GPU(s)", file=sys.stderr)
        sys.exit(2)
    # one rank per GPU; PJ_BENCH_BACKEND=gloo rehearses the N>1 bookkeeping with several
    # ranks sharing fewer GPUs (the driver's runs use RCCL, one GPU per rank)
    backend = os.environ.get("PJ_BENCH_BACKEND", "nccl")
    if args.launch_check:
        return launch_check(rank, world, backend)

    import torch
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend=backend)

    import paralleljohnson_amd as pj

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    t_ctx = time.perf_counter()
    ctx = pj.Context(local)
    ctx_s = time.perf_counter() - t_ctx
    tts_dir = tempfile.TemporaryDirectory()
    tts = None
    if rank == 0 and WORKLOADS[args.workload]["kind"] == "kronecker" and not args.no_tts:
        tts = tts_process(args, WORKLOADS[args.workload], tts_dir.name)
        # the driver reclaims the tool's ~40 GB of device memory after it exits; allocations
        # made right then wait for it (seen as 1-3 s of "graph build" in whichever process
        # allocated next), so the GPU is left idle for a few seconds before this one builds
        time.sleep(5.0)
    main_res = run_workload(ctx, args.workload, args, rank, world, barrier, args.steps, args.warmup)
    elapsed, m_sum, b_sum, t_kernel = main_res["elapsed"], main_res["m_sum"], main_res["b_sum"], main_res["t_kernel"]
    w_sum, scanned, probes = main_res["w_sum"], main_res["scanned"], main_res["probes"]
    if dist is not None:
        t = torch.tensor([elapsed, m_sum, b_sum, t_kernel, w_sum, scanned, probes], dtype=torch.float64, device="cuda")
        tmax = t[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed = float(tmax[0])
        m_sum, b_sum, t_kernel, w_sum, scanned, probes = (float(x) for x in t[1:])
    wl = main_res["wl"]
    g = main_res["g"]
    value = m_sum / elapsed / 1e9
    work = {"achieved": w_sum / t_kernel / 1e9,  # GB/s: scanned-work bytes per solve / device time per solve
            "model_8d": b_sum / t_kernel / 1e9, "scanned": scanned, "probes": probes, "w_sum": w_sum}
    if not wl["weighted"]:  # (the unit-weight BFS has no device work counters: SURVEY.md §8d's model)
        work["achieved"] = work["model_8d"]
    traffic = measured_traffic(args) if wl["weighted"] else None

    tts_s, tts_phases = time_to_solution(ctx_s, main_res, tts, tts_dir.name) if tts else (None, None)
    tts_dir.cleanup()
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(g, main_res, args)
    n_vertices, nnz = g.n, g.nnz
    r0 = main_res["roots"][0]
    k26w_batch = None
    if world == 1 and not args.no_secondary and not args.scale and wl["weighted"]:
        k26w_batch = run_weighted_batch(g, args)
    g.close()

    secondary = {}
    if k26w_batch:
        secondary["k26w_batch"] = k26w_batch
    if world == 1 and not args.no_secondary and not args.scale:
        for key in ("k22", "wg"):
            if key == args.workload:
                continue
            res = run_workload(ctx, key, args, 0, 1, barrier, 8, 2)
            gg, rr = res["g"], res["roots"][0]
            secondary[key] = {
                "workload": res["wl"]["name"], "n_vertices": gg.n, "nnz": gg.nnz,
                "gteps": round(res["m_sum"] / res["elapsed"] / 1e9, 3),
                "ms_per_sssp": round(1000.0 * res["elapsed"] / 8, 4),
                "kernel_ms_mean": round(1000.0 * res["t_kernel"] / 8, 4),
                "hbm_frac_algorithmic": round(res["b_sum"] / res["t_kernel"] / 1e9 / HBM_PEAK_GBS, 4),
                "reached": res["reach"][rr][0], "m_r": res["reach"][rr][1],
                "levels_td_bu": list(res["levels"][rr][1:3]),
            }
            gg.close()

    if world == 1 and not args.no_secondary and not args.scale and not args.no_cpu_baseline:
        secondary["wg_cli"] = run_wg_cli(ctx, args)

    def max_sum(el, m):
        if dist is None:
            return el, m
        t = torch.tensor([el, m], dtype=torch.float64, device="cuda")
        tm = t[:1].clone()
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(tm[0]), float(t[1])

    if not args.no_secondary and not args.scale:
        ms = run_multisource(ctx, args, rank, world, barrier)
        el, m = max_sum(ms["elapsed"], ms["m"])
        _, bsum = max_sum(ms["elapsed"], ms["b"])
        secondary["ms1024"] = {
            "workload": "web-google-shaped-synthetic, 1024 sources (smallest ids with out-degree >= 1), "
                        "up to 512 per batched pass (one 64-bit mask word per 64 sources), source-sharded over the ranks",
            "sources_per_rank": ms["n_src"], "batch_ms": round(1000.0 * el, 3),
            "batch_ms_stat": f"median of {len(ms['reps'])} timed batches (max over ranks of each rank's median)",
            "batch_ms_min_max_rank0": [round(1000.0 * min(ms["reps"]), 3), round(1000.0 * max(ms["reps"]), 3)],
            "gteps": round(m / el / 1e9, 3), "scaling": "strong (1024 sources in total)",
            # B summed over the sources; the batched passes share the CSR reads,
            # so this "effective" rate can exceed the HBM peak: a reuse factor, not a fraction
            "algorithmic_bytes_sum": bsum,
            "reuse_factor_vs_hbm_peak": round(bsum / el / 1e9 / (HBM_PEAK_GBS * world), 3),
        }
        if ms["cpu"]:
            secondary["ms1024"]["cpu_baseline"] = ms["cpu"]
    mean_ms = 1000.0 * elapsed / args.steps

    def emit():
        if rank == 0:
            print(json.dumps(line(main_res, wl, value, mean_ms, work, traffic, tts_s, tts_phases, cpu, secondary,
                                  n_vertices, nnz, t_kernel, world, args)), flush=True)

    force_part = os.environ.get("PJ_BENCH_FORCE_PART") == "1"  # (tests the guard under a gloo rehearsal)
    if not args.no_partitioned and not args.scale and (world == 1 or backend == "nccl" or force_part):
        # (a gloo rehearsal shares one GPU between ranks; RCCL needs a GPU per rank)
        # The partitioned leg is the only one with a data-path collective (libpj's RCCL
        # group). Guard it: an exception becomes an error entry, and a watchdog on every
        # rank emits the line without it and ends the process if a collective hangs.
        import threading

        def on_timeout():
            secondary["k28_partitioned"] = {"error": f"not finished within {args.part_timeout:.0f} s (watchdog)"}
            emit()
            os._exit(3)  # the line is out; a hung collective still fails the run

        wd = threading.Timer(args.part_timeout, on_timeout)
        wd.daemon = True
        wd.start()
        try:
            pr = run_partitioned(ctx, args, rank, world, barrier, backend)
        except Exception as e:  # noqa: BLE001 (reported in the line, not fatal to it)
            pr = None
            secondary["k28_partitioned"] = {"error": f"rank {rank}: {type(e).__name__}: {e}"[:300]}
        # every rank reaches this collective (the watchdog covers a rank stuck in RCCL)
        el, n_ok = max_sum(pr["elapsed"] if pr else 0.0, 1.0 if pr else 0.0)
        wd.cancel()
        if pr is not None and int(round(n_ok)) != world:
            pr = None
            secondary["k28_partitioned"] = {"error": f"failed on {world - int(round(n_ok))} rank(s)"}
    else:
        pr = None
    if world == 1 and pr is not None and not args.no_part_host:
        try:
            secondary["k28_partitioned_host_w2"] = run_partitioned_host(args)
        except Exception as e:  # noqa: BLE001
            secondary["k28_partitioned_host_w2"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        try:
            secondary["k26w_partitioned_host_w2"] = run_wpartitioned_host(args)
        except Exception as e:  # noqa: BLE001
            secondary["k26w_partitioned_host_w2"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    if pr is not None:
        per = el / pr["roots"]
        secondary["k28_partitioned"] = {
            "workload": f"graph500-kronecker-s{args.part_scale}-ef{args.edgefactor}-unit-bfs, 1D vertex "
                        f"partition over {world} GPU(s), libpj level loop, transport {pr['transport']['transport']}",
            **pr["transport"],
            "n_vertices": pr["n"], "nnz": 2 * (args.edgefactor << args.part_scale),
            "nnz_local_rank0": pr["nnz_local"], "roots": pr["roots"],
            "time_to_solution_ms": round(1000.0 * per, 3),
            "gteps": round(pr["m"] / el / 1e9, 3), "gteps_graph500": round(pr["m"] / el / 2e9, 3),
            "hbm_frac_algorithmic": round(pr["b"] / el / 1e9 / (HBM_PEAK_GBS * world), 4),
            "levels_td_bu": [pr["st0"]["td_levels"], pr["st0"]["bu_levels"]],
            "build_s": round(pr["build_s"], 2), "build_phases_rank0": pr["build_phases"],
            "scaling": "strong (one graph, all ranks)",
        }

    emit()
    if dist is not None:
        dist.destroy_process_group()


def measured_traffic(args):
    """The DRAM-side bytes per k26w solve of the last per-kernel table (tools/cycle.sh wtable ->
    profiles/traffic_k26w.json) and its per-kernel rows -- only when the table was measured on
    the loaded build (pj_build_id(): a digest of libpj's sources and flags); otherwise the
    line carries traffic null and says why."""
    import paralleljohnson_amd as pj
    path = os.path.join(ROOT, "profiles", f"traffic_{args.workload}.json")
    if args.scale or args.opt:
        return {"bytes": None, "note": "not measured for this configuration"}
    if not os.path.exists(path):
        return {"bytes": None, "note": f"{os.path.relpath(path, ROOT)} missing"}
    with open(path) as f:
        tj = json.load(f)
    if tj.get("build_id") != pj.build_id():
        return {"bytes": None, "note": f"{os.path.relpath(path, ROOT)} was measured on build {tj.get('build_id')}, "
                                       f"the loaded libpj is {pj.build_id()}: stale, not reported"}
    return {"bytes": tj["hbm_bytes_per_sssp"], "table": tj, "path": os.path.relpath(path, ROOT)}


def gather_ceiling(probes_per_solve, t_solve):
    """The probes' rate against the chip's random-gather ceiling, measured by the FETCH_SIZE
    calibration (profiles/r06/gather_calib.json: random 4-byte words from a 4 GiB table, each
    a 128-byte memory-side request): the bound of a latency- and line-bound kernel whose bytes
    fraction says little (a 4-byte probe moves a 128-byte line)."""
    path = os.path.join(ROOT, "profiles", "r06", "gather_calib.json")
    if not probes_per_solve or not os.path.exists(path):
        return {}
    with open(path) as f:
        cal = json.load(f)
    ceil = cal["random_dword_gathers_per_s"]
    rate = probes_per_solve / t_solve
    return {"probe_rate_per_s": round(rate), "probe_ceiling_per_s": round(ceil),
            "probe_frac": round(rate / ceil, 4),
            "probe_ceiling_source": "profiles/r06/gather_calib.json (tools/calib/gather_calib.hip, cal_dwords_k)"}


def line(main_res, wl, value, mean_ms, work, traffic, tts_s, tts_phases, cpu, secondary, n_vertices, nnz,
         t_kernel, world, args):
    """The one JSON line of the run (rank 0)."""
    r0 = main_res["roots"][0]
    lv = main_res["levels"][r0]
    solves = args.steps * world
    t_solve = t_kernel / solves  # device seconds per solve
    roofline = {
        "bound": "hbm",
        "achieved": round(work["achieved"], 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(work["achieved"] / HBM_PEAK_GBS, 4),
        "traffic": None,
        "traffic_frac": None,
        "model": ("scanned work, counted on the device in every timed solve: 4N + n_r(12 + 2*O) + the edge records "
                  "read as stored (4-byte packed light CSR, 5-byte u32 id + u8 weight) + the probes of their other "
                  "ends (4-byte dist, 1-byte heavy-pull map); time = HIP events on libpj's stream, all kernels of a "
                  "solve" if wl["weighted"] else "SURVEY.md §8d (unit-weight BFS: no work counters)"),
        "bytes_per_sssp": round(work["w_sum"] / solves),
        "scanned_edges_per_sssp": round(work["scanned"] / solves),
        "probes_per_sssp": round(work["probes"] / solves),
        "frac_model_8d": round(work["model_8d"] / HBM_PEAK_GBS, 4),
        **gather_ceiling(work["probes"] / solves, t_solve),
        "model_8d": "SURVEY.md §8d: 4N + n_r(12 + 2*O) + m_r(8 + 4*weighted), every reached edge read; the solve "
                    "scans a fraction of them (a pull stops a row at its first useless weight), so this figure can "
                    "exceed 1 and bounds nothing",
    }
    if traffic is not None:
        roofline["traffic_note"] = traffic.get("note")
        if traffic.get("bytes"):
            tb, tab = traffic["bytes"], traffic["table"]
            roofline["traffic"] = round(tb)
            roofline["traffic_frac"] = round(tb / t_solve / 1e9 / HBM_PEAK_GBS, 4)
            roofline["traffic_note"] = (f"DRAM-side bytes per solve of {traffic['path']} (build {tab['build_id']}, "
                                        f"the loaded one): (RDREQ - RDREQ_32B) x {tab['bytes_per_request']:.0f} + "
                                        f"RDREQ_32B x 32 + WRITE_SIZE, calibrated by {tab['calibration']}; "
                                        f"Infinity-Cache hits included (an upper bound)")
            dom = max(tab["kernels"], key=lambda r: r["ms"])
            roofline["dominant_kernel"] = {
                "kernel": dom["kernel"], "ms_per_sssp": round(dom["ms"], 4),
                "work_bytes": round(dom["work_bytes"]), "dram_bytes": round(dom["dram_bytes"]),
                "work_frac": round(dom["work_bytes"] / (dom["ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "dram_frac": round(dom["dram_bytes"] / (dom["ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "source": traffic["path"] + " (rocprofv3 kernel trace + --pmc passes of tools/traffic_probe.py)"}
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
        "data": (f"synthetic: Graph500 Kronecker (A,B,C=0.57,0.19,0.19) generated on the device, seed "
                 f"{args.seed}, both directions" + (", weights 1 + hash mod 255" if wl["weighted"] else "")
                 if wl["kind"] == "kronecker" else "synthetic web-Google-shaped graph (SNAP file absent)"),
        "config": {
            "workload": wl["name"] if not args.scale else f"{wl['name']} (scale override {args.scale})",
            "n_vertices": n_vertices, "nnz": nnz, "roots_per_rank": args.steps,
            "parallelism": f"source-sharded x{world} (graph replicated, no data-path collective)",
        },
        "gteps_graph500": round(value / 2, 3),
        "ms_per_sssp": round(mean_ms, 4),
        "scanned_edges_per_sssp": round(work["scanned"] / solves),
        "m_r_per_sssp": round(main_res["m_sum"] / args.steps),
        "time_to_solution_s": tts_s,
        "time_to_solution_phases": tts_phases,
        "scaling_note": ("N>1: the graph is replicated and the roots are sharded (no exchange between GPUs), "
                         "i.e. ideal weak scaling; the partitioned multi-GPU solve is secondary.k28_partitioned"),
        "kernel_ms_mean": round(1000.0 * t_solve, 4),
        "step": ("one SSSP: distances initialised -> final in the solver's degree-ordered ids on the device; the "
                 "gather to input ids (0.2 ms at s26) runs with the first read of the result (D2H, sol_file, "
                 "pj_dist_device) and is inside time_to_solution_s"),
        "bands_or_levels": lv[0], "relax_launches": lv[3],
        "roofline": roofline,
        "cpu_baseline": cpu,
        "secondary": secondary or None,
    }
    return out


def run_wg_cli(ctx, args):
    """configs[0] end to end: the web-Google-shaped synthetic written as a SNAP text file, the
    parallel_johnson CLI timed from process start to sol_file closed (time-to-solution: HIP
    init, GPU parse + CSR, solve, output), next to the reference's BSP algorithm at np = 4
    (oracle port of :466-594, the `mpirun -np 4` analogue) on the same graph, sol_file bytes
    compared."""
    import hashlib
    import subprocess
    import tempfile

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # cpu_baseline leg only (reference timing and the byte comparison)
    import paralleljohnson_amd as pj

    O.build()
    g = ctx.generate_webgraph(seed=args.seed)
    row, col, _ = g.get_csr()
    g.close()
    col = col.view(np.uint32)
    src = np.repeat(np.arange(len(row) - 1, dtype=np.int64), np.diff(row))
    with tempfile.TemporaryDirectory() as td:
        path, out = os.path.join(td, "web-Google-synthetic.txt"), os.path.join(td, "sol.txt")
        body = np.char.add(np.char.add(src.astype(str), "\t"), col.astype(np.int64).astype(str))
        with open(path, "wb") as f:
            f.write(("# Directed graph (synthetic, web-Google-shaped)\n# FromNodeId\tToNodeId\n" +
                     "\n".join(body.tolist()) + "\n").encode())
        del body, src
        walls = []
        for _ in range(3):
            t0 = time.perf_counter()
            r = subprocess.run([pj.cli_path(), path, "0", out], capture_output=True, text=True, timeout=300)
            walls.append(time.perf_counter() - t0)
            if r.returncode != 0:
                raise RuntimeError(f"parallel_johnson failed: {r.stderr[-500:]}")
        t_line = r.stdout.strip()
        got = open(out, "rb").read()
        text_mb = os.path.getsize(path) / 1e6
        # configs[4] through the drop-in: 1024 sources (PJ_SOURCES), one sol_file each
        srcs = np.nonzero(np.diff(row) >= 1)[0][:1024]
        lst, odir = os.path.join(td, "sources.txt"), os.path.join(td, "ms")
        os.makedirs(odir)
        with open(lst, "w") as f:
            f.write("\n".join(map(str, srcs)) + "\n")
        t0 = time.perf_counter()
        r = subprocess.run([pj.cli_path(), path, "0", os.path.join(odir, "sol_{s}.txt")], capture_output=True, text=True,
                           timeout=600, env=dict(os.environ, PJ_SOURCES="@" + lst))
        ms_wall = time.perf_counter() - t0
        if r.returncode != 0:
            raise RuntimeError(f"parallel_johnson PJ_SOURCES failed: {r.stderr[-500:]}")
        ms_files = os.listdir(odir)
        ms_bytes = sum(os.path.getsize(os.path.join(odir, x)) for x in ms_files)
        ms_first = open(os.path.join(odir, f"sol_{srcs[0]}.txt"), "rb").read()
        ms_cli = {"sources": int(len(srcs)), "files": len(ms_files), "bytes_written": ms_bytes,
                  "time_to_solution_s": round(ms_wall, 3), "time_line": r.stdout.strip()}
    ms_cli["first_file_identical_to_oracle"] = ms_first == O.format_sol(O.bfs(row, col, int(srcs[0])))
    t0 = time.perf_counter()
    ref, st = O.reference_sssp(row, col, 0, 4)
    ref_s = time.perf_counter() - t0
    exp = O.format_sol(ref)
    m_r = int(np.diff(row)[ref < 100000].sum())
    np_scan = {}  # np = 1, 4 and the host threads bench.py uses
    for p in sorted({1, 4, max(1, min(args.cpu_threads, cpu_share()))}):
        if p == 4:
            np_scan[p] = round(st.solve_s, 4)
            continue
        d_p, st_p = O.reference_sssp(row, col, 0, p)
        if not (d_p == ref).all():
            raise RuntimeError(f"reference algorithm at np={p} disagrees with np=4")
        np_scan[p] = round(st_p.solve_s, 4)
    return {
        "workload": "web-google-shaped-synthetic, SNAP text file, source 0, parallel_johnson CLI end to end",
        "text_mb": round(text_mb, 1), "n_vertices": len(row) - 1, "nnz": int(len(col)),
        "time_to_solution_s": round(min(walls), 3), "time_line": t_line,
        "sol_bytes_identical_to_reference_np4": got == exp,
        "sol_sha256": hashlib.sha256(got).hexdigest()[:16],
        "reference_np4_solve_s": round(st.solve_s, 3), "reference_np4_wall_s": round(ref_s, 3),
        "reference_np4_gteps": round(m_r / st.solve_s / 1e9, 5), "reference_cores": 4,
        "reference_kind": "port (oracle restatement of the reference's BSP heap algorithm, 4 host threads)",
        "reference_solve_s_by_np": np_scan,
        "ms1024_drop_in": ms_cli,
        **host_cpu(),
    }


def cpu_baseline(g, res, args):
    """The reference algorithm (oracle port of :466-594) on host threads, bounded sample of one
    solve, at np = 1, 4 and the box's CPU share; `value` is the fastest leg."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # cpu_baseline leg only

    O.build()
    row, col, w = g.get_csr()
    col = col.view(np.uint32)
    share = max(1, min(args.cpu_threads, cpu_share()))
    r = res["roots"][0]
    m_r = res["reach"][r][1]
    legs = {}
    for p in sorted({1, 4, share}):
        if p > share:
            continue
        _, st = O.reference_sssp(row, col, r, p, w=w, budget_s=args.cpu_seconds)
        rate = (st.scans if st.truncated else m_r) / st.solve_s
        legs[p] = {"gteps": round(rate / 1e9, 5), "solve_s": round(st.solve_s, 3), "truncated": bool(st.truncated),
                   "scans": int(st.scans), "rounds": int(st.rounds)}
    best = max(legs, key=lambda p: legs[p]["gteps"])
    del row, col, w
    return {
        "value": legs[best]["gteps"],
        "unit": "GTEPS",
        "cores": best,
        "kind": "port",
        "sample": (f"one solve (root {r}) of the same graph per leg, each bounded to {args.cpu_seconds:g} s of "
                   f"solve time (a truncated leg stops at a round boundary and counts CSR entries scanned/s); "
                   f"reference BSP heap algorithm, 30 pops/round, np partitions on np host threads; value = the "
                   f"fastest leg (np = {best})"),
        "by_np": legs,
        "cpu_share": share,
        **host_cpu(),
    }


if __name__ == "__main__":
    main()
