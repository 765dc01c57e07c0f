"""1D vertex-partitioned solves: libpj's C++ protocol loops
(engine.cpp: the BFS level loop and the delta-stepping band loop, the analogue of
the reference's BSP round loop ParallelJohnson.cpp:488-594 with its
Alltoall(v) / Allreduce exchange :522-554 / :589-590).

CPU: the same C++ loops over a numpy restatement of the device steps
(tests/part_numpy.py), at world 1 and over gloo at world 2-3 (pj_engine_bfs /
pj_engine_delta with a callback transport). GPU: the product path -- libpj's
kernels (pj_part_* / pj_wpart_*), the loops inside pj_part_bfs / pj_wpart_delta,
over the in-process transports (ranks sharing the one GPU through device copies;
RCCL at world 1) and through the CLI at P = 1, 2, 3.

Bar: bit-exact distances against the oracle BFS / Dijkstra (the reference's R9
contract); partitioning is result-neutral."""
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from conftest import ROOT
from helpers import random_graph, to_text

INF = 100000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _csr(oracle, s, d, n, w=None):
    return oracle.coo2csr(np.asarray(s, np.int64), np.asarray(d, np.int64), n, w)


def _oracle_dist(oracle, src, dst, n, source):
    if not 0 <= source < n:
        return np.full(n, INF, np.int32)
    row, col, _ = _csr(oracle, src, dst, n)
    return oracle.bfs(row, col, source)


def _cases():
    rng = np.random.default_rng(2024)
    out = []
    for kind, n in (("uniform", 300), ("hub", 700), ("chain", 257), ("uniform", 64), ("hub", 1500)):
        s, d = random_graph(rng, kind, n)
        out.append((kind, n, s.astype(np.int64), d.astype(np.int64)))
    # symmetric (both directions written, like the Kronecker inputs)
    s, d = random_graph(rng, "hub", 900)
    out.append(("sym", 900, np.concatenate([s, d]).astype(np.int64), np.concatenate([d, s]).astype(np.int64)))
    return out


def _wcases():
    rng = np.random.default_rng(99)
    out = []
    for kind, n, wmax in (("uniform", 500, 300), ("hub", 900, 40), ("chain", 300, 5), ("uniform", 64, 2)):
        s, d = random_graph(rng, kind, n)
        w = rng.integers(0 if kind == "uniform" else 1, wmax, len(s)).astype(np.uint32)
        out.append((kind, n, s.astype(np.int64), d.astype(np.int64), w))
    return out


class LocalTransport:
    """world 1: the collectives are copies (CPU tests of the loops without gloo)."""

    def allreduce(self, vals, is_min):
        pass

    def alltoall_counts(self, send, recv):
        recv[:] = send

    def alltoallv(self, send_ptr, scounts, recv_ptr, rcounts, elem):
        from paralleljohnson_amd.partition import _host
        nb = int(scounts[0]) * elem
        if nb:
            _host(recv_ptr, nb)[:] = _host(send_ptr, nb)

    def allgather(self, own_ptr, all_ptr, nbytes):
        from paralleljohnson_amd.partition import _host
        if own_ptr != all_ptr:
            _host(all_ptr, nbytes)[:] = _host(own_ptr, nbytes)


# ----------------------------------------------------------------- CPU ----

def test_block_geometry():
    from paralleljohnson_amd.partition import block_geometry
    for n in (0, 1, 63, 64, 65, 1000, 4096, 100003):
        for world in (1, 2, 3, 8):
            block, ranges = block_geometry(n, world)
            assert block % 64 == 0 and block >= 64
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            for r in range(world - 1):
                assert ranges[r][1] == ranges[r + 1][0]
            for v in range(0, n, max(1, n // 97)):
                r = v // block
                assert ranges[r][0] <= v < ranges[r][1]


@pytest.mark.parametrize("force", [0, 1, 2])
def test_engine_world1_numpy(oracle, force):
    """libpj's BFS level loop (pj_engine_bfs) over numpy steps, one rank."""
    from part_numpy import NumpyPart
    from paralleljohnson_amd.partition import Comm, engine_bfs
    comm = Comm.from_callbacks(LocalTransport(), 0, 1)
    for kind, n, s, d in _cases():
        ops = NumpyPart(s, d, n, 0, 1, symmetric=(kind == "sym"))
        for source in (0, n // 3, n - 1, n + 5, -1):
            st = engine_bfs(ops, comm, source, force=force)
            exp = _oracle_dist(oracle, s, d, n, source)
            assert np.array_equal(ops.dist_local(), exp), (kind, source, force)
            assert st["reached"] == int((exp < INF).sum())
            if force == 1:
                assert st["bu_levels"] == 0
            if force == 2 and st["levels"]:
                assert st["td_levels"] == 0


def _rank_main(rank, world, port, path, force, weighted):
    """One rank of a gloo job running libpj's C++ loop over numpy steps; rank 0 saves."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from gloo_transport import GlooTransport, gather_blocks
    from part_numpy import NumpyPart, NumpyWPart
    from paralleljohnson_amd.partition import Comm, engine_bfs, engine_delta
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Comm.from_callbacks(GlooTransport(), rank, world)
    res = {}
    if not weighted:
        for ci, (kind, n, s, d) in enumerate(_cases()):
            ops = NumpyPart(s, d, n, rank, world, symmetric=(kind == "sym"))
            for source in (0, n // 3, n - 1, n + 5):
                st = engine_bfs(ops, comm, source, force=force)
                res[f"{ci}_{source}"] = gather_blocks(ops.dist_local(), ops.block, world, n)
                res[f"{ci}_{source}_st"] = np.array([st["reached"], st["reached_edges"], st["sent"]])
    else:
        for i, (_, n, s, d, w) in enumerate(_wcases()):
            ops = NumpyWPart(s, d, w, n, rank, world)
            for delta in (0, 7, 60):
                for source in (0, n // 3, n - 1, n + 2):
                    st = engine_delta(ops, comm, source, delta)
                    res[f"c{i}_{delta}_{source}"] = gather_blocks(ops.dist_local(), ops.block, world, n)
                    res[f"c{i}_{delta}_{source}_reached"] = np.array([st["reached"], st["reached_edges"]])
    if rank == 0:
        np.savez(path, **res)
    dist.barrier()
    dist.destroy_process_group()


def _run_world(world, force=0, weighted=False):
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "res.npz")
        mp.spawn(_rank_main, args=(world, _free_port(), path, force, weighted), nprocs=world, join=True)
        with np.load(path) as z:
            return {k: z[k] for k in z.files}


@pytest.mark.parametrize("world,force", [(2, 0), (2, 1), (2, 2), (3, 0)])
def test_engine_gloo_numpy(oracle, world, force):
    """The C++ level loop at world 2-3 over gloo: count exchange, Alltoallv of claimed ids,
    all-gathered visited bitmaps around pull levels, sum termination."""
    res = _run_world(world, force)
    for ci, (kind, n, s, d) in enumerate(_cases()):
        for source in (0, n // 3, n - 1, n + 5):
            exp = _oracle_dist(oracle, s, d, n, source)
            assert np.array_equal(res[f"{ci}_{source}"], exp), (world, force, kind, source)
            row, _, _ = _csr(oracle, s, d, n)
            reached = exp < INF
            assert res[f"{ci}_{source}_st"][:2].tolist() == [int(reached.sum()), int(np.diff(row)[reached].sum())]
    # push levels exchange ids between the ranks (the protocol is exercised, not bypassed)
    assert any(res[k][2] > 0 for k in res if k.endswith("_st")) or force == 2


def _wexpected(oracle):
    out = []
    for i, (_, n, s, d, w) in enumerate(_wcases()):
        row, col, wc = oracle.coo2csr(s.astype(np.uint32), d.astype(np.uint32), n, w)
        out.append((f"c{i}", n, row, col, wc))
    return out


def _wcheck(res, exp_graphs, oracle, deltas, world):
    for name, n, row, col, wc in exp_graphs:
        for source in (0, n // 3, n - 1, n + 2):
            exp = oracle.dijkstra(row, col, wc, source) if source < n else np.full(n, INF, np.int32)
            reached = exp < INF
            for delta in deltas:
                got = res[f"{name}_{delta}_{source}"]
                assert np.array_equal(got, exp), (name, delta, source, world)
                assert res[f"{name}_{delta}_{source}_reached"].tolist() == [
                    int(reached.sum()), int(np.diff(row)[reached].sum())], (name, delta, source)


def test_wengine_world1_numpy(oracle):
    """libpj's band loop (pj_engine_delta) without an exchange, numpy device steps."""
    from part_numpy import NumpyWPart
    from paralleljohnson_amd.partition import Comm, engine_delta
    comm = Comm.from_callbacks(LocalTransport(), 0, 1)
    res = {}
    for i, (_, n, s, d, w) in enumerate(_wcases()):
        ops = NumpyWPart(s, d, w, n, 0, 1)
        for delta in (0, 1, 7, 60):
            for source in (0, n // 3, n - 1, n + 2):
                st = engine_delta(ops, comm, source, delta)
                res[f"c{i}_{delta}_{source}"] = ops.dist_local()
                res[f"c{i}_{delta}_{source}_reached"] = np.array([st["reached"], st["reached_edges"]])
    _wcheck(res, _wexpected(oracle), oracle, (0, 1, 7, 60), 1)


@pytest.mark.parametrize("world", [2, 3])
def test_wengine_gloo_numpy(oracle, world):
    """The C++ band loop at world 2-3 over gloo: Alltoallv of packed (id, cand) pairs,
    all-reduced sum/min termination; bit-exact vs the oracle Dijkstra."""
    res = _run_world(world, weighted=True)
    _wcheck(res, _wexpected(oracle), oracle, (0, 7, 60), world)


def test_engine_step_failure_is_reported(oracle):
    """A failing step surfaces as an exception, not a hang or a wrong answer."""
    from part_numpy import NumpyPart
    from paralleljohnson_amd.partition import Comm, engine_bfs
    kind, n, s, d = _cases()[0]
    ops = NumpyPart(s, d, n, 0, 1)

    def boom(level):
        raise RuntimeError("step failed")
    ops.push = boom
    with pytest.raises(RuntimeError, match="step failed"):
        engine_bfs(ops, Comm.from_callbacks(LocalTransport(), 0, 1), 0)


# ----------------------------------------------------------------- GPU ----

def _group(pj, world, transport="host"):
    from paralleljohnson_amd.partition import Comm
    ctxs = [pj.Context(0) for _ in range(world)]
    return ctxs, Comm.group(ctxs, transport)


@pytest.mark.gpu
@pytest.mark.parametrize("force", [0, 1, 2])
@pytest.mark.parametrize("transport", ["self", "rccl"])
def test_part_world1_gpu(ctx, oracle, force, transport):
    """pj_part_bfs at world 1: no transport, and a one-rank RCCL group (the RCCL calls
    of the loop -- allreduce, allgather, grouped send/recv -- with nothing to send). Option
    single_gpu 1 (default) solves with bfs.hip's single-GPU BFS on the partition's borrowed
    rows, 0 with the level loop; both alternate on one partition (the arrays go back after
    each borrowed solve)."""
    from paralleljohnson_amd.partition import Comm, load_coo
    comm = Comm.for_rank(ctx, 1, 0, Comm.unique_id() if transport == "rccl" else None)
    assert comm.kind == transport
    for kind, n, s, d in _cases():
        ops = load_coo(ctx, s, d, n, 0, 1, symmetric=(kind == "sym"))
        ops.set_option("direction", force)
        row, _, _ = _csr(oracle, s, d, n)
        for source in (0, n // 3, n - 1, n + 5, -1):
            exp = _oracle_dist(oracle, s, d, n, source)
            reached = exp < INF
            for single in (1, 0):
                ops.set_option("single_gpu", single)
                st = ops.bfs(comm, source)
                got = ops.gather_dist(comm)
                assert np.array_equal(got, exp), (kind, source, force, single)
                assert st["reached"] == int(reached.sum()) and ops.reach()[0] == st["reached"]
                assert st["reached_edges"] == int(np.diff(row)[reached].sum()), (kind, source, force, single)
                if force == 1:
                    assert st["bu_levels"] == 0
        ops.close()
    comm.close()


@pytest.mark.gpu
def test_part_kronecker_matches_single_gpu(ctx, pj, oracle):
    """The partitioned generator yields the same graph: s16, world 1, vs pj.Graph and the oracle."""
    from paralleljohnson_amd.partition import Comm, load_kronecker
    g = ctx.generate_kronecker(16, 16, 3)
    row, col, _ = g.get_csr()
    ops = load_kronecker(ctx, 16, 16, 3, 0, 1)
    comm = Comm.for_rank(ctx, 1, 0)
    assert ops.nnz_local == g.nnz
    for r in g.sample_roots(5, 4):
        exp = oracle.bfs(row, col.view(np.uint32), int(r))
        for single in (1, 0):  # (bfs.hip on the borrowed rows, then the level loop)
            ops.set_option("single_gpu", single)
            st = ops.bfs(comm, int(r))
            got = ops.gather_dist(comm)
            assert np.array_equal(got, g.sssp(int(r))), (r, single)
            assert np.array_equal(got, exp), (r, single)
            rs = g.reach_stats()
            assert (st["reached"], st["reached_edges"]) == (rs["reached"], rs["reached_edges"])
            assert st["td_levels"] >= 1 and st["bu_levels"] >= 1  # both directions exercised
    ops.close()
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world,force,cap", [(2, 0, -1), (2, 1, -1), (2, 2, -1), (3, 0, -1), (2, 1, 64), (3, 0, 200)])
def test_part_group_one_gpu(pj, oracle, world, force, cap):
    """world ranks of one process sharing the one GPU (host transport: device copies between
    the ranks' buffers, one host thread per rank): libpj kernels + the C++ level loop + the
    exchange end to end, on random graphs and Kronecker s14; with a small exchange_cap the
    big push levels go out in pieces (word ranges of the owners' slices)."""
    from paralleljohnson_amd.partition import bfs_group, gather_group, load_coo, load_kronecker
    ctxs, comms = _group(pj, world)
    assert all(c.kind == "host" for c in comms)
    sent = 0
    for kind, n, s, d in _cases():
        parts = [load_coo(ctxs[r], s, d, n, r, world, symmetric=(kind == "sym")) for r in range(world)]
        for p in parts:
            p.set_option("direction", force)
            p.set_option("exchange_cap", cap)
        row, _, _ = _csr(oracle, s, d, n)
        for source in (0, n // 3, n - 1, n + 5):
            st = bfs_group(parts, comms, source)
            exp = _oracle_dist(oracle, s, d, n, source)
            assert np.array_equal(gather_group(parts, comms), exp), (kind, source)
            reached = exp < INF
            assert [st[0]["reached"], st[0]["reached_edges"]] == [int(reached.sum()),
                                                                  int(np.diff(row)[reached].sum())]
            assert len({x["levels"] for x in st}) == 1  # every rank ran the same levels
            sent += sum(x["sent"] for x in st)
        for p in parts:
            p.close()
    assert sent > 0 or force == 2
    k = oracle.kronecker(14, 16, 7)
    krow, kcol, _ = oracle.coo2csr(k[0], k[1], 1 << 14)
    parts = [load_kronecker(ctxs[r], 14, 16, 7, r, world) for r in range(world)]
    for p in parts:
        p.set_option("direction", force)
        p.set_option("exchange_cap", cap)
    for source in (1, 777, 12345):
        bfs_group(parts, comms, source)
        assert np.array_equal(gather_group(parts, comms), oracle.bfs(krow, kcol, source)), source
    if cap > 0:  # the buffers stay near the cap (pieces are word ranges: up to ~2x on skew)
        for p in parts:
            assert p.device_bytes()["exchange"] <= 2 * 4 * 1.25 * 3 * cap + 64, p.device_bytes()
    for p in parts:
        p.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world,transport", [(1, "rccl"), (2, "host"), (3, "host")])
def test_wpart_group(pj, oracle, world, transport):
    """Weighted SSSP over the 1D partition (wpart.hip + the C++ band loop): every rank on the
    one GPU; bit-exact against the oracle Dijkstra for several band widths and sources, with
    the tail switch (all-reduced unsettled-edge count, then a 64x / 3x light threshold) at its
    default, forced right after the first band, and off; heavy steps pushed, pulled (the
    Kronecker case: unsettled vertices scan their heavy rows through the all-gathered member
    map) by the default rule, and pulled whenever the graph allows; light rounds pushed, pulled by
    the default rule and pulled whenever the frontier is big enough."""
    from paralleljohnson_amd.partition import delta_group, gather_group, load_weighted
    ctxs, comms = _group(pj, world, transport)
    cases = [(f"c{i}", n, ctxs[0].load_coo(s, d, w=w, n=n)) for i, (_, n, s, d, w) in enumerate(_wcases())]
    cases.append(("k12", 1 << 12, ctxs[0].generate_kronecker(12, 16, 3, weighted=True)))
    for name, n, g0 in cases:
        row, col, wc = g0.get_csr()
        col = col.view(np.uint32)
        parts = []
        for r in range(world):
            gr = g0 if r == 0 else None
            if gr is None:  # each rank cuts its block from a graph on its own context
                gr = ctxs[r].load_coo(np.repeat(np.arange(n), np.diff(row)), col, w=wc, n=n)
            parts.append(load_weighted(ctxs[r], gr, r, world))
            if r:
                gr.close()
        g0.close()
        # (delta 60, light pull always: light rows of hundreds of edges, the long-row chunk list)
        # (world 1: the single-GPU solver, option single_gpu 1, then the band loop over
        # wpart.hip's kernels that every rank runs at world > 1)
        for single in ((1, 0) if world == 1 else (1,)):
            for delta, tf, tm, pf, lp in ((0, 0.1, 64, 4, 3), (7, 2.0, 3, 1e9, 1e9), (60, 0.0, 64, 0, 0),
                                          (7, 0.1, 64, 1e9, 3), (0, 0.0, 64, 4, 1e9), (60, 0.1, 64, 4, 1e9)):
                for p in parts:
                    p.set_option("single_gpu", single)
                    p.set_option("tail_frac", tf)
                    p.set_option("tail_mult", tm)
                    p.set_option("pull_factor", pf)
                    p.set_option("light_pull", lp)
                for source in (0, n // 3, n - 1, n + 2):
                    st = delta_group(parts, comms, source, delta)
                    exp = oracle.dijkstra(row, col, wc, source) if source < n else np.full(n, INF, np.int32)
                    assert np.array_equal(gather_group(parts, comms), exp), (name, delta, tf, tm, pf, lp, source,
                                                                             world, single)
                    reached = exp < INF
                    assert [st[0]["reached"], st[0]["reached_edges"]] == [int(reached.sum()),
                                                                          int(np.diff(row)[reached].sum())]
        for p in parts:
            p.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_wpart_generate_kronecker_blocks(pj, oracle, world):
    """pj_wpart_generate_kronecker: each rank enumerates the weighted generator and keeps its
    block's rows only. The blocks' entry counts are the single-GPU CSR's row sums over the
    block, every rank has the whole graph's nnz (the automatic delta's mean weight), and the
    gathered distances equal the oracle Dijkstra on the single-GPU CSR; the exchange buffers
    stay traffic-sized."""
    from paralleljohnson_amd.partition import delta_group, gather_group, load_weighted_kronecker
    ctxs, comms = _group(pj, world, "host")
    for scale, ef, seed in ((10, 16, 5), (12, 8, 6)):
        g0 = ctxs[0].generate_kronecker(scale, ef, seed, weighted=True)
        row, col, wc = g0.get_csr()
        col = col.view(np.uint32)
        n = g0.n
        g0.close()
        parts = [load_weighted_kronecker(ctxs[r], scale, ef, seed, r, world) for r in range(world)]
        for p in parts:
            assert p.nnz == row[-1] and p.nnz_local == row[p.hi] - row[p.lo], (scale, p.rank)
        sent = [0] * world
        for source in (0, n // 3, n - 1):
            st = delta_group(parts, comms, source)
            exp = oracle.dijkstra(row, col, wc, source)
            assert np.array_equal(gather_group(parts, comms), exp), (scale, world, source)
            assert st[0]["reached"] == int((exp < INF).sum())
            sent = [max(a, x["sent"]) for a, x in zip(sent, st)]
        for p in parts:
            b = p.device_bytes()
            # the receive buffer (at most 2n pairs), the claim queue (shards at twice a round's
            # average, a spill of its pairs, <= the pairs the rank sent in a solve, beyond the
            # initial 96 x 16 + 4096) and the send buffer the engine packs into (the queue's capacity)
            q0 = 96 * 16 + 4096 + 16 * 64
            assert b["rows"] > 0 and b["exchange"] <= 8 * (2 * n + 2 * (3 * sent[p.rank] + q0)), (b, sent)
            p.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_wpart_claim_queue_overflow(pj, oracle, world):
    """A light or heavy step whose remote pairs overflow a claim-queue shard runs again on a
    grown queue (all the band's members as the frontier, the sent-pair cache cleared): with
    the shard capacity cut to a few pairs before every solve, the gathered distances still
    equal the oracle Dijkstra, and the queue has grown past what was set."""
    from paralleljohnson_amd.partition import delta_group, gather_group, load_weighted_kronecker
    ctxs, comms = _group(pj, world, "host")
    g0 = ctxs[0].generate_kronecker(12, 16, 9, weighted=True)
    row, col, wc = g0.get_csr()
    col = col.view(np.uint32)
    n = g0.n
    g0.close()
    parts = [load_weighted_kronecker(ctxs[r], 12, 16, 9, r, world) for r in range(world)]
    for cap in (1, 3, 40):
        for source in (0, n // 3, n - 1):
            for p in parts:
                p.set_option("queue_shard", cap)
            delta_group(parts, comms, source)
            exp = oracle.dijkstra(row, col, wc, source)
            assert np.array_equal(gather_group(parts, comms), exp), (cap, world, source)
        assert max(p.device_bytes()["exchange"] for p in parts) > 64 * 8 * cap
    with pytest.raises(pj.PJError):
        parts[0].set_option("queue_shard", 0)
    for p in parts:
        p.close()


@pytest.mark.gpu
def test_wpart_relax_refuses_a_send_buffer_at_world2(pj):
    """no bound on a relax's queued pairs is known before it runs, so at world > 1
    pj_wpart_relax takes no send buffer (PJ_ERR_ARG): the caller sizes one from the counts and
    calls pj_wpart_pack."""
    import ctypes
    from paralleljohnson_amd.partition import load_weighted
    ctx = pj.Context(0)
    g = ctx.load_coo([0, 1, 2, 3], [1, 2, 3, 0], [1, 2, 3, 4], n=200)
    parts = [load_weighted(ctx, g, r, 2) for r in range(2)]
    counts = np.zeros(2, np.int64)
    rc = pj._lib.pj_wpart_relax(parts[0]._h, 1, 0, 10, ctypes.c_void_p(4096), counts.ctypes.data_as(ctypes.c_void_p))
    assert rc == -1 and b"pass send = NULL" in pj._lib.pj_last_error()
    for p in parts:
        p.close()
    g.close()
    ctx.close()


@pytest.mark.gpu
def test_multi_weighted_partition_state_shrinks(pj, oracle):
    """pj_multi with a weighted partitioned Kronecker s24 (every rank enumerates the tuples
    and keeps its block's rows: pj_wpart_generate_kronecker) at world 2, 4 and 8 (ranks
    sharing the one GPU over the host transport): the per-rank O(block) vertex state --
    distances, frontier bitmaps, light prefixes, long-row queue, sent-pair cache -- at world
    8 is at most a third of world 2's, the rows shrink with the world, and the distances
    equal the single-GPU solver's on the same graph."""
    from paralleljohnson_amd.partition import Multi
    ctx = pj.Context(0)
    g = ctx.generate_kronecker(24, 16, 1, weighted=True)
    root = int(g.sample_roots(2, 1)[0])
    exp = g.sssp(root)
    g.close()
    ctx.close()
    state, rows = {}, {}
    for world in (2, 4, 8):
        with Multi(world, "host") as m:
            m.generate_kronecker(24, 16, 1, weighted=True)
            got, st = m.sssp(root)
            assert np.array_equal(got, exp), world
            b = [m.device_bytes(r) for r in range(world)]
            state[world] = max(x["state"] for x in b)
            rows[world] = max(x["rows"] for x in b)
            print(f"world {world}: per-rank bytes {b[0]}")
    assert state[8] * 3 <= state[2], state
    assert rows[8] * 3 <= rows[2], rows


@pytest.mark.gpu
@pytest.mark.parametrize("weighted", [False, True])
def test_cli_processes_byte_identical(pj, oracle, tmp_path, weighted):
    """`parallel_johnson` at P = 1 (single-GPU solver), P = 2 and 3 (PJ_GPUS: the 1D partition
    in one process, ranks sharing the GPU over the host transport) and under an MPI-style
    launcher (OMPI_COMM_WORLD_SIZE = 2: rank 0 runs both ranks, rank 1 exits): the same
    sol_file bytes as the oracle, and the `Time:` line names P (:603-604)."""
    rng = np.random.default_rng(77 + weighted)
    s, d = random_graph(rng, "hub", 3000)
    w = rng.integers(1, 200, len(s)).astype(np.uint32) if weighted else None
    text = to_text(s, d, w=w, style=1)
    path = tmp_path / "g.txt"
    path.write_bytes(text)
    src = int(s[0])
    ps, pd, pw, n = oracle.parse_snap(text, weighted=weighted)
    row, col, wc = oracle.coo2csr(ps, pd, n, pw)
    exp = oracle.format_sol(oracle.dijkstra(row, col, wc, src) if weighted else oracle.bfs(row, col, src))
    base = dict(os.environ, PJ_WEIGHTED=str(int(weighted)))
    base.pop("PJ_GPUS", None)
    runs = [("1", {}), ("2", {"PJ_GPUS": "2"}), ("3", {"PJ_GPUS": "3"}),
            ("2", {"OMPI_COMM_WORLD_SIZE": "2", "OMPI_COMM_WORLD_RANK": "0"})]
    for p, extra in runs:
        out = tmp_path / f"sol_{p}_{len(extra)}.txt"
        r = subprocess.run([pj.cli_path(), str(path), str(src), str(out)], capture_output=True, text=True,
                           env=dict(base, **extra), timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        assert out.read_bytes() == exp, (p, extra)
        assert r.stdout.startswith("Time: ") and r.stdout.endswith(f" seconds when using {p} processes.\n")
        assert r.stderr.splitlines()[-1] == f"the shortest path distance vector has been saved in file {out}"
    # the other launcher ranks do nothing and exit 0 (only rank 0 works)
    r = subprocess.run([pj.cli_path(), str(path), str(src), str(tmp_path / "rank1.txt")], capture_output=True,
                       env=dict(base, OMPI_COMM_WORLD_SIZE="2", OMPI_COMM_WORLD_RANK="1"), timeout=120)
    assert r.returncode == 0 and not (tmp_path / "rank1.txt").exists()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 3])
def test_wpart_load_snap(pj, oracle, tmp_path, world):
    """pj_wpart_load_snap: each rank parses the weighted text and keeps only its block's
    rows; the band loop over the host transport equals the oracle Dijkstra, and the block
    holds exactly the block's out-edges."""
    from paralleljohnson_amd.partition import block_geometry, delta_group, gather_group, load_weighted_snap
    rng = np.random.default_rng(41 + world)
    n = 2000
    s, d = random_graph(rng, "hub", n)
    w = rng.integers(1, 120, len(s)).astype(np.uint32)
    text = to_text(s, d, w=w, style=2)
    path = tmp_path / "w.txt"
    path.write_bytes(text)
    ps, pd, pw, nn = oracle.parse_snap(text, weighted=True)
    row, col, wc = oracle.coo2csr(ps, pd, nn, pw)
    ctxs, comms = _group(pj, world)
    parts = [load_weighted_snap(ctxs[r], str(path), r, world) for r in range(world)]
    block, ranges = block_geometry(nn, world)
    for r, p in enumerate(parts):
        assert (p.lo, p.hi, p.n) == (ranges[r][0], ranges[r][1], nn)
        assert p.nnz_local == int(row[ranges[r][1]] - row[ranges[r][0]])
    for source in (int(ps[0]), 0, nn - 1, nn + 3):
        delta_group(parts, comms, source)
        exp = oracle.dijkstra(row, col, wc, source) if source < nn else np.full(nn, INF, np.int32)
        assert np.array_equal(gather_group(parts, comms), exp), source
    for p in parts:
        p.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 3])
def test_multi_handle(pj, oracle, tmp_path, world):
    """The n-GPU handle (pj_multi_*, SURVEY.md §8b `pj_create(n_gpus)`), ranks sharing the one
    GPU over the host transport: partitioned single-source solves (unit and weighted) equal the
    oracle; replicated batches (sources sharded over the ranks) equal per-source oracle rows;
    batch_write files are byte-identical to the oracle's sol_files in both layouts; a CSR cache
    written by rank 0 serves the next replicated load."""
    from paralleljohnson_amd.partition import PARTITIONED, REPLICATED, Multi
    rng = np.random.default_rng(90 + world)
    s, d = random_graph(rng, "hub", 2500)
    w = rng.integers(1, 150, len(s)).astype(np.uint32)
    for weighted in (False, True):
        text = to_text(s, d, w=w if weighted else None, style=1)
        path = tmp_path / f"g{int(weighted)}.txt"
        path.write_bytes(text)
        ps, pd, pw, n = oracle.parse_snap(text, weighted=weighted)
        row, col, wc = oracle.coo2csr(ps, pd, n, pw)

        def ref(src):
            if src < 0 or src >= n:
                return np.full(n, INF, np.int32)
            return oracle.dijkstra(row, col, wc, src) if weighted else oracle.bfs(row, col, src)

        sources = [int(ps[0]), 0, n - 1, n + 5, int(ps[len(ps) // 2])]
        with Multi(world, "host" if world > 1 else "auto") as m:
            assert m.info()["layout"] == -1
            with pytest.raises(pj.PJError):
                m.sssp(0)
            m.load_snap(str(path), weighted=weighted, layout=PARTITIONED)
            info = m.info()
            assert (info["n"], info["world"], info["layout"], info["weighted"]) == (n, world, PARTITIONED, weighted)
            for src in sources:
                dist, st = m.sssp(src)
                exp = ref(src)
                assert np.array_equal(dist, exp), (weighted, src)
                assert st["reached"] == int((exp < INF).sum())
            paths = [str(tmp_path / f"p{world}_{weighted}_{i}.txt") for i in range(len(sources))]
            m.sssp_batch_write(sources, paths)
            for src, p in zip(sources, paths):
                assert open(p, "rb").read() == oracle.format_sol(ref(src)), (src, p)

            cache = str(tmp_path / f"c{world}_{int(weighted)}.pjcsr")
            m.set_csr_cache(cache)
            m.load_snap(str(path), weighted=weighted, layout=REPLICATED)
            assert m.info()["transport"] == "replicated" and os.path.exists(cache)
            rows = m.sssp_batch(sources)
            for i, src in enumerate(sources):
                assert np.array_equal(rows[i], ref(src)), (weighted, src)
            m.load_snap(str(path), weighted=weighted, layout=REPLICATED)  # from the cache now
            paths = [str(tmp_path / f"r{world}_{weighted}_{i}.txt") for i in range(len(sources))]
            m.sssp_batch_write(sources, paths)
            for src, p in zip(sources, paths):
                assert open(p, "rb").read() == oracle.format_sol(ref(src)), (src, p)
            dist, _ = m.sssp(sources[0])
            assert np.array_equal(dist, ref(sources[0]))
    # Kronecker through the handle: partitioned (unit) equals the single-GPU solver
    with Multi(world, "host" if world > 1 else "auto") as m:
        m.generate_kronecker(11, 16, 5, layout=PARTITIONED)
        with pj.Context(0) as c:
            g = c.generate_kronecker(11, 16, 5)
            for root in g.sample_roots(3, 2):
                assert np.array_equal(m.sssp(int(root))[0], g.sssp(int(root)))
            g.close()
