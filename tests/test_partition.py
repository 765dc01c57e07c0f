"""1D vertex-partitioned BFS: protocol tests on CPU (gloo,
world_size 1-3, numpy restatement of the device steps) and parity of the HIP
kernels (libpj pj_part_*) against the oracle on the GPU, at world_size 1 and
at world_size 2 with both ranks sharing the one GPU (gloo, host-staged).

Bar: bit-exact distances against the oracle BFS (the reference's R9 contract);
partitioning is result-neutral."""
import os
import socket
import sys
import tempfile

import numpy as np
import pytest

from conftest import ROOT
from helpers import random_graph

INF = 100000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_dist(oracle, src, dst, n, source):
    row, col, _ = oracle.coo2csr(np.asarray(src, np.int64), np.asarray(dst, np.int64), n)
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
def test_protocol_world1_numpy(oracle, force):
    from part_numpy import NumpyPart
    from paralleljohnson_amd.partition import PartitionedBFS, gather_dist
    for kind, n, s, d in _cases():
        sym = kind == "sym"
        ops = NumpyPart(s, d, n, 0, 1, symmetric=sym)
        bfs = PartitionedBFS(ops, None, force=force)
        for source in (0, n // 3, n - 1, n + 5, -1):
            bfs.solve(source)
            got = gather_dist(ops, None)
            exp = _oracle_dist(oracle, s, d, n, source) if 0 <= source < n else np.full(n, INF, np.int32)
            assert np.array_equal(got, exp), (kind, source, force)


def _rank_main(rank, world, port, path, force, device, backend="gloo"):
    """One rank of a gloo (or nccl) job: every case, every source; rank 0 saves the results."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    from paralleljohnson_amd.partition import Exchange, PartitionedBFS, gather_dist
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    ex = Exchange()
    res = {}
    if device:
        import paralleljohnson_amd as pj
        from paralleljohnson_amd.partition import load_coo, load_kronecker
        ctx = pj.Context(0)
        cases = [(k, n, s, d) for k, n, s, d in _cases()]
        for ci, (kind, n, s, d) in enumerate(cases):
            ops = load_coo(ctx, s, d, n, rank, world, symmetric=(kind == "sym"))
            bfs = PartitionedBFS(ops, ex, force=force)
            for source in (0, n // 3, n - 1):
                st = bfs.solve(source)
                res[f"{ci}_{source}"] = gather_dist(ops, ex)
                res[f"{ci}_{source}_reached"] = np.array([st["reached"], st["reached_edges"]])
            ops.close()
        ops = load_kronecker(ctx, 14, 16, 7, rank, world)
        bfs = PartitionedBFS(ops, ex, force=force)
        for source in (1, 777, 12345):
            bfs.solve(source)
            res[f"k14_{source}"] = gather_dist(ops, ex)
        ops.close()
    else:
        from part_numpy import NumpyPart
        for ci, (kind, n, s, d) in enumerate(_cases()):
            ops = NumpyPart(s, d, n, rank, world, symmetric=(kind == "sym"))
            bfs = PartitionedBFS(ops, ex, force=force)
            for source in (0, n // 3, n - 1, n + 5):
                bfs.solve(source)
                res[f"{ci}_{source}"] = gather_dist(ops, ex)
    if rank == 0:
        np.savez(path, **res)
    dist.barrier()
    dist.destroy_process_group()


def _run_world(world, force, device=False, backend="gloo"):
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "res.npz")
        mp.spawn(_rank_main, args=(world, _free_port(), path, force, device, backend), nprocs=world, join=True)
        with np.load(path) as z:
            return {k: z[k] for k in z.files}


@pytest.mark.parametrize("world,force", [(2, 0), (2, 1), (2, 2), (3, 0)])
def test_protocol_gloo_numpy(oracle, world, force):
    res = _run_world(world, force)
    for ci, (kind, n, s, d) in enumerate(_cases()):
        for source in (0, n // 3, n - 1, n + 5):
            exp = _oracle_dist(oracle, s, d, n, source) if source < n else np.full(n, INF, np.int32)
            assert np.array_equal(res[f"{ci}_{source}"], exp), (world, force, kind, source)


# ----------------------------------------------------------------- GPU ----

@pytest.mark.gpu
@pytest.mark.parametrize("force", [0, 1, 2])
def test_part_world1_gpu(ctx, oracle, force):
    from paralleljohnson_amd.partition import PartitionedBFS, gather_dist, load_coo
    for kind, n, s, d in _cases():
        ops = load_coo(ctx, s, d, n, 0, 1, symmetric=(kind == "sym"))
        bfs = PartitionedBFS(ops, None, force=force)
        for source in (0, n // 3, n - 1, n + 5, -1):
            st = bfs.solve(source)
            got = gather_dist(ops, None)
            exp = _oracle_dist(oracle, s, d, n, source) if 0 <= source < n else np.full(n, INF, np.int32)
            assert np.array_equal(got, exp), (kind, source, force)
            assert st["reached"] == int(np.sum(exp < INF))
            assert ops.reach()[0] == st["reached"]
        ops.close()


@pytest.mark.gpu
def test_part_kronecker_matches_single_gpu(ctx, pj, oracle):
    """The partitioned generator yields the same graph: s16, world 1, vs pj.Graph and the oracle."""
    from paralleljohnson_amd.partition import PartitionedBFS, gather_dist, load_kronecker
    g = ctx.generate_kronecker(16, 16, 3)
    row, col, _ = g.get_csr()
    ops = load_kronecker(ctx, 16, 16, 3, 0, 1)
    assert ops.nnz_local == g.nnz
    bfs = PartitionedBFS(ops, None)
    for r in g.sample_roots(5, 4):
        st = bfs.solve(int(r))
        got = gather_dist(ops, None)
        assert np.array_equal(got, g.sssp(int(r))), r
        assert np.array_equal(got, oracle.bfs(row, col.view(np.uint32), int(r))), r
        rs = g.reach_stats()
        assert (st["reached"], st["reached_edges"]) == (rs["reached"], rs["reached_edges"])
        assert st["td_levels"] >= 1 and st["bu_levels"] >= 1  # both directions exercised
    ops.close()
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world,force,backend", [(2, 0, "gloo"), (2, 2, "gloo"), (1, 0, "nccl")])
def test_part_world2_one_gpu(oracle, world, force, backend):
    """Two ranks on the one GPU (gloo, host-staged): kernels + exchange end to end; and the
    RCCL (nccl backend) code path of the exchange at world 1, device tensors, no staging."""
    res = _run_world(world, force, device=True, backend=backend)
    for ci, (kind, n, s, d) in enumerate(_cases()):
        for source in (0, n // 3, n - 1):
            exp = _oracle_dist(oracle, s, d, n, source)
            assert np.array_equal(res[f"{ci}_{source}"], exp), (kind, source)
            row, col, _ = _csr(oracle, s, d, n)
            reached = exp < INF
            assert res[f"{ci}_{source}_reached"].tolist() == [int(reached.sum()),
                                                             int(np.diff(row)[reached].sum())]
    k = oracle.kronecker(14, 16, 7)
    row, col, _ = oracle.coo2csr(k[0], k[1], 1 << 14)
    for source in (1, 777, 12345):
        assert np.array_equal(res[f"k14_{source}"], oracle.bfs(row, col, source)), source


def _csr(oracle, s, d, n):
    return oracle.coo2csr(np.asarray(s, np.int64), np.asarray(d, np.int64), n)


@pytest.mark.gpu
def test_run_module_matches_cli(pj, oracle, tmp_path):
    """`python -m paralleljohnson_amd.run` (1 process, and 2 ranks on the one GPU under
    torchrun with gloo) writes the same sol_file bytes as the single-GPU CLI and the oracle."""
    import subprocess
    from helpers import to_text
    rng = np.random.default_rng(77)
    s, d = random_graph(rng, "hub", 3000)
    path = tmp_path / "g.txt"
    path.write_bytes(to_text(s, d, style=1))
    src = int(s[0])
    env = dict(os.environ, PJ_DEVICE="0")
    ref = tmp_path / "cli.sol"
    subprocess.run([pj.cli_path(), str(path), str(src), str(ref)], check=True, capture_output=True, env=env)
    row, col, _ = oracle.coo2csr(np.asarray(s, np.int64), np.asarray(d, np.int64), int(max(s.max(), d.max())) + 1)
    assert ref.read_bytes() == oracle.format_sol(oracle.bfs(row, col, src))
    one = tmp_path / "one.sol"
    r = subprocess.run([sys.executable, "-m", "paralleljohnson_amd.run", str(path), str(src), str(one)],
                       check=True, capture_output=True, text=True, env=env, cwd=ROOT)
    assert one.read_bytes() == ref.read_bytes()
    assert r.stdout.startswith("Time: ") and r.stdout.rstrip().endswith("seconds when using 1 processes.")
    assert "parallel Johnson's algorithm completes." in r.stderr
    two = tmp_path / "two.sol"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        "-m", "paralleljohnson_amd.run", str(path), str(src), str(two)],
                       capture_output=True, text=True, env=dict(env, PJ_BACKEND="gloo"), cwd=ROOT, timeout=200)
    assert r.returncode == 0, r.stderr[-2000:]
    assert two.read_bytes() == ref.read_bytes()
    assert "when using 2 processes." in r.stdout


@pytest.mark.gpu
def test_run_module_weighted(pj, oracle, tmp_path):
    """PJ_WEIGHTED=1: the single-GPU CLI (delta-stepping) and `python -m
    paralleljohnson_amd.run` at 1 and 2 ranks (PartitionedDelta, gloo) write the
    oracle Dijkstra's sol_file bytes."""
    import subprocess
    from helpers import to_text
    rng = np.random.default_rng(78)
    s, d = random_graph(rng, "hub", 2500)
    w = rng.integers(1, 200, len(s)).astype(np.uint32)
    text = to_text(s, d, w=w, style=1)
    path = tmp_path / "gw.txt"
    path.write_bytes(text)
    src = int(s[0])
    ps, pd, pw, n = oracle.parse_snap(text, weighted=True)
    row, col, wc = oracle.coo2csr(ps, pd, n, pw)
    exp = oracle.format_sol(oracle.dijkstra(row, col, wc, src))
    env = dict(os.environ, PJ_DEVICE="0", PJ_WEIGHTED="1")
    ref = tmp_path / "cli.sol"
    subprocess.run([pj.cli_path(), str(path), str(src), str(ref)], check=True, capture_output=True, env=env)
    assert ref.read_bytes() == exp
    one = tmp_path / "one.sol"
    subprocess.run([sys.executable, "-m", "paralleljohnson_amd.run", str(path), str(src), str(one)],
                   check=True, capture_output=True, text=True, env=env, cwd=ROOT)
    assert one.read_bytes() == exp
    two = tmp_path / "two.sol"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        "-m", "paralleljohnson_amd.run", str(path), str(src), str(two)],
                       capture_output=True, text=True, env=dict(env, PJ_BACKEND="gloo"), cwd=ROOT, timeout=200)
    assert r.returncode == 0, r.stderr[-2000:]
    assert two.read_bytes() == exp
    assert "when using 2 processes." in r.stdout


# ------------------------------------------- weighted (delta-stepping) ----

def _wcases():
    rng = np.random.default_rng(99)
    out = []
    for kind, n, wmax in (("uniform", 500, 300), ("hub", 900, 40), ("chain", 300, 5), ("uniform", 64, 2)):
        s, d = random_graph(rng, kind, n)
        w = rng.integers(0 if kind == "uniform" else 1, wmax, len(s)).astype(np.uint32)
        out.append((kind, n, s.astype(np.int64), d.astype(np.int64), w))
    return out


def _wrank_main(rank, world, port, path, backend):
    """One rank: weighted delta-stepping over the partition for every case; rank 0 saves."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import paralleljohnson_amd as pj
    from paralleljohnson_amd.partition import Exchange, PartitionedDelta, gather_dist, load_weighted
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    ex = Exchange()
    ctx = pj.Context(0)
    res = {}
    graphs = [(f"c{i}", ctx.load_coo(s, d, w=w, n=n)) for i, (_, n, s, d, w) in enumerate(_wcases())]
    graphs.append(("k12", ctx.generate_kronecker(12, 16, 3, weighted=True)))
    for name, g in graphs:
        ops = load_weighted(ctx, g, rank, world)
        n = g.n
        g.close()
        for delta in (0, 7, 60):
            sp = PartitionedDelta(ops, ex, delta=delta)
            for source in (0, n // 3, n - 1, n + 2):
                st = sp.solve(source)
                res[f"{name}_{delta}_{source}"] = gather_dist(ops, ex)
                res[f"{name}_{delta}_{source}_reached"] = np.array([st["reached"], st["reached_edges"]])
        ops.close()
    if rank == 0:
        np.savez(path, **res)
    dist.barrier()
    dist.destroy_process_group()


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


def _wrank_numpy(rank, world, port, path):
    """One rank of the weighted protocol on CPU (gloo), device steps restated in numpy."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from part_numpy import NumpyWPart
    from paralleljohnson_amd.partition import Exchange, PartitionedDelta, gather_dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ex = Exchange()
    res = {}
    for i, (_, n, s, d, w) in enumerate(_wcases()):
        ops = NumpyWPart(s, d, w, n, rank, world)
        for delta in (0, 7, 60):
            sp = PartitionedDelta(ops, ex, delta=delta)
            for source in (0, n // 3, n - 1, n + 2):
                st = sp.solve(source)
                res[f"c{i}_{delta}_{source}"] = gather_dist(ops, ex)
                res[f"c{i}_{delta}_{source}_reached"] = np.array([st["reached"], st["reached_edges"]])
    if rank == 0:
        np.savez(path, **res)
    dist.barrier()
    dist.destroy_process_group()


def test_wprotocol_world1_numpy(oracle):
    """The band loop (PartitionedDelta) without an exchange, numpy device steps."""
    from part_numpy import NumpyWPart
    from paralleljohnson_amd.partition import PartitionedDelta, gather_dist
    res = {}
    for i, (_, n, s, d, w) in enumerate(_wcases()):
        ops = NumpyWPart(s, d, w, n, 0, 1)
        for delta in (0, 1, 7, 60):
            sp = PartitionedDelta(ops, None, delta=delta)
            for source in (0, n // 3, n - 1, n + 2):
                st = sp.solve(source)
                res[f"c{i}_{delta}_{source}"] = gather_dist(ops, None)
                res[f"c{i}_{delta}_{source}_reached"] = np.array([st["reached"], st["reached_edges"]])
    _wcheck(res, _wexpected(oracle), oracle, (0, 1, 7, 60), 1)


@pytest.mark.parametrize("world", [2, 3])
def test_wprotocol_gloo_numpy(oracle, world):
    """Weighted band loop at world 2-3 over gloo: all_to_all of packed (id, cand)
    pairs, all_reduce sum/min termination; bit-exact vs the oracle Dijkstra."""
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "res.npz")
        mp.spawn(_wrank_numpy, args=(world, _free_port(), path), nprocs=world, join=True)
        with np.load(path) as z:
            res = {k: z[k] for k in z.files}
    _wcheck(res, _wexpected(oracle), oracle, (0, 7, 60), world)


@pytest.mark.gpu
@pytest.mark.parametrize("world,backend", [(1, "nccl"), (2, "gloo"), (3, "gloo")])
def test_wpart_delta_stepping(pj, oracle, world, backend):
    """Weighted SSSP over the 1D partition (wpart.hip + PartitionedDelta): every
    rank on the one GPU; distances bit-exact against the oracle Dijkstra, for
    several band widths and sources (including one outside [0, n))."""
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "res.npz")
        mp.spawn(_wrank_main, args=(world, _free_port(), path, backend), nprocs=world, join=True)
        with np.load(path) as z:
            res = {k: z[k] for k in z.files}
    exp_graphs = []
    for i, (_, n, s, d, w) in enumerate(_wcases()):
        row, col, wc = oracle.coo2csr(s.astype(np.uint32), d.astype(np.uint32), n, w)
        exp_graphs.append((f"c{i}", n, row, col, wc))
    ctx = pj.Context(0)
    g = ctx.generate_kronecker(12, 16, 3, weighted=True)
    row, col, wc = g.get_csr()
    exp_graphs.append(("k12", g.n, row, col.astype(np.uint32), wc))
    g.close()
    ctx.close()
    for name, n, row, col, wc in exp_graphs:
        for source in (0, n // 3, n - 1, n + 2):
            exp = oracle.dijkstra(row, col, wc, source) if source < n else np.full(n, INF, np.int32)
            reached = exp < INF
            for delta in (0, 7, 60):
                got = res[f"{name}_{delta}_{source}"]
                assert np.array_equal(got, exp), (name, delta, source, world)
                assert res[f"{name}_{delta}_{source}_reached"].tolist() == [
                    int(reached.sum()), int(np.diff(row)[reached].sum())], (name, delta, source)
