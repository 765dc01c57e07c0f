"""Batched multi-source (Johnson-style) rows: BASELINE.json configs[4] at full size, the
multi-source drop-in (pj_sssp_batch_write, CLI PJ_SOURCES) and the weighted batch.

The reference answers one source per run (atoi(argv[2]), ParallelJohnson.cpp:448) and
writes one sol_file (:615-620); a batch must therefore give, per source, exactly the
bytes of a single-source run. Rows are checked against the oracle BFS / Dijkstra."""
import os
import subprocess

import numpy as np
import pytest

from helpers import random_graph, to_text

INF = 100000

pytestmark = pytest.mark.gpu


def ms1024_sources(row, k=1024):
    """bench.py run_multisource / SURVEY.md §8d: the k smallest ids with out-degree >= 1."""
    return np.nonzero(np.diff(row) >= 1)[0][:k]


@pytest.mark.parametrize("hub_first", [0, 1])
def test_ms1024_full_size(ctx, oracle, hub_first):
    """configs[4] exactly as bench.py times it: the web-Google-shaped graph (916,428 ids,
    5,105,039 edges, seed 1), the 1024 smallest ids with out-degree >= 1, the default
    pass width (512 sources per pass); every one of the 1024 rows equals the oracle BFS.
    hub_first = 1: the pull levels probe the in-rows ordered highest in-degree first."""
    g = ctx.generate_webgraph(916428, 5105039, 1)
    g.set_option("hub_first", hub_first)
    row, col, _ = g.get_csr()
    col = col.view(np.uint32)
    sources = ms1024_sources(row)
    assert len(sources) == 1024
    out = g.sssp_batch(sources)
    st = g.stats()
    assert out.shape == (1024, 916428) and st["levels"] > 0 and st["kernel_ms"] > 0
    threads = max(1, min(16, os.cpu_count() or 1))
    reached = 0
    for c in range(0, 1024, 128):
        exp = oracle.bfs_batch(row, col, sources[c:c + 128], threads)
        bad = np.nonzero((out[c:c + 128] != exp).any(axis=1))[0]
        assert len(bad) == 0, f"rows {list(c + bad[:8])} differ from the oracle"
        reached += int((exp < INF).sum())
    assert reached > 1024 * 1000  # the sources reach real components, not just themselves
    g.close()


def test_batch_write_matches_single_runs(ctx, oracle, tmp_path):
    """pj_sssp_batch_write: row i as the sol_file paths[i], byte-identical to
    pj_write_sol of a single-source solve; 300 sources (two passes, partial last word),
    out-of-range sources (all inf) and duplicates."""
    rng = np.random.default_rng(11)
    n = 15000
    src, dst = random_graph(rng, "hub", n)
    g = ctx.load_coo(src, dst, n=n)
    row, col, _ = oracle.coo2csr(src.astype(np.uint32), dst.astype(np.uint32), n)
    sources = [int(x) for x in rng.integers(0, n, 296)] + [-1, n, 3, 3]
    paths = [str(tmp_path / f"sol_{i}.txt") for i in range(len(sources))]
    g.sssp_batch_write(sources, paths)
    for i, s in enumerate(sources):
        assert open(paths[i], "rb").read() == oracle.format_sol(oracle.bfs(row, col, s)), (i, s)
    with pytest.raises(Exception):  # strict: an unopenable path is an error
        g.sssp_batch_write([0], [str(tmp_path / "no_such_dir" / "x.txt")])
    g.close()


def test_weighted_batch(ctx, oracle, tmp_path):
    """Weighted graphs: concurrent delta-stepping solves (default 2 streams); rows equal
    the oracle Dijkstra, the batch's stats are summed, copy_dist refuses a batch result."""
    rng = np.random.default_rng(5)
    n = 6000
    src, dst = random_graph(rng, "uniform", n)
    w = rng.integers(1, 200, len(src)).astype(np.uint32)
    g = ctx.load_coo(src, dst, w=w, n=n)
    row, col, wc = oracle.coo2csr(src.astype(np.uint32), dst.astype(np.uint32), n, w=w)
    sources = [0, 17, -5, n - 1, 17]
    one = [g.sssp(s) for s in sources]
    single_ms = g.stats()["kernel_ms"]  # the last single solve
    out = g.sssp_batch(sources)
    st = g.stats()
    for i, s in enumerate(sources):
        exp = oracle.dijkstra(row, col, wc, s)
        assert (out[i] == exp).all() and (one[i] == exp).all(), (i, s)
    assert st["kernel_ms"] > single_ms * 0.5 and st["levels"] >= 1
    with pytest.raises(Exception):
        g.copy_dist()
    paths = [str(tmp_path / f"w_{i}.txt") for i in range(len(sources))]
    g.sssp_batch_write(sources, paths)
    for i, s in enumerate(sources):
        assert open(paths[i], "rb").read() == oracle.format_sol(out[i])
    g.close()


@pytest.mark.parametrize("slots", [1, 2, 3, 4])
def test_weighted_batch_streams(ctx, oracle, tmp_path, slots):
    """Johnson-style weighted batches with 1-4 solves in flight (delta.hip delta_batch: one
    stream, frontier ring, counter block and distance rows per slot, the light CSR shared):
    every row, duplicates and out-of-range sources included, equals the oracle Dijkstra on a
    weighted Kronecker graph (light / heavy pulls, tail) and on a directed random graph; a
    single-source solve between batches is unaffected; the sol_files equal the rows."""
    gk = ctx.generate_kronecker(13, 16, 91, weighted=True)
    row, col, wc = gk.get_csr()
    col = col.astype(np.uint32)
    roots = [int(r) for r in gk.sample_roots(7, 12)]
    sources = roots + [roots[0], -1, gk.n, roots[3], 0]
    gk.set_option("batch_streams", slots)
    out = gk.sssp_batch(sources)
    exp = {s: oracle.dijkstra(row, col, wc, s) for s in set(sources)}
    for i, s in enumerate(sources):
        assert (out[i] == exp[s]).all(), (slots, i, s)
    assert (gk.sssp(roots[1]) == exp[roots[1]]).all()
    paths = [str(tmp_path / f"k_{i}.txt") for i in range(len(sources))]
    gk.sssp_batch_write(sources, paths)
    for i, s in enumerate(sources):
        assert open(paths[i], "rb").read() == oracle.format_sol(exp[s]), (slots, i)
    out2 = gk.sssp_batch(sources[::-1])
    for i, s in enumerate(sources[::-1]):
        assert (out2[i] == exp[s]).all(), (slots, "rev", i, s)
    gk.close()
    rng = np.random.default_rng(40 + slots)
    n = 9000
    src, dst = random_graph(rng, "hub", n)
    w = rng.integers(0, 300, len(src)).astype(np.uint32)
    g = ctx.load_coo(src, dst, w=w, n=n)
    row, col, wc = oracle.coo2csr(src.astype(np.uint32), dst.astype(np.uint32), n, w=w)
    g.set_option("batch_streams", slots)
    sources = [int(x) for x in rng.integers(0, n, 11)] + [int(src[0])]
    out = g.sssp_batch(sources)
    for i, s in enumerate(sources):
        assert (out[i] == oracle.dijkstra(row, col, wc, s)).all(), (slots, "directed", i, s)
    with pytest.raises(Exception):
        g.set_option("batch_streams", 9)
    g.close()


@pytest.mark.parametrize("gpus", [1, 2])
def test_cli_multi_source(pj, oracle, tmp_path, gpus):
    """`PJ_SOURCES=... parallel_johnson webfile x pattern`: one sol_file per source, each
    byte-identical to the single-source CLI run (atoi per token, as argv[2] :448);
    PJ_GPUS = 2 shards the sources over two GPU contexts (one GPU on the test box)."""
    rng = np.random.default_rng(3)
    n = 5000
    src, dst = random_graph(rng, "hub", n)
    f = tmp_path / "g.txt"
    f.write_bytes(to_text(src, dst, style=1))
    s2, d2, _, nn = oracle.parse_snap(f.read_bytes())
    row, col, _ = oracle.coo2csr(s2, d2, nn)
    env = dict(os.environ, PJ_SOURCES="0, 7,abc\n-1,12x", PJ_GPUS=str(gpus))
    r = subprocess.run([pj.cli_path(), str(f), "ignored", str(tmp_path / "out_{s}_{i}.txt")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("Time: ") and r.stdout.endswith(f" seconds when using {gpus} processes.\n")
    for i, s in enumerate([0, 7, 0, -1, 12]):  # atoi("abc") = 0, atoi("12x") = 12
        got = (tmp_path / f"out_{s}_{i}.txt").read_bytes()
        assert got == oracle.format_sol(oracle.bfs(row, col, s)), (i, s)
        single = tmp_path / f"single_{i}.txt"
        r1 = subprocess.run([pj.cli_path(), str(f), str(s), str(single)], capture_output=True, timeout=300)
        assert r1.returncode == 0 and single.read_bytes() == got
    # "@file" list, pattern without a token -> <pattern>.<source>
    lst = tmp_path / "sources.txt"
    lst.write_text("5\n9\n")
    env["PJ_SOURCES"] = "@" + str(lst)
    r = subprocess.run([pj.cli_path(), str(f), "0", str(tmp_path / "plain.txt")], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    for s in (5, 9):
        assert (tmp_path / f"plain.txt.{s}").read_bytes() == oracle.format_sol(oracle.bfs(row, col, s))


def test_cli_multi_source_weighted(pj, oracle, tmp_path):
    rng = np.random.default_rng(9)
    n = 3000
    src, dst = random_graph(rng, "uniform", n)
    w = rng.integers(1, 50, len(src))
    f = tmp_path / "gw.txt"
    f.write_bytes(to_text(src, dst, w=w))
    s2, d2, w2, nn = oracle.parse_snap(f.read_bytes(), weighted=True)
    row, col, wc = oracle.coo2csr(s2, d2, nn, w=w2)
    env = dict(os.environ, PJ_SOURCES="1,2,3", PJ_WEIGHTED="1", PJ_GPUS="2")
    r = subprocess.run([pj.cli_path(), str(f), "0", str(tmp_path / "w{s}.txt")], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    for s in (1, 2, 3):
        assert (tmp_path / f"w{s}.txt").read_bytes() == oracle.format_sol(oracle.dijkstra(row, col, wc, s))
