"""Ingestion (read_webgraph :66-105, coord2csr :117-159) at sizes
where the radix sort runs several passes over many tiles: the CSR must equal a stable
counting sort by src (file order inside rows, :143-149), and weighted rows must be
ordered by (weight, file order) for delta-stepping. Also the Kronecker SNAP text
writer used as the ingestion benchmark's input, round-tripped through the oracle
parser and the CLI."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

INF = 100000


@pytest.mark.parametrize("n,m,wmax", [(1 << 22, 20_000_000, 0), (3_000_000, 9_000_000, 70000),
                                      (300, 100_000, 255), (70_000, 1_000_000, 1)])
def test_csr_build_matches_stable_sort(ctx, n, m, wmax):
    rng = np.random.default_rng(n + m)
    src = rng.integers(0, n, m)
    src[: m // 4] = rng.integers(0, 64, m // 4)  # heavy rows: long runs of one digit
    dst = rng.integers(0, n, m)
    w = rng.integers(1, wmax + 1, m).astype(np.uint32) if wmax else None
    g = ctx.load_coo(src, dst, w=w, n=n)
    row, col, wc = g.get_csr()
    g.close()
    order = np.lexsort((np.arange(m), w, src)) if wmax else np.argsort(src, kind="stable")
    exp_row = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(src, minlength=n), out=exp_row[1:])
    assert np.array_equal(row, exp_row)
    assert np.array_equal(col.view(np.uint32), dst[order].astype(np.uint32))
    if wmax:
        assert np.array_equal(wc, w[order])


def test_kronecker_text_roundtrip(ctx, pj, oracle, tmp_path):
    """pj_kronecker_write_snap: the oracle parser reads back exactly the tuples of the
    oracle's Kronecker restatement (generation order, both directions, weights), and the
    CLI on that text equals the oracle BFS."""
    for weighted in (False, True):
        path = tmp_path / f"k10_{int(weighted)}.txt"
        ctx.kronecker_write_snap(str(path), 10, 16, 5, weighted=weighted)
        s, d, w, n = oracle.parse_snap(path.read_bytes(), weighted=weighted)
        ks, kd, kw = oracle.kronecker(10, 16, 5, weighted=weighted)
        assert np.array_equal(s, ks) and np.array_equal(d, kd)
        if weighted:
            assert np.array_equal(w, kw)
    path = tmp_path / "k10_0.txt"
    s, d, _, n = oracle.parse_snap(path.read_bytes())
    row, col, _ = oracle.coo2csr(s, d, n)
    out = tmp_path / "sol.txt"
    r = subprocess.run([pj.cli_path(), str(path), str(int(s[0])), str(out)], capture_output=True, text=True,
                       env=dict(os.environ, PJ_PHASES="1"), timeout=120)
    assert r.returncode == 0, r.stderr
    assert out.read_bytes() == oracle.format_sol(oracle.bfs(row, col, int(s[0])))
    assert "phase load: file->HBM" in r.stderr
    g = ctx.load_snap(str(path))
    st = g.load_stats()
    assert st["text_bytes"] == path.stat().st_size and st["parse_ms"] > 0 and st["csr_ms"] > 0
    g.close()


def test_file_loader_pieces(ctx, oracle, tmp_path):
    """pj_load_snap streams the file into HBM in 8 MiB pinned pieces on several threads:
    lines crossing piece boundaries, a last partial piece and comment lines must give the
    same CSR as the in-memory path and the oracle parser; a directory and an empty file
    read as an empty graph (the reference's unchecked ifstream, :67)."""
    rng = np.random.default_rng(5)
    m = 1_700_000  # ~21 MB of text: two full pieces and a partial one
    src = rng.integers(0, 3_000_000, m)
    dst = rng.integers(0, 3_000_000, m)
    body = np.char.add(np.char.add(src.astype(str), "\t"), dst.astype(str))
    text = ("# header\n" + "\n".join(body.tolist()) + "\n# trailer without newline").encode()
    path = tmp_path / "big.txt"
    path.write_bytes(text)
    assert len(text) > 2 * (8 << 20)
    g = ctx.load_snap(str(path))
    row, col, _ = g.get_csr()
    st = g.load_stats()
    g.close()
    h = ctx.load_snap_buffer(text)
    hrow, hcol, _ = h.get_csr()
    h.close()
    assert np.array_equal(row, hrow) and np.array_equal(col, hcol)
    s, d, _, n = oracle.parse_snap(text)
    orow, ocol, _ = oracle.coo2csr(s, d, n)
    assert np.array_equal(row, orow) and np.array_equal(col.view(np.uint32), ocol)
    assert st["text_bytes"] == len(text) and st["read_ms"] > 0
    empty = tmp_path / "empty.txt"
    empty.write_bytes(b"")
    for p in (tmp_path, empty, tmp_path / "missing.txt"):
        e = ctx.load_snap(str(p))
        assert e.n == 0 and e.nnz == 0
        e.close()
