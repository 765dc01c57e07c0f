"""Binary CSR cache (pj_graph_save / pj_load_csr_file) and the CLI's
PJ_CSR_CACHE: a loaded graph has byte-identical CSR/CSC/weights and the same distances as
the graph it was saved from, and the CLI's sol_file is the same with and without the cache."""
import os
import subprocess

import numpy as np
import pytest

from helpers import random_graph, to_text

pytestmark = pytest.mark.gpu


def _same_graph(a, b):
    assert (a.n, a.nnz, a.weighted) == (b.n, b.nnz, b.weighted)
    ra, ca, wa = a.get_csr()
    rb, cb, wb = b.get_csr()
    assert (ra == rb).all() and (ca == cb).all()
    if wa is not None:
        assert (wa == wb).all()


def test_cache_roundtrip_directed(ctx, oracle, tmp_path):
    """Non-symmetric (CSR + CSC on disk): distances in push, pull and auto modes."""
    rng = np.random.default_rng(11)
    n = 30000
    src, dst = random_graph(rng, "hub", n)
    g = ctx.load_coo(src, dst, n=n)
    p = str(tmp_path / "g.pjcsr")
    g.save(p)
    h = ctx.load_csr_file(p)
    _same_graph(g, h)
    row, col, _ = g.get_csr()
    col = col.astype(np.uint32)
    for r in (int(src[0]), 5, n - 1):
        exp = oracle.bfs(row, col, r)
        for mode in (0, 1, 2):
            h.set_option("direction", mode)
            assert (h.sssp(r) == exp).all()
    assert (h.sssp_batch([int(src[0]), 5]) == g.sssp_batch([int(src[0]), 5])).all()


def test_cache_roundtrip_weighted_kronecker(ctx, oracle, tmp_path):
    """Symmetric weighted graph (no CSC on disk): delta-stepping on the loaded copy."""
    g = ctx.generate_kronecker(12, 16, 3, weighted=True)
    p = str(tmp_path / "k.pjcsr")
    g.save(p, src_size=123, src_mtime_ns=456)
    h = ctx.load_csr_file(p, 123, 456)
    _same_graph(g, h)
    row, col, w = h.get_csr()
    for r in g.sample_roots(5, 3):
        assert (h.sssp(int(r)) == oracle.dijkstra(row, col.astype(np.uint32), w, int(r))).all()


def test_cache_errors(ctx, pj, tmp_path):
    g = ctx.generate_webgraph(5000, 40000, 2)
    p = tmp_path / "w.pjcsr"
    g.save(str(p), 10, 20)
    with pytest.raises(pj.PJError) as e:
        ctx.load_csr_file(str(p), 11, 20)  # stale stamp
    assert e.value.name == "PJ_ERR_STATE"
    with pytest.raises(pj.PJError) as e:
        ctx.load_csr_file(str(tmp_path / "absent.pjcsr"))
    assert e.value.name == "PJ_ERR_IO"
    data = p.read_bytes()
    (tmp_path / "t.pjcsr").write_bytes(data[:-4])  # truncated
    (tmp_path / "m.pjcsr").write_bytes(b"X" + data[1:])  # bad magic
    for bad in ("t.pjcsr", "m.pjcsr"):
        with pytest.raises(pj.PJError) as e:
            ctx.load_csr_file(str(tmp_path / bad))
        assert e.value.name == "PJ_ERR_PARSE"
    e0 = ctx.load_snap_buffer(b"")
    e0.save(str(tmp_path / "e.pjcsr"))
    assert ctx.load_csr_file(str(tmp_path / "e.pjcsr")).n == 0


def test_cli_csr_cache(pj, oracle, tmp_path):
    rng = np.random.default_rng(5)
    src, dst = random_graph(rng, "uniform", 8000)
    f = tmp_path / "g.txt"
    f.write_bytes(to_text(src, dst, style=0))
    out = tmp_path / "sol.txt"
    env = dict(os.environ, PJ_CSR_CACHE="1")
    r = subprocess.run([pj.cli_path(), str(f), "3", str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    plain = out.read_bytes()
    for _ in range(2):  # first run writes the cache, the second loads it
        out.unlink()
        r = subprocess.run([pj.cli_path(), str(f), "3", str(out)], capture_output=True, text=True, timeout=120,
                           env=env)
        assert r.returncode == 0, r.stderr
        assert out.read_bytes() == plain
        assert os.path.exists(str(f) + ".pjcsr")
    # a changed text file invalidates the cache
    f.write_bytes(to_text(dst, src, style=0) + b"")
    os.utime(f, ns=(1, 1))
    r = subprocess.run([pj.cli_path(), str(f), "3", str(out)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    r2 = subprocess.run([pj.cli_path(), str(f), "3", str(tmp_path / "p.txt")], capture_output=True, text=True,
                        timeout=120)
    assert out.read_bytes() == (tmp_path / "p.txt").read_bytes()


@pytest.mark.parametrize("where", ["row", "col", "csc"])
def test_cache_corrupted_payload(ctx, pj, tmp_path, where):
    """A cache file with a valid header but a corrupted payload fails with PJ_ERR_PARSE
    (checked on the device) instead of faulting a kernel; the CLI then re-parses."""
    n = 5000
    rng = np.random.default_rng(3)
    src, dst = random_graph(rng, "uniform", n)
    g = ctx.load_coo(src, dst, n=n)
    p = tmp_path / "c.pjcsr"
    g.save(str(p))
    raw = bytearray(p.read_bytes())
    nnz = g.nnz
    rowb = 4 * (n + 1)
    if where == "row":  # a decreasing offset in the middle of the row array
        off = 64 + 4 * (n // 2)
        raw[off:off + 4] = (0xFFFFFF).to_bytes(4, "little")
    elif where == "col":  # a column id past n
        off = 64 + rowb + 4 * (nnz // 3)
        raw[off:off + 4] = (n + 7).to_bytes(4, "little")
    else:  # the in-edge CSC of a directed graph
        off = 64 + rowb + 4 * nnz + rowb + 4 * (nnz // 2)
        raw[off:off + 4] = (2 ** 31).to_bytes(4, "little")
    p.write_bytes(bytes(raw))
    with pytest.raises(pj.PJError) as e:
        ctx.load_csr_file(str(p))
    assert e.value.name == "PJ_ERR_PARSE"
    g.close()
