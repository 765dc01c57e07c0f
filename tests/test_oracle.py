"""CPU tests of the oracle (test infrastructure) against the reference's known answers.

Pinning: SURVEY.md Appendix B (behaviours measured on the reference binary,
committed as tests/golden/appendix_b.json) and scipy.sparse.csgraph (an
independent implementation of the R9 output contract). No reference-held
fixtures exist.
"""
import ctypes
import hashlib

import numpy as np
import pytest

from helpers import chain_text, random_graph, to_text

INF = 100000


def _atoi(s: str) -> int:
    return ctypes.CDLL(None).atoi(s.encode())


def _oracle_sol(O, text, source):
    src, dst, _, n = O.parse_snap(text)
    row, col, _ = O.coo2csr(src, dst, n)
    return O.bfs(row, col, source), row, col


def test_appendix_b_known_answers(oracle, appendix_b):
    for case in appendix_b:
        if case.get("generator"):
            continue
        text = case["text"].encode()
        if case["expect"] == "parse_error":
            with pytest.raises(oracle.ParseError):
                oracle.parse_snap(text)
            continue
        src = _atoi(case["source"])
        dist, row, col = _oracle_sol(oracle, text, src)
        assert dist.tolist() == case["expect"], case["name"]
        assert oracle.format_sol(dist).decode() == case["sol"], case["name"]
        # the restated BSP heap algorithm agrees at every partition count
        for p in (1, 2, 3, 8):
            r, _ = oracle.reference_sssp(row, col, src, p)
            assert r.tolist() == case["expect"], (case["name"], p)


def test_appendix_b_chain_cap(oracle, appendix_b):
    case = next(c for c in appendix_b if c.get("generator") == "chain")
    dist, row, col = _oracle_sol(oracle, chain_text(case["n"]), 0)
    out = oracle.format_sol(dist)
    assert len(out) == case["sol_bytes"]
    assert hashlib.sha256(out).hexdigest() == case["sol_sha256"]
    assert dist[99999] == 99999 and dist[100000] == INF


def test_parse_semantics(oracle):
    # `istringstream >> int >> int` details (:92-93)
    s, d, _, n = oracle.parse_snap(b"12abc 3\n7\t+5\n4 -0\n9 -\n0x1 8\n")
    assert s.tolist() == [12, 7, 4, 9, 0] and d.tolist() == [0, 5, 0, 0, 0] and n == 13
    for bad in (b"5\n", b"5 \n", b"5\r\n", b"1 -3\n", b"1 99999999999\n", b"99999999999 1\n"):
        with pytest.raises(oracle.ParseError):
            oracle.parse_snap(bad)
    # no trailing newline, NUL bytes, weights column
    s, d, w, n = oracle.parse_snap(b"0 1 9\n1\x002 4\n2 3 x", weighted=True)
    assert s.tolist() == [0, 1, 2] and d.tolist() == [1, 0, 3] and w.tolist() == [9, 0, 0]


def test_coo2csr_stable(oracle):
    src = np.array([2, 0, 2, 1, 0, 2], np.uint32)
    dst = np.array([5, 1, 3, 4, 0, 1], np.uint32)
    row, col, _ = oracle.coo2csr(src, dst, 6)
    assert row.tolist() == [0, 2, 3, 6, 6, 6, 6]
    assert col.tolist() == [1, 0, 4, 5, 3, 1]  # file order inside each row (:143-149)


@pytest.mark.parametrize("kind", ["uniform", "hub", "chain"])
def test_oracle_vs_scipy(oracle, kind):
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import shortest_path
    rng = np.random.default_rng(hash(kind) % 2**32)
    for trial in range(6):
        n = int(rng.integers(2, 2500))
        src, dst = random_graph(rng, kind, n)
        text = to_text(src, dst, style=trial % 3)
        s, d, _, N = oracle.parse_snap(text)
        row, col, _ = oracle.coo2csr(s, d, N)
        root = int(s[0]) if len(s) else 0
        dist = oracle.bfs(row, col, root)
        A = csr_matrix((np.ones(len(col)), col.astype(np.int64), row), shape=(N, N))
        sp = shortest_path(A, unweighted=True, indices=root)
        exp = np.where(np.isinf(sp) | (sp >= INF), INF, sp).astype(np.int32)
        assert (dist == exp).all()
        for p in (1, 2, 4, 7):
            r, st = oracle.reference_sssp(row, col, root, p)
            assert (r == dist).all(), p


def test_dijkstra_vs_scipy(oracle):
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import shortest_path
    rng = np.random.default_rng(7)
    for trial in range(8):
        n = int(rng.integers(2, 1500))
        src, dst = random_graph(rng, ["uniform", "hub"][trial % 2], n)
        w = rng.integers(0 if trial % 3 == 0 else 1, 2000, len(src)).astype(np.uint32)
        s, d, ww, N = oracle.parse_snap(to_text(src, dst, w), weighted=True)
        row, col, wc = oracle.coo2csr(s, d, N, ww)
        root = int(s[0]) if len(s) else 0
        dist = oracle.dijkstra(row, col, wc, root)
        A = csr_matrix((wc.astype(float) + 1e-9, col.astype(np.int64), row), shape=(N, N))
        sp = shortest_path(A, indices=root)
        exp = np.where(np.isinf(sp) | (sp >= INF), INF, np.round(sp)).astype(np.int32)
        assert (dist == exp).all()
        r, _ = oracle.reference_sssp(row, col, root, 3, w=wc)
        assert (r == dist).all()


def test_kronecker_spec(oracle):
    s, d, w = oracle.kronecker(10, 16, 3, weighted=True)
    assert len(s) == 2 * 16 * 1024
    assert (s[0::2] == d[1::2]).all() and (d[0::2] == s[1::2]).all()
    assert (w[0::2] == w[1::2]).all() and w.min() >= 1 and w.max() <= 255
    assert s.max() < 1024
    # permutation: the generator's label map is a bijection on [0, 2^scale)
    s2, _, _ = oracle.kronecker(10, 16, 3)
    assert (s2 == s).all()
    deg = np.bincount(s, minlength=1024)
    assert deg.max() > 20 * deg.mean()  # skewed (Kronecker), not uniform


@pytest.mark.parametrize("weighted", [False, True])
def test_row_digest_pins(oracle, weighted):
    """The order-free row digest computed from the generator spec (no COO, no CSR) equals
    the digest of coord2csr's CSR of pjo_kronecker's COO; a weight-sorted row order keeps
    the digest and has no out-of-order entries; one changed entry changes the digest."""
    s, d, w = oracle.kronecker(12, 16, 5, weighted=weighted)
    row, col, wc = oracle.coo2csr(s, d, 1 << 12, w)
    deg, hs = oracle.kronecker_row_digest(12, 16, 5, weighted, threads=3)
    cdeg, chs, _ = oracle.csr_row_digest(row, col, wc, threads=2)
    assert (deg == cdeg).all() and (hs == chs).all()
    assert (deg == np.diff(row)).all()
    if weighted:
        rid = np.repeat(np.arange(1 << 12), np.diff(row))
        o = np.lexsort((wc, rid))  # stable: ties keep file order
        sdeg, shs, bad = oracle.csr_row_digest(row, col[o], wc[o])
        assert bad == 0 and (shs == hs).all()
        assert oracle.csr_row_digest(row, col, wc)[2] > 0  # file order is not weight order
    col2 = col.copy()
    col2[len(col2) // 2] ^= 1
    assert (oracle.csr_row_digest(row, col2, wc)[1] != hs).sum() == 1


def test_sssp_certificate_checker(oracle):
    """The full-size GPU tests prove exactness with helpers.sssp_certificate (no CPU
    solve at 2^31 entries); here the checker itself is pinned: it accepts the oracle's
    distances and rejects single-entry corruptions, unit and weighted, capped."""
    from helpers import sssp_certificate
    rng = np.random.default_rng(77)
    for trial in range(6):
        n = int(rng.integers(2, 3000))
        src, dst = random_graph(rng, ["uniform", "hub", "chain"][trial % 3], n)
        w = None if trial % 2 else rng.integers(1, [3, 40000, 60000][trial % 3], len(src)).astype(np.uint32)
        row, col, wc = oracle.coo2csr(src.astype(np.uint32), dst.astype(np.uint32), n, w)
        r = int(src[0]) if len(src) else 0
        d = oracle.bfs(row, col, r) if w is None else oracle.dijkstra(row, col, wc, r)
        assert sssp_certificate(row, col, wc, d, r, chunk=997) == [], trial
        reached = np.nonzero((d < INF) & (np.arange(n) != r))[0]
        if len(reached):
            v = int(reached[len(reached) // 2])
            for delta in (-1, 1):
                bad = d.copy()
                bad[v] += delta
                assert sssp_certificate(row, col, wc, bad, r, chunk=997), (trial, v, delta)
        unreached = np.nonzero(d == INF)[0]
        if len(unreached):
            bad = d.copy()
            bad[unreached[0]] = INF - 1
            assert sssp_certificate(row, col, wc, bad, r), trial
    # chain longer than the cap: the R9 cut at 100000 is exact, not a violation
    n = 100010
    row = np.arange(n + 1, dtype=np.int64).clip(max=n - 1)
    col = np.arange(1, n, dtype=np.int32)
    d = np.minimum(np.arange(n), INF).astype(np.int32)
    assert sssp_certificate(row, col, None, d, 0) == []
