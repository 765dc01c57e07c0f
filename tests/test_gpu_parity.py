"""GPU parity tests: libpj (HIP, via the C-ABI) against the oracle.

Bar: bit-exact distances (integer work). Small cases compare every vertex
with the oracle; the full-size Kronecker s22 case is checked vertex by vertex
against the oracle BFS too (the CPU BFS finishes in seconds).
"""
import hashlib
import subprocess

import numpy as np
import pytest

from helpers import chain_text, csr_to_text, random_graph, to_text

pytestmark = pytest.mark.gpu
INF = 100000


def _oracle_csr(oracle, text, weighted=False):
    s, d, w, n = oracle.parse_snap(text, weighted=weighted)
    row, col, wc = oracle.coo2csr(s, d, n, w)
    return row, col, wc


def test_appendix_b_on_gpu(ctx, pj, appendix_b):
    import ctypes
    atoi = ctypes.CDLL(None).atoi
    for case in appendix_b:
        if case.get("generator"):
            continue
        text = case["text"].encode()
        if case["expect"] == "parse_error":
            with pytest.raises(pj.PJError) as e:
                ctx.load_snap_buffer(text)
            assert e.value.name == "PJ_ERR_PARSE" and "line 2" in str(e.value)
            continue
        g = ctx.load_snap_buffer(text)
        d = g.sssp(atoi(case["source"].encode()))
        assert d.tolist() == case["expect"], case["name"]
        assert pj.format_sol(d).decode() == case["sol"], case["name"]
        g.close()


def test_chain_cap(ctx, pj, appendix_b):
    case = next(c for c in appendix_b if c.get("generator") == "chain")
    g = ctx.load_snap_buffer(chain_text(case["n"]))
    d = g.sssp(0)
    out = pj.format_sol(d)
    assert hashlib.sha256(out).hexdigest() == case["sol_sha256"]
    assert d[99999] == 99999 and d[100000] == INF
    assert g.stats()["levels"] == 99999


@pytest.mark.parametrize("style", [0, 1, 2])
def test_parse_and_csr_bit_exact(ctx, oracle, style):
    rng = np.random.default_rng(11 + style)
    for kind in ("uniform", "hub", "chain"):
        n = int(rng.integers(2, 30000))
        src, dst = random_graph(rng, kind, n)
        text = to_text(src, dst, style=style)
        row, col, _ = _oracle_csr(oracle, text)
        g = ctx.load_snap_buffer(text)
        grow, gcol, _ = g.get_csr()
        assert g.n == len(row) - 1
        assert (grow == row).all()
        assert (gcol.astype(np.uint32) == col).all()  # stable: file order inside rows


def test_parse_weird_lines(ctx, oracle):
    text = b"12abc 3\n7\t+5\n4 -0\n9 -\n0x1 8\n#x\n \t1 2\n1\x002\n3 4 5 6\r\n"
    row, col, _ = _oracle_csr(oracle, text)
    g = ctx.load_snap_buffer(text)
    grow, gcol, _ = g.get_csr()
    assert (grow == row).all() and (gcol.astype(np.uint32) == col).all()
    for bad in (b"0 1\n5\n", b"0 1\n5 \n", b"0 1\n1 -3\n", b"0 1\n1 99999999999\n"):
        with pytest.raises(Exception):
            ctx.load_snap_buffer(bad)


@pytest.mark.parametrize("small", [0, 1])
@pytest.mark.parametrize("kind", ["uniform", "hub", "chain"])
@pytest.mark.parametrize("direction", [0, 1, 2])
def test_bfs_random_graphs(ctx, oracle, kind, direction, small):
    """small = 1: levels with small push frontiers run on one workgroup (bfs.hip small_levels)."""
    rng = np.random.default_rng(100 + 7 * direction + len(kind))
    for trial in range(4):
        n = int(rng.integers(2, 60000))
        src, dst = random_graph(rng, kind, n)
        g = ctx.load_coo(src, dst, n=n)
        g.set_option("direction", direction)
        g.set_option("bfs_small", small)
        row, col, _ = oracle.coo2csr(src.astype(np.uint32), dst.astype(np.uint32), n)
        roots = [int(src[0]) if len(src) else 0, int(rng.integers(0, n)), n, -5]
        for r in roots:
            exp = oracle.bfs(row, col, r)
            for hf, pv, pf in ((0, 0, 1), (1, 0, 1), (1, 2, 1), (1, 0.1, 1), (1, 2, 0), (0, 0.1, 0)):
                # (file-order in-rows, then the hub-first copy the pull levels probe; the
                # vertex-count direction rule off, at its default and eager; the pulls' first
                # two probes from the dense copy of the rows' first entries, or from the rows)
                g.set_option("hub_first", hf)
                g.set_option("pull_vertex", pv)
                g.set_option("pull_first", pf)
                d = g.sssp(r)
                assert (d == exp).all(), (kind, direction, trial, r, hf, pv, pf)
                st = g.stats()  # (n_r, m_r from the levels' counters, small levels included)
                reached = exp < INF
                assert (st["reached"], st["reached_edges"]) == (int(reached.sum()), int(np.diff(row)[reached].sum()))
        g.close()


def test_kronecker_generator_matches_spec(ctx, oracle):
    for scale, ef, seed in ((1, 1, 5), (8, 4, 9), (12, 16, 1)):
        g = ctx.generate_kronecker(scale, ef, seed)
        assert g.symmetric and g.n == 1 << scale and g.nnz == 2 * (ef << scale)
        s, d, _ = oracle.kronecker(scale, ef, seed)
        row, col, _ = oracle.coo2csr(s, d, 1 << scale)
        grow, gcol, _ = g.get_csr()
        assert (grow == row).all() and (gcol.astype(np.uint32) == col).all()


@pytest.mark.parametrize("weighted", [False, True])
def test_kronecker_csr_s20_exact(ctx, oracle, weighted):
    """The GPU Kronecker -> radix sort -> CSR build at s20 (2^25 entries) against the
    oracle's independent pjo_kronecker + coord2csr (:117-159): identical row offsets and
    columns; weighted rows are weight-sorted with ties in file order (a stable sort of the
    oracle's file-order rows by weight)."""
    g = ctx.generate_kronecker(20, 16, 1, weighted=weighted)
    grow, gcol, gw = g.get_csr()
    g.close()
    s, d, w = oracle.kronecker(20, 16, 1, weighted=weighted)
    row, col, wc = oracle.coo2csr(s, d, 1 << 20, w)
    del s, d, w
    assert (grow == row).all()
    if weighted:
        o = np.lexsort((wc, np.repeat(np.arange(1 << 20), np.diff(row))))
        col, wc = col[o], wc[o]
        assert (np.asarray(gw, np.uint32) == wc).all()
    assert (gcol.view(np.uint32) == col).all()


def test_kronecker_csr_s26w_full_size_digest(ctx, oracle):
    """configs[2]'s graph at full size (s26, 2^31 entries, weights 1..255, built by two
    radix sorts on the GPU): every row's entry count and order-free (col, w) hash sum
    equal the digest computed on the host straight from the generator spec (no sort, no
    CSR; symmetric with equal weights by construction), and every row is weight-sorted."""
    import os
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "8") or 8)))
    g = ctx.generate_kronecker(26, 16, 1, weighted=True)
    row, col, w = g.get_csr()
    g.close()
    assert len(col) == 1 << 31
    gdeg, ghs, unsorted = oracle.csr_row_digest(row, col, w, threads=threads)
    del col, w
    assert unsorted == 0
    deg, hs = oracle.kronecker_row_digest(26, 16, 1, True, threads=threads)
    assert (gdeg == deg).all()
    assert (ghs == hs).all()


@pytest.mark.parametrize("scale", [10, 14, 16])
def test_bfs_kronecker(ctx, oracle, scale):
    g = ctx.generate_kronecker(scale, 16, 2)
    row, col, _ = g.get_csr()
    col = col.astype(np.uint32)
    for r in g.sample_roots(3, 4):
        d = g.sssp(int(r))
        exp = oracle.bfs(row, col, int(r))
        assert (d == exp).all()
        for direction in (1, 2, 0):  # push only, pull whenever possible, automatic
            g.set_option("direction", direction)
            for hf, pf in ((1, 1), (0, 1), (1, 0)):
                g.set_option("hub_first", hf)
                g.set_option("pull_first", pf)
                assert (g.sssp(int(r)) == exp).all(), (direction, hf, pf)
            g.set_option("pull_first", 1)
        st = g.reach_stats()
        reached = exp < INF
        assert st["reached"] == reached.sum()
        assert st["reached_edges"] == np.diff(row)[reached].sum()


def test_bfs_kronecker_s22_full_size(ctx, oracle):
    """BASELINE.json configs[1] at full size, every vertex against the oracle."""
    g = ctx.generate_kronecker(22, 16, 1)
    assert g.nnz == 134217728
    row, col, _ = g.get_csr()
    col = col.astype(np.uint32)
    r = int(g.sample_roots(1, 1)[0])
    d = g.sssp(r)
    exp = oracle.bfs(row, col, r)
    assert (d == exp).all()
    st = g.stats()
    assert st["bu_levels"] > 0 and st["td_levels"] > 0  # direction switching exercised
    # edges scanned (pj_stats): at least the frontier edges of the push levels, at most every
    # reached edge once per level
    assert 0 < st["scanned_edges"] <= (st["levels"] + 1) * int(np.diff(row)[exp < INF].sum())
    for hf in (1, 0):  # pull levels over the hub-first in-rows, and back
        g.set_option("hub_first", hf)
        assert (g.sssp(r) == exp).all(), hf
    g.set_option("hub_first", 1)
    # the bench's root whose second level the vertex-count rule turns from a 6.18M-edge push
    # into a pull (profiles/r06/k22_levels_pmc_*.txt), with the rule off, at its default, eager
    r2 = 3377866
    exp2 = oracle.bfs(row, col, r2)
    bu = {}
    for pv in (0, 2, 0.1):
        g.set_option("pull_vertex", pv)
        assert (g.sssp(r2) == exp2).all(), pv
        bu[pv] = g.stats()["bu_levels"]
    assert bu[2] > bu[0]  # (the rule fired)
    g.set_option("pull_vertex", 2)
    # push-only levels of millions of vertices overflow the per-block hub staging (the
    # overflow path once lost hubs in about 1 of 50 such solves), with and without the
    # one-workgroup small levels
    g.set_option("direction", 1)
    for small in (1, 0, 1):
        g.set_option("bfs_small", small)
        assert (g.sssp(r) == exp).all(), small
    g.close()


def test_device_cache_slices_and_trim(ctx, pj):
    """devmem.cpp: freed device blocks >= 1 GiB stay cached and serve later big allocations
    whole or in slices (two live s23 graphs inside one s24 build's freed blocks); a graph built
    from cached memory answers as one built from fresh memory; trim returns the free blocks."""
    pj.trim_device_cache()
    g = ctx.generate_kronecker(24, 16, 1, weighted=True)
    r = int(g.sample_roots(1, 7)[0])
    d24 = g.sssp(r)
    g.close()
    assert pj.trim_device_cache() >= 2**30  # the build's temporaries and the graph's arrays
    g = ctx.generate_kronecker(23, 16, 1, weighted=True)  # (fresh memory)
    r = int(g.sample_roots(1, 7)[0])
    exp = g.sssp(r)
    g.close()
    a = ctx.generate_kronecker(24, 16, 1, weighted=True)  # caches s24-sized blocks again
    assert (a.sssp(int(a.sample_roots(1, 7)[0])) == d24).all()
    a.close()
    g1 = ctx.generate_kronecker(23, 16, 1, weighted=True)  # slices of the cached blocks
    g2 = ctx.generate_kronecker(23, 16, 1, weighted=True)
    assert (g1.sssp(r) == exp).all() and (g2.sssp(r) == exp).all()
    g1.close()
    assert (g2.sssp(r) == exp).all()
    g2.close()
    assert pj.trim_device_cache() >= 2**30


def test_partitions_built_in_poisoned_cached_blocks(ctx, pj, monkeypatch):
    """the partitioned builds are why the device cache exists, and a cached slice
    is handed out as the last owner left it, not zeroed like fresh driver memory. With
    PJ_DEVMEM_POISON every cached slice comes out full of 0xFF; the weighted and unit-weight
    partitions (world 2, host transport) built twice through such slices -- the second build in
    the first one's freed blocks -- must still answer as the single-GPU solvers do."""
    from paralleljohnson_amd.partition import (Comm, bfs_group, delta_group, gather_group, load_kronecker,
                                               load_weighted_kronecker)
    pj.trim_device_cache()
    exp = {}
    for weighted in (True, False):
        g = ctx.generate_kronecker(24, 16, 3, weighted=weighted)
        roots = [int(r) for r in g.sample_roots(5, 2)]
        exp[weighted] = {r: g.sssp(r) for r in roots}
        g.close()  # (its >= 1 GiB arrays stay cached for the partitions below)
    monkeypatch.setenv("PJ_DEVMEM_POISON", "1")
    ctxs = [pj.Context(0) for _ in range(2)]
    comms = Comm.group(ctxs, "host")
    try:
        for build in range(2):
            for weighted in (True, False):
                load = load_weighted_kronecker if weighted else load_kronecker
                parts = [load(ctxs[k], 24, 16, 3, k, 2) for k in range(2)]
                for r, d in exp[weighted].items():
                    (delta_group if weighted else bfs_group)(parts, comms, r)
                    assert (gather_group(parts, comms) == d).all(), (build, weighted, r)
                for p in parts:
                    p.close()
    finally:
        for c in comms:
            c.close()
        for c in ctxs:
            c.close()
        monkeypatch.delenv("PJ_DEVMEM_POISON")
        pj.trim_device_cache()


def test_weighted_delta_stepping(ctx, oracle):
    rng = np.random.default_rng(21)
    for trial in range(6):
        n = int(rng.integers(2, 40000))
        src, dst = random_graph(rng, ["uniform", "hub", "chain"][trial % 3], n)
        w = rng.integers(0 if trial % 2 else 1, [3, 300, 5000][trial % 3], len(src)).astype(np.uint32)
        g = ctx.load_coo(src, dst, w=w, n=n)
        row, col, wc = oracle.coo2csr(src.astype(np.uint32), dst.astype(np.uint32), n, w)
        # weighted rows are stored weight-sorted, ties in file order (graph.hip)
        grow, gcol, gw = g.get_csr()
        rid = np.repeat(np.arange(n), np.diff(row))
        perm = np.lexsort((wc, rid))
        assert (grow == row).all()
        assert (gcol.astype(np.uint32) == col[perm]).all() and (gw == wc[perm]).all()
        for delta in (0, 1, 37):
            g.set_option("delta", delta)
            for r in (int(src[0]) if len(src) else 0, int(rng.integers(0, n))):
                assert (g.sssp(r) == oracle.dijkstra(row, col, wc, r)).all(), (trial, delta, r)
        g.close()


def test_weighted_fan_cascades(ctx, oracle):
    """A light row longer than the hub threshold reached by a light edge, followed by
    thousands of in-band improvements in one round (hub queue, tile-dense rounds)."""
    rng = np.random.default_rng(5)
    fan = 9000
    leaves = np.arange(2, 2 + fan)
    nxt = 2 + fan + rng.integers(0, 3000, fan)
    src = np.concatenate([[0], np.ones(fan, np.int64), leaves, nxt[:500]])
    dst = np.concatenate([[1], leaves, nxt, rng.integers(0, 2 + fan + 3000, 500)])
    n = 2 + fan + 3000
    for wmax in (1, 4):
        w = rng.integers(0, wmax, len(src)).astype(np.uint32)
        g = ctx.load_coo(src, dst, w=w, n=n)
        row, col, wc = oracle.coo2csr(src.astype(np.uint32), dst.astype(np.uint32), n, w)
        for delta in (0, 8, 1000):
            g.set_option("delta", delta)
            assert (g.sssp(0) == oracle.dijkstra(row, col, wc, 0)).all(), (wmax, delta)
        g.close()


def test_weighted_text_and_kronecker(ctx, oracle):
    text = b"0 1 5\n0 2 1\n2 1 1\n1 3 99999\n3 4 1\n2 4 200000\n"
    g = ctx.load_snap_buffer(text, weighted=True)
    row, col, wc = _oracle_csr(oracle, text, weighted=True)
    assert g.sssp(0).tolist() == oracle.dijkstra(row, col, wc, 0).tolist() == [0, 2, 1, INF, INF]
    g = ctx.generate_kronecker(14, 16, 4, weighted=True)
    row, col, wc = g.get_csr()
    col = col.astype(np.uint32)
    for r in g.sample_roots(8, 3):
        assert (g.sssp(int(r)) == oracle.dijkstra(row, col, wc, int(r))).all()


def test_weighted_dense_rounds_and_light_filter(ctx, oracle):
    """Tile-dense light rounds (dense_frac: never / whenever the frontier is non-empty /
    the default threshold), the has-light-edge filter (on / off), the packed 32-bit light
    CSR (on / off) and the split whole-CSR records, light pulls in the tail (on / off), the
    deferred band check (on / off), with light pulls never / by the default rule / in every
    round and with and without the tail switch: directed random graphs (no pulls), a star whose
    light segment exceeds the dense mode's hub threshold (4096), and Kronecker graphs.
    Bit-exact against the oracle Dijkstra."""
    rng = np.random.default_rng(33)
    graphs = []
    for kind, n in (("uniform", 30000), ("hub", 20000)):
        src, dst = random_graph(rng, kind, n)
        w = rng.integers(1, 200, len(src)).astype(np.uint32)
        graphs.append((kind, ctx.load_coo(src, dst, w=w, n=n)))
    fan = 9000  # vertex 1 -> 9000 leaves at weight 1: one light segment > 4096 edges
    src = np.concatenate([[0], np.ones(fan, np.int64), 2 + rng.integers(0, fan, 20000)])
    dst = np.concatenate([[1], 2 + np.arange(fan), 2 + rng.integers(0, fan, 20000)])
    w = np.concatenate([[3], np.ones(fan), rng.integers(1, 90, 20000)]).astype(np.uint32)
    graphs.append(("star", ctx.load_coo(src, dst, w=w, n=2 + fan)))
    graphs.append(("k13", ctx.generate_kronecker(13, 16, 17, weighted=True)))
    graphs.append(("k15ef4", ctx.generate_kronecker(15, 4, 18, weighted=True)))
    for name, g in graphs:
        row, col, wc = g.get_csr()
        col = col.astype(np.uint32)
        roots = [0] + [int(r) for r in g.sample_roots(4, 2)]
        exp = {r: oracle.dijkstra(row, col, wc, r) for r in roots}
        for i, (dense, pk, tp) in enumerate(((0.0, 0, 0), (1e-12, 1, 1), (0.02, 1, 1), (0.1, 2, 0), (0.1, 0, 1))):
            lf = i & 1
            for lp, tf in ((2.0, 0.1), (0.0, 0.1), (2.0, 0.0), (1e15, 0.1)):
                g.set_option("dense_frac", dense)
                g.set_option("light_pack", min(pk, 1))
                g.set_option("split_w", int(pk != 2))
                g.set_option("tail_pull", tp)
                g.set_option("defer_check", int(dense != 0.02))
                g.set_option("light_filter", lf)
                g.set_option("light_pull", lp)
                g.set_option("tail_frac", tf)
                for delta in (0, 40):
                    g.set_option("delta", delta)
                    for r in roots:
                        assert (g.sssp(r) == exp[r]).all(), (name, dense, pk, tp, lf, lp, tf, delta, r)
        g.close()


@pytest.mark.parametrize("scale,ef", [(13, 16), (15, 4)])
def test_weighted_band_width(ctx, oracle, scale, ef):
    """Bands narrower than the light threshold (delta.hip band_width): light edges
    may then leave the band; the band's rounds must still settle it exactly. And
    the switch to a wider tail threshold/band after tail_after bands."""
    g = ctx.generate_kronecker(scale, ef, 3 + scale, weighted=True)
    row, col, wc = g.get_csr()
    col = col.astype(np.uint32)
    roots = [int(r) for r in g.sample_roots(5 + ef, 3)]
    exp = {r: oracle.dijkstra(row, col, wc, r) for r in roots}
    for pf, lp in ((0.0, 0.0), (4.0, 2.0), (1e15, 1e15)):
        g.set_option("pull_factor", pf)
        g.set_option("light_pull", lp)
        for delta, bw, td, ta in ((24, 1, 0, 0), (24, 5, 0, 0), (24, 12, 0, 0), (60, 7, 0, 0), (7, 100, 0, 0),
                                  (24, 0, 96, 0), (24, 0, 96, 1), (24, 0, 96, 3), (7, 3, 50, 2), (24, 0, 10, 2)):
            g.set_option("delta", delta)
            g.set_option("band_width", bw)
            g.set_option("tail_delta", td)
            g.set_option("tail_after", ta)
            g.set_option("tail_frac", 2.0 if td else 0.0)  # (switch as soon as tail_after allows)
            for r in roots:
                for sr in (0, 1, 2):
                    g.set_option("spec_round", sr)
                    assert (g.sssp(r) == exp[r]).all(), (pf, lp, delta, bw, td, ta, r, sr)
    g.close()


@pytest.mark.parametrize("scale,ef", [(12, 16), (14, 4), (15, 16)])
def test_weighted_defer_heavy(ctx, oracle, scale, ef):
    """Deferred far heavy edges (defer_heavy, delta.hip): a heavy push relaxes only the edges
    that land in the next band and leaves the rest to the next heavy step (a pull whose stop
    rule starts at the deferring band, or a whole push of the deferred members), and pushes
    them whole before an empty band's jump or the end. Every heavy push deferred (1e-12),
    the default threshold, never (0); pull rules that make the next step a pull or a push;
    small deltas and narrow bands (empty bands, jumps); with and without the tail and the
    deferred band check. Bit-exact against the oracle Dijkstra."""
    g = ctx.generate_kronecker(scale, ef, 21 + scale, weighted=True)
    row, col, wc = g.get_csr()
    col = col.astype(np.uint32)
    roots = [int(r) for r in g.sample_roots(11 + ef, 3)]
    exp = {r: oracle.dijkstra(row, col, wc, r) for r in roots}
    pushed_any = False  # (with defer_heavy 1e-12 every heavy push outside the tail switch defers)
    for dh in (1e-12, 0.002, 0.0):
        g.set_option("defer_heavy", dh)
        for pf in (4.0, 0.3, 40.0):
            g.set_option("pull_factor", pf)
            # (deltas above 127: bands too wide for the heavy pull's byte map, whose probes then read
            # dist, the deferred members included: ADVICE r05)
            for delta, bw, tf, dc in ((0, 0, 0.2, 1), (3, 0, 0.0, 1), (7, 2, 0.0, 0), (24, 0, 0.1, 1), (2, 1, 0.3, 0),
                                      (160, 0, 0.0, 1), (200, 130, 0.0, 0)):
                g.set_option("delta", delta)
                g.set_option("band_width", bw)
                g.set_option("tail_frac", tf)
                g.set_option("defer_check", dc)
                for r in roots:
                    for sr in (0, 1, 2):  # (spec_round: light rounds enqueued behind every check's publish)
                        g.set_option("spec_round", sr)
                        assert (g.sssp(r) == exp[r]).all(), (dh, pf, delta, bw, tf, dc, r, sr)
                        pushed_any |= dh > 0 and g.stats()["td_levels"] > 0
    assert pushed_any
    g.close()


@pytest.mark.parametrize("scale,ef", [(12, 16), (14, 4), (16, 1), (15, 16)])
def test_weighted_pull_heavy(ctx, oracle, scale, ef):
    """Heavy edges by pull (symmetric graphs): never (push only), by the default
    rule, and in every band; several deltas, with and without the tail switch. Bit-exact against the oracle Dijkstra."""
    g = ctx.generate_kronecker(scale, ef, 9 + scale, weighted=True)
    row, col, wc = g.get_csr()
    col = col.astype(np.uint32)
    roots = [int(r) for r in g.sample_roots(3 + ef, 3)]
    exp = {r: oracle.dijkstra(row, col, wc, r) for r in roots}
    # (heavy pull factor, light pull factor): push only, default rules, pull whenever possible
    for pf, lp in ((0.0, 0.0), (4.0, 2.0), (1e15, 1e15)):
        g.set_option("pull_factor", pf)
        g.set_option("light_pull", lp)
        for delta, tf in ((0, 0.1), (7, 0.0), (60, 0.1), (7, 0.1), (60, 0.0)):
            g.set_option("delta", delta)
            g.set_option("tail_frac", tf)
            for r in roots:
                assert (g.sssp(r) == exp[r]).all(), (pf, lp, delta, tf, r)
                st = g.stats()
                if pf == 0.0:
                    assert st["bu_levels"] == 0
                if pf == 1e15:
                    assert st["td_levels"] == 0
    g.close()


def test_batch_and_empty(ctx, oracle):
    g = ctx.generate_kronecker(11, 8, 6)
    row, col, _ = g.get_csr()
    col = col.astype(np.uint32)
    roots = list(g.sample_roots(1, 5)) + [-1, 1 << 11]
    out = g.sssp_batch(roots)
    for i, r in enumerate(roots):
        assert (out[i] == oracle.bfs(row, col, int(r))).all()
    e = ctx.load_snap_buffer(b"")
    assert e.n == 0 and e.sssp(0).size == 0


def test_copy_dist_into_pinned_rows(ctx, pj, oracle):
    """pj_host_pin'd rows take the direct DMA path of pj_copy_dist (> 1 MiB), pageable rows
    the staged one: the same distances either way."""
    g = ctx.generate_kronecker(19, 8, 4)
    row, col, _ = g.get_csr()
    r = int(g.sample_roots(2, 1)[0])
    g.sssp(r, copy=False)
    staged = g.copy_dist()
    rows = np.empty(g.n + 17, np.int32)  # (larger than n, and not page-aligned at its end)
    pj.host_pin(rows)
    try:
        pinned = g.copy_dist(rows)
    finally:
        pj.host_unpin(rows)
    assert 4 * g.n > (1 << 20)
    assert (pinned == staged).all() and (staged == oracle.bfs(row, col.astype(np.uint32), r)).all()
    rows2 = np.empty(g.n, np.int32)
    with pj.host_pin(rows2):  # the handle form: unpinned at the end of the block
        with pytest.raises(ValueError):
            pj.host_pin(rows2)  # (already registered)
        assert (g.copy_dist(rows2) == staged).all()
    with pytest.raises(ValueError):
        pj.host_unpin(rows2)  # (no longer registered)
    with pytest.raises(ValueError):
        g.copy_dist(np.empty(g.n - 1, np.int32))
    g.close()


def test_cli_end_to_end(pj, oracle, tmp_path):
    rng = np.random.default_rng(3)
    src, dst = random_graph(rng, "hub", 5000)
    text = to_text(src, dst, style=1)
    f = tmp_path / "g.txt"
    f.write_bytes(text)
    out = tmp_path / "sol.txt"
    r = subprocess.run([pj.cli_path(), str(f), "7", str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    row, col, _ = _oracle_csr(oracle, text)
    assert out.read_bytes() == oracle.format_sol(oracle.bfs(row, col, 7))
    lines = r.stderr.splitlines()
    assert lines == [
        "process 0 reads in the web graph data......",
        f"N = {len(row) - 1}",
        "read in the webgraph is done.",
        "distribute sparse matrix is done.",
        "compute shortest paths from source node: 7",
        "parallel Johnson's algorithm starts......",
        "parallel Johnson's algorithm completes.",
        f"the shortest path distance vector has been saved in file {out}",
    ]
    assert r.stdout.startswith("Time: ") and r.stdout.endswith(" seconds when using 1 processes.\n")
    # missing input file -> N = 0, header-only sol_file, rc 0 (Appendix B)
    r = subprocess.run([pj.cli_path(), str(tmp_path / "missing.txt"), "0", str(out)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and out.read_bytes() == b"the vector is:\n" and "N = 0" in r.stderr
    # atoi source semantics
    r = subprocess.run([pj.cli_path(), str(f), "7abc", str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and out.read_bytes() == oracle.format_sol(oracle.bfs(row, col, 7))


@pytest.mark.parametrize("kind", ["uniform", "hub", "chain"])
def test_msbfs_batch_rows(ctx, oracle, kind):
    """pj_sssp_batch (64 x W sources per pass, msbfs.hip): every row equals a single-source run."""
    rng = np.random.default_rng(77 + len(kind))
    n = 20000
    src, dst = random_graph(rng, kind, n)
    g = ctx.load_coo(src, dst, n=n)
    row, col, _ = oracle.coo2csr(src.astype(np.uint32), dst.astype(np.uint32), n)
    sources = [int(x) for x in rng.integers(0, n, 70)] + [-1, n, int(src[0]), int(src[0])]
    out = g.sssp_batch(sources)
    assert out.shape == (len(sources), n)
    for i, r in enumerate(sources):
        assert (out[i] == oracle.bfs(row, col, r)).all(), (kind, i, r)


def test_msbfs_levels_past_the_end_in_poisoned_memory(ctx, oracle, monkeypatch):
    """Regression (round 6, the intermittent illegal address of test_multi_handle): the first
    batch of a fresh graph launches 16 levels, far past a shallow pass's end, and its level
    archive is whatever memory the allocator handed back. The level ring must stay ended once a
    level finds nothing (no later level may run on entries the pass never wrote, whose row
    bitmaps can hold bits past n). With PJ_DEVMEM_POISON every allocation starts full of 0xFF;
    fresh graphs with n not a multiple of 64, 2-3 source batches (one out of range), rows equal
    the oracle BFS."""
    monkeypatch.setenv("PJ_DEVMEM_POISON", "1")
    try:
        for t, (kind, n) in enumerate([("hub", 2500), ("uniform", 3001), ("hub", 777), ("chain", 130)]):
            rng = np.random.default_rng(4100 + t)
            src, dst = random_graph(rng, kind, n)
            row, col, _ = oracle.coo2csr(src.astype(np.uint32), dst.astype(np.uint32), n)
            a, b = (int(src[0]), int(src[len(src) // 2])) if len(src) else (1, 2)
            for sources in ([a, n + 5], [0, n - 1, b]):
                g = ctx.load_coo(src, dst, n=n)
                for _ in range(2):  # (the second batch starts from the first one's level count)
                    out = g.sssp_batch(sources)
                    for i, r in enumerate(sources):
                        assert (out[i] == oracle.bfs(row, col, r)).all(), (kind, n, sources, i)
                g.close()
    finally:
        monkeypatch.delenv("PJ_DEVMEM_POISON")


@pytest.mark.parametrize("streams", [1, 2, 3])
def test_msbfs_stream_slots(ctx, oracle, tmp_path, streams):
    """Batched BFS passes on 1-3 concurrent slots (msbfs.hip: one stream, mask set and distance
    block per slot, a host thread each): 64-source passes (ms_width 1), every row of a
    300-source batch with duplicates and out-of-range sources equals the oracle BFS, and the
    sol_files of the drop-in equal the rows."""
    rng = np.random.default_rng(900 + streams)
    n = 12000
    src, dst = random_graph(rng, "hub", n)
    g = ctx.load_coo(src, dst, n=n)
    row, col, _ = oracle.coo2csr(src.astype(np.uint32), dst.astype(np.uint32), n)
    g.set_option("ms_width", 1)
    g.set_option("ms_streams", streams)
    sources = [int(x) for x in rng.integers(0, n, 290)] + [-1, n, int(src[0]), int(src[0])] + list(range(6))
    out = g.sssp_batch(sources)
    exp = {s: oracle.bfs(row, col, s) for s in set(sources)}
    for i, s in enumerate(sources):
        assert (out[i] == exp[s]).all(), (streams, i, s)
    paths = [str(tmp_path / f"m_{i}.txt") for i in range(0, len(sources), 37)]
    g.sssp_batch_write(sources[::37], paths)
    for p, s in zip(paths, sources[::37]):
        assert open(p, "rb").read() == oracle.format_sol(exp[s]), (streams, s)
    with pytest.raises(Exception):
        g.set_option("ms_streams", 5)
    g.close()


@pytest.mark.parametrize("width,alpha", [(1, 16), (2, 0), (4, 16), (4, 1e9), (8, 16), (8, 0), (16, 16)])
def test_msbfs_pass_widths(ctx, oracle, width, alpha):
    """Passes of 64 x W sources (W words per vertex mask): 300 sources cross several
    passes and a partial last word; push and pull levels; rows equal single-source runs."""
    rng = np.random.default_rng(5 + width)
    n = 12000
    src, dst = random_graph(rng, "hub", n)
    g = ctx.load_coo(src, dst, n=n)
    g.set_option("ms_width", width)
    g.set_option("ms_alpha", alpha)  # push levels: default rule, never, always
    row, col, _ = oracle.coo2csr(src.astype(np.uint32), dst.astype(np.uint32), n)
    sources = [int(x) for x in rng.integers(-2, n + 2, {8: 700, 16: 1100}.get(width, 300))]
    out = g.sssp_batch(sources)
    exp = {r: oracle.bfs(row, col, r) for r in set(sources)}
    for i, r in enumerate(sources):
        assert (out[i] == exp[r]).all(), (width, i, r)
    g.close()


def test_msbfs_kronecker_and_chain_cap(ctx, oracle, pj):
    g = ctx.generate_kronecker(14, 16, 3)
    row, col, _ = g.get_csr()
    col = col.astype(np.uint32)
    roots = list(g.sample_roots(5, 64))
    out = g.sssp_batch(roots)
    for i, r in enumerate(roots):
        assert (out[i] == oracle.bfs(row, col, int(r))).all()
    # R9 cap applies per source in batch mode too
    c = ctx.load_snap_buffer(chain_text(100010))
    out = c.sssp_batch([0, 5])
    assert out[0][99999] == 99999 and out[0][100000] == INF and out[1][100004] == 99999 and out[1][100005] == INF


def test_webgraph_cli_config0(ctx, pj, oracle, tmp_path):
    """BASELINE configs[0] on the web-Google-shaped synthetic (the SNAP file is not
    available): sol_file bytes equal the oracle BFS and the reference's BSP algorithm
    at np=4 (the mpirun -np 4 analogue)."""
    g = ctx.generate_webgraph(916428, 5105039, 1)
    assert g.n == 916428 and g.nnz == 5105039
    row, col, _ = g.get_csr()
    col = col.astype(np.uint32)
    f = tmp_path / "web-Google-synthetic.txt"
    f.write_bytes(csr_to_text(row, col))
    out = tmp_path / "sol.txt"
    r = subprocess.run([pj.cli_path(), str(f), "0", str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    exp = oracle.bfs(row, col, 0)
    ref4, st = oracle.reference_sssp(row, col, 0, 4)
    assert (ref4 == exp).all()
    assert out.read_bytes() == oracle.format_sol(exp)
    assert (exp < INF).sum() > 100000  # source 0 reaches a large part of the graph
    # the in-process solver with and without the one-workgroup small levels, several sources
    for small in (0, 1):
        g.set_option("bfs_small", small)
        assert (g.sssp(0) == exp).all(), small
        for s in (1, 77, 5000):
            assert (g.sssp(s) == oracle.bfs(row, col, s)).all(), (small, s)
    g.close()


def test_weighted_kronecker_s26_full_size(ctx):
    """BASELINE.json configs[2] at full size (2^31 entries, weights 1..255), the bench's
    first roots: every distance proven exact by the shortest-path certificate
    (helpers.sssp_certificate: no edge relaxes further, every reached vertex has a
    tight in-edge), which needs no CPU solve. Also checks reach_stats against dist."""
    import torch
    from helpers import sssp_certificate
    g = ctx.generate_kronecker(26, 16, 1, weighted=True)
    assert g.nnz == 1 << 31 and g.weighted
    roots = [int(r) for r in g.sample_roots(2, 2)]  # bench.py: sample_roots(seed + 1, 64)
    dists = {r: g.sssp(r) for r in roots}
    row, col, w = g.get_csr()
    g.close()
    assert int(w.min()) >= 1 and int(w.max()) <= 255
    deg = np.diff(row)
    for r, d in dists.items():
        assert sssp_certificate(row, col, w, d, r, device="cuda", chunk=1 << 28) == [], r
        reached = d < INF
        assert reached.sum() > (1 << 24)  # the giant component (~49% of the ids at s26)
        assert d[reached].max() > 255  # multi-hop weighted paths, several bands
    torch.cuda.empty_cache()


def test_partitioned_bfs_s28_full_size(ctx, pj):
    """BASELINE.json configs[3] at full size: Kronecker s28 (2^33 entries, 64-bit row
    offsets), 1D vertex partition at world 1 (no exchange), and at world 2, 4 and 8 with
    every rank on the one GPU over the host transport (each rank builds only its own
    rows; per level: the claimed remote ids packed owner-major into traffic-sized
    buffers, the count exchange, the alltoallv of ids
    (the reference's :522-554, buffers sized at :495-501), the visited all-gather around
    pull levels and the termination allreduce :589-590). Every world must give the same
    gathered distances, which are proven exact by the certificate against the CSR of the
    same graph built by the single-GPU loader (kronecker -> radix sort -> CSR)."""
    import torch
    from helpers import sssp_certificate
    from paralleljohnson_amd.partition import Comm, bfs_group, gather_group, load_kronecker
    roots, dists = [], {}
    ops = load_kronecker(ctx, 28, 16, 1, 0, 1)
    comm = Comm.for_rank(ctx, 1, 0)
    for c in np.random.default_rng(8).integers(0, 1 << 28, 64):  # bench.py's root rule: reached > 1
        st = ops.bfs(comm, int(c))
        if st["reached"] > 1:
            d = ops.gather_dist(comm)
            assert st["reached"] == int((d < INF).sum())
            roots.append(int(c))
            dists[int(c)] = d
        if len(roots) == 2:
            break
    ops.close()
    comm.close()
    torch.cuda.empty_cache()
    mem = {}
    for world in (2, 4, 8):
        ctxs = [pj.Context(0) for _ in range(world)]
        comms = Comm.group(ctxs, "host")
        parts = [load_kronecker(ctxs[r], 28, 16, 1, r, world) for r in range(world)]
        assert sum(p.nnz_local for p in parts) == 1 << 33
        sent = [0] * world
        for r in roots:
            st = bfs_group(parts, comms, r)
            assert len({(x["levels"], x["td_levels"], x["bu_levels"]) for x in st}) == 1  # same loop on every rank
            assert sum(x["sent"] for x in st) > 0  # the owner exchange ran
            assert st[0]["reached"] == int((dists[r] < INF).sum()), (world, r)
            got = gather_group(parts, comms)
            assert np.array_equal(got, dists[r]), (world, r)
            sent = [max(a, x["sent"]) for a, x in zip(sent, st)]
        # per-rank device bytes: the exchange buffers follow the traffic (at most the ids one
        # BFS sends / receives, x1.25 growth slack, x2 for send + recv), no longer world x block
        # sized regions (round 3: 40 N bytes per rank at every world)
        b = [p.device_bytes() for p in parts]
        mem[world] = {k: max(x[k] for x in b) for k in b[0]}
        n = 1 << 28
        assert mem[world]["exchange"] <= 2 * 1.25 * 4 * max(sent) * world + 64, (world, mem[world], sent)
        assert mem[world]["exchange"] < 40 * n / 16, (world, mem[world])
        for p in parts:
            p.close()
        for c in comms:
            c.close()
        for c in ctxs:
            c.close()
        torch.cuda.empty_cache()
    # rows and vertex state shrink with the world size; the N-bit bitmaps stay
    assert mem[8]["rows"] < mem[2]["rows"] / 3 and mem[8]["state"] < mem[2]["state"] / 3, mem
    # the exchange buffers are capped at block / 16 ids per direction (bigger push levels go
    # out in pieces): O(N / P) like the rest of the rank's state
    assert mem[8]["exchange"] <= 0.3 * mem[2]["exchange"], mem
    print("per-rank device bytes by world:", mem)  # (shown with pytest -s)
    total = {w: sum(m.values()) for w, m in mem.items()}
    assert total[8] < total[4] < total[2], mem
    g = ctx.generate_kronecker(28, 16, 1)
    assert g.nnz == 1 << 33
    row, col, _ = g.get_csr()
    g.close()
    for r, d in dists.items():
        assert sssp_certificate(row, col, None, d, r, device="cuda", chunk=1 << 28) == [], r
        assert (d < INF).sum() > (1 << 26)
    torch.cuda.empty_cache()


def test_partitioned_weighted_s22_world2(ctx, pj):
    """The weighted 1D partition (wpart.hip + the C++ band loop) on the full Kronecker s22
    with weights 1..255 at world 2 (ranks sharing the GPU over the host transport), each
    rank generating only its own block's rows:
    gathered distances equal the single-GPU delta-stepping solver's and are proven exact
    by the certificate; the remote-candidate exchange ran, in buffers sized to its traffic."""
    import torch
    from helpers import sssp_certificate
    from paralleljohnson_amd.partition import Comm, delta_group, gather_group, load_weighted_kronecker
    world = 2
    ctxs = [pj.Context(0) for _ in range(world)]
    comms = Comm.group(ctxs, "host")
    gs = [ctxs[0].generate_kronecker(22, 16, 1, weighted=True)]  # (the single-GPU reference solve)
    # each rank generates only its block's rows (pj_wpart_generate_kronecker)
    parts = [load_weighted_kronecker(ctxs[r], 22, 16, 1, r, world) for r in range(world)]
    assert sum(p.nnz_local for p in parts) == gs[0].nnz and all(p.nnz == gs[0].nnz for p in parts)
    roots = [int(r) for r in gs[0].sample_roots(2, 2)]
    sent = 0
    for r in roots:
        st = delta_group(parts, comms, r)
        assert sum(x["sent"] for x in st) > 0
        assert len({(x["bands"], x["rounds"]) for x in st}) == 1
        got = gather_group(parts, comms)
        exp = gs[0].sssp(r)
        assert np.array_equal(got, exp), r
        assert st[0]["reached"] == int((exp < INF).sum())
        sent = max(sent, max(x["sent"] for x in st))
    # the (id, candidate) exchange follows the traffic, not world x block regions (round 3: 24 N
    # bytes per rank): the claim queue and the send buffer packed from it (each at most twice a
    # round's pairs over the shards plus once as spill, <= the solve's pairs, beyond their initial
    # 96 x block / 256 pairs) and the receive buffer (x1.25 growth slack)
    for p in parts:
        b = p.device_bytes()
        q0 = 96 * max(16, p.block // 256) + 4096 + 16 * 64
        assert 0 < b["exchange"] <= 8 * (2 * (3 * sent + q0) + 1.25 * sent * world), (b, sent)
        assert b["exchange"] < 24 * (1 << 22) / 4, b
    row, col, w = gs[0].get_csr()
    # the automatic delta (both solvers' rule, internal.h auto_delta): c(n) x mean weight /
    # mean out-degree, c = 0.1875 log2(n) - 1.875 within [2, 3.5] -- 2.25 at s22
    n = len(row) - 1
    mean_w = int(w.astype(np.int64).sum()) / len(col)  # (the generator's exact sum / 2M, as wpart's)
    exp_delta = int(np.floor(2.25 * mean_w / (len(col) / n) + 0.5))
    assert st[0]["delta"] == exp_delta, (st[0]["delta"], exp_delta)
    for p in parts:
        p.close()
    for g in gs:
        g.close()
    for c in comms:
        c.close()
    for c in ctxs:
        c.close()
    torch.cuda.empty_cache()
    # the certificate of the last solve's distances (got) against the single-GPU CSR
    assert sssp_certificate(row, col, w, got, roots[-1], device="cuda", chunk=1 << 27) == []


@pytest.mark.gpu
def test_weighted_work_counters_and_deferred_gather(ctx, oracle):
    """The always-on work counters of a weighted solve (pj_stats.scanned_edges / probes /
    work_bytes, per kernel class) are consistent, and the input-id distances gathered lazily
    from the solver's ids (delta_materialize) are exact through every reader: the host copy,
    pj_dist_device, the reach pass and the parent tree; a source without edges gets its 0."""
    g = ctx.generate_kronecker(14, 16, 5, weighted=True)
    row, col, wc = g.get_csr()
    col = col.astype(np.uint32)
    deg = np.diff(row)
    roots = [int(r) for r in g.sample_roots(3, 3)]
    for r in roots:
        exp = oracle.dijkstra(row, col, wc, r)
        g.sssp(r, copy=False)
        st = g.stats()
        byk = st["work_by_kernel"]
        assert st["scanned_edges"] == sum(v[0] for v in byk.values()) > 0
        assert st["probes"] == sum(v[1] for v in byk.values()) > 0
        assert st["work_bytes"] == sum(v[2] for v in byk.values())
        for rec, prb, nb in byk.values():
            assert 0 <= prb <= rec + rec  # (a probe per record at most, a pull's stop record unprobed)
            assert rec + prb <= nb <= 8 * rec + 4 * prb
        assert byk["light_round"][0] > 0
        # a solve scans fewer records than the reached vertices' rows hold, and never 4x more
        m_r = int(deg[exp < oracle.INT_INF].sum())
        assert st["scanned_edges"] <= 4 * m_r
        assert g.dist_device_ptr() != 0  # (materializes the input-id row)
        assert (g.copy_dist() == exp).all()
        g.sssp(r, copy=False)
        rs = g.reach_stats()
        assert rs["reached"] == int((exp < oracle.INT_INF).sum()) and rs["reached_edges"] == m_r
        par = g.parent_tree()
        assert all(v == 0 for k, v in g.validate_tree(r, par).items() if k.startswith("bad"))
        assert (g.sssp(r) == exp).all()
    iso = int(np.nonzero(deg == 0)[0][0])
    g.sssp(iso, copy=False)
    assert g.stats()["scanned_edges"] == 0
    d = g.copy_dist()
    assert d[iso] == 0 and (np.delete(d, iso) == oracle.INT_INF).all()
    g.close()
