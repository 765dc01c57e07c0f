"""Shortest-path tree output and its Graph500-style validation (SURVEY.md §8f rank 4;
no reference counterpart: the reference writes distances only, output_vector :32-46).

The tree is a function of the distances (the smallest tight in-neighbour), so the GPU
parent array must equal the CPU restatement (helpers.tight_parents) bit for bit, and
pj_validate_tree must count exactly what helpers.graph500_checks counts, for valid and
for corrupted parent arrays. Parity of the distances themselves is test_gpu_parity's.
"""
import os
import subprocess

import numpy as np
import pytest

from helpers import graph500_checks, random_graph, tight_parents

INF = 100000
ZERO = dict(bad_root=0, bad_reach=0, bad_tree_edge=0, bad_edge=0, bad_cycle=0)


def _bad(rep):
    return {k: v for k, v in rep.items() if k.startswith("bad_")}


def _corruptions(par, dist, source, rng):
    """Parent arrays that break one Graph500 check each (name, array)."""
    n = len(par)
    reached = np.nonzero((dist < INF) & (np.arange(n) != source))[0]
    unreached = np.nonzero(dist >= INF)[0]
    out = []
    p = par.copy()
    p[source] = -1
    out.append(("root", p))
    if len(unreached):
        p = par.copy()
        p[unreached[0]] = source
        out.append(("reach", p))
    if len(reached) >= 2:
        a, b = reached[0], reached[-1]
        p = par.copy()
        p[a], p[b] = b, a  # a 2-cycle: not tight, and their subtrees no longer reach the root
        out.append(("cycle", p))
        # a parent at least as far from the source: never joined by a tight edge (w >= 1)
        near = reached[np.argmin(dist[reached])]
        far = reached[np.argmax(dist[reached])]
        if far == near:
            far = reached[1] if reached[0] == near else reached[0]
        p = par.copy()
        p[near] = far
        out.append(("tree", p))
        p = par.copy()
        p[a] = n + 5
        out.append(("range", p))
    return out


# ---------------------------------------------------------------- CPU (checker) --

def test_checks_pin_on_small_graph(oracle):
    """The CPU checker on a hand-made graph: the tight tree passes, each corruption is
    caught by the check it breaks."""
    src = np.array([0, 0, 1, 2, 3, 5, 5], np.uint32)  # 4 has no in-edge; 6 only from 5
    dst = np.array([1, 2, 3, 3, 0, 6, 6], np.uint32)
    n = 7
    row, col, _ = oracle.coo2csr(src, dst, n)
    dist = oracle.bfs(row, col, 0)
    assert dist.tolist() == [0, 1, 1, 2, INF, INF, INF]
    par = tight_parents(row, col, None, dist, 0)
    assert par.tolist() == [0, 0, 0, 1, -1, -1, -1]  # 3: smallest tight in-neighbour (1, not 2)
    assert _bad(graph500_checks(row, col, None, dist, par, 0)) == ZERO
    p = par.copy(); p[3] = 2
    assert _bad(graph500_checks(row, col, None, dist, p, 0)) == ZERO  # any tight parent is valid
    p = par.copy(); p[3] = 0
    assert graph500_checks(row, col, None, dist, p, 0)["bad_tree_edge"] == 1  # no edge 0 -> 3
    p = par.copy(); p[6] = 5
    assert graph500_checks(row, col, None, dist, p, 0)["bad_reach"] == 1
    p = par.copy(); p[1], p[2] = 2, 1
    r = graph500_checks(row, col, None, dist, p, 0)
    assert r["bad_tree_edge"] == 2 and r["bad_cycle"] == 3  # 1, 2 and 3 (child of 1) lose the root
    d = dist.copy(); d[3] = 3
    assert graph500_checks(row, col, None, d, tight_parents(row, col, None, d, 0), 0)["bad_edge"] == 2
    p = par.copy(); p[0] = 1
    assert graph500_checks(row, col, None, dist, p, 0)["bad_root"] == 1


def test_checks_weighted_cpu(oracle):
    rng = np.random.default_rng(3)
    n = 3000
    s, d = random_graph(rng, "hub", n)
    w = rng.integers(1, 20, len(s)).astype(np.uint32)
    row, col, wc = oracle.coo2csr(s.astype(np.uint32), d.astype(np.uint32), n, w)
    dist = oracle.dijkstra(row, col, wc, int(s[0]))
    par = tight_parents(row, col, wc, dist, int(s[0]))
    assert _bad(graph500_checks(row, col, wc, dist, par, int(s[0]))) == ZERO
    for name, p in _corruptions(par, dist, int(s[0]), rng):
        assert sum(_bad(graph500_checks(row, col, wc, dist, p, int(s[0]))).values()) > 0, name


def test_zero_weight_tree_is_acyclic(oracle):
    """Zero-weight edges: two vertices at the same distance must not parent each other
    (source 9 -> 2 (w 1), 1 <-> 2 (w 0), 2 -> 3 (w 0), 3 -> 1 (w 0)): 2 takes its positive
    tight in-edge, 1 and 3 are parented by hop depth through the zero-weight edges."""
    src = np.array([9, 1, 2, 2, 3], np.uint32)
    dst = np.array([2, 2, 1, 3, 1], np.uint32)
    w = np.array([1, 0, 0, 0, 0], np.uint32)
    row, col, wc = oracle.coo2csr(src, dst, 10, w)
    dist = oracle.dijkstra(row, col, wc, 9)
    assert dist[[1, 2, 3, 9]].tolist() == [1, 1, 1, 0]
    par = tight_parents(row, col, wc, dist, 9)
    assert par[[1, 2, 3, 9]].tolist() == [2, 9, 2, 9]
    assert _bad(graph500_checks(row, col, wc, dist, par, 9)) == ZERO
    p = par.copy(); p[2] = 1  # the old smallest-tight-parent rule: 1 <-> 2 cycle
    assert graph500_checks(row, col, wc, dist, p, 9)["bad_cycle"] > 0


# ---------------------------------------------------------------------- GPU --

def _check_graph(g, root, rng, corrupt=True):
    row, col, w = g.get_csr()
    dist = g.sssp(root)
    par = g.parent_tree()
    exp = tight_parents(row, col, w, dist, root)
    assert (par == exp).all()
    rep = g.validate_tree(root, par)
    assert _bad(rep) == ZERO and rep["reached"] == int((dist < INF).sum())
    if corrupt:
        for name, p in _corruptions(par, dist, root, rng):
            got = g.validate_tree(root, p)
            assert got == graph500_checks(row, col, w, dist, p, root), name
            assert sum(_bad(got).values()) > 0, name


@pytest.mark.gpu
@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("kind", ["uniform", "hub", "chain"])
def test_parent_tree_random_graphs(ctx, kind, weighted):
    rng = np.random.default_rng(40 + len(kind) + weighted)
    for trial in range(3):
        n = int(rng.integers(2, 40000))
        s, d = random_graph(rng, kind, n)
        w = rng.integers(1, 30, len(s)).astype(np.uint32) if weighted else None
        g = ctx.load_coo(s, d, w=w, n=n)
        _check_graph(g, int(s[0]) if len(s) else 0, rng)
        g.close()


@pytest.mark.gpu
def test_parent_tree_zero_weights(ctx, oracle):
    """Weights 0..3 (zero-weight cycles at equal distance): the tree is acyclic, equal to
    the CPU restatement, and passes every Graph500 check (advisor case included)."""
    rng = np.random.default_rng(77)
    g = ctx.load_coo(np.array([9, 1, 2, 2, 3]), np.array([2, 2, 1, 3, 1]), w=np.array([1, 0, 0, 0, 0], np.uint32), n=10)
    _check_graph(g, 9, rng, corrupt=False)
    assert g.parent_tree()[[1, 2, 3, 9]].tolist() == [2, 9, 2, 9]
    g.close()
    for kind in ("uniform", "hub", "chain"):
        n = int(rng.integers(1000, 30000))
        s, d = random_graph(rng, kind, n)
        w = rng.integers(0, 4, len(s)).astype(np.uint32)
        g = ctx.load_coo(s, d, w=w, n=n)
        _check_graph(g, int(s[0]), rng)
        g.close()


@pytest.mark.gpu
def test_parent_tree_kronecker_and_webgraph(ctx):
    """Every solver path gives the smallest-tight-parent tree: Kronecker BFS (push / pull
    levels, hubs), weighted Kronecker (delta bands), and configs[0]'s web-Google-shaped
    graph at full size."""
    rng = np.random.default_rng(7)
    g = ctx.generate_kronecker(16, 16, 2)
    for r in g.sample_roots(5, 2):
        _check_graph(g, int(r), rng)
    g.close()
    g = ctx.generate_kronecker(14, 16, 3, weighted=True)
    for r in g.sample_roots(5, 2):
        _check_graph(g, int(r), rng)
    g.close()
    g = ctx.generate_webgraph()
    _check_graph(g, 0, rng, corrupt=False)
    g.close()


@pytest.mark.gpu
def test_parent_tree_state_errors(ctx, pj):
    g = ctx.generate_kronecker(10, 16, 1)
    with pytest.raises(pj.PJError) as e:
        g.parent_tree()
    assert e.value.name == "PJ_ERR_STATE"
    g.sssp(1)
    with pytest.raises(pj.PJError) as e:
        g.validate_tree(2, np.full(g.n, -1, np.int64))  # not the last solve's source
    assert e.value.name == "PJ_ERR_STATE"
    g.sssp_batch([1, 2])
    with pytest.raises(pj.PJError):
        g.parent_tree()
    g.close()


@pytest.mark.gpu
def test_cli_parents(pj, oracle, tmp_path):
    rng = np.random.default_rng(11)
    n = 5000
    s, d = random_graph(rng, "hub", n)
    text = "".join(f"{a}\t{b}\n" for a, b in zip(s, d)).encode()
    web = tmp_path / "g.txt"
    web.write_bytes(text)
    row, col, _ = oracle.coo2csr(s.astype(np.uint32), d.astype(np.uint32), int(max(s.max(), d.max())) + 1)
    src = int(s[0])
    dist = oracle.bfs(row, col, src)
    exp = tight_parents(row, col, None, dist, src)
    env = dict(os.environ, PJ_PARENTS=str(tmp_path / "par.txt"))
    env.pop("PJ_GPUS", None)
    r = subprocess.run([pj.cli_path(), str(web), str(src), str(tmp_path / "sol.txt")], env=env,
                       capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert b"validation passed" in r.stderr
    body = (tmp_path / "par.txt").read_bytes().split(b"\n")
    assert body[0] == b"the parent tree is:"
    assert [int(x) for x in body[1:-1]] == exp.tolist()
    r = subprocess.run([pj.cli_path(), str(web), str(src), str(tmp_path / "sol2.txt")],
                       env=dict(env, PJ_GPUS="2"), capture_output=True, timeout=120)
    assert r.returncode == 255 and b"PJ_PARENTS" in r.stderr
