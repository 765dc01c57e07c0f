"""Shared graph builders for the parity tests (seeded, deterministic)."""
import numpy as np


def chain_text(n):
    return "".join(f"{i} {i + 1}\n" for i in range(n - 1)).encode()


def random_graph(rng, kind, n):
    """Directed multigraph edges (src, dst) of a few shapes the reference's fuzz used
    (uniform, power-law hub, chain + noise)."""
    if kind == "uniform":
        m = int(rng.integers(0, 6 * n + 1))
        return rng.integers(0, n, m), rng.integers(0, n, m)
    if kind == "hub":
        m = 8 * n
        a = rng.zipf(1.6, m) % n
        b = rng.integers(0, n, m)
        flip = rng.random(m) < 0.5
        return np.where(flip, a, b), np.where(flip, b, a)
    if kind == "chain":
        s = np.arange(n - 1)
        noise = max(1, n // 20)
        return (np.concatenate([s, rng.integers(0, n, noise)]),
                np.concatenate([s + 1, rng.integers(0, n, noise)]))
    raise ValueError(kind)


def to_text(src, dst, w=None, style=0):
    """Edge-list text in a few of the layouts the reference accepts."""
    lines = ["# FromNodeId\tToNodeId\n"] if style else []
    for i, (a, b) in enumerate(zip(src, dst)):
        sep = "\t" if (style == 0 or i % 3) else "  "
        tail = f"\t{w[i]}" if w is not None else ""
        eol = "\r\n" if (style == 2 and i % 2) else "\n"
        lines.append(f"{a}{sep}{b}{tail}{eol}")
        if style and i % 97 == 0:
            lines.append("\n# comment line\n")
    return "".join(lines).encode()


def sssp_certificate(row, col, w, dist, root, inf=100000, device="cpu", chunk=1 << 27):
    """Size-independent proof that `dist` is the capped shortest-path vector of the CSR
    graph from `root` (the R9 contract): returns a list of violations
    (empty = exact).

    With weights >= 1 (w is None = unit), `dist` is exact iff
      (1) dist[root] == 0 when 0 <= root < n, every entry in [0, inf];
      (2) no edge u->v with dist[u] + w < inf has dist[v] > dist[u] + w;
      (3) every v != root with dist[v] < inf has a tight in-edge u->v,
          dist[u] + w == dist[v] (so dist[v] is the length of a real path).
    (2) bounds dist from above by induction along shortest paths; (3) gives a
    strictly decreasing predecessor chain that ends at the root, so dist is a path
    length; a true distance >= inf therefore forces dist = inf. Edges are streamed
    in row chunks of about `chunk` entries, on `device` (torch)."""
    import torch
    n = len(row) - 1
    d = torch.as_tensor(np.asarray(dist, dtype=np.int64)).to(device)
    bad = []
    if n == 0:
        return bad
    if int(d.min()) < 0 or int(d.max()) > inf:
        bad.append("entry outside [0, inf]")
    if 0 <= root < n and int(d[root]) != 0:
        bad.append(f"dist[root] = {int(d[root])}")
    best = torch.full((n,), inf, dtype=torch.int64, device=device)  # min over in-edges of dist[u] + w
    row = np.asarray(row, dtype=np.int64)
    r0 = 0
    while r0 < n:
        r1 = int(np.searchsorted(row, row[r0] + chunk, side="right")) - 1
        r1 = min(max(r1, r0 + 1), n)
        e0, e1 = int(row[r0]), int(row[r1])
        if e1 > e0:
            deg = torch.as_tensor(np.diff(row[r0:r1 + 1])).to(device)
            u = torch.repeat_interleave(torch.arange(r0, r1, device=device), deg)
            v = torch.as_tensor(np.asarray(col[e0:e1]).view(np.uint32).astype(np.int64)).to(device)
            cand = d[u] + (1 if w is None else torch.as_tensor(np.asarray(w[e0:e1], dtype=np.int64)).to(device))
            cand = torch.where(d[u] < inf, cand, torch.full_like(cand, inf)).clamp_(max=inf)
            if bool((d[v] > cand).any()):
                bad.append(f"edge rows [{r0}, {r1}): an edge relaxes further (condition 2)")
            best.scatter_reduce_(0, v, cand, reduce="amin")
        r0 = r1
    reached = d < inf
    if 0 <= root < n:
        reached[root] = False
    if bool((best[reached] != d[reached]).any()):
        bad.append("a reached vertex has no tight in-edge (condition 3)")
    return bad


def csr_to_text(row, col):
    """SNAP-style edge list (tab-separated, '#' header) of a CSR, rows in order."""
    import numpy as np
    src = np.repeat(np.arange(len(row) - 1, dtype=np.int64), np.diff(row))
    body = np.char.add(np.char.add(src.astype(str), "\t"), np.asarray(col, dtype=np.int64).astype(str))
    return ("# Directed graph (synthetic, web-Google-shaped)\n# FromNodeId\tToNodeId\n" +
            "\n".join(body.tolist()) + "\n").encode()


def tight_parents(row, col, w, dist, source, inf=100000):
    """CPU restatement of pj_parent_tree (tree.hip): parent[v] = the smallest u with an
    edge u -> v of weight w > 0 and dist[u] + w == dist[v] < inf; a reached v without
    one is parented through zero-weight tight edges, level by level from the vertices
    parented so far (hop depth h, 0 for the source and every vertex with a positive tight
    in-edge): the smallest u with w == 0, dist[u] == dist[v], h(u) == h(v) - 1.
    parent[source] = source, -1 when unreached."""
    row = np.asarray(row, dtype=np.int64)
    n = len(row) - 1
    d = np.asarray(dist, dtype=np.int64)
    u = np.repeat(np.arange(n, dtype=np.int64), np.diff(row))
    v = np.asarray(col).view(np.uint32).astype(np.int64)
    wt = np.ones_like(v) if w is None else np.asarray(w, dtype=np.int64)
    tight = (d[u] < inf) & (d[v] < inf) & (d[u] + wt == d[v])
    big = np.iinfo(np.int64).max
    par = np.full(n, big, np.int64)
    pos = tight & (wt > 0)
    np.minimum.at(par, v[pos], u[pos])
    zero = tight & (wt == 0)
    if zero.any():
        hop = np.where(par != big, 0, -1)
        if 0 <= source < n:
            hop[source] = 0
        zu, zv = u[zero], v[zero]
        lvl = 0
        while True:
            e = (hop[zu] == lvl) & (hop[zv] < 0)
            if 0 <= source < n:
                e &= zv != source
            if not e.any():
                break
            np.minimum.at(par, zv[e], zu[e])
            hop[zv[e]] = lvl + 1
            lvl += 1
    par[par == big] = -1
    if 0 <= source < n:
        par[source] = source
    return par


def graph500_checks(row, col, w, dist, parent, source, inf=100000):
    """CPU restatement of pj_validate_tree (the Graph500 BFS / SSSP validation, for the
    capped int32 distances): counts per check, all bad_* zero = valid."""
    row = np.asarray(row, dtype=np.int64)
    n = len(row) - 1
    d = np.asarray(dist, dtype=np.int64)
    p = np.asarray(parent, dtype=np.int64)
    u = np.repeat(np.arange(n, dtype=np.int64), np.diff(row))
    v = np.asarray(col).view(np.uint32).astype(np.int64)
    wt = np.ones_like(v) if w is None else np.asarray(w, dtype=np.int64)
    reached = d < inf
    out = dict(reached=int(reached.sum()), bad_root=0, bad_reach=0, bad_tree_edge=0, bad_edge=0, bad_cycle=0)
    fu = reached[u]
    via = d[u] + wt
    out["bad_edge"] = int((d[v][fu] > np.minimum(via[fu], inf)).sum())
    ok = np.zeros(n, bool)
    t = fu & (d[v] < inf) & (via == d[v]) & (p[v] == u)
    ok[v[t]] = True
    idx = np.arange(n)
    other = idx != source
    out["bad_root"] = int(0 <= source < n and (p[source] != source or d[source] != 0))
    out["bad_reach"] = int(((~reached) & other & (p != -1)).sum())
    inner = reached & other
    badp = inner & ((p < 0) | (p >= n) | (p == idx))
    out["bad_reach"] += int(badp.sum())
    good = inner & ~badp
    out["bad_tree_edge"] = int((good & ~ok).sum())
    anc = np.where(good, p, -1)
    if 0 <= source < n:
        anc[source] = source
    for _ in range(max(1, int(np.ceil(np.log2(max(n, 2))))) + 1):
        anc = np.where(anc >= 0, anc[np.maximum(anc, 0)], -1)
    out["bad_cycle"] = int((inner & (anc != source)).sum())
    return out
