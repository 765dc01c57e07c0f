"""Numpy restatement of the pj_part_* / pj_wpart_* device steps (part.hip,
wpart.hip), for the CPU tests of libpj's partitioned protocol loops
(engine.cpp, driven through pj_engine_bfs / pj_engine_delta) under gloo.

Test infrastructure only: it lets the world_size > 1 exchange, termination and
direction logic of the C++ loops run without a GPU. The product path runs the
same loops over libpj's kernels (pj_part_bfs / pj_wpart_delta). Semantics per
step are those documented in include/pj.h. The buffers the loop hands to the
transport (vis, iso, zown, send, recv) are numpy arrays with fixed addresses."""
import numpy as np

from paralleljohnson_amd.partition import block_geometry

INF = 100000


class NumpyPart:
    def __init__(self, src, dst, n, rank, world, symmetric=False):
        src = np.asarray(src, np.int64)
        dst = np.asarray(dst, np.int64)
        self.n, self.rank, self.world = n, rank, world
        self.block, ranges = block_geometry(n, world)
        self.bw = self.block // 64
        self.lo, self.hi = ranges[rank]
        self.nl = self.hi - self.lo
        self.symmetric = symmetric

        def rows(key, val):
            m = (key >= self.lo) & (key < self.hi)
            k, v = key[m] - self.lo, val[m]
            order = np.argsort(k, kind="stable")
            row = np.zeros(self.nl + 1, np.int64)
            np.add.at(row, k + 1, 1)
            return np.cumsum(row), v[order]

        self.row, self.col = rows(src, dst)
        self.crow, self.ccol = (self.row, self.col) if symmetric else rows(dst, src)
        self.nnz_local = len(self.col)
        self.vis = np.zeros(world * self.bw, np.uint64)
        self.iso = np.zeros_like(self.vis)
        self.zown = np.zeros(self.bw, np.uint64)
        cap = world * self.block if world > 1 else 1
        self.send = np.zeros(cap, np.uint32)
        self.recv = np.zeros(cap, np.uint32)
        self.dist = np.full(max(self.nl, 1), INF, np.int32)[: self.nl]
        self.fr = np.zeros(self.bw, np.uint64)
        self.frn = np.zeros(self.bw, np.uint64)

    def _v(self):
        return self.vis

    @staticmethod
    def _get(words, ids):
        ids = np.asarray(ids, np.int64)
        return (words[ids >> 6] >> (ids & 63).astype(np.uint64)) & np.uint64(1)

    @staticmethod
    def _set(words, ids):
        ids = np.asarray(ids, np.int64)
        np.bitwise_or.at(words, ids >> 6, np.uint64(1) << (ids & 63).astype(np.uint64))

    def zmask(self):
        """Own isolated-vertex words -> zown (padding past the last owned vertex counts as isolated)."""
        self.zown[:] = 0
        v = np.arange(self.block)
        iso = np.ones(self.block, bool)
        iso[: self.nl] = (np.diff(self.row) == 0) & (np.diff(self.crow) == 0)
        self._set(self.zown, v[iso])

    def _settle(self, ids, level):
        """ids: global ids owned by this rank, newly claimed."""
        loc = np.asarray(ids, np.int64) - self.lo
        self.dist[loc] = level + 1
        self._set(self.frn, loc)

    def begin(self, s):
        self._v()[:] = self.iso
        self.dist[:] = INF
        self.fr[:] = 0
        self.frn[:] = 0
        if 0 <= s < self.n:
            self._set(self._v(), [s])
            if self.lo <= s < self.hi:
                self.dist[s - self.lo] = 0
                self._set(self.frn, [s - self.lo])
        return self.end_level()

    def _frontier(self, words):
        ids = np.nonzero(np.unpackbits(words.view(np.uint8), bitorder="little"))[0]
        return ids[ids < self.nl]

    def push(self, level):
        vis = self._v()
        f = self._frontier(self.fr)
        if len(f):
            tg = np.concatenate([self.col[self.row[u]:self.row[u + 1]] for u in f])
        else:
            tg = np.zeros(0, np.int64)
        tg = tg[self._get(vis, tg) == 0]
        tg = np.unique(tg)
        self._set(vis, tg)
        owner = tg // self.block
        mine = owner == self.rank
        self._settle(tg[mine], level)
        out = tg[~mine]
        counts = [int(np.sum(owner[~mine] == o)) for o in range(self.world)]
        packed = np.concatenate([out[owner[~mine] == o] for o in range(self.world)]) if len(out) else out
        if len(packed):
            self.send[: len(packed)] = packed.astype(np.uint32)
        return counts

    def apply(self, level, nr):
        vis = self._v()
        ids = self.recv[:nr].astype(np.int64)
        assert np.all((ids >= self.lo) & (ids < self.hi)), "received ids owned by another rank"
        ids = np.unique(ids[self._get(vis, ids) == 0])
        self._set(vis, ids)
        self._settle(ids, level)

    def pull(self, level):
        vis = self._v().copy()  # snapshot: pull writes only frn
        own = vis[self.rank * self.bw:(self.rank + 1) * self.bw]
        cand = np.nonzero(np.unpackbits(own.view(np.uint8), bitorder="little") == 0)[0]
        found = [v for v in cand
                 if v < self.nl and np.any(self._get(vis, self.ccol[self.crow[v]:self.crow[v + 1]]))]
        if found:
            self._settle(np.asarray(found, np.int64) + self.lo, level)

    def end_level(self):
        self.fr[:] = self.frn
        self.frn[:] = 0
        own = self._v()[self.rank * self.bw:(self.rank + 1) * self.bw]
        own |= self.fr
        f = self._frontier(self.fr)
        deg = np.diff(self.row)[f] if len(f) else np.zeros(0, np.int64)
        return [int(len(f)), int(deg.sum()), int(np.sum(deg > 0))]

    def reach(self):
        r = self.dist < INF
        return int(r.sum()), int(np.diff(self.row)[r].sum())

    def dist_local(self):
        return self.dist.copy()


class NumpyWPart:
    """Numpy restatement of the pj_wpart_* steps (wpart.hip; semantics as in
    include/pj.h), driven by libpj's band loop (pj_engine_delta) under gloo on CPU.
    Same block geometry; send/recv are int64 (id | cand << 32), owner-major."""

    def __init__(self, src, dst, w, n, rank, world):
        src = np.asarray(src, np.int64)
        dst = np.asarray(dst, np.int64)
        w = np.asarray(w, np.int64)
        self.n, self.rank, self.world = n, rank, world
        self.block, ranges = block_geometry(n, world)
        self.lo, self.hi = ranges[rank]
        self.nl = self.hi - self.lo
        self.nnz = len(src)
        self.mean_w = float(w.sum()) / len(w) if len(w) else 1.0
        m = (src >= self.lo) & (src < self.hi)
        k = src[m] - self.lo
        order = np.argsort(k, kind="stable")
        row = np.zeros(self.nl + 1, np.int64)
        np.add.at(row, k + 1, 1)
        self.row, self.col, self.w = np.cumsum(row), dst[m][order], w[m][order]
        self.nnz_local = len(self.col)
        cap = world * self.block if world > 1 else 1
        self.send = np.zeros(cap, np.int64)
        self.recv = np.zeros(cap, np.int64)
        self.dist = np.full(self.nl, INF, np.int64)
        self.cand = np.full(n, INF, np.int64)
        self.fr = np.zeros(self.nl, bool)
        self.frn = np.zeros(self.nl, bool)
        self.mb = np.zeros(self.nl, bool)
        self.delta = 1

    def begin(self, source, delta=0):
        if delta <= 0:
            mean_deg = self.nnz / self.n if self.n else 1.0
            delta = int(max(1.0, min(65536.0, np.floor(3.5 * self.mean_w / max(1.0, mean_deg) + 0.5))))
        self.delta = delta
        self.dist[:] = INF
        self.cand[:] = INF
        if 0 <= source < self.n and self.lo <= source < self.hi:
            self.dist[source - self.lo] = 0
        return delta

    def select(self, lo, hi):
        self.fr = (self.dist >= lo) & (self.dist < hi)
        self.frn[:] = False
        self.mb[:] = False
        above = self.dist[self.dist >= lo]
        return int(self.fr.sum()), int(above.min()) if len(above) else INF

    def _lower(self, v, c, hi, light):
        """Owned target v (global) gets candidate c (atomicMin; light: joins frn below hi)."""
        i = v - self.lo
        if c < self.dist[i]:
            self.dist[i] = c
            if light and c < hi:
                self.frn[i] = True

    def relax(self, light, lo, hi):
        if light:
            self.mb |= self.fr
            us = np.nonzero(self.fr)[0]
        else:
            us = np.nonzero(self.mb)[0]
        touched = {}
        for u in us:
            a, b = self.row[u], self.row[u + 1]
            for v, wt in zip(self.col[a:b], self.w[a:b]):
                if (wt < self.delta) != bool(light):
                    continue
                c = self.dist[u] + wt
                if c >= INF:
                    continue
                if self.lo <= v < self.hi:
                    self._lower(v, c, hi, light)
                elif c < self.cand[v]:  # re-sent only when this rank improves on it
                    self.cand[v] = c
                    touched[int(v)] = True
        ids = np.array(sorted(touched), np.int64)
        owner = ids // self.block
        counts = [int(np.sum(owner == o)) for o in range(self.world)]
        if len(ids):
            packed = ids | (self.cand[ids] << 32)  # ids are sorted, hence owner-major
            self.send[: len(ids)] = packed
        return counts

    def apply(self, nr, light, lo, hi):
        rec = self.recv[:nr]
        ids, cs = rec & 0xFFFFFFFF, rec >> 32
        assert np.all((ids >= self.lo) & (ids < self.hi)), "received ids owned by another rank"
        for v, c in zip(ids, cs):
            self._lower(int(v), int(c), hi, light)

    def end_round(self):
        self.fr = self.frn.copy()
        self.frn[:] = False
        return int(self.fr.sum())

    def reach(self):
        r = self.dist < INF
        return int(r.sum()), int(np.diff(self.row)[r].sum())

    def dist_local(self):
        return self.dist.astype(np.int32)

    def close(self):
        pass
