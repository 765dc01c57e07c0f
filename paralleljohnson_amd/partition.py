"""1D vertex-partitioned BFS across GPUs, one process per GPU.

The reference distributes contiguous vertex blocks over MPI ranks (nn2rank /
get_start_nn, ParallelJohnson.cpp:169-200; row scatter :344-410) and, every
round, exchanges (vertex, distance) pairs with MPI_Alltoall + MPI_Alltoallv
(:522-554) and tests termination with MPI_Allreduce (:589-590). Here:

  * each rank holds the rows of its block on its GPU (pj_part_* in libpj);
  * a level is a top-down (push) or bottom-up (pull) step chosen with Beamer's
    rule from global frontier counts, identical on every rank;
  * push levels exchange the claimed target ids with all_to_all_single (the
    analogue of :522-554; the distance is implicit: level + 1);
  * the per-level counts are summed with all_reduce (the analogue of :589-590);
  * pull levels read a replicated visited bitmap, refreshed by an all-gather of
    the owned slices (N/8 bytes in total) before and after each pull level.

Collectives go through torch.distributed: backend "nccl" is RCCL over xGMI on
MI355X. With the gloo backend (CPU tests, or several ranks sharing one GPU for
rehearsal) device tensors are staged through host memory.

The device steps are an `ops` object (DevicePart: libpj kernels on the GPU).
There is no CPU fallback in the product path; tests substitute a numpy
restatement of the same steps to exercise the protocol on CPU.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional

import numpy as np

from . import INT_INF, PJError, _check, _lib, _ptr

_I64 = ctypes.c_int64


class PartInfo(ctypes.Structure):
    _fields_ = [("n", _I64), ("lo", _I64), ("hi", _I64), ("block", _I64), ("words_per_rank", _I64),
                ("nnz_local", _I64), ("nnz_in_local", _I64), ("rank", ctypes.c_int32),
                ("world", ctypes.c_int32), ("symmetric", ctypes.c_int32), ("off64", ctypes.c_int32)]


def block_geometry(n: int, world: int):
    """Vertex block per rank (multiple of 64) and the owned range of each rank."""
    per = (n + world - 1) // world
    block = max(64, (per + 63) // 64 * 64)
    ranges = [(min(r * block, n), min(r * block + block, n)) for r in range(world)]
    return block, ranges


class Exchange:
    """The collectives of one level (torch.distributed; `None` group = default)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.stage = dist.get_backend(group) == "gloo"

    def _dev(self, like):
        return "cpu" if self.stage else like.device

    def allreduce_sum(self, vals: List[int], like) -> List[int]:
        import torch
        t = torch.tensor(vals, dtype=torch.int64, device=self._dev(like))
        self.dist.all_reduce(t, group=self.group)
        return t.tolist()

    def allreduce_min(self, vals: List[int], like) -> List[int]:
        import torch
        t = torch.tensor(vals, dtype=torch.int64, device=self._dev(like))
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN, group=self.group)
        return t.tolist()

    def alltoall_counts(self, counts: List[int], like) -> List[int]:
        import torch
        s = torch.tensor(counts, dtype=torch.int64, device=self._dev(like))
        r = torch.empty_like(s)
        self.dist.all_to_all_single(r, s, group=self.group)
        return r.tolist()

    def alltoall_ids(self, send, send_counts: List[int], recv, recv_counts: List[int]):
        ns, nr = sum(send_counts), sum(recv_counts)
        src = send[:ns]
        dst = recv[:nr]
        if self.stage and send.device.type != "cpu":
            s_cpu = src.cpu()
            r_cpu = dst.new_empty(nr, device="cpu")
            self.dist.all_to_all_single(r_cpu, s_cpu, output_split_sizes=recv_counts,
                                        input_split_sizes=send_counts, group=self.group)
            dst.copy_(r_cpu)
        else:
            self.dist.all_to_all_single(dst, src, output_split_sizes=recv_counts,
                                        input_split_sizes=send_counts, group=self.group)

    def allgather_slices(self, out, own):
        """out (world * w words) := concatenation of every rank's `own` (w words)."""
        if self.stage and out.device.type != "cpu":
            o = out.cpu()
            self.dist.all_gather_into_tensor(o, own.cpu().clone(), group=self.group)
            out.copy_(o)
        else:
            self.dist.all_gather_into_tensor(out, own.clone(), group=self.group)


class DevicePart:
    """This rank's block on its GPU: libpj's pj_part_* kernels (the product path).

    Device buffers shared with the collectives are torch tensors; libpj is put
    on torch's current stream so kernels and RCCL calls are stream-ordered."""

    def __init__(self, ctx, handle):
        import torch
        self._ctx = ctx
        self._h = handle
        info = PartInfo()
        _check(_lib.pj_part_info_get(self._h, ctypes.byref(info)))
        self.n, self.lo, self.hi = info.n, info.lo, info.hi
        self.block, self.bw = info.block, info.words_per_rank
        self.rank, self.world = info.rank, info.world
        self.nnz_local, self.symmetric = info.nnz_local, bool(info.symmetric)
        self.nl = self.hi - self.lo
        dev = torch.device("cuda", ctx.device)
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        self.vis = torch.zeros(self.world * self.bw, dtype=torch.int64, device=dev)
        self.iso = torch.zeros_like(self.vis)
        cap = self.world * self.block if self.world > 1 else 1
        self.send = torch.empty(cap, dtype=torch.int32, device=dev)
        self.recv = torch.empty(cap, dtype=torch.int32, device=dev)
        self._counts = (_I64 * max(self.world, 1))()
        self._st = (_I64 * 3)()

    # buffers ---------------------------------------------------------------
    def own_slice(self):
        return self.vis[self.rank * self.bw:(self.rank + 1) * self.bw]

    def zmask(self):
        import torch
        z = torch.empty(self.bw, dtype=torch.int64, device=self.vis.device)
        _check(_lib.pj_part_zmask(self._h, ctypes.c_void_p(z.data_ptr())))
        return z

    @staticmethod
    def _p(t):
        return ctypes.c_void_p(t.data_ptr())

    # steps -------------------------------------------------------------------
    def begin(self, source: int):
        _check(_lib.pj_part_begin(self._h, int(source), self._p(self.iso), self._p(self.vis), self._st))
        return list(self._st)

    def push(self, level: int) -> List[int]:
        _check(_lib.pj_part_push(self._h, int(level), self._p(self.vis), self._p(self.send), self._counts))
        return list(self._counts)[: self.world]

    def apply(self, level: int, n_recv: int):
        _check(_lib.pj_part_apply(self._h, int(level), self._p(self.vis), self._p(self.recv), int(n_recv)))

    def pull(self, level: int):
        _check(_lib.pj_part_pull(self._h, int(level), self._p(self.vis)))

    def end_level(self):
        _check(_lib.pj_part_end_level(self._h, self._p(self.vis), self._st))
        return list(self._st)

    # results -----------------------------------------------------------------
    def reach(self):
        out = (_I64 * 2)()
        _check(_lib.pj_part_reach(self._h, out))
        return int(out[0]), int(out[1])

    def dist_local(self) -> np.ndarray:
        out = np.empty(max(self.nl, 1), np.int32)
        _check(_lib.pj_part_copy_dist(self._h, _ptr(out)))
        return out[: self.nl]

    def close(self):
        if self._h:
            _check(_lib.pj_part_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def load_kronecker(ctx, scale: int, edgefactor: int, seed: int, rank: int, world: int) -> DevicePart:
    h = ctypes.c_void_p()
    _check(_lib.pj_part_generate_kronecker(ctx._h, int(scale), int(edgefactor), ctypes.c_uint64(seed),
                                           int(rank), int(world), ctypes.byref(h)))
    return DevicePart(ctx, h)


def load_snap(ctx, path: str, rank: int, world: int) -> DevicePart:
    """The rank's share of a SNAP edge list (pj_part_load_snap)."""
    h = ctypes.c_void_p()
    _check(_lib.pj_part_load_snap(ctx._h, os.fsencode(path), int(rank), int(world), ctypes.byref(h)))
    return DevicePart(ctx, h)


def load_coo(ctx, src, dst, n: int, rank: int, world: int, symmetric: bool = False) -> DevicePart:
    s = np.ascontiguousarray(np.asarray(src, dtype=np.int64))
    d = np.ascontiguousarray(np.asarray(dst, dtype=np.int64))
    if len(s) != len(d):
        raise ValueError("src and dst differ in length")
    h = ctypes.c_void_p()
    _check(_lib.pj_part_load_coo(ctx._h, _ptr(s), _ptr(d), len(s), int(n), int(symmetric), int(rank),
                                 int(world), ctypes.byref(h)))
    return DevicePart(ctx, h)


class PartitionedBFS:
    """The level loop of one rank. Every rank calls solve() with the same source.

    alpha / beta: Beamer's direction-switch parameters (as the single-GPU
    solver's defaults); force: 0 auto, 1 push only, 2 pull from level 1 on."""

    def __init__(self, ops, exchange: Optional[Exchange] = None, nnz_global: Optional[int] = None,
                 alpha: float = 14.0, beta: float = 24.0, force: int = 0):
        self.ops = ops
        self.ex = exchange
        self.alpha, self.beta, self.force = alpha, beta, force
        self.world = 1 if exchange is None else exchange.world
        if self.world != ops.world:
            raise PJError(-9, f"exchange has {self.world} ranks, the partition {ops.world}")
        if nnz_global is None:
            nnz_global = self._sum([ops.nnz_local])[0]
        self.nnz_global = nnz_global
        # replicated isolated-vertex mask: one all-gather per graph
        z = ops.zmask()
        if self.ex is None:
            ops.iso.copy_(z)
        else:
            self.ex.allgather_slices(ops.iso, z)
        self.stats = {}

    def _sum(self, vals):
        return vals if self.ex is None else self.ex.allreduce_sum(vals, self.ops.vis)

    def _allgather_vis(self):
        if self.ex is not None:
            self.ex.allgather_slices(self.ops.vis, self.ops.own_slice())

    def solve(self, source: int) -> dict:
        ops = self.ops
        n_f, m_f, nz = self._sum(ops.begin(source))
        n_r, m_r = n_f, m_f
        m_u = self.nnz_global - m_f
        mode, level, td, bu, sent = 0, 0, 0, 0, 0
        if self.force == 2:
            mode = 1
            self._allgather_vis()
        while n_f > 0 and level + 1 < INT_INF:
            prev_n_f = n_f
            if mode == 0:
                counts = ops.push(level)
                if self.ex is not None:
                    rc = self.ex.alltoall_counts(counts, ops.vis)
                    self.ex.alltoall_ids(ops.send, counts, ops.recv, rc)
                    sent += sum(counts)
                    ops.apply(level, sum(rc))
                td += 1
            else:
                ops.pull(level)
                bu += 1
            n_f, m_f, nz = self._sum(ops.end_level())
            n_r += n_f
            m_r += m_f
            m_u -= m_f
            # Beamer: switch to pull when the frontier's edges exceed the unexplored
            # edges / alpha, back to push when the frontier is small and shrinking
            nxt = mode
            if self.force == 1:
                nxt = 0
            elif self.force == 2:
                nxt = 1
            elif mode == 0 and m_f > m_u / self.alpha:
                nxt = 1
            elif mode == 1 and n_f < ops.n / self.beta and n_f < prev_n_f:
                nxt = 0
            if n_f > 0 and (nxt == 1 or mode == 1):
                self._allgather_vis()
            mode = nxt
            level += 1
        self.stats = dict(levels=level, td_levels=td, bu_levels=bu, reached=n_r, reached_edges=m_r,
                          ids_sent=sent)
        return self.stats


def gather_dist(ops, exchange: Optional[Exchange]) -> np.ndarray:
    """Full distance vector on every rank (test/CLI helper; not in the timed path)."""
    import torch
    local = ops.dist_local()
    if exchange is None:
        return local
    block, ranges = block_geometry(ops.n, ops.world)
    buf = torch.full((block,), INT_INF, dtype=torch.int32)
    buf[: len(local)] = torch.from_numpy(local)
    out = torch.empty(block * ops.world, dtype=torch.int32)
    if exchange.stage:
        exchange.dist.all_gather_into_tensor(out, buf, group=exchange.group)
    else:
        dev = (ops.vis if hasattr(ops, "vis") else ops.send).device
        o = out.to(dev)
        exchange.dist.all_gather_into_tensor(o, buf.to(dev), group=exchange.group)
        out = o.cpu()
    return out.numpy()[: ops.n]


# ---- weighted SSSP over the 1D partition (delta-stepping; wpart.hip) --------

class DeviceWPart:
    """This rank's block of a weighted graph on its GPU (libpj pj_wpart_*)."""

    def __init__(self, ctx, graph, rank: int, world: int):
        import torch
        h = ctypes.c_void_p()
        _check(_lib.pj_wpart_from_graph(graph._h, int(rank), int(world), ctypes.byref(h)))
        self._ctx = ctx
        self._h = h
        info = (_I64 * 8)()
        _check(_lib.pj_wpart_info(self._h, info))
        self.n, self.lo, self.hi, self.block, self.nnz_local, self.world, self.rank, self.nnz = list(info)
        self.nl = self.hi - self.lo
        dev = torch.device("cuda", ctx.device)
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        cap = self.world * self.block if self.world > 1 else 1
        self.send = torch.empty(cap, dtype=torch.int64, device=dev)
        self.recv = torch.empty(cap, dtype=torch.int64, device=dev)
        self._counts = (_I64 * max(self.world, 1))()
        self._o2 = (_I64 * 2)()

    @staticmethod
    def _p(t):
        return ctypes.c_void_p(t.data_ptr())

    def begin(self, source: int, delta: int = 0) -> int:
        d = ctypes.c_int32()
        _check(_lib.pj_wpart_begin(self._h, int(source), int(delta), ctypes.byref(d)))
        return d.value

    def select(self, lo: int, hi: int):
        _check(_lib.pj_wpart_select(self._h, int(lo), int(hi), self._o2))
        return int(self._o2[0]), int(self._o2[1])

    def relax(self, light: bool, lo: int, hi: int) -> List[int]:
        _check(_lib.pj_wpart_relax(self._h, int(light), int(lo), int(hi), self._p(self.send), self._counts))
        return list(self._counts)[: self.world]

    def apply(self, n_recv: int, light: bool, lo: int, hi: int):
        _check(_lib.pj_wpart_apply(self._h, self._p(self.recv), int(n_recv), int(light), int(lo), int(hi)))

    def end_round(self) -> int:
        nf = _I64()
        _check(_lib.pj_wpart_end_round(self._h, ctypes.byref(nf)))
        return nf.value

    def reach(self):
        _check(_lib.pj_wpart_reach(self._h, self._o2))
        return int(self._o2[0]), int(self._o2[1])

    def dist_local(self) -> np.ndarray:
        out = np.empty(max(self.nl, 1), np.int32)
        _check(_lib.pj_wpart_copy_dist(self._h, _ptr(out)))
        return out[: self.nl]

    def close(self):
        if self._h:
            _check(_lib.pj_wpart_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PartitionedDelta:
    """The band loop of one rank (delta-stepping, Meyer & Sanders) over a 1D
    vertex partition; every rank calls solve() with the same source. The
    reference's round loop (:488-594) with its exchange (:522-554) and its
    termination all-reduce (:579-593); R9 makes the result independent of the
    partition and of the band structure."""

    def __init__(self, ops, exchange: Optional[Exchange] = None, delta: int = 0):
        self.ops = ops
        self.ex = exchange
        self.delta = delta
        self.world = 1 if exchange is None else exchange.world
        if self.world != ops.world:
            raise PJError(-9, f"exchange has {self.world} ranks, the partition {ops.world}")
        self.stats = {}

    def _sum(self, vals):
        return vals if self.ex is None else self.ex.allreduce_sum(vals, self.ops.send)

    def _min(self, vals):
        return vals if self.ex is None else self.ex.allreduce_min(vals, self.ops.send)

    def _exchange_apply(self, light, lo, hi):
        ops = self.ops
        counts = ops.relax(light, lo, hi)
        nr = 0
        if self.ex is not None:
            rc = self.ex.alltoall_counts(counts, ops.send)
            self.ex.alltoall_ids(ops.send, counts, ops.recv, rc)
            nr = sum(rc)
            self.sent += sum(counts)
        ops.apply(nr, light, lo, hi)

    def solve(self, source: int) -> dict:
        ops = self.ops
        delta = ops.begin(source, self.delta)
        lo, bands, rounds = 0, 0, 0
        self.sent = 0
        while lo < INT_INF:
            hi = min(lo + delta, INT_INF)
            cnt, mn = ops.select(lo, hi)
            cnt = self._sum([cnt])[0]
            if cnt == 0:
                mn = self._min([mn])[0]
                if mn >= INT_INF:
                    break
                lo = max(mn // delta * delta, hi)  # jump to the next occupied band
                continue
            bands += 1
            while True:  # light rounds until no rank has a frontier
                self._exchange_apply(True, lo, hi)
                rounds += 1
                if self._sum([ops.end_round()])[0] == 0:
                    break
            self._exchange_apply(False, lo, hi)  # heavy edges of the band's members
            lo = hi
        r, m = self._sum(list(ops.reach()))
        self.stats = dict(delta=delta, bands=bands, rounds=rounds, reached=r, reached_edges=m, sent=self.sent)
        return self.stats


def load_weighted(ctx, graph, rank: int, world: int) -> DeviceWPart:
    """The rank's block of a weighted pj Graph (the graph may be closed afterwards)."""
    return DeviceWPart(ctx, graph, rank, world)
