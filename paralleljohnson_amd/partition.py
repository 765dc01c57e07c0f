"""1D vertex-partitioned solves across GPUs: Python binding of
libpj's pj_comm / pj_part_* / pj_wpart_* (include/pj.h).

The reference distributes contiguous vertex blocks over MPI ranks (nn2rank /
get_start_nn, ParallelJohnson.cpp:169-200; row scatter :344-410) and, every
round, exchanges (vertex, distance) pairs with MPI_Alltoall + MPI_Alltoallv
(:522-554) and tests termination with MPI_Allreduce (:589-590). In libpj:

  * each rank holds the rows of its block on its GPU (pj_part_load_* /
    pj_wpart_from_graph: no scatter);
  * the level loop (BFS) and the band loop (delta-stepping) run in C++
    (engine.cpp), one call per rank: pj_part_bfs / pj_wpart_delta;
  * the collectives go through a pj_comm (Comm below): RCCL over xGMI (one
    process per GPU, or one process driving several GPUs), device copies
    between ranks that are threads of one process (several ranks may share a
    GPU), or caller callbacks (any transport: the CPU tests use gloo).

There is no torch and no CPU fallback on this path; the protocol loop is the
same C++ code whatever the transport. `engine_bfs` / `engine_delta` run that
loop over caller-supplied device steps (the CPU tests pass a numpy
restatement, tests/part_numpy.py).
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence

import numpy as np

from . import INT_INF, PJError, _check, _lib, _ptr  # noqa: F401

_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_INT = ctypes.c_int
_P = ctypes.c_void_p
_PP = ctypes.POINTER(ctypes.c_void_p)
_PI64 = ctypes.POINTER(ctypes.c_int64)


class PartInfo(ctypes.Structure):
    _fields_ = [("n", _I64), ("lo", _I64), ("hi", _I64), ("block", _I64), ("words_per_rank", _I64),
                ("nnz_local", _I64), ("nnz_in_local", _I64), ("rank", _I32),
                ("world", _I32), ("symmetric", _I32), ("off64", _I32), ("bytes_rows", _I64),
                ("bytes_state", _I64), ("bytes_bitmaps", _I64), ("bytes_exchange", _I64),
                ("build_us", _I64 * 10)]

BUILD_PHASES = ("enumerate_count_s", "enumerate_write_s", "sort_s", "csr_s", "alloc_s", "state_s", "total_s", "free_s",
                "slowest_alloc_s", "slowest_alloc_gb")


class PartStats(ctypes.Structure):
    _fields_ = [("solve_ms", ctypes.c_double), ("levels", _I64), ("td_levels", _I64), ("bu_levels", _I64),
                ("bands", _I64), ("rounds", _I64), ("reached", _I64), ("reached_edges", _I64), ("sent", _I64),
                ("delta", _I32), ("heavy_pulls", _I32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_CB_ALLREDUCE = ctypes.CFUNCTYPE(_INT, _P, _PI64, _INT, _INT)
_CB_A2A_COUNTS = ctypes.CFUNCTYPE(_INT, _P, _PI64, _PI64)
_CB_A2AV = ctypes.CFUNCTYPE(_INT, _P, _P, _PI64, _P, _PI64, _I64)
_CB_ALLGATHER = ctypes.CFUNCTYPE(_INT, _P, _P, _P, _I64)


class CommCallbacks(ctypes.Structure):
    _fields_ = [("user", _P), ("rank", _INT), ("world", _INT), ("allreduce", _CB_ALLREDUCE),
                ("alltoall_counts", _CB_A2A_COUNTS), ("alltoallv", _CB_A2AV), ("allgather", _CB_ALLGATHER)]


_ST_ZMASK = ctypes.CFUNCTYPE(_INT, _P)
_ST_BEGIN = ctypes.CFUNCTYPE(_INT, _P, _I64, _PI64)
_ST_PUSH = ctypes.CFUNCTYPE(_INT, _P, _INT, _PI64)
_ST_APPLY = ctypes.CFUNCTYPE(_INT, _P, _INT, _I64)
_ST_PULL = ctypes.CFUNCTYPE(_INT, _P, _INT)
_ST_END = ctypes.CFUNCTYPE(_INT, _P, _PI64)


class BfsSteps(ctypes.Structure):
    _fields_ = [("user", _P), ("n", _I64), ("nnz_local", _I64), ("words_per_rank", _I64), ("block", _I64),
                ("rank", _I32), ("world", _I32), ("vis", _P), ("iso", _P), ("zown", _P), ("send", _P), ("recv", _P),
                ("zmask", _ST_ZMASK), ("begin", _ST_BEGIN), ("push", _ST_PUSH), ("apply", _ST_APPLY),
                ("pull", _ST_PULL), ("end_level", _ST_END)]


_DS_BEGIN = ctypes.CFUNCTYPE(_INT, _P, _I64, _I32, ctypes.POINTER(_I32))
_DS_SELECT = ctypes.CFUNCTYPE(_INT, _P, _I32, _I32, _PI64)
_DS_RELAX = ctypes.CFUNCTYPE(_INT, _P, _INT, _I32, _I32, _PI64)
_DS_APPLY = ctypes.CFUNCTYPE(_INT, _P, _I64, _INT, _I32, _I32)
_DS_END = ctypes.CFUNCTYPE(_INT, _P, _PI64)
_DS_REACH = ctypes.CFUNCTYPE(_INT, _P, _PI64)


class DeltaSteps(ctypes.Structure):
    _fields_ = [("user", _P), ("n", _I64), ("rank", _I32), ("world", _I32), ("send", _P), ("recv", _P),
                ("begin", _DS_BEGIN), ("select", _DS_SELECT), ("relax", _DS_RELAX), ("apply", _DS_APPLY),
                ("end_round", _DS_END), ("reach", _DS_REACH)]


TRANSPORTS = {"auto": 0, "rccl": 1, "host": 2}


def block_geometry(n: int, world: int):
    """Vertex block per rank (multiple of 64) and the owned range of each rank."""
    per = (n + world - 1) // world
    block = max(64, (per + 63) // 64 * 64)
    ranges = [(min(r * block, n), min(r * block + block, n)) for r in range(world)]
    return block, ranges


def _host(ptr: int, nbytes: int) -> np.ndarray:
    """uint8 view of nbytes of host memory at ptr (callback transports and steps)."""
    if nbytes <= 0:
        return np.zeros(0, np.uint8)
    return np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(ptr))


# ---------------------------------------------------------------- transport ---

class Comm:
    """One rank's endpoint of a pj_comm group (the reference's MPI_COMM_WORLD)."""

    def __init__(self, handle, keep=None):
        self._h = handle
        self._keep = keep  # callback objects that must outlive the handle
        r, w, k = _INT(), _INT(), ctypes.c_char_p()
        _check(_lib.pj_comm_info(self._h, ctypes.byref(r), ctypes.byref(w), ctypes.byref(k)))
        self.rank, self.world, self.kind = r.value, w.value, k.value.decode()

    def transport_ranks(self):
        """(group size, this rank's index) as the transport itself reports them
        (pj_comm_transport_ranks: ncclCommCount / ncclCommUserRank for RCCL)."""
        c, i = _INT(), _INT()
        _check(_lib.pj_comm_transport_ranks(self._h, ctypes.byref(c), ctypes.byref(i)))
        return c.value, i.value

    @staticmethod
    def unique_id() -> bytes:
        """RCCL group id made by rank 0 and handed to every rank by the launcher."""
        buf = (ctypes.c_uint8 * 128)()
        _check(_lib.pj_comm_unique_id(buf))
        return bytes(buf)

    @classmethod
    def for_rank(cls, ctx, world: int, rank: int, uid: Optional[bytes] = None) -> "Comm":
        """This process's rank of an RCCL group (one process per GPU); world 1
        without an id is a single-rank transport with no RCCL."""
        h = ctypes.c_void_p()
        idb = None if uid is None else (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        _check(_lib.pj_comm_create_rank(ctx._h, int(world), int(rank), idb, ctypes.byref(h)))
        return cls(h)

    @classmethod
    def group(cls, ctxs: Sequence, transport: str = "auto") -> List["Comm"]:
        """world ranks in this process, rank r bound to ctxs[r] (one host thread per rank)."""
        world = len(ctxs)
        arr = (ctypes.c_void_p * world)(*[c._h.value for c in ctxs])
        out = (ctypes.c_void_p * world)()
        _check(_lib.pj_comm_create_group(arr, world, TRANSPORTS[transport], out))
        return [cls(ctypes.c_void_p(out[r])) for r in range(world)]

    @classmethod
    def from_callbacks(cls, transport, rank: int, world: int) -> "Comm":
        """A transport object with allreduce(vals, is_min), alltoall_counts(send, recv),
        alltoallv(send_ptr, scounts, recv_ptr, rcounts, elem) and
        allgather(own_ptr, all_ptr, nbytes) (int64 arrays in place, raw pointers)."""
        err = []

        def wrap(fn):
            def call(*a):
                try:
                    fn(*a)
                    return 0
                except BaseException as e:  # noqa: BLE001 - reported through the status
                    err.append(e)
                    return 1
            return call

        def allreduce(_, vals, k, is_min):
            v = np.ctypeslib.as_array(vals, shape=(k,))
            transport.allreduce(v, bool(is_min))

        def a2a(_, send, recv):
            transport.alltoall_counts(np.ctypeslib.as_array(send, shape=(world,)),
                                      np.ctypeslib.as_array(recv, shape=(world,)))

        def a2av(_, send, scounts, recv, rcounts, elem):
            transport.alltoallv(send or 0, np.ctypeslib.as_array(scounts, shape=(world,)).copy(), recv or 0,
                                np.ctypeslib.as_array(rcounts, shape=(world,)).copy(), int(elem))

        def allgather(_, own, all_, nbytes):
            transport.allgather(own or 0, all_ or 0, int(nbytes))

        cb = CommCallbacks(None, int(rank), int(world), _CB_ALLREDUCE(wrap(allreduce)),
                           _CB_A2A_COUNTS(wrap(a2a)), _CB_A2AV(wrap(a2av)), _CB_ALLGATHER(wrap(allgather)))
        h = ctypes.c_void_p()
        _check(_lib.pj_comm_create_callbacks(ctypes.byref(cb), ctypes.byref(h)))
        c = cls(h, keep=(cb, transport))
        c.errors = err
        return c

    def close(self):
        if self._h:
            _check(_lib.pj_comm_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------- partitions ---

class DevicePart:
    """This rank's block of a unit-weight graph on its GPU (pj_part_*)."""

    def __init__(self, ctx, handle):
        self._ctx = ctx
        self._h = handle
        info = PartInfo()
        _check(_lib.pj_part_info_get(self._h, ctypes.byref(info)))
        self.n, self.lo, self.hi = info.n, info.lo, info.hi
        self.block, self.bw = info.block, info.words_per_rank
        self.rank, self.world = info.rank, info.world
        self.nnz_local, self.symmetric = info.nnz_local, bool(info.symmetric)
        self.nl = self.hi - self.lo

    def device_bytes(self) -> dict:
        """pj_part_info_get's per-rank device bytes (rows, vertex state, N-bit bitmaps,
        exchange buffers sized to the largest level's traffic)."""
        info = PartInfo()
        _check(_lib.pj_part_info_get(self._h, ctypes.byref(info)))
        return {"rows": info.bytes_rows, "state": info.bytes_state, "bitmaps": info.bytes_bitmaps,
                "exchange": info.bytes_exchange}

    def build_phases(self) -> dict:
        """pj_part_info_get's build phases in seconds (BUILD_PHASES)."""
        info = PartInfo()
        _check(_lib.pj_part_info_get(self._h, ctypes.byref(info)))
        return {k: round(info.build_us[i] * (1e-3 if k.endswith("_gb") else 1e-6), 4)  # ([9] is in MB)
                for i, k in enumerate(BUILD_PHASES)}

    def set_option(self, key: str, value: float):
        _check(_lib.pj_part_set_option(self._h, key.encode(), float(value)))

    def bfs(self, comm: Comm, source: int) -> dict:
        """pj_part_bfs: every rank of comm calls it with the same source."""
        st = PartStats()
        _check(_lib.pj_part_bfs(self._h, comm._h, int(source), ctypes.byref(st)))
        return st.as_dict()

    def gather_dist(self, comm: Comm, want: bool = True) -> Optional[np.ndarray]:
        """The whole distance vector (every rank must call; the :612-614 Gatherv)."""
        out = np.empty(max(self.n, 1), np.int32) if want else None
        _check(_lib.pj_part_gather_dist(self._h, comm._h, _ptr(out)))
        return out[: self.n] if want else None

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


class DeviceWPart:
    """This rank's block of a weighted graph on its GPU (pj_wpart_*)."""

    def __init__(self, ctx, graph, rank: int, world: int, handle=None):
        h = handle
        if h is None:
            h = ctypes.c_void_p()
            _check(_lib.pj_wpart_from_graph(graph._h, int(rank), int(world), ctypes.byref(h)))
        self._ctx = ctx
        self._h = h
        info = (_I64 * 8)()
        _check(_lib.pj_wpart_info(self._h, info))
        self.n, self.lo, self.hi, self.block, self.nnz_local, self.world, self.rank, self.nnz = list(info)
        self.nl = self.hi - self.lo

    def device_bytes(self) -> dict:
        """pj_wpart_device_bytes: rows, O(block) vertex state, replicated maps, queue + exchange buffers."""
        out = np.zeros(4, np.int64)
        _check(_lib.pj_wpart_device_bytes(self._h, _ptr(out)))
        return {"rows": int(out[0]), "state": int(out[1]), "maps": int(out[2]), "exchange": int(out[3])}

    def set_option(self, key: str, value: float):
        """pj_wpart_set_option: "tail_frac", "tail_mult", "pull_factor", "light_pull",
        "tail_light_pull" or "queue_shard" (the claim queue's shard capacity, this rank).

        Every rank of a group must set the same values (the ranks take the tail switch and
        the pull decisions from all-reduced counts, and agree once per solve whether every
        rank allows each pull)."""
        _check(_lib.pj_wpart_set_option(self._h, key.encode(), float(value)))

    def delta(self, comm: Comm, source: int, delta: int = 0) -> dict:
        """pj_wpart_delta: every rank of comm calls it with the same source and delta."""
        st = PartStats()
        _check(_lib.pj_wpart_delta(self._h, comm._h, int(source), int(delta), ctypes.byref(st)))
        return st.as_dict()

    def gather_dist(self, comm: Comm, want: bool = True) -> Optional[np.ndarray]:
        out = np.empty(max(self.n, 1), np.int32) if want else None
        _check(_lib.pj_wpart_gather_dist(self._h, comm._h, _ptr(out)))
        return out[: self.n] if want else None

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


def load_weighted(ctx, graph, rank: int, world: int) -> DeviceWPart:
    """The rank's block of a weighted pj Graph (the graph may be closed afterwards)."""
    return DeviceWPart(ctx, graph, rank, world)


def load_weighted_kronecker(ctx, scale: int, edgefactor: int, seed: int, rank: int, world: int) -> DeviceWPart:
    """The rank's block of the weighted Kronecker graph, generated per block on its GPU
    (pj_wpart_generate_kronecker: no rank ever holds the whole graph)."""
    h = ctypes.c_void_p()
    _check(_lib.pj_wpart_generate_kronecker(ctx._h, int(scale), int(edgefactor), ctypes.c_uint64(seed), int(rank),
                                            int(world), ctypes.byref(h)))
    return DeviceWPart(ctx, None, rank, world, handle=h)


def load_weighted_snap(ctx, path: str, rank: int, world: int) -> DeviceWPart:
    """The rank's block of a weighted SNAP file (pj_wpart_load_snap: only the block's rows are kept)."""
    h = ctypes.c_void_p()
    _check(_lib.pj_wpart_load_snap(ctx._h, os.fsencode(path), int(rank), int(world), ctypes.byref(h)))
    return DeviceWPart(ctx, None, rank, world, handle=h)


def bfs_group(parts: Sequence[DevicePart], comms: Sequence[Comm], source: int) -> List[dict]:
    """pj_part_bfs_group: every rank of a one-process group at once (a host thread each)."""
    w = len(parts)
    st = (PartStats * w)()
    _check(_lib.pj_part_bfs_group(w, (ctypes.c_void_p * w)(*[p._h.value for p in parts]),
                                  (ctypes.c_void_p * w)(*[c._h.value for c in comms]), int(source), st))
    return [s.as_dict() for s in st]


def delta_group(parts: Sequence[DeviceWPart], comms: Sequence[Comm], source: int, delta: int = 0) -> List[dict]:
    w = len(parts)
    st = (PartStats * w)()
    _check(_lib.pj_wpart_delta_group(w, (ctypes.c_void_p * w)(*[p._h.value for p in parts]),
                                     (ctypes.c_void_p * w)(*[c._h.value for c in comms]), int(source), int(delta), st))
    return [s.as_dict() for s in st]


# ------------------------------------------- the loops over caller steps ---

def _put(ptr, vals):
    for i, v in enumerate(vals):
        ptr[i] = int(v)


def _step_call(err, fn):
    def call(*a):
        try:
            fn(*a)
            return 0
        except BaseException as e:  # noqa: BLE001 - reported through the status
            err.append(e)
            return 1
    return call


def _raise_first(err, exc):
    if err:
        raise err[0]
    raise exc


def engine_bfs(steps, comm: Comm, source: int, alpha: float = 14.0, beta: float = 24.0, force: int = 0) -> dict:
    """libpj's partitioned BFS loop (pj_engine_bfs) over caller steps: an object with
    n, nnz_local, bw, block, rank, world, numpy buffers vis / iso / zown / send /
    recv and the pj_part_* step methods zmask(), begin(source) -> [3],
    push(level) -> counts, apply(level, n_recv), pull(level), end_level() -> [3]."""
    err = []
    world = int(steps.world)

    def begin(_, s, st):
        _put(st, steps.begin(int(s)))

    def push(_, level, counts):
        _put(counts, list(steps.push(int(level)))[:world])

    def end_level(_, st):
        _put(st, steps.end_level())

    cs = BfsSteps(None, int(steps.n), int(steps.nnz_local), int(steps.bw), int(steps.block), int(steps.rank), world,
                  steps.vis.ctypes.data, steps.iso.ctypes.data, steps.zown.ctypes.data, steps.send.ctypes.data,
                  steps.recv.ctypes.data,
                  _ST_ZMASK(_step_call(err, lambda _: steps.zmask())), _ST_BEGIN(_step_call(err, begin)),
                  _ST_PUSH(_step_call(err, push)), _ST_APPLY(_step_call(err, lambda _, l, nr: steps.apply(l, nr))),
                  _ST_PULL(_step_call(err, lambda _, l: steps.pull(l))), _ST_END(_step_call(err, end_level)))
    st = PartStats()
    rc = _lib.pj_engine_bfs(ctypes.byref(cs), comm._h, int(source), float(alpha), float(beta), int(force),
                            ctypes.byref(st))
    if rc != 0:
        _raise_first(err + getattr(comm, "errors", []), PJError(rc, (_lib.pj_last_error() or b"").decode()))
    return st.as_dict()


def engine_delta(steps, comm: Comm, source: int, delta: int = 0) -> dict:
    """libpj's partitioned delta-stepping loop (pj_engine_delta) over caller steps:
    n, rank, world, numpy send / recv and the pj_wpart_* step methods begin(source,
    delta) -> delta, select(lo, hi) -> (count, min), relax(light, lo, hi) -> counts,
    apply(n_recv, light, lo, hi), end_round() -> n_f, reach() -> (n_r, m_r)."""
    err = []
    world = int(steps.world)

    def begin(_, s, d, out):
        out[0] = int(steps.begin(int(s), int(d)))

    def select(_, lo, hi, out):
        _put(out, steps.select(int(lo), int(hi)))

    def relax(_, light, lo, hi, counts):
        _put(counts, list(steps.relax(bool(light), int(lo), int(hi)))[:world])

    def end_round(_, out):
        out[0] = int(steps.end_round())

    def reach(_, out):
        _put(out, steps.reach())

    cs = DeltaSteps(None, int(steps.n), int(steps.rank), world, steps.send.ctypes.data, steps.recv.ctypes.data,
                    _DS_BEGIN(_step_call(err, begin)), _DS_SELECT(_step_call(err, select)),
                    _DS_RELAX(_step_call(err, relax)),
                    _DS_APPLY(_step_call(err, lambda _, nr, light, lo, hi: steps.apply(nr, bool(light), lo, hi))),
                    _DS_END(_step_call(err, end_round)), _DS_REACH(_step_call(err, reach)))
    st = PartStats()
    rc = _lib.pj_engine_delta(ctypes.byref(cs), comm._h, int(source), int(delta), ctypes.byref(st))
    if rc != 0:
        _raise_first(err + getattr(comm, "errors", []), PJError(rc, (_lib.pj_last_error() or b"").decode()))
    return st.as_dict()


def gather_group(parts: Sequence, comms: Sequence[Comm]) -> np.ndarray:
    """The whole distance vector of a one-process group: every rank gathers on its own
    host thread (the collective needs all of them at once); rank 0's copy is returned."""
    import threading
    out, errs = [None], []

    def run(r):
        try:
            d = parts[r].gather_dist(comms[r], want=(r == 0))
            if r == 0:
                out[0] = d
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=run, args=(r,)) for r in range(len(parts))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    return out[0]


class MultiInfo(ctypes.Structure):
    _fields_ = [("n", _I64), ("world", _I32), ("layout", _I32), ("weighted", _I32), ("transport", ctypes.c_char_p)]


PARTITIONED, REPLICATED = 0, 1
TRANSPORTS = {"auto": 0, "rccl": 1, "host": 2}


class Multi:
    """The n-GPU handle (pj_multi_*, SURVEY.md §8b `pj_create(int n_gpus, ...)`):
    P ranks in this process, one pj_ctx and host thread each, the transport
    between them, and the graph partitioned (the reference's np = P run) or
    replicated (sources sharded over the ranks)."""

    def __init__(self, n_gpus: int, transport: str = "auto"):
        h = ctypes.c_void_p()
        _check(_lib.pj_multi_create(int(n_gpus), TRANSPORTS[transport], ctypes.byref(h)))
        self._h = h

    def close(self):
        if self._h:
            _check(_lib.pj_multi_destroy(self._h))
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def info(self) -> dict:
        i = MultiInfo()
        _check(_lib.pj_multi_info(self._h, ctypes.byref(i)))
        return {"n": i.n, "world": i.world, "layout": i.layout, "weighted": bool(i.weighted),
                "transport": (i.transport or b"").decode()}

    def device_bytes(self, rank: int) -> dict:
        """pj_multi_device_bytes: rank's rows, O(block) vertex state, replicated maps, exchange."""
        out = np.zeros(4, np.int64)
        _check(_lib.pj_multi_device_bytes(self._h, int(rank), _ptr(out)))
        return {"rows": int(out[0]), "state": int(out[1]), "maps": int(out[2]), "exchange": int(out[3])}

    def set_csr_cache(self, path: Optional[str]):
        _check(_lib.pj_multi_set_csr_cache(self._h, None if path is None else os.fsencode(path)))

    def load_snap(self, path: str, weighted: bool = False, layout: int = PARTITIONED):
        _check(_lib.pj_multi_load_snap(self._h, os.fsencode(path), int(weighted), int(layout)))

    def generate_kronecker(self, scale: int, edgefactor: int = 16, seed: int = 1, weighted: bool = False,
                           layout: int = PARTITIONED):
        _check(_lib.pj_multi_generate_kronecker(self._h, int(scale), int(edgefactor), ctypes.c_uint64(seed),
                                                int(weighted), int(layout)))

    def sssp(self, source: int):
        """(distances, stats) of one solve from `source`."""
        n = self.info()["n"]
        out = np.empty(max(n, 1), np.int32)
        st = PartStats()
        _check(_lib.pj_multi_sssp(self._h, int(source), _ptr(out), ctypes.byref(st)))
        return out[:n], st.as_dict()

    def sssp_batch(self, sources: Sequence[int]) -> np.ndarray:
        n = self.info()["n"]
        src = np.ascontiguousarray(np.asarray(sources, dtype=np.int64))
        out = np.empty((len(src), max(n, 1)), np.int32)
        _check(_lib.pj_multi_sssp_batch(self._h, _ptr(src), len(src), _ptr(out)))
        return out[:, :n]

    def sssp_batch_write(self, sources: Sequence[int], paths: Sequence[str], strict: bool = True) -> float:
        """One sol_file per source; returns the device solve time (ms)."""
        src = np.ascontiguousarray(np.asarray(sources, dtype=np.int64))
        if len(paths) != len(src):
            raise ValueError("one path per source")
        arr = (ctypes.c_char_p * max(len(paths), 1))(*[os.fsencode(p) for p in paths])
        ms = ctypes.c_double()
        _check(_lib.pj_multi_sssp_batch_write(self._h, _ptr(src), len(src), ctypes.cast(arr, ctypes.c_void_p),
                                              int(strict), ctypes.byref(ms)))
        return ms.value


class TorchDistTransport:
    """The callbacks of pj_comm_create_callbacks over torch.distributed on HOST buffers (e.g.
    the gloo backend): libpj's protocol loops at world > 1 without a GPU (the CPU tests over
    numpy steps). Its buffers must be host memory, so it cannot carry libpj's own partitions
    (device buffers): bench.py's partitioned leg rejects it at world > 1."""

    def __init__(self):
        import torch.distributed as dist
        self._dist = dist
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()

    def allreduce(self, vals, is_min):
        import torch
        t = torch.from_numpy(vals.copy())
        self._dist.all_reduce(t, op=self._dist.ReduceOp.MIN if is_min else self._dist.ReduceOp.SUM)
        vals[:] = t.numpy()

    def alltoall_counts(self, send, recv):
        import torch
        s = torch.from_numpy(send.copy())
        r = torch.empty_like(s)
        self._dist.all_to_all_single(r, s)
        recv[:] = r.numpy()

    def alltoallv(self, send_ptr, scounts, recv_ptr, rcounts, elem):
        import torch
        sb, rb = (scounts * elem).tolist(), (rcounts * elem).tolist()
        src = torch.from_numpy(_host(send_ptr, sum(sb)).copy()) if sum(sb) else torch.zeros(0, dtype=torch.uint8)
        dst = torch.empty(sum(rb), dtype=torch.uint8)
        self._dist.all_to_all_single(dst, src, output_split_sizes=rb, input_split_sizes=sb)
        if sum(rb):
            _host(recv_ptr, sum(rb))[:] = dst.numpy()

    def allgather(self, own_ptr, all_ptr, nbytes):
        import torch
        own = torch.from_numpy(_host(own_ptr, nbytes).copy())
        out = torch.empty(nbytes * self.world, dtype=torch.uint8)
        self._dist.all_gather_into_tensor(out, own)
        _host(all_ptr, nbytes * self.world)[:] = out.numpy()
