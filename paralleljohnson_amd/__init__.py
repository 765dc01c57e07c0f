"""paralleljohnson_amd — MI355X-native shortest-path relaxation.

Python binding (ctypes) of libpj, the C-ABI in include/pj.h. The compute path
is the HIP library paralleljohnson_amd/lib/libpj.so; this module only moves
arguments across the ABI. There is no CPU fallback: importing fails loudly if
the library is missing, and every call raises PJError when libpj reports an
error (e.g. no gfx950 device).

The reference's only interface is its CLI (`parallel_johnson webfile
source_node sol_file`, ParallelJohnson.cpp:286-303); the same CLI is built as
paralleljohnson_amd/bin/parallel_johnson (see cli_path()).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np

INT_INF = 100000  # ParallelJohnson.cpp:29

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PJ_LIB_OVERRIDE") or os.path.join(_HERE, "lib", "libpj.so")
CLI_PATH = os.path.join(_HERE, "bin", "parallel_johnson")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
        "(make -C paralleljohnson_amd/csrc)")

# PyTorch-ROCm bundles its own libamdhip64 (same SONAME as /opt/rocm's). Load it
# first when it is installed, so that libpj binds to the same HIP runtime and
# torch streams / RCCL collectives and libpj kernels share one device context
# (two runtimes in one process make the second one report "no GPUs").
try:
    import torch  # noqa: F401
except ImportError:  # the C-ABI path does not need torch
    pass

_lib = ctypes.CDLL(LIB_PATH)

PJ_OK = 0
_STATUS = {
    -1: "PJ_ERR_ARG", -2: "PJ_ERR_IO", -3: "PJ_ERR_PARSE", -4: "PJ_ERR_HIP", -5: "PJ_ERR_OOM",
    -6: "PJ_ERR_RANGE", -7: "PJ_ERR_NODEVICE", -8: "PJ_ERR_STATE", -9: "PJ_ERR_COMM",
}


class PJError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{_STATUS.get(code, code)}: {msg}")
        self.code = code
        self.name = _STATUS.get(code, str(code))


class Stats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_double), ("wall_ms", ctypes.c_double), ("levels", ctypes.c_int64),
                ("td_levels", ctypes.c_int64), ("bu_levels", ctypes.c_int64), ("reached", ctypes.c_int64),
                ("reached_edges", ctypes.c_int64), ("relax_rounds", ctypes.c_int64),
                ("scanned_edges", ctypes.c_int64), ("probes", ctypes.c_int64), ("work_bytes", ctypes.c_int64),
                ("work_by_kernel", (ctypes.c_int64 * 3) * 4)]
    # rows of work_by_kernel (pj.h): (records, probes, bytes) per kernel class
    WORK_KERNELS = ("light_round", "light_hub", "heavy_pull", "heavy_push")

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k != "work_by_kernel"}
        d["work_by_kernel"] = {name: [int(x) for x in self.work_by_kernel[i]]
                               for i, name in enumerate(self.WORK_KERNELS)}
        return d


class TreeReport(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int64) for k in ("reached", "bad_root", "bad_reach", "bad_tree_edge", "bad_edge",
                                              "bad_cycle")]


class LoadStats(ctypes.Structure):
    _fields_ = [("read_ms", ctypes.c_double), ("h2d_ms", ctypes.c_double), ("parse_ms", ctypes.c_double),
                ("csr_ms", ctypes.c_double), ("text_bytes", ctypes.c_int64)]


_P = ctypes.c_void_p
_PP = ctypes.POINTER(ctypes.c_void_p)
_I64 = ctypes.c_int64
_INT = ctypes.c_int

_SIGS = {
    "pj_create": ([_INT, _PP], _INT),
    "pj_destroy": ([_P], _INT),
    "pj_stream": ([_P], _P),
    "pj_last_error": ([], ctypes.c_char_p),
    "pj_version": ([], ctypes.c_char_p),
    "pj_build_id": ([], ctypes.c_char_p),
    "pj_trim_device_cache": ([_P], _INT),
    "pj_load_snap": ([_P, ctypes.c_char_p, _INT, _PP], _INT),
    "pj_load_snap_buffer": ([_P, ctypes.c_char_p, _I64, _INT, _PP], _INT),
    "pj_load_coo": ([_P, _P, _P, _P, _I64, _I64, _PP], _INT),
    "pj_generate_kronecker": ([_P, _INT, _INT, ctypes.c_uint64, _INT, _PP], _INT),
    "pj_generate_webgraph": ([_P, _I64, _I64, ctypes.c_uint64, _PP], _INT),
    "pj_kronecker_write_snap": ([_P, _INT, _INT, ctypes.c_uint64, _INT, ctypes.c_char_p], _INT),
    "pj_graph_save": ([_P, ctypes.c_char_p, _I64, _I64], _INT),
    "pj_load_csr_file": ([_P, ctypes.c_char_p, _I64, _I64, _PP], _INT),
    "pj_load_snap_cached": ([_P, ctypes.c_char_p, _INT, ctypes.c_char_p, _INT, _PP], _INT),
    "pj_graph_destroy": ([_P], _INT),
    "pj_graph_load_stats": ([_P, _P], _INT),
    "pj_graph_info": ([_P, _P, _P, _P, _P], _INT),
    "pj_graph_get_csr": ([_P, _P, _P, _P], _INT),
    "pj_graph_out_degree": ([_P, _I64, _P], _INT),
    "pj_sample_roots": ([_P, ctypes.c_uint64, _INT, _P, _P], _INT),
    "pj_sssp": ([_P, _I64, _P], _INT),
    "pj_copy_dist": ([_P, _P], _INT),
    "pj_dist_device": ([_P], _P),
    "pj_host_pin": ([_P, ctypes.c_size_t], _INT),
    "pj_host_unpin": ([_P], _INT),
    "pj_sssp_batch": ([_P, _P, _INT, _P], _INT),
    "pj_sssp_batch_write": ([_P, _P, _INT, _P, _INT], _INT),
    "pj_device_count": ([_P], _INT),
    "pj_last_stats": ([_P, _P], _INT),
    "pj_reach_stats": ([_P, _P], _INT),
    "pj_set_option": ([_P, ctypes.c_char_p, ctypes.c_double], _INT),
    "pj_write_sol": ([_P, _I64, ctypes.c_char_p, _INT], _INT),
    "pj_format_sol": ([_P, _I64, _P, _I64, _P], _INT),
    "pj_set_stream": ([_P, _P], _INT),
    "pj_parent_tree": ([_P, _P], _INT),
    "pj_validate_tree": ([_P, _I64, _P, _P], _INT),
    "pj_write_parents": ([_P, _I64, ctypes.c_char_p], _INT),
    "pj_part_generate_kronecker": ([_P, _INT, _INT, ctypes.c_uint64, _INT, _INT, _PP], _INT),
    "pj_part_load_coo": ([_P, _P, _P, _I64, _I64, _INT, _INT, _INT, _PP], _INT),
    "pj_part_load_snap": ([_P, ctypes.c_char_p, _INT, _INT, _PP], _INT),
    "pj_part_destroy": ([_P], _INT),
    "pj_part_info_get": ([_P, _P], _INT),
    "pj_part_zmask": ([_P, _P], _INT),
    "pj_part_begin": ([_P, _I64, _P, _P, _P], _INT),
    "pj_part_push": ([_P, _INT, _P, _P, _P], _INT),
    "pj_part_apply": ([_P, _INT, _P, _P, _I64], _INT),
    "pj_part_pull": ([_P, _INT, _P], _INT),
    "pj_part_end_level": ([_P, _P, _P], _INT),
    "pj_part_reach": ([_P, _P], _INT),
    "pj_part_copy_dist": ([_P, _P], _INT),
    "pj_part_dist_device": ([_P], _P),
    "pj_wpart_from_graph": ([_P, _INT, _INT, _PP], _INT),
    "pj_wpart_load_snap": ([_P, ctypes.c_char_p, _INT, _INT, _PP], _INT),
    "pj_wpart_destroy": ([_P], _INT),
    "pj_wpart_info": ([_P, _P], _INT),
    "pj_wpart_device_bytes": ([_P, _P], _INT),
    "pj_wpart_generate_kronecker": ([_P, _INT, _INT, ctypes.c_uint64, _INT, _INT, _PP], _INT),
    "pj_wpart_begin": ([_P, _I64, ctypes.c_int32, _P], _INT),
    "pj_wpart_select": ([_P, ctypes.c_int32, ctypes.c_int32, _P], _INT),
    "pj_wpart_relax": ([_P, _INT, ctypes.c_int32, ctypes.c_int32, _P, _P], _INT),
    "pj_wpart_apply": ([_P, _P, _I64, _INT, ctypes.c_int32, ctypes.c_int32], _INT),
    "pj_wpart_pack": ([_P, _P], _INT),
    "pj_part_load_snap_group": ([_INT, _P, ctypes.c_char_p, _P], _INT),
    "pj_wpart_load_snap_group": ([_INT, _P, ctypes.c_char_p, _P], _INT),
    "pj_wpart_end_round": ([_P, _P], _INT),
    "pj_wpart_reach": ([_P, _P], _INT),
    "pj_wpart_copy_dist": ([_P, _P], _INT),
    # transport and partitioned solves (partition.py wraps them)
    "pj_comm_unique_id": ([_P], _INT),
    "pj_comm_create_rank": ([_P, _INT, _INT, _P, _PP], _INT),
    "pj_comm_create_group": ([_P, _INT, _INT, _P], _INT),
    "pj_comm_create_callbacks": ([_P, _PP], _INT),
    "pj_comm_info": ([_P, _P, _P, _P], _INT),
    "pj_comm_transport_ranks": ([_P, _P, _P], _INT),
    "pj_comm_destroy": ([_P], _INT),
    "pj_part_bfs": ([_P, _P, _I64, _P], _INT),
    "pj_part_set_option": ([_P, ctypes.c_char_p, ctypes.c_double], _INT),
    "pj_part_bfs_group": ([_INT, _P, _P, _I64, _P], _INT),
    "pj_part_gather_dist": ([_P, _P, _P], _INT),
    "pj_wpart_delta": ([_P, _P, _I64, ctypes.c_int32, _P], _INT),
    "pj_wpart_set_option": ([_P, ctypes.c_char_p, ctypes.c_double], _INT),
    "pj_wpart_delta_group": ([_INT, _P, _P, _I64, ctypes.c_int32, _P], _INT),
    "pj_wpart_gather_dist": ([_P, _P, _P], _INT),
    "pj_engine_bfs": ([_P, _P, _I64, ctypes.c_double, ctypes.c_double, _INT, _P], _INT),
    "pj_engine_delta": ([_P, _P, _I64, ctypes.c_int32, _P], _INT),
    # the n-GPU handle (partition.Multi wraps it)
    "pj_multi_create": ([_INT, _INT, _PP], _INT),
    "pj_multi_destroy": ([_P], _INT),
    "pj_multi_ctx": ([_P, _INT, _PP], _INT),
    "pj_multi_set_csr_cache": ([_P, ctypes.c_char_p], _INT),
    "pj_multi_load_snap": ([_P, ctypes.c_char_p, _INT, _INT], _INT),
    "pj_multi_generate_kronecker": ([_P, _INT, _INT, ctypes.c_uint64, _INT, _INT], _INT),
    "pj_multi_info": ([_P, _P], _INT),
    "pj_multi_device_bytes": ([_P, _INT, _P], _INT),
    "pj_multi_sssp": ([_P, _I64, _P, _P], _INT),
    "pj_multi_sssp_batch": ([_P, _P, _INT, _P], _INT),
    "pj_multi_sssp_batch_write": ([_P, _P, _INT, _P, _INT, _P], _INT),
}
for _name, (_args, _res) in _SIGS.items():
    _fn = getattr(_lib, _name)
    _fn.argtypes = _args
    _fn.restype = _res

EXPORTS = tuple(_SIGS)


def _check(rc: int):
    if rc != PJ_OK:
        raise PJError(rc, (_lib.pj_last_error() or b"").decode(errors="replace"))


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def version() -> str:
    return _lib.pj_version().decode()


def build_id() -> str:
    """Digest of libpj's sources and compile flags (pj_build_id): measurements kept under
    profiles/ carry it, so a reader can tell whether they were taken on the loaded build."""
    return _lib.pj_build_id().decode()


def trim_device_cache() -> int:
    """Return libpj's cached free device blocks (>= 1 GiB each) to the driver; bytes
    released (pj_trim_device_cache)."""
    r = ctypes.c_int64(0)
    _check(_lib.pj_trim_device_cache(ctypes.byref(r)))
    return int(r.value)


def cli_path() -> str:
    return CLI_PATH


class Graph:
    """A graph resident on one GPU (CSR, plus CSC for pull levels)."""

    def __init__(self, ctx: "Context", handle: ctypes.c_void_p):
        self._ctx = ctx
        self._h = handle
        n, m, w, s = _I64(), _I64(), _INT(), _INT()
        _check(_lib.pj_graph_info(self._h, ctypes.byref(n), ctypes.byref(m), ctypes.byref(w), ctypes.byref(s)))
        self.n, self.nnz, self.weighted, self.symmetric = n.value, m.value, bool(w.value), bool(s.value)

    def close(self):
        if self._h:
            _check(_lib.pj_graph_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- relaxation ------------------------------------------------------
    def sssp(self, source: int, copy: bool = True) -> Optional[np.ndarray]:
        """Distances from `source` (int32, INT_INF = unreachable)."""
        out = np.empty(max(self.n, 1), np.int32) if copy else None
        _check(_lib.pj_sssp(self._h, int(source), _ptr(out)))
        return out[: self.n] if copy else None

    def copy_dist(self, out: Optional[np.ndarray] = None) -> np.ndarray:
        """The last result into `out` (int32, >= n entries, e.g. pinned with host_pin) or a new array."""
        if out is None:
            out = np.empty(max(self.n, 1), np.int32)
        elif out.dtype != np.int32 or out.size < self.n or not out.flags.c_contiguous:
            raise ValueError("copy_dist: out must be a contiguous int32 array of >= n entries")
        _check(_lib.pj_copy_dist(self._h, _ptr(out)))
        return out[: self.n]

    def dist_device_ptr(self) -> int:
        return _lib.pj_dist_device(self._h) or 0

    def sssp_batch(self, sources: Sequence[int], copy: bool = True) -> Optional[np.ndarray]:
        """Rows of the all-pairs distance matrix for `sources` (n_src x n int32)."""
        src = np.ascontiguousarray(np.asarray(sources, dtype=np.int64))
        out = np.empty((len(src), max(self.n, 1)), np.int32) if copy else None
        _check(_lib.pj_sssp_batch(self._h, _ptr(src), len(src), _ptr(out)))
        return out[:, : self.n] if copy else None

    def sssp_batch_write(self, sources: Sequence[int], paths: Sequence[str], strict: bool = True):
        """Row i of the batch written as the sol_file paths[i] (pj_sssp_batch_write)."""
        src = np.ascontiguousarray(np.asarray(sources, dtype=np.int64))
        if len(paths) != len(src):
            raise ValueError("one path per source")
        arr = (ctypes.c_char_p * max(len(paths), 1))(*[os.fsencode(p) for p in paths])
        _check(_lib.pj_sssp_batch_write(self._h, _ptr(src), len(src), ctypes.cast(arr, ctypes.c_void_p),
                                        int(strict)))

    def load_stats(self) -> dict:
        """Ingestion phase times of this graph (pj_graph_load_stats)."""
        st = LoadStats()
        _check(_lib.pj_graph_load_stats(self._h, ctypes.byref(st)))
        return {k: getattr(st, k) for k, _ in st._fields_}

    def stats(self) -> dict:
        st = Stats()
        _check(_lib.pj_last_stats(self._h, ctypes.byref(st)))
        return st.as_dict()

    def stats_into(self, st: "Stats") -> "Stats":
        """The last solve's statistics into a caller's Stats (no dict built: timed loops)."""
        _check(_lib.pj_last_stats(self._h, ctypes.byref(st)))
        return st

    def reach_stats(self) -> dict:
        st = Stats()
        _check(_lib.pj_reach_stats(self._h, ctypes.byref(st)))
        return st.as_dict()

    def set_option(self, key: str, value: float):
        _check(_lib.pj_set_option(self._h, key.encode(), float(value)))

    # -- shortest-path tree (pj_parent_tree / pj_validate_tree) --------------
    def parent_tree(self) -> np.ndarray:
        """Parents of the last single-source solve (int64, -1 = unreached)."""
        out = np.empty(max(self.n, 1), np.int64)
        _check(_lib.pj_parent_tree(self._h, _ptr(out)))
        return out[: self.n]

    def validate_tree(self, source: int, parent: np.ndarray) -> dict:
        """Graph500-style checks of `parent` against the last solve from `source` (all bad_* 0 = valid)."""
        p = np.ascontiguousarray(parent, dtype=np.int64)
        if len(p) != self.n:
            raise ValueError("one parent per vertex")
        rep = TreeReport()
        _check(_lib.pj_validate_tree(self._h, int(source), _ptr(p), ctypes.byref(rep)))
        return {k: getattr(rep, k) for k, _ in rep._fields_}

    # -- inspection --------------------------------------------------------
    def save(self, path: str, src_size: int = -1, src_mtime_ns: int = -1):
        """Binary CSR cache of this graph (pj_graph_save)."""
        _check(_lib.pj_graph_save(self._h, os.fsencode(path), int(src_size), int(src_mtime_ns)))

    def get_csr(self):
        row = np.empty(self.n + 1, np.int64)
        col = np.empty(max(self.nnz, 1), np.int32)
        w = np.empty(max(self.nnz, 1), np.uint32) if self.weighted else None
        _check(_lib.pj_graph_get_csr(self._h, _ptr(row), _ptr(col), _ptr(w)))
        return row, col[: self.nnz], (w[: self.nnz] if w is not None else None)

    def out_degree(self, v: int) -> int:
        d = _I64()
        _check(_lib.pj_graph_out_degree(self._h, int(v), ctypes.byref(d)))
        return d.value

    def sample_roots(self, seed: int, n: int) -> np.ndarray:
        out = np.empty(max(n, 1), np.int64)
        found = _INT()
        _check(_lib.pj_sample_roots(self._h, ctypes.c_uint64(seed), int(n), _ptr(out), ctypes.byref(found)))
        return out[: found.value]


class Context:
    """One GPU (pj_ctx). Not thread-safe; one thread per context."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        _check(_lib.pj_create(int(device), ctypes.byref(h)))
        self._h = h
        self.device = device

    def close(self):
        if self._h:
            _check(_lib.pj_destroy(self._h))
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def stream(self) -> int:
        return _lib.pj_stream(self._h) or 0

    def set_stream(self, stream: Optional[int]):
        """Launch later work on an external hipStream_t (e.g. torch's current stream); None = own."""
        _check(_lib.pj_set_stream(self._h, ctypes.c_void_p(stream) if stream else None))

    def load_snap(self, path: str, weighted: bool = False) -> Graph:
        g = ctypes.c_void_p()
        _check(_lib.pj_load_snap(self._h, os.fsencode(path), int(weighted), ctypes.byref(g)))
        return Graph(self, g)

    def load_snap_buffer(self, text: bytes, weighted: bool = False) -> Graph:
        g = ctypes.c_void_p()
        _check(_lib.pj_load_snap_buffer(self._h, text, len(text), int(weighted), ctypes.byref(g)))
        return Graph(self, g)

    def load_coo(self, src, dst, w=None, n: int = -1) -> Graph:
        s = np.ascontiguousarray(np.asarray(src, dtype=np.int64))
        d = np.ascontiguousarray(np.asarray(dst, dtype=np.int64))
        if len(s) != len(d):
            raise ValueError("src and dst differ in length")
        wa = None if w is None else np.ascontiguousarray(np.asarray(w, dtype=np.uint32))
        g = ctypes.c_void_p()
        _check(_lib.pj_load_coo(self._h, _ptr(s), _ptr(d), _ptr(wa), len(s), int(n), ctypes.byref(g)))
        return Graph(self, g)

    def load_snap_cached(self, path: str, cache_path: Optional[str], weighted: bool = False,
                         write_back: bool = True) -> Graph:
        """pj_load_snap through the CSR cache file cache_path (pj_load_snap_cached)."""
        h = ctypes.c_void_p()
        _check(_lib.pj_load_snap_cached(self._h, os.fsencode(path), int(weighted),
                                        None if cache_path is None else os.fsencode(cache_path), int(write_back),
                                        ctypes.byref(h)))
        return Graph(self, h)

    def load_csr_file(self, path: str, expect_src_size: int = -1, expect_src_mtime_ns: int = -1) -> "Graph":
        """A graph saved by Graph.save (pj_load_csr_file): no parse, no sort."""
        g = ctypes.c_void_p()
        _check(_lib.pj_load_csr_file(self._h, os.fsencode(path), int(expect_src_size), int(expect_src_mtime_ns),
                                     ctypes.byref(g)))
        return Graph(self, g)

    def generate_webgraph(self, n_ids: int = 916428, n_edges: int = 5105039, seed: int = 1) -> Graph:
        """web-Google-shaped synthetic graph."""
        g = ctypes.c_void_p()
        _check(_lib.pj_generate_webgraph(self._h, int(n_ids), int(n_edges), ctypes.c_uint64(seed), ctypes.byref(g)))
        return Graph(self, g)

    def kronecker_write_snap(self, path: str, scale: int, edgefactor: int = 16, seed: int = 1,
                             weighted: bool = False):
        """The Kronecker tuples as a SNAP text file in generation order (ingestion benchmarks)."""
        _check(_lib.pj_kronecker_write_snap(self._h, int(scale), int(edgefactor), ctypes.c_uint64(seed),
                                            int(weighted), os.fsencode(path)))

    def generate_kronecker(self, scale: int, edgefactor: int = 16, seed: int = 1, weighted: bool = False) -> Graph:
        g = ctypes.c_void_p()
        _check(_lib.pj_generate_kronecker(self._h, int(scale), int(edgefactor), ctypes.c_uint64(seed),
                                          int(weighted), ctypes.byref(g)))
        return Graph(self, g)


def format_sol(dist) -> bytes:
    """output_vector (:32-46) as bytes."""
    d = np.ascontiguousarray(np.asarray(dist, dtype=np.int32))
    ln = _I64()
    _check(_lib.pj_format_sol(_ptr(d), len(d), None, 0, ctypes.byref(ln)))
    buf = np.empty(max(ln.value, 1), np.uint8)
    _check(_lib.pj_format_sol(_ptr(d), len(d), _ptr(buf), ln.value, ctypes.byref(ln)))
    return buf[: ln.value].tobytes()


def write_sol(dist, path: str, strict: bool = False):
    d = np.ascontiguousarray(np.asarray(dist, dtype=np.int32))
    _check(_lib.pj_write_sol(_ptr(d), len(d), os.fsencode(path), int(strict)))


def write_parents(parent, path: str):
    p = np.ascontiguousarray(parent, dtype=np.int64)
    _check(_lib.pj_write_parents(_ptr(p), len(p), os.fsencode(path)))


class Pinned:
    """A host array page-locked by host_pin. Holds the array, so its pages cannot be freed
    (and the address reused by another array) while the registration stands. The module's
    registry keeps the handle too (so that host_unpin(array) finds it), so dropping the
    handle does NOT unpin: close(), the end of a `with` block or host_unpin(array) does."""

    def __init__(self, a: np.ndarray):
        self.array = a
        self.addr = a.ctypes.data
        _check(_lib.pj_host_pin(self.addr, a.nbytes))
        _PINNED[self.addr] = self

    def close(self):
        if self.array is not None:
            _PINNED.pop(self.addr, None)
            self.array = None
            _check(_lib.pj_host_unpin(self.addr))

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            if self.array is not None and _lib is not None:
                _lib.pj_host_unpin(self.addr)
        except Exception:  # noqa: BLE001 (interpreter shutdown)
            pass


_PINNED = {}  # address -> Pinned (keeps the handle and its array alive until close / host_unpin)


def host_pin(a: np.ndarray) -> Pinned:
    """Page-lock a (contiguous) host array for direct device -> host copies (pj_host_pin).
    Returns a Pinned handle (also a context manager); host_unpin(a) or handle.close() undoes it."""
    if not a.flags.c_contiguous or a.nbytes == 0:
        raise ValueError("host_pin: a contiguous, non-empty array")
    if a.ctypes.data in _PINNED:
        raise ValueError("host_pin: this address is already pinned")
    return Pinned(a)


def host_unpin(a: np.ndarray):
    h = _PINNED.get(a.ctypes.data)
    if h is None:
        raise ValueError("host_unpin: not pinned through host_pin")
    h.close()


def device_count() -> int:
    """Number of visible HIP devices (pj_device_count)."""
    n = _INT()
    _check(_lib.pj_device_count(ctypes.byref(n)))
    return n.value
