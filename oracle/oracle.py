"""ORACLE — test infrastructure only.

ctypes wrapper around oracle/_build/liboracle.so, the plain-C restatement of
/root/reference/ParallelJohnson.cpp (see pj_oracle.h for the per-function
citations and for how parity is pinned). Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module; the product path
(paralleljohnson_amd) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

INT_INF = 100000  # ParallelJohnson.cpp:29

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        i64 = ctypes.c_int64
        L.pjo_parse_snap.argtypes = [P, i64, ctypes.c_int, P, P, P, i64, P, P, P]
        L.pjo_parse_snap.restype = ctypes.c_int
        L.pjo_coo2csr.argtypes = [P, P, P, i64, i64, P, P, P]
        L.pjo_coo2csr.restype = None
        L.pjo_bfs.argtypes = [P, P, i64, i64, P]
        L.pjo_bfs.restype = None
        L.pjo_bfs_batch.argtypes = [P, P, i64, P, i64, ctypes.c_int, P]
        L.pjo_bfs_batch.restype = None
        L.pjo_dijkstra.argtypes = [P, P, P, i64, i64, P]
        L.pjo_dijkstra.restype = None
        L.pjo_reference_sssp.argtypes = [P, P, P, i64, i64, ctypes.c_int, P, P]
        L.pjo_reference_sssp.restype = ctypes.c_int
        L.pjo_reference_sssp_budget.argtypes = [P, P, P, i64, i64, ctypes.c_int, ctypes.c_double, P, P]
        L.pjo_reference_sssp_budget.restype = ctypes.c_int
        L.pjo_format_sol.argtypes = [P, i64, P]
        L.pjo_format_sol.restype = i64
        L.pjo_kronecker.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int, P, P, P]
        L.pjo_kronecker.restype = None
        L.pjo_kronecker_row_digest.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                               P, P]
        L.pjo_kronecker_row_digest.restype = None
        L.pjo_csr_row_digest.argtypes = [P, P, P, i64, ctypes.c_int, P, P]
        L.pjo_csr_row_digest.restype = i64
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class ParseError(ValueError):
    def __init__(self, line):
        super().__init__(f"edge list line {line}: not a well-defined edge for the reference")
        self.line = line


def parse_snap(text: bytes, weighted: bool = False):
    """read_webgraph :66-105 -> (src u32, dst u32, w u32|None, N)."""
    L = lib()
    buf = np.frombuffer(text, dtype=np.uint8) if len(text) else np.zeros(1, np.uint8)
    nnz = ctypes.c_int64()
    mx = ctypes.c_int64()
    bad = ctypes.c_int64()
    rc = L.pjo_parse_snap(_p(buf), len(text), int(weighted), None, None, None, 0,
                          ctypes.byref(nnz), ctypes.byref(mx), ctypes.byref(bad))
    if rc != 0:
        raise ParseError(bad.value)
    m = nnz.value
    src = np.zeros(max(m, 1), np.uint32)
    dst = np.zeros(max(m, 1), np.uint32)
    w = np.zeros(max(m, 1), np.uint32) if weighted else None
    rc = L.pjo_parse_snap(_p(buf), len(text), int(weighted), _p(src), _p(dst), _p(w), m,
                          ctypes.byref(nnz), ctypes.byref(mx), ctypes.byref(bad))
    if rc != 0:
        raise ParseError(bad.value)
    return src[:m], dst[:m], (w[:m] if w is not None else None), mx.value + 1


def coo2csr(src, dst, n, w=None):
    """coord2csr :117-159 -> (row_ptr int64[n+1], col u32[nnz], w u32|None)."""
    src = np.ascontiguousarray(src, np.uint32)
    dst = np.ascontiguousarray(dst, np.uint32)
    m = len(src)
    row = np.zeros(n + 1, np.int64)
    col = np.zeros(max(m, 1), np.uint32)
    wo = None
    if w is not None:
        w = np.ascontiguousarray(w, np.uint32)
        wo = np.zeros(max(m, 1), np.uint32)
    lib().pjo_coo2csr(_p(src), _p(dst), _p(w), m, n, _p(row), _p(col), _p(wo))
    return row, col[:m], (wo[:m] if wo is not None else None)


def bfs(row, col, source):
    n = len(row) - 1
    dist = np.zeros(max(n, 1), np.int32)
    lib().pjo_bfs(_p(row), _p(np.ascontiguousarray(col, np.uint32)), n, int(source), _p(dist))
    return dist[:n]


def bfs_batch(row, col, sources, threads=8):
    """pjo_bfs for every source (rows of a k x n int32 matrix), on host threads."""
    n = len(row) - 1
    src = np.ascontiguousarray(np.asarray(sources, dtype=np.int64))
    out = np.zeros((max(len(src), 1), max(n, 1)), np.int32)
    lib().pjo_bfs_batch(_p(row), _p(np.ascontiguousarray(col, np.uint32)), n, _p(src), len(src), int(threads),
                        _p(out))
    return out[: len(src), :n]


def dijkstra(row, col, w, source):
    n = len(row) - 1
    dist = np.zeros(max(n, 1), np.int32)
    lib().pjo_dijkstra(_p(row), _p(np.ascontiguousarray(col, np.uint32)),
                       _p(np.ascontiguousarray(w, np.uint32)), n, int(source), _p(dist))
    return dist[:n]


class RefStats(ctypes.Structure):
    _fields_ = [("solve_s", ctypes.c_double), ("rounds", ctypes.c_int64), ("pops", ctypes.c_int64),
                ("scans", ctypes.c_int64), ("decreases", ctypes.c_int64),
                ("reinserts", ctypes.c_int64), ("messages", ctypes.c_int64), ("truncated", ctypes.c_int64)]


def reference_sssp(row, col, source, nproc=1, w=None, budget_s=0.0):
    """The reference's BSP heap algorithm (:466-594) on nproc host threads.
    budget_s > 0 stops it at the first round boundary after that much solve time
    (st.truncated = 1, dist incomplete): the bounded CPU-baseline sample."""
    n = len(row) - 1
    dist = np.zeros(max(n, 1), np.int32)
    st = RefStats()
    wa = None if w is None else np.ascontiguousarray(w, np.uint32)
    rc = lib().pjo_reference_sssp_budget(_p(row), _p(np.ascontiguousarray(col, np.uint32)), _p(wa), n,
                                         int(source), int(nproc), ctypes.c_double(budget_s), _p(dist),
                                         ctypes.byref(st))
    if rc != 0:
        raise ValueError("nproc out of range")
    return dist[:n], st


def format_sol(dist) -> bytes:
    """output_vector :32-46."""
    d = np.ascontiguousarray(dist, np.int32)
    n = len(d)
    ln = lib().pjo_format_sol(_p(d), n, None)
    buf = np.zeros(ln, np.uint8)
    lib().pjo_format_sol(_p(d), n, _p(buf))
    return buf.tobytes()


def kronecker(scale, edgefactor, seed, weighted=False):
    m = 2 * (edgefactor << scale)
    src = np.zeros(m, np.uint32)
    dst = np.zeros(m, np.uint32)
    w = np.zeros(m, np.uint32)
    lib().pjo_kronecker(scale, edgefactor, seed, int(weighted), _p(src), _p(dst), _p(w))
    return src, dst, (w if weighted else None)


def kronecker_row_digest(scale, edgefactor, seed, weighted=False, threads=8):
    """Per-vertex (entries, order-free hash sum of (col, w)) of the Kronecker spec, both
    directions, without building the COO or CSR (full-size cross-check of a GPU build)."""
    n = 1 << scale
    deg = np.zeros(n, np.uint32)
    hs = np.zeros(n, np.uint64)
    lib().pjo_kronecker_row_digest(scale, edgefactor, seed, int(weighted), int(threads), _p(deg), _p(hs))
    return deg, hs


def csr_row_digest(row, col, w=None, threads=8):
    """The same digest of a CSR, plus the count of rows entries out of weight order."""
    row = np.ascontiguousarray(row, np.int64)
    n = len(row) - 1
    deg = np.zeros(max(n, 1), np.uint32)
    hs = np.zeros(max(n, 1), np.uint64)
    col = np.ascontiguousarray(np.asarray(col).view(np.uint32))
    wv = None if w is None else np.ascontiguousarray(w, np.uint32)
    bad = lib().pjo_csr_row_digest(_p(row), _p(col), _p(wv), n, int(threads), _p(deg), _p(hs))
    return deg[:n], hs[:n], int(bad)
