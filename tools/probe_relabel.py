"""Does a degree-ordered relabel help the MS-BFS (configs[4]) and the unit BFS (configs[1])?
Loads each graph twice through pj_load_coo -- input ids, and relabeled on the host by out-degree
descending (ties by id) -- and times the same work on both, interleaved; the relabeled results are
mapped back and compared. The un-permute itself is not timed here (the level kernels' gain first).
Usage: python tools/probe_relabel.py [ms|k22|both]"""
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import numpy as np  # noqa: E402

import paralleljohnson_amd as pj  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "both"
ctx = pj.Context(0)


def relabeled(g):
    row, col, _ = g.get_csr()
    n = len(row) - 1
    deg = np.diff(row)
    perm = np.lexsort((np.arange(n), -deg.astype(np.int64)))  # new id i holds input id perm[i]
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n)
    src = np.repeat(np.arange(n, dtype=np.int64), deg)
    dst = col.astype(np.int64)
    a = ctx.load_coo(src, dst, n=n)
    b = ctx.load_coo(inv[src], inv[dst], n=n)
    return row, a, b, perm, inv


if what in ("ms", "both"):
    g = ctx.generate_webgraph()
    row, a, b, perm, inv = relabeled(g)
    g.close()
    srcs = np.nonzero(np.diff(row) > 0)[0][:1024]
    for gg, ss, tag in ((a, srcs, "input ids"), (b, inv[srcs], "relabeled")):
        gg.sssp_batch([int(x) for x in ss[:64]], copy=False)
        gg.sssp_batch([int(x) for x in ss], copy=False)
    da = a.sssp_batch([int(x) for x in srcs[:64]])
    db = b.sssp_batch([int(x) for x in inv[srcs[:64]]])
    assert (db[:, inv] == da).all(), "relabeled MS-BFS rows differ"
    for rep in range(3):
        for gg, ss, tag in ((a, srcs, "input ids"), (b, inv[srcs], "relabeled")):
            ts, ks = [], []
            for _ in range(7):
                t = time.perf_counter()
                gg.sssp_batch([int(x) for x in ss], copy=False)
                ts.append(time.perf_counter() - t)
                ks.append(gg.stats()["kernel_ms"])
            print(f"ms1024 {tag:10s} rep {rep}: batch {1e3 * np.median(ts):.3f} ms (min {1e3 * min(ts):.3f}) "
                  f"kernel {np.median(ks):.3f} ms", flush=True)
    a.close()
    b.close()

if what in ("k22", "both"):
    g = ctx.generate_kronecker(22, 16, 1)
    roots = [int(r) for r in g.sample_roots(2, 8)]
    row, a, b, perm, inv = relabeled(g)
    g.close()
    for r in roots[:2]:
        assert (b.sssp(int(inv[r]))[inv] == a.sssp(r)).all(), "relabeled BFS differs"
    for rep in range(3):
        for gg, rs, tag in ((a, roots, "input ids"), (b, [int(inv[r]) for r in roots], "relabeled")):
            for r in rs:
                gg.sssp(r, copy=False)
            ks = []
            t = time.perf_counter()
            for r in rs:
                gg.sssp(r, copy=False)
                ks.append(gg.stats()["kernel_ms"])
            el = time.perf_counter() - t
            print(f"k22 {tag:10s} rep {rep}: {1e3 * el / len(rs):.4f} ms per BFS, kernel {np.mean(ks):.4f} ms",
                  flush=True)
    a.close()
    b.close()
