import sys, os, ctypes
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (R, os.path.join(R, "oracle"), os.path.join(R, "tests")):
    sys.path.insert(0, p)
import numpy as np
import oracle as O
import paralleljohnson_amd as pj
from helpers import random_graph

ctx = pj.Context(0)
direction, kind = 2, "uniform"
rng = np.random.default_rng(100 + 7 * direction + len(kind))
for trial in range(4):
    n = int(rng.integers(2, 60000))
    src, dst = random_graph(rng, kind, n)
    roots = [int(src[0]) if len(src) else 0, int(rng.integers(0, n)), n, -5]
g = ctx.load_coo(src, dst, n=n)
row, col, _ = O.coo2csr(src.astype(np.uint32), dst.astype(np.uint32), n)
grow, gcol, _ = g.get_csr()
r = 7305
exp = O.bfs(row, col, r)
iso = (np.diff(row) == 0)
# in-degree via CSC
indeg = np.bincount(dst, minlength=n)
iso &= indeg == 0
nw = (n + 63) // 64
lib = pj._lib
lib.pj_debug_bitmaps.argtypes = [ctypes.c_void_p] * 4
def bits(words):
    b = np.unpackbits(words.view(np.uint8), bitorder="little")[:n].astype(bool)
    return b
g.set_option("direction", 2)
for L in range(1, 9):
    g.set_option("max_levels", L)
    d = g.sssp(r)
    v0 = np.zeros(nw, np.uint64); v1 = np.zeros(nw, np.uint64); fn = np.zeros(nw, np.uint64)
    lib.pj_debug_bitmaps(g._h, v0.ctypes.data, v1.ctypes.data, fn.ctypes.data)
    want = (exp <= L) | iso
    b0, b1, bf = bits(v0), bits(v1), bits(fn)
    cur = b0 if L % 2 == 0 else b1   # pull levels flip vsel each level: after L levels the current is vis[L % 2]
    print(f"L={L}: dist mismatches {(d != np.where(exp <= L, exp, 100000)).sum()}  vis[L%2] vs want: missing {(want & ~cur).sum()} extra {(cur & ~want).sum()}  fnew vs (exp==L): missing {((exp == L) & ~bf).sum()} extra {(bf & (exp != L)).sum()}", flush=True)
    miss = np.nonzero(want & ~cur)[0][:5]
    extra = np.nonzero(cur & ~want)[0][:5]
    if len(miss) or len(extra):
        print("   missing", miss.tolist(), "exp", exp[miss].tolist(), "got", d[miss].tolist())
        print("   extra", extra.tolist(), "exp", exp[extra].tolist(), "got", d[extra].tolist())
