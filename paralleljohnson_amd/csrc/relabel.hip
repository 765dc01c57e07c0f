// relabel.hip — degree-ordered copy of a weighted graph for delta-stepping.
//
// The relaxations of delta.hip read and atomicMin dist[target] for every edge.
// In a Kronecker graph half the ids are isolated and the edge targets are
// concentrated on a few hubs scattered over the id space by the label
// permutation, so with input ids every target access is a random 4-byte read
// that costs a whole 64-byte line from HBM (measured: ~1.2 L2 misses per edge
// at s26). New ids: vertices with any edge first (n_scan of them), ordered by
// out-degree descending (ties by input id). The touched part of dist is then
// dense (half the size at s26, inside the 256 MB Infinity Cache) and the hot
// entries share lines. The band selection passes only scan [0, n_scan).
// Distances are mapped back to input ids at the end of every solve, inside
// the timed region. This is a pure relabeling: it changes no distance.
#include "devutil.h"

namespace pj {

namespace {

template <typename Off>
__global__ void degree_k(const Off* __restrict__ row, i64 n, u32* __restrict__ deg) {
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x)
        deg[v] = (u32)(row[v + 1] - row[v]);
}

// touched[v] = 1 if v is the target of an edge (idempotent plain stores)
__global__ void mark_targets_k(const u32* __restrict__ col, i64 nnz, uint8_t* __restrict__ touched) {
    for (i64 e = (i64)blockIdx.x * blockDim.x + threadIdx.x; e < nnz; e += (i64)gridDim.x * blockDim.x)
        if (!touched[col[e]]) touched[col[e]] = 1;  // (most targets repeat: skip the store)
}

__global__ void max_u32_k(const u32* __restrict__ in, i64 n, u32* __restrict__ out) {
    u32 m = 0;
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) m = max(m, in[i]);
    m = wave_max(m);
    if (lane_id() == 0 && m) atomicMax(out, m);
}

// sort key: vertices with edges first, by out-degree descending; the rest last
__global__ void order_key_k(const u32* __restrict__ deg, const uint8_t* __restrict__ touched, i64 n, u32 maxdeg,
                            u32* __restrict__ key, u32* __restrict__ ids, u32* __restrict__ nscan) {
    u32 c = 0;
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x) {
        const bool any = deg[v] > 0 || touched[v];
        key[v] = any ? maxdeg - deg[v] : maxdeg + 1;
        ids[v] = (u32)v;
        c += any;
    }
    c = wave_sum(c);
    if (lane_id() == 0 && c) atomicAdd(nscan, c);
}

__global__ void invert_k(const u32* __restrict__ perm, i64 n, u32* __restrict__ inv, const u32* __restrict__ deg,
                         u32* __restrict__ ndeg) {
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) {
        const u32 o = perm[i];
        inv[o] = (u32)i;
        ndeg[i] = deg[o];
    }
}

__global__ void narrow_k(const u64* __restrict__ in, i64 n, u32* __restrict__ out) {
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x)
        out[i] = (u32)in[i];
}

// one wave per new row: copy the old row in order, targets renamed
template <typename Off>
__global__ __launch_bounds__(256) void copy_rows_k(const u32* __restrict__ perm, const u32* __restrict__ inv,
                                                   const Off* __restrict__ orow, const u32* __restrict__ ocol,
                                                   const u32* __restrict__ ow, const Off* __restrict__ nrow,
                                                   u32* __restrict__ ncol, u32* __restrict__ nw, i64 nrows) {
    // (bound by the random id lookups inv[ocol[k]]: a lane-per-row and an
    // edge-parallel form over 64 rows per wave measured no faster, 50-56 ms at s26)
    const i64 nwaves = (i64)gridDim.x * (blockDim.x / WAVE);
    for (i64 i = (i64)blockIdx.x * (blockDim.x / WAVE) + wave_id(); i < nrows; i += nwaves) {
        const u32 o = perm[i];
        const Off b = orow[o], d = orow[o + 1] - b, nb = nrow[i];
        for (Off k = (Off)lane_id(); k < d; k += WAVE) {
            ncol[nb + k] = inv[ocol[b + k]];
            nw[nb + k] = ow[b + k];
        }
    }
}

#ifndef PJ_RL_COPY
#define PJ_RL_COPY 1  // 0: one wave per new row; 1: edge tiles (below)
#endif
#ifndef PJ_RL_PASSES
#define PJ_RL_PASSES 1  // target-id range passes of the tile copy
#endif

constexpr int CT = 256;          // threads of a tile block
constexpr int CE = 8;            // edges per thread
constexpr int CTILE = CT * CE;   // new-CSR entries per tile
constexpr int CROWS = CTILE + 1; // rows staged per tile (more: per-edge global search)

// tile_row[t] = the new row holding entry t * CTILE; tile_row[ntiles] = the row of
// the last entry (only rows with entries are written)
template <typename Off>
__global__ void tile_rows_k(const Off* __restrict__ nrow, i64 n, i64 nnz, u32* __restrict__ tile_row) {
    const i64 ntiles = (nnz + CTILE - 1) / CTILE;
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x) {
        const i64 b = (i64)nrow[v], e = (i64)nrow[v + 1];
        if (e <= b) continue;
        for (i64 t = (b + CTILE - 1) / CTILE; t * CTILE < e; ++t) tile_row[t] = (u32)v;
        if (e == nnz) tile_row[ntiles] = (u32)v;
    }
}

// Edge-balanced copy: a block takes CTILE consecutive entries of the new CSR, stages
// the new and old row starts of the rows they belong to in LDS, and every thread
// copies CE entries (stride CT: coalesced stores), each found by a binary search
// over the staged starts. All CE loads of a thread are independent, so the random
// id lookups inv[ocol[k]] overlap (the wave-per-row form walks short rows with
// mostly idle lanes, one dependent row chain per wave). A pass renames only the
// targets in [lo, hi) (PJ_RL_PASSES > 1: each pass's slice of inv stays cached).
template <typename Off>
__global__ __launch_bounds__(CT) void copy_tiles_k(const u32* __restrict__ perm, const u32* __restrict__ inv,
                                                   const Off* __restrict__ orow, const u32* __restrict__ ocol,
                                                   const u32* __restrict__ ow, const Off* __restrict__ nrow,
                                                   u32* __restrict__ ncol, u32* __restrict__ nw, i64 nnz,
                                                   const u32* __restrict__ tile_row, u32 lo, u32 hi, int first) {
    __shared__ Off s_nb[CROWS], s_ob[CROWS];
    const i64 ntiles = (nnz + CTILE - 1) / CTILE;
    for (i64 t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const i64 e0 = t * CTILE, e1 = min(e0 + CTILE, nnz);
        const u32 r0 = tile_row[t], r1 = tile_row[t + 1];
        const i64 nr = (i64)r1 - r0 + 1;
        const bool staged = nr <= CROWS;
        if (staged)
            for (i64 j = threadIdx.x; j < nr; j += CT) {
                s_nb[j] = nrow[r0 + j];
                s_ob[j] = orow[perm[r0 + j]];
            }
        __syncthreads();
        i64 src[CE];
#pragma unroll
        for (int m = 0; m < CE; ++m) {
            const i64 k = e0 + threadIdx.x + m * CT;
            src[m] = -1;
            if (k >= e1) continue;
            i64 a = 0, b = nr - 1;  // largest j with start(j) <= k
            while (a < b) {
                const i64 mid = (a + b + 1) >> 1;
                const Off st = staged ? s_nb[mid] : nrow[r0 + mid];
                if ((i64)st <= k) a = mid;
                else b = mid - 1;
            }
            const Off nb = staged ? s_nb[a] : nrow[r0 + a];
            const Off ob = staged ? s_ob[a] : orow[perm[r0 + a]];
            src[m] = (i64)ob + (k - (i64)nb);
        }
        u32 c[CE], wv[CE];
#pragma unroll
        for (int m = 0; m < CE; ++m)
            if (src[m] >= 0) {
                c[m] = ocol[src[m]];
                if (first) wv[m] = ow[src[m]];
            }
#pragma unroll
        for (int m = 0; m < CE; ++m)
            if (src[m] >= 0) {
                const i64 k = e0 + threadIdx.x + m * CT;
                if (c[m] >= lo && c[m] < hi) ncol[k] = inv[c[m]];
                if (first) nw[k] = wv[m];
            }
        __syncthreads();
    }
}

template <typename Off>
void build(Graph& g) {
    hipStream_t s = g.ctx->stream;
    const i64 n = g.n, nnz = g.nnz;
    const Off* orow = static_cast<const Off*>(g.row_ptr());
    std::unique_ptr<Relabeled> R(new Relabeled());
    const unsigned grid = (unsigned)g.ctx->cu_count * 16u;
    DevBuf<u32> deg((size_t)n + 1), key((size_t)n + 1), kalt((size_t)n + 1), ids((size_t)n + 1),
        ialt((size_t)n + 1);
    DevBuf<uint8_t> touched((size_t)n + 1);
    DevBuf<u32> scal(2);
    PJ_HIP(hipMemsetAsync(touched.p, 0, (size_t)n + 1, s));
    PJ_HIP(hipMemsetAsync(scal.p, 0, 2 * sizeof(u32), s));
    degree_k<Off><<<grid_for(n, 256, grid), 256, 0, s>>>(orow, n, deg.p);
    // vertices that are only targets also get an id below n_scan; a symmetric graph has
    // none (every target has the reverse edge), so the random byte stores are skipped
    if (nnz && !g.symmetric) mark_targets_k<<<grid_for(nnz, 256, grid), 256, 0, s>>>(g.col.p, nnz, touched.p);
    max_u32_k<<<grid_for(n, 256, grid), 256, 0, s>>>(deg.p, n, scal.p);
    PJ_LAUNCH_CHECK();
    u32 h[2] = {0, 0};
    PJ_HIP(hipMemcpyAsync(h, scal.p, sizeof(u32), hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
    const u32 maxdeg = h[0];
    order_key_k<<<grid_for(n, 256, grid), 256, 0, s>>>(deg.p, touched.p, n, maxdeg, key.p, ids.p, scal.p + 1);
    PJ_LAUNCH_CHECK();
    PJ_HIP(hipMemcpyAsync(h + 1, scal.p + 1, sizeof(u32), hipMemcpyDeviceToHost, s));
    int bits = 0;
    while (bits < 32 && ((u64)1 << bits) < (u64)maxdeg + 2) ++bits;
    SortWs ws;
    u32 *kr, *pr;
    radix_sort_pairs<u32>(key.p, kalt.p, ids.p, ialt.p, n, bits, ws, s, &kr, &pr);
    R->perm.alloc((size_t)n);
    R->inv.alloc((size_t)n);
    PJ_HIP(hipMemcpyAsync(R->perm.p, pr, sizeof(u32) * (size_t)n, hipMemcpyDeviceToDevice, s));
    u32* ndeg = kr == key.p ? kalt.p : key.p;  // free buffer
    invert_k<<<grid_for(n, 256, grid), 256, 0, s>>>(R->perm.p, n, R->inv.p, deg.p, ndeg);
    PJ_LAUNCH_CHECK();
    DevBuf<u64> off((size_t)n + 1);
    exclusive_scan_u32(ndeg, off.p, n, g.scan, s);
    Off* nrow;
    if (sizeof(Off) == 8) {
        R->row64 = std::move(off);
        nrow = reinterpret_cast<Off*>(R->row64.p);
    } else {
        R->row32.alloc((size_t)n + 1);
        narrow_k<<<grid_for(n + 1, 256, grid), 256, 0, s>>>(off.p, n + 1, R->row32.p);
        PJ_LAUNCH_CHECK();
        nrow = reinterpret_cast<Off*>(R->row32.p);
    }
    R->col.alloc((size_t)(nnz ? nnz : 1));
    R->w.alloc((size_t)(nnz ? nnz : 1));
    if (nnz && PJ_RL_COPY == 0) {
        copy_rows_k<Off><<<grid, 256, 0, s>>>(R->perm.p, R->inv.p, orow, g.col.p, g.w.p, nrow, R->col.p, R->w.p,
                                              n);
    } else if (nnz) {
        const i64 ntiles = (nnz + CTILE - 1) / CTILE;
        DevBuf<u32> trow((size_t)ntiles + 1);
        tile_rows_k<Off><<<grid_for(n, 256, grid), 256, 0, s>>>(nrow, n, nnz, trow.p);
        PJ_LAUNCH_CHECK();
        const unsigned tgrid = (unsigned)std::min<i64>(ntiles, (i64)g.ctx->cu_count * 8);
        const u64 span = ((u64)n + PJ_RL_PASSES - 1) / PJ_RL_PASSES;
        for (int p = 0; p < PJ_RL_PASSES; ++p) {
            const u64 lo = span * (u64)p, hi = std::min<u64>((u64)n, lo + span);
            copy_tiles_k<Off><<<tgrid, CT, 0, s>>>(R->perm.p, R->inv.p, orow, g.col.p, g.w.p, nrow, R->col.p,
                                                   R->w.p, nnz, trow.p, (u32)lo,
                                                   p + 1 == PJ_RL_PASSES ? 0xFFFFFFFFu : (u32)hi, p == 0);
            PJ_LAUNCH_CHECK();
        }
        PJ_HIP(hipStreamSynchronize(s));  // trow is freed on return
    }
    PJ_LAUNCH_CHECK();
    R->dist.alloc((size_t)n);
    PJ_HIP(hipStreamSynchronize(s));
    R->n_scan = h[1];
    g.rl = std::move(R);
}

}  // namespace

// The relabeled id of one input vertex (4-byte read of inv; a whole host copy of
// inv cost ~0.1 s of the first solve on a 2^26-vertex graph).
i64 relabeled_id(const Relabeled& R, i64 v, hipStream_t s) {
    u32 x = 0;
    PJ_HIP(hipMemcpyAsync(&x, R.inv.p + v, sizeof(u32), hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
    return (i64)x;
}

void build_relabeled(Graph& g) {
    if (g.n == 0) {
        g.rl.reset(new Relabeled());
        return;
    }
    if (g.off64) build<u64>(g);
    else build<u32>(g);
}

}  // namespace pj
