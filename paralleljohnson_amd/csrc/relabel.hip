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
// id lookups inv[ocol[k]] overlap (a wave-per-row form walked short rows with mostly
// idle lanes, one dependent row chain per wave: 53.7 against 43.7 ms at s26, and
// target-range passes that keep a slice of inv cached measured 49-61 ms,
// profiles/r03/relabel_copy_variants.txt). The weights are written as WT (u8 when
// every weight fits, the solver's split records) and their sum and maximum reduced on
// the way (wacc[0], wacc[1]: the auto delta's mean weight and the u8 test), so no
// separate pass reads the 2^31 input weights again.
template <typename Off, typename WT>
__global__ __launch_bounds__(CT) void copy_tiles_k(const u32* __restrict__ perm, const u32* __restrict__ inv,
                                                   const Off* __restrict__ orow, const u32* __restrict__ ocol,
                                                   const u32* __restrict__ ow, const Off* __restrict__ nrow,
                                                   u32* __restrict__ ncol, WT* __restrict__ nw, i64 nnz,
                                                   const u32* __restrict__ tile_row, u64* __restrict__ wacc) {
    __shared__ Off s_nb[CROWS], s_ob[CROWS];
    __shared__ u64 red[CT / WAVE];
    const i64 ntiles = (nnz + CTILE - 1) / CTILE;
    u64 wsum = 0;
    u32 wmax = 0;
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
                wv[m] = ow[src[m]];
            }
#pragma unroll
        for (int m = 0; m < CE; ++m)
            if (src[m] >= 0) {
                const i64 k = e0 + threadIdx.x + m * CT;
                ncol[k] = inv[c[m]];
                nw[k] = (WT)wv[m];
                wsum += wv[m];
                wmax = max(wmax, wv[m]);
            }
        __syncthreads();
    }
    wsum = block_sum<CT / WAVE>(wsum, red);
    wmax = wave_max(wmax);
    if (lane_id() == 0) red[wave_id()] = wmax;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 0; k < CT / WAVE; ++k) wmax = max(wmax, (u32)red[k]);
        if (wsum) atomicAdd(&wacc[0], wsum);
        if (wmax) atomicMax(&wacc[1], (u64)wmax);
    }
}

template <typename Off>
void build(Graph& g) {
    hipStream_t s = g.ctx->stream;
    const i64 n = g.n, nnz = g.nnz;
    const Off* orow = static_cast<const Off*>(g.row_ptr());
    std::unique_ptr<Relabeled> R(new Relabeled());
    const unsigned grid = (unsigned)g.ctx->cu_count * 16u;
    // the temporaries in ONE allocation: a hipFree costs ~0.19 ms of host time at s26
    // (it waits for the device), and there were twelve of them behind the copy
    const i64 ntiles = (nnz + CTILE - 1) / CTILE;
    const size_t nb = ((size_t)n + 1) * sizeof(u32), al = 256;
    auto up = [&](size_t b) { return (b + al - 1) / al * al; };
    const size_t sz_off = sizeof(Off) == 8 ? 0 : up(((size_t)n + 1) * sizeof(u64));
    DevBuf<uint8_t> arena(5 * up(nb) + up((size_t)n + 1) + up(4 * sizeof(u64)) + sz_off +
                          up(((size_t)ntiles + 1) * sizeof(u32)));
    uint8_t* cur = arena.p;
    auto carve = [&](size_t b) {
        uint8_t* q = cur;
        cur += up(b);
        return q;
    };
    u32* deg = reinterpret_cast<u32*>(carve(nb));
    u32* key = reinterpret_cast<u32*>(carve(nb));
    u32* kalt = reinterpret_cast<u32*>(carve(nb));
    u32* ids = reinterpret_cast<u32*>(carve(nb));
    u32* ialt = reinterpret_cast<u32*>(carve(nb));
    uint8_t* touched = carve((size_t)n + 1);
    u64* scal64 = reinterpret_cast<u64*>(carve(4 * sizeof(u64)));  // [0] max degree, [1] n_scan (u32), [2..3] wacc
    u32* scal = reinterpret_cast<u32*>(scal64);
    u64* wacc = scal64 + 2;
    PJ_HIP(hipMemsetAsync(touched, 0, (size_t)n + 1, s));
    PJ_HIP(hipMemsetAsync(scal64, 0, 4 * sizeof(u64), s));
    degree_k<Off><<<grid_for(n, 256, grid), 256, 0, s>>>(orow, n, deg);
    // vertices that are only targets also get an id below n_scan; a symmetric graph has
    // none (every target has the reverse edge), so the random byte stores are skipped
    if (nnz && !g.symmetric) mark_targets_k<<<grid_for(nnz, 256, grid), 256, 0, s>>>(g.col.p, nnz, touched);
    max_u32_k<<<grid_for(n, 256, grid), 256, 0, s>>>(deg, n, scal);
    PJ_LAUNCH_CHECK();
    u32 h[2] = {0, 0};
    PJ_HIP(hipMemcpyAsync(h, scal, sizeof(u32), hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
    const u32 maxdeg = h[0];
    order_key_k<<<grid_for(n, 256, grid), 256, 0, s>>>(deg, touched, n, maxdeg, key, ids, scal + 1);
    PJ_LAUNCH_CHECK();
    PJ_HIP(hipMemcpyAsync(h + 1, scal + 1, sizeof(u32), hipMemcpyDeviceToHost, s));
    int bits = 0;
    while (bits < 32 && ((u64)1 << bits) < (u64)maxdeg + 2) ++bits;
    SortWs ws;
    u32 *kr, *pr;
    radix_sort_pairs<u32>(key, kalt, ids, ialt, n, bits, ws, s, &kr, &pr);
    R->perm.alloc((size_t)n);
    R->inv.alloc((size_t)n);
    PJ_HIP(hipMemcpyAsync(R->perm.p, pr, sizeof(u32) * (size_t)n, hipMemcpyDeviceToDevice, s));
    u32* ndeg = kr == key ? kalt : key;  // free buffer
    invert_k<<<grid_for(n, 256, grid), 256, 0, s>>>(R->perm.p, n, R->inv.p, deg, ndeg);
    PJ_LAUNCH_CHECK();
    Off* nrow;
    if (sizeof(Off) == 8) {  // the scan writes the 64-bit row offsets in place
        R->row64.alloc((size_t)n + 1);
        exclusive_scan_u32(ndeg, R->row64.p, n, g.scan, s);
        nrow = reinterpret_cast<Off*>(R->row64.p);
    } else {
        u64* off = reinterpret_cast<u64*>(carve(((size_t)n + 1) * sizeof(u64)));
        exclusive_scan_u32(ndeg, off, n, g.scan, s);
        R->row32.alloc((size_t)n + 1);
        narrow_k<<<grid_for(n + 1, 256, grid), 256, 0, s>>>(off, n + 1, R->row32.p);
        PJ_LAUNCH_CHECK();
        nrow = reinterpret_cast<Off*>(R->row32.p);
    }
    R->col.alloc((size_t)(nnz ? nnz : 1));
    R->w8.alloc((size_t)(nnz ? nnz : 1));
    if (nnz) {
        u32* trow = reinterpret_cast<u32*>(carve(((size_t)ntiles + 1) * sizeof(u32)));
        tile_rows_k<Off><<<grid_for(n, 256, grid), 256, 0, s>>>(nrow, n, nnz, trow);
        PJ_LAUNCH_CHECK();
        const unsigned tgrid = (unsigned)std::min<i64>(ntiles, (i64)g.ctx->cu_count * 8);
        copy_tiles_k<Off, uint8_t><<<tgrid, CT, 0, s>>>(R->perm.p, R->inv.p, orow, g.col.p, g.w.p, nrow, R->col.p,
                                                       R->w8.p, nnz, trow, wacc);
        PJ_LAUNCH_CHECK();
        preload_delta_module();  // host work hidden behind the copy
        u64 hw[2] = {0, 0};
        PJ_HIP(hipMemcpyAsync(hw, wacc, sizeof(hw), hipMemcpyDeviceToHost, s));
        PJ_HIP(hipStreamSynchronize(s));
        if (hw[1] > 255) {  // wide weights: the copy again with u32 weights (ids rewritten unchanged)
            R->w8.release();
            R->w.alloc((size_t)nnz);
            PJ_HIP(hipMemsetAsync(wacc, 0, 2 * sizeof(u64), s));
            copy_tiles_k<Off, u32><<<tgrid, CT, 0, s>>>(R->perm.p, R->inv.p, orow, g.col.p, g.w.p, nrow, R->col.p,
                                                       R->w.p, nnz, trow, wacc);
            PJ_LAUNCH_CHECK();
        }
        if (g.mean_weight < 0.0) {
            g.mean_weight = (double)hw[0] / (double)nnz;
            g.max_weight = (long long)hw[1];
        }
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
