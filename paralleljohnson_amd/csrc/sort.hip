// sort.hip — stable LSD radix sort of (key, value) pairs and CSR row bounds.
//
// This is the GPU form of coord2csr (ParallelJohnson.cpp:117-159): the
// reference does a stable counting sort of the COO by src; here each 8-bit
// digit pass is a stable counting sort over 4096-key tiles:
//   hist    : per-tile digit histogram (LDS atomics)        -> hist[digit][tile]
//   scan    : exclusive scan of hist in digit-major order     -> global offsets
//   scatter : per tile, stable in-tile rank by wave64 ballot peer masks, then
//             position = offset[digit][tile] + rank
// Order inside a tile is (item j, wave, lane) = global index order, so every
// pass is stable and the result keeps file order inside each row, exactly
// like the reference's scatter loop :143-149.
#include "devutil.h"

namespace pj {

namespace {

constexpr int RB = 256;
constexpr int RIPT = 16;
constexpr int RTILE = RB * RIPT;
constexpr int RW = RB / WAVE;

__global__ __launch_bounds__(RB) void radix_hist_k(const u32* __restrict__ keys, i64 n, int shift,
                                                   u32* __restrict__ hist, i64 ntiles) {
    __shared__ u32 cnt[256];
    const int t = threadIdx.x;
    cnt[t] = 0;
    __syncthreads();
    const i64 base = (i64)blockIdx.x * RTILE;
#pragma unroll 4
    for (int k = 0; k < RIPT; ++k) {
        i64 i = base + (i64)k * RB + t;
        if (i < n) atomicAdd(&cnt[(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[(i64)t * ntiles + blockIdx.x] = cnt[t];
}

template <typename V>
__global__ __launch_bounds__(RB) void radix_scatter_k(const u32* __restrict__ keys,
                                                      const V* __restrict__ vals,
                                                      u32* __restrict__ kout, V* __restrict__ vout,
                                                      i64 n, int shift, const u64* __restrict__ offs,
                                                      i64 ntiles) {
    __shared__ u32 cnt[RW][256];
    __shared__ u32 pre[RW][256];
    __shared__ u64 toff[256];
    const int t = threadIdx.x, wid = wave_id();
    const i64 base = (i64)blockIdx.x * RTILE;
    toff[t] = offs[(i64)t * ntiles + blockIdx.x];
#pragma unroll
    for (int w = 0; w < RW; ++w) cnt[w][t] = 0;

    u32 key[RIPT];
    V val[RIPT];
#pragma unroll
    for (int j = 0; j < RIPT; ++j) {
        i64 i = base + (i64)j * RB + t;
        key[j] = i < n ? keys[i] : 0u;
        val[j] = i < n ? vals[i] : V(0);
    }
    u32 run = 0;  // thread t owns digit t's running count inside this tile
    __syncthreads();

#pragma unroll 1
    for (int j = 0; j < RIPT; ++j) {
        const i64 i = base + (i64)j * RB + t;
        const bool valid = i < n;
        const u32 d = (key[j] >> shift) & 255u;
        u64 peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const u64 m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const u32 rank_in = (u32)__popcll(peers & lanemask_lt());
        if (valid && rank_in == 0) cnt[wid][d] = (u32)__popcll(peers);
        __syncthreads();
        {
            u32 b = run;
#pragma unroll
            for (int w = 0; w < RW; ++w) {
                pre[w][t] = b;
                b += cnt[w][t];
                cnt[w][t] = 0;
            }
            run = b;
        }
        __syncthreads();
        if (valid) {
            const u64 pos = toff[d] + pre[wid][d] + rank_in;
            kout[pos] = key[j];
            vout[pos] = val[j];
        }
    }
}

template <typename Off>
__global__ void csr_bounds_k(const u32* __restrict__ keys, i64 nnz, i64 nv, Off* __restrict__ row) {
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v <= nv; v += (i64)gridDim.x * blockDim.x) {
        i64 lo = 0, hi = nnz;  // first index with key >= v
        while (lo < hi) {
            i64 mid = (lo + hi) >> 1;
            if ((i64)keys[mid] < v) lo = mid + 1;
            else hi = mid;
        }
        row[v] = (Off)lo;
    }
}

}  // namespace

template <typename V>
void radix_sort_pairs(u32* keys, u32* keys_alt, V* vals, V* vals_alt, i64 n, int bits, SortWs& ws,
                      hipStream_t s, u32** kout, V** vout) {
    u32 *kc = keys, *ka = keys_alt;
    V *vc = vals, *va = vals_alt;
    if (n > 0 && bits > 0) {
        const i64 ntiles = (n + RTILE - 1) / RTILE;
        ws.hist.ensure((size_t)(256 * ntiles));
        ws.offs.ensure((size_t)(256 * ntiles + 1));
        for (int shift = 0; shift < bits; shift += 8) {
            radix_hist_k<<<(unsigned)ntiles, RB, 0, s>>>(kc, n, shift, ws.hist.p, ntiles);
            PJ_LAUNCH_CHECK();
            exclusive_scan_u32(ws.hist.p, ws.offs.p, 256 * ntiles, ws.scan, s);
            radix_scatter_k<V><<<(unsigned)ntiles, RB, 0, s>>>(kc, vc, ka, va, n, shift, ws.offs.p, ntiles);
            PJ_LAUNCH_CHECK();
            std::swap(kc, ka);
            std::swap(vc, va);
        }
    }
    *kout = kc;
    *vout = vc;
}

template void radix_sort_pairs<u32>(u32*, u32*, u32*, u32*, i64, int, SortWs&, hipStream_t, u32**, u32**);
template void radix_sort_pairs<u64>(u32*, u32*, u64*, u64*, i64, int, SortWs&, hipStream_t, u32**, u64**);

template <typename Off>
void csr_bounds(const u32* sorted_keys, i64 nnz, i64 nv, Off* row, hipStream_t s) {
    csr_bounds_k<Off><<<grid_for(nv + 1, 256, 8192), 256, 0, s>>>(sorted_keys, nnz, nv, row);
    PJ_LAUNCH_CHECK();
}
template void csr_bounds<u32>(const u32*, i64, i64, u32*, hipStream_t);
template void csr_bounds<u64>(const u32*, i64, i64, u64*, hipStream_t);

}  // namespace pj
