// sort.hip — stable LSD radix sort of (key, value) pairs and CSR row bounds.
//
// This is the GPU form of coord2csr (ParallelJohnson.cpp:117-159): the
// reference does one stable counting sort of the COO by src; here the key is
// split into P = ceil(bits / 8) digits of equal width (at most 8 bits: 22-bit
// keys -> 8 + 7 + 7), and each digit pass is a stable counting sort over
// tiles of TILE pairs:
//   hist    : per-tile digit histograms (wave-private LDS counters) -> hist[tile][digit],
//             and per chunk of tiles                             -> csum[digit][chunk]
//   scan    : exclusive scan of csum in digit-major order, then per tile -> offs[tile][digit]
//   scatter : the tile is ranked by digit inside each wave (ballot peer masks,
//             wave-private running counters in LDS, no block barrier per
//             item), reordered by digit in LDS, and written out in LDS order,
//             so consecutive lanes store consecutive addresses of one digit's
//             run: coalesced writes instead of 64 lanes hitting up to 256
//             buckets.
// Tile order is (wave, item, lane) = global index order, so every pass is
// stable and the result keeps file order inside each row, exactly like the
// reference's scatter loop :143-149.
#include "devutil.h"

namespace pj {

namespace {

constexpr int RB = 256;  // threads per tile block (4 waves)
constexpr int RNW = RB / WAVE;
#ifndef PJ_SORT_XCD
#define PJ_SORT_XCD 1
#endif
#ifndef PJ_SORT_IPT32
#define PJ_SORT_IPT32 16
#endif
#ifndef PJ_SORT_CHUNK
#define PJ_SORT_CHUNK 16
#endif
constexpr int HC = PJ_SORT_CHUNK;  // tiles per histogram block (one chunk)
#ifndef PJ_SORT_HIST_ATOMIC
#define PJ_SORT_HIST_ATOMIC 1  // s24: 985 -> 596 us per pass over the ballot counting
#endif
#ifndef PJ_SORT_IPT64
#define PJ_SORT_IPT64 16
#endif

// Tile of a block. With PJ_SORT_XCD, consecutive tiles go to blocks b, b + 8, ...
// (one XCD under round-robin placement, speed only): the line shared by tile t's
// run of a digit and tile t + 1's run is then written through one L2.
__device__ __forceinline__ i64 tile_of(i64 ntiles) {
    const i64 b = blockIdx.x;
    if (!PJ_SORT_XCD || ntiles < 64) return b;
    const i64 per = ntiles / 8, rem = ntiles % 8;  // XCD x gets per (+1 for x < rem) consecutive tiles
    const i64 x = b % 8, k = b / 8;  // blocks with b % 8 == x number exactly per + (x < rem)
    return x * per + (x < rem ? x : rem) + k;
}

// pairs per thread: 16 (4096-pair tiles; 32 KB of LDS with u32 values, 48 KB with u64):
// 32 gave longer digit runs but half the resident tiles per CU and measured slower
template <typename V>
constexpr int ipt() {
    return sizeof(V) == 8 ? PJ_SORT_IPT64 : PJ_SORT_IPT32;
}
template <typename V>
constexpr int tile() {
    return RB * ipt<V>();
}

// Per-tile digit histograms of a chunk of HC consecutive tiles. Each wave counts
// into wave-private LDS counters with returnless LDS atomics (default; counting
// 64 keys per step with ballot peer masks and one read-modify-write per distinct
// digit measured 1.65x slower: the dependent LDS round trips). Outputs are laid
// out for coalesced stores: hist[tile][256] (tile-major) and the chunk's digit
// sums csum[digit][chunk] (one scattered store per digit per HC tiles; a
// digit-major hist[digit][tile] costs one partial-line store per digit per tile).
template <int TILE>
__global__ __launch_bounds__(RB) void radix_hist_k(const u32* __restrict__ keys, i64 n, int shift, int dbits,
                                                   u32* __restrict__ hist, u32* __restrict__ csum, i64 ntiles,
                                                   i64 nchunks) {
    __shared__ u32 cnt[RNW][256];
    const int t = threadIdx.x, lane = lane_id(), w = wave_id();
    const u32 dmask = (1u << dbits) - 1u;
    constexpr int ROWS = TILE / RB;
    u32 chunk_sum = 0;
    const i64 t0 = (i64)blockIdx.x * HC, t1 = min(t0 + HC, ntiles);
    for (i64 tl = t0; tl < t1; ++tl) {
        for (int d = lane; d < 256; d += WAVE) cnt[w][d] = 0;
        const i64 wbase = tl * TILE + (i64)w * (TILE / RNW) + lane;
        u32 key[ROWS];  // every load issued before the first ballot
#pragma unroll
        for (int j = 0; j < ROWS; ++j) {
            const i64 i = wbase + (i64)j * WAVE;
            key[j] = i < n ? keys[i] : 0u;
        }
#if PJ_SORT_HIST_ATOMIC
        // returnless LDS atomics into the wave's own counters (nothing waits on them)
#pragma unroll
        for (int j = 0; j < ROWS; ++j)
            if (wbase + (i64)j * WAVE < n) atomicAdd(&cnt[w][(key[j] >> shift) & dmask], 1u);
#else
#pragma unroll
        for (int j = 0; j < ROWS; ++j) {
            const bool valid = wbase + (i64)j * WAVE < n;
            const u32 d = (key[j] >> shift) & dmask;
            u64 peers = __ballot(valid);
            for (int b = 0; b < dbits; ++b) {
                const bool bit = (d >> b) & 1u;
                const u64 m = __ballot(bit);
                peers &= bit ? m : ~m;
            }
            if (valid && lane == __ffsll((long long)peers) - 1) cnt[w][d] += (u32)__popcll(peers);
        }
#endif
        __syncthreads();
        u32 c = 0;
#pragma unroll
        for (int q = 0; q < RNW; ++q) c += cnt[q][t];
        hist[tl * 256 + t] = c;
        chunk_sum += c;
        __syncthreads();  // the counters are reset for the next tile
    }
    if ((u32)t <= dmask) csum[(i64)t * nchunks + blockIdx.x] = chunk_sum;
}

// offs[tile][digit] = (digit-major exclusive prefix of the chunk sums) + the digit's
// counts in the chunk's earlier tiles: the global start of the tile's run of each digit.
__global__ __launch_bounds__(RB) void radix_offs_k(const u32* __restrict__ hist, const u64* __restrict__ cpre,
                                                   u64* __restrict__ offs, i64 ntiles, i64 nchunks) {
    const int t = threadIdx.x;
    const i64 t0 = (i64)blockIdx.x * HC, t1 = min(t0 + HC, ntiles);
    u64 run = cpre[(i64)t * nchunks + blockIdx.x];
    for (i64 tl = t0; tl < t1; ++tl) {
        offs[tl * 256 + t] = run;
        run += hist[tl * 256 + t];
    }
}

template <typename V>
__global__ __launch_bounds__(RB) void radix_scatter_k(const u32* __restrict__ keys, const V* __restrict__ vals,
                                                      u32* __restrict__ kout, V* __restrict__ vout, i64 n, int shift,
                                                      int dbits, const u64* __restrict__ offs, i64 ntiles) {
    constexpr int IPT = ipt<V>();
    constexpr int TILE = tile<V>();
    __shared__ u32 s_key[TILE];
    __shared__ V s_val[TILE];
    __shared__ u32 s_cnt[RNW][256];  // per-wave running counters, then per-wave exclusive bases
    __shared__ u32 s_start[256];     // tile-local exclusive start of each digit
    __shared__ u64 s_goff[256];      // global position of the tile's run of each digit
    __shared__ u32 s_red[RNW];
    const int t = threadIdx.x, lane = lane_id(), w = wave_id();
    const u32 dmask = (1u << dbits) - 1u;
    const i64 tl = tile_of(ntiles);
    const i64 base = tl * TILE;
    for (int d = lane; d < 256; d += WAVE) s_cnt[w][d] = 0;
    s_goff[t] = offs[tl * 256 + t];

    // wave w owns tile items [w * 64 * IPT, (w + 1) * 64 * IPT), row j = 64 consecutive items
    u32 key[IPT];
    V val[IPT];
    u32 rk[IPT];
    const i64 wbase = base + (i64)w * WAVE * IPT + lane;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const i64 i = wbase + (i64)j * WAVE;
        key[j] = i < n ? keys[i] : 0u;
        val[j] = i < n ? vals[i] : V(0);
    }
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const bool valid = wbase + (i64)j * WAVE < n;
        const u32 d = (key[j] >> shift) & dmask;
        u64 peers = __ballot(valid);
        for (int b = 0; b < dbits; ++b) {
            const bool bit = (d >> b) & 1u;
            const u64 m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const int leader = __ffsll((long long)peers) - 1;
        u32 c = 0;
        if (valid && lane == leader) {
            c = s_cnt[w][d];
            s_cnt[w][d] = c + (u32)__popcll(peers);
        }
        c = __shfl(c, leader < 0 ? 0 : leader, 64);
        rk[j] = c + (u32)__popcll(peers & lanemask_lt());
    }
    __syncthreads();
    // digit t: per-wave exclusive bases and the tile total, then the tile-local starts
    u32 tot = 0;
#pragma unroll
    for (int q = 0; q < RNW; ++q) {
        const u32 c = s_cnt[q][t];
        s_cnt[q][t] = tot;
        tot += c;
    }
    u32 all;
    s_start[t] = block_excl_scan<RNW>(tot, s_red, all);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        if (wbase + (i64)j * WAVE < n) {
            const u32 d = (key[j] >> shift) & dmask;
            const u32 pos = s_start[d] + s_cnt[w][d] + rk[j];
            s_key[pos] = key[j];
            s_val[pos] = val[j];
        }
    }
    __syncthreads();
    // LDS order = digit-major, stable: lane-consecutive positions within a digit's run
    const i64 count = min((i64)TILE, n - base);
#pragma unroll 4
    for (int k = 0; k < IPT; ++k) {
        const int i = k * RB + t;
        if (i < count) {
            const u32 kk = s_key[i];
            const u32 d = (kk >> shift) & dmask;
            const u64 g = s_goff[d] + (u64)(i - (int)s_start[d]);
            kout[g] = kk;
            vout[g] = s_val[i];
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
        constexpr i64 TILE = tile<V>();
        const i64 ntiles = (n + TILE - 1) / TILE;
        const int passes = (bits + 7) / 8;
        const int dbits = (bits + passes - 1) / passes;  // equal digits: fewer buckets, longer runs
        const i64 nchunks = (ntiles + HC - 1) / HC;
        ws.hist.ensure((size_t)(256 * ntiles));
        ws.csum.ensure((size_t)(256 * nchunks));
        ws.offs.ensure((size_t)(256 * std::max(ntiles, nchunks) + 1));
        ws.cpre.ensure((size_t)(256 * nchunks + 1));
        for (int shift = 0; shift < bits; shift += dbits) {
            const int db = std::min(dbits, bits - shift);
            const i64 nh = (i64)(1 << db) * nchunks;
            radix_hist_k<tile<V>()><<<(unsigned)nchunks, RB, 0, s>>>(kc, n, shift, db, ws.hist.p, ws.csum.p, ntiles,
                                                                     nchunks);
            PJ_LAUNCH_CHECK();
            exclusive_scan_u32(ws.csum.p, ws.cpre.p, nh, ws.scan, s);
            radix_offs_k<<<(unsigned)nchunks, RB, 0, s>>>(ws.hist.p, ws.cpre.p, ws.offs.p, ntiles, nchunks);
            PJ_LAUNCH_CHECK();
            radix_scatter_k<V><<<(unsigned)ntiles, RB, 0, s>>>(kc, vc, ka, va, n, shift, db, ws.offs.p, ntiles);
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
