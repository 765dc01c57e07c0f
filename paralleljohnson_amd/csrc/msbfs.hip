// msbfs.hip — batched multi-source unit-weight SSSP (Johnson-style rows of
// the all-pairs matrix), up to 64 x W sources per pass (W = 1, 2, 4, 8 or 16 words;
// 8 by default).
//
// The reference answers one source per run (`atoi(argv[2])`, :448); a batch of
// 64 W runs shares every CSR read here. Per vertex v the pass keeps three masks
// of W 64-bit words, one bit per source of the batch:
//   V[v]  sources that have reached v          (the reference's sp[] arrays, as bits)
//   F[v]  sources that reached v at the last level (their frontier)
//   Fn[v] the same for the level being computed
// A level is a pull over in-edges: Fn[v] = (OR over in-neighbours u of F[u]) & ~V[v],
// with the scan stopping as soon as every source still missing at v is covered.
// Distances follow the R9 contract per source: the level number, capped at INT_INF.
//
// Distance output (round 5): the levels do not store distances. Each level's new masks go
// to a level archive (entry L+1 for level L, entry 0 = the sources; a level writes only
// the rows with new bits, and a row bitmap Z per entry says which), and one expansion
// kernel at the end of the pass writes the whole 64 W x n distance block with full-line
// stores: every (source, vertex) bit is set in exactly one entry, the arrival level. Per
// level stores of the new pairs' distances into the source-major block were masked
// partial-line writes, 64 W of them per wave and level: 8 of the 11.5 ms of an MS1024
// batch (profiles/r05/ms_dist_r5k.txt). A pass deeper than the archive expands it when it
// fills and stores the later levels' distances directly, as before.
//
// Work mapping: one wave per 64 consecutive vertices; each lane walks its first
// MS_SERIAL in-edges in a wave-uniform loop (predicated body), then the whole wave
// scans the rest of long rows (web-graph in-hubs) 64 edges at a time. The masks
// are stored vertex-major (W words contiguous), so a probe of F[u] is one 8W-byte
// access: wider passes do the same number of random probes for more sources
// (the levels are probe-latency-bound, profiles/r01). W = 8 (512 sources) measured
// best on MS1024; 16 is 3% slower (two passes' latency saved, but twice the mask
// bytes per probe and per vertex).
#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>
#include <vector>

#include "devutil.h"

namespace pj {

namespace {

constexpr int MB = 256;
#ifndef PJ_MS_SERIAL
#define PJ_MS_SERIAL 16
#endif
constexpr int MS_SERIAL = PJ_MS_SERIAL;  // in-edges a lane scans alone before the wave helps
#ifndef PJ_MS_U
#define PJ_MS_U 4  // swept (round 3, MS1024): 2 / 4 / 8 at 4 workgroups per CU, 4 / 8 at 8: 4 at 8 best
#endif
constexpr int MS_U = PJ_MS_U;  // pull: in-edges a lane loads per serial step
constexpr int MS_WMAX = 16;  // widest pass: 1024 sources (option ms_width)
constexpr int MS_WDEF = 8;   // default widest pass: 512 sources

constexpr int MS_NSH = 16;  // shards of the per-level edge counter (one 64-B line each)

struct MsCtl {
    u64 active[3];  // ring: level L reads [(L+2)%3] (level L-1), writes [L%3], block 0 zeroes [(L+1)%3]
    u64 done;       // set once by block 0 of the first level that finds nothing to do
    u64 pad[4];
    // same ring: out-edges of the vertices newly reached by a level (its frontier's push
    // cost), summed over MS_NSH shards: every workgroup of a level adds its count, and one
    // word taking them all saturates at ~88 atomics per microsecond
    u64 fedges[3][MS_NSH][8];
    // (PJ_MS_UF) same ring: the sources that reached some vertex at that level (the OR of
    // the level's new masks, sharded like fedges): only they can extend the next level
    u64 uf[3][MS_NSH][MS_WMAX];
};

// PJ_MS_UF 1: a pull level looks only for the sources whose frontier is not empty (the
// previous level's uf): a vertex that all still-active sources have reached needs no scan,
// and its scan stops once those are covered (late levels, where few sources' searches are
// still running, otherwise scan every in-edge of every vertex some source never reaches)
// MS1024: 11.66 / 11.64 -> 11.54 / 11.51 ms per batch interleaved (r4e, profiles/r04/ms_uf_r4e.txt)
#ifndef PJ_MS_UF
#define PJ_MS_UF 1
#endif
template <int W>
__device__ __forceinline__ void ms_uf_read(const MsCtl* c, int slot, u64 (&m)[W]) {
#pragma unroll
    for (int j = 0; j < W; ++j) m[j] = 0;
    for (int i = 0; i < MS_NSH; ++i)
#pragma unroll
        for (int j = 0; j < W; ++j) m[j] |= c->uf[slot][i][j];
}
// the block's OR of the lanes' masks into shard blockIdx % MS_NSH of slot (block-uniform call)
template <int W>
__device__ __forceinline__ void ms_uf_add(MsCtl* c, int slot, const u64 (&m)[W], u64 (*red)[MS_WMAX]) {
#pragma unroll
    for (int j = 0; j < W; ++j) {
        u64 x = m[j];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x |= __shfl_xor(x, off, 64);
        if (lane_id() == 0) red[threadIdx.x / WAVE][j] = x;
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)W) {
        u64 o = 0;
        for (int w = 0; w < MB / WAVE; ++w) o |= red[w][threadIdx.x];
        if (o) atomicOr(&c->uf[slot][blockIdx.x % MS_NSH][threadIdx.x], o);
    }
}

__device__ __forceinline__ u64 ms_fedges(const MsCtl* c, int slot) {
    u64 t = 0;
#pragma unroll
    for (int i = 0; i < MS_NSH; ++i) t += c->fedges[slot][i][0];
    return t;
}
__device__ __forceinline__ void ms_add_fedges(MsCtl* c, int slot, u64 x) {
    atomicAdd(&c->fedges[slot][blockIdx.x % MS_NSH][0], x);
}

// Direction of level L, identical in every kernel of the level: push (top-down,
// atomicOr of the frontier masks into the targets' next masks) while the last
// frontier's out-edges are few, else pull over in-edges.
__device__ __forceinline__ bool ms_is_push(const MsCtl* c, int32_t L, u64 push_max) {
    return ms_fedges(c, (L + 2) % 3) < push_max;
}
// (done first: once level D's prep finds level D-1 empty it returns before zeroing ring slot
// (D+1) % 3, which still holds level D-2's 1, so without it level D+2 of a batch launched past
// the end would run again on archive entries this pass never wrote -- recycled memory whose
// row bitmap may hold bits past n, which the push takes as vertices: the intermittent illegal
// address of round 6, test_multi_handle, the first batch of a freshly loaded graph)
__device__ __forceinline__ bool ms_live(const MsCtl* c, int32_t L) {
    return c->done == 0 && c->active[(L + 2) % 3] != 0 && L + 1 < INT_INF;
}

template <int W>
struct Mask {
    u64 w[W];
};

template <int W>
__device__ __forceinline__ Mask<W> mload(const u64* __restrict__ p, i64 v) {
    Mask<W> m;
    if constexpr (W >= 8) {
        const ulonglong2* q = reinterpret_cast<const ulonglong2*>(p + v * W);
#pragma unroll
        for (int k = 0; k < W / 2; ++k) {
            const ulonglong2 x = q[k];
            m.w[2 * k] = x.x;
            m.w[2 * k + 1] = x.y;
        }
    } else if constexpr (W == 4) {
        const ulonglong2* q = reinterpret_cast<const ulonglong2*>(p + v * 4);
        const ulonglong2 x = q[0], y = q[1];
        m.w[0] = x.x; m.w[1] = x.y; m.w[2] = y.x; m.w[3] = y.y;
    } else if constexpr (W == 2) {
        const ulonglong2 x = reinterpret_cast<const ulonglong2*>(p)[v];
        m.w[0] = x.x; m.w[1] = x.y;
    } else {
        m.w[0] = p[v];
    }
    return m;
}
template <int W>
__device__ __forceinline__ void mstore(u64* __restrict__ p, i64 v, const Mask<W>& m) {
#pragma unroll
    for (int j = 0; j < W; ++j) p[v * W + j] = m.w[j];
}
template <int W>
__device__ __forceinline__ bool many(const Mask<W>& m) {
    u64 x = 0;
#pragma unroll
    for (int j = 0; j < W; ++j) x |= m.w[j];
    return x != 0;
}
template <int W>
__device__ __forceinline__ bool mopen(const Mask<W>& need, const Mask<W>& acc) {  // need & ~acc != 0
    u64 x = 0;
#pragma unroll
    for (int j = 0; j < W; ++j) x |= need.w[j] & ~acc.w[j];
    return x != 0;
}

__device__ __forceinline__ u64 wave_or(u64 x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x |= __shfl_xor(x, off, 64);
    return x;
}

// PJ_MS_FZ 1: a bitmap Z (one bit per vertex, "F[v] is nonzero", written whole by every
// level, a wave's 64 vertices as one word) beside the masks: the pull probes Z[u] (n / 8
// bytes, cache-resident) before the 8W-byte F[u] and skips zero rows, the push skips
// waves whose 64 vertices have no frontier, and a pull level stores only nonzero Fn rows
// (readers consult Zn first).
// MS1024: 11.72 / 11.73 -> 11.59 / 11.65 ms per batch interleaved (r4b, profiles/r04/ms_fz_r4b.txt)
#ifndef PJ_MS_FZ
#define PJ_MS_FZ 1
#endif
__device__ __forceinline__ bool zbit(const u64* __restrict__ Z, u32 u) { return (Z[u >> 6] >> (u & 63)) & 1ull; }

#ifndef PJ_MS_GPC
#define PJ_MS_GPC 8  // level-kernel workgroups per CU (MS1024: 12.8 -> 12.4 ms with MS_U 4, round 3)
#endif
// (filling the distance block here, ~0.43 ms per 512-source pass at 4.4 TB/s on the
// web-Google-shaped graph, is cheaper than writing INT_INF for the unreached pairs at
// the end of the pass, measured 0.72 ms: that loop's stores are mostly partial)
__global__ __launch_bounds__(MB) void ms_init_k(u64* __restrict__ V, u64* __restrict__ F, i64 nw,
                                                int32_t* __restrict__ dist, i64 nb_dist, MsCtl* ctl,
                                                int64_t* host_done, u64* __restrict__ Z, i64 nzw) {
    const i64 tid = (i64)blockIdx.x * MB + threadIdx.x, nth = (i64)gridDim.x * MB;
    if (tid == 0) {
        for (int i = 0; i < 3; ++i) {
            ctl->active[i] = 0;
            for (int j = 0; j < MS_NSH; ++j) ctl->fedges[i][j][0] = 0;
        }
        ctl->done = 0;
        *host_done = -1;
    }
    for (i64 i = tid; i < 3 * MS_NSH * MS_WMAX; i += nth) (&ctl->uf[0][0][0])[i] = 0;
    for (i64 i = tid; i < nw; i += nth) {
        V[i] = 0;
        F[i] = 0;
    }
    for (i64 i = tid; i < nzw; i += nth) Z[i] = 0;
    if (!dist) return;  // (the archive's expansion writes every distance)
    int4* d4 = reinterpret_cast<int4*>(dist);
    const i64 n4 = nb_dist / 4;
    for (i64 i = tid; i < n4; i += nth) d4[i] = make_int4(INT_INF, INT_INF, INT_INF, INT_INF);
    for (i64 i = n4 * 4 + tid; i < nb_dist; i += nth) dist[i] = INT_INF;
}

// one thread per source (sources may repeat: atomics on the masks)
template <typename Off>
__global__ void ms_sources_k(const int64_t* __restrict__ src, int ns, int W, i64 n, const Off* __restrict__ row,
                             u64* __restrict__ V, u64* __restrict__ F, int32_t* __restrict__ dist, MsCtl* ctl,
                             u64* __restrict__ Z) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ns) return;
    const int64_t s = src[i];
    if (s < 0 || s >= n) return;
    atomicOr(&V[s * W + (i >> 6)], 1ull << (i & 63));
    atomicOr(&F[s * W + (i >> 6)], 1ull << (i & 63));
    atomicOr(&Z[s >> 6], 1ull << (s & 63));
    if (dist) dist[(i64)i * n + s] = 0;
    ctl->active[2] = 1;  // "level -1" found the sources
    atomicOr(&ctl->uf[2][0][i >> 6], 1ull << (i & 63));
    atomicAdd(&ctl->fedges[2][0][0], (u64)(row[s + 1] - row[s]));
}

// First kernel of level L: ends the pass when level L-1 found nothing, zeroes
// the ring slots level L+1 writes, and (push levels) clears the output masks.
template <int W>
__global__ __launch_bounds__(MB) void ms_prep_k(i64 n, u64* __restrict__ Fn, int32_t L, u64 push_max, MsCtl* ctl,
                                                int64_t* host_done) {
    if (!ms_live(ctl, L)) {
        if (blockIdx.x == 0 && threadIdx.x == 0 && !ctl->done) {
            ctl->done = 1;
            *host_done = L;
        }
        return;
    }
    if (blockIdx.x == 0 && threadIdx.x < MS_NSH) {
        if (threadIdx.x == 0) ctl->active[(L + 1) % 3] = 0;
        ctl->fedges[(L + 1) % 3][threadIdx.x][0] = 0;
    }
    if (PJ_MS_UF && blockIdx.x == 0)
        for (int i = threadIdx.x; i < MS_NSH * MS_WMAX; i += MB) (&ctl->uf[(L + 1) % 3][0][0])[i] = 0;
    if (!ms_is_push(ctl, L, push_max)) return;
    ulonglong2* p = reinterpret_cast<ulonglong2*>(Fn);
    const i64 n2 = n * W / 2;
    for (i64 i = (i64)blockIdx.x * MB + threadIdx.x; i < n2; i += (i64)gridDim.x * MB) p[i] = make_ulonglong2(0, 0);
    if ((n * W) & 1) {
        if (blockIdx.x == 0 && threadIdx.x == 0) Fn[n * W - 1] = 0;
    }
}

// distances of newly reached (source, v) pairs: loop over the sources any lane
// reached (wave-uniform), so each store is one coalesced run of the wave's 64
// consecutive vertices in that source's row
template <int W>
__device__ __forceinline__ void ms_write_dist(const Mask<W>& newb, int32_t* __restrict__ dist, i64 n, i64 v,
                                              int32_t val) {
    if (!dist) return;  // (archive mode: ms_expand_k writes them)
#pragma unroll
    for (int j = 0; j < W; ++j) {
        u64 un = wave_or(newb.w[j]);
        while (un) {
            const int sbit = __ffsll((long long)un) - 1;
            un &= un - 1;
            if ((newb.w[j] >> sbit) & 1ull) dist[(i64)(sbit + 64 * j) * n + v] = val;
        }
    }
}

// Push level: every vertex u with a nonzero frontier mask ORs it into the next
// mask of each out-neighbour (no-return atomics); ms_fin_k then keeps the bits
// not yet in V.
template <typename Off, int W>
__global__ __launch_bounds__(MB) void ms_push_k(i64 n, const Off* __restrict__ row, const u32* __restrict__ col,
                                                const u64* __restrict__ F, u64* __restrict__ Fn, int32_t L,
                                                u64 push_max, const MsCtl* ctl, const u64* __restrict__ Z) {
    if (!ms_live(ctl, L) || !ms_is_push(ctl, L, push_max)) return;
    const int lane = lane_id();
    const i64 nwaves = (i64)gridDim.x * (MB / WAVE);
    for (i64 base = ((i64)blockIdx.x * (MB / WAVE) + wave_id()) * 64; base < n; base += nwaves * 64) {
        const i64 u = base + lane;
        Mask<W> f{};
        if (PJ_MS_FZ) {
            const u64 zw = Z[base >> 6];
            if (!zw) continue;
            if (u < n && ((zw >> lane) & 1ull)) f = mload<W>(F, u);
        } else if (u < n) {
            f = mload<W>(F, u);
        }
        const bool act = many<W>(f);
        if (!__ballot(act)) continue;
        Off b = 0, e = 0;
        if (act) {
            b = row[u];
            e = row[u + 1];
        }
        const Off lim = (e - b > (Off)MS_SERIAL) ? b + (Off)MS_SERIAL : e;
        for (Off k = b; k < lim; ++k) {
            const u32 v = col[k];
#pragma unroll
            for (int j = 0; j < W; ++j)
                if (f.w[j]) atomicOr(&Fn[(i64)v * W + j], f.w[j]);
        }
        u64 open = __ballot(lim < e);
        while (open) {
            const int l = __ffsll((long long)open) - 1;
            open &= open - 1;
            const Off kb = __shfl(lim, l, 64), ke = __shfl(e, l, 64);
            Mask<W> fl;
#pragma unroll
            for (int j = 0; j < W; ++j) fl.w[j] = __shfl(f.w[j], l, 64);
            for (Off kk = kb + lane; kk < ke; kk += WAVE) {
                const u32 v = col[kk];
#pragma unroll
                for (int j = 0; j < W; ++j)
                    if (fl.w[j]) atomicOr(&Fn[(i64)v * W + j], fl.w[j]);
            }
        }
    }
}

template <typename Off, int W>
__global__ __launch_bounds__(MB) void ms_fin_k(i64 n, const Off* __restrict__ row, u64* __restrict__ V,
                                               u64* __restrict__ Fn, int32_t* __restrict__ dist, int32_t L,
                                               Mask<W> smask, u64 push_max, MsCtl* ctl, u64* __restrict__ Zn) {
    if (!ms_live(ctl, L) || !ms_is_push(ctl, L, push_max)) return;
    __shared__ u64 red[MB / WAVE];
    __shared__ u64 ured[MB / WAVE][MS_WMAX];
    const int lane = lane_id();
    u64 found_any = 0, fe = 0;
    u64 ufl[W] = {};
    const i64 nwaves = (i64)gridDim.x * (MB / WAVE);
    for (i64 base = ((i64)blockIdx.x * (MB / WAVE) + wave_id()) * 64; base < n; base += nwaves * 64) {
        const i64 v = base + lane;
        Mask<W> fn{};
        if (v < n) fn = mload<W>(Fn, v);
        const bool act = many<W>(fn);
        if (!__ballot(act)) {
            if (PJ_MS_FZ && lane == 0) Zn[base >> 6] = 0;
            continue;
        }
        Mask<W> newb{};
        bool anynew = false;
        if (act) {
            const Mask<W> vv = mload<W>(V, v);
            Mask<W> nv;
#pragma unroll
            for (int j = 0; j < W; ++j) {
                newb.w[j] = fn.w[j] & ~vv.w[j] & smask.w[j];
                nv.w[j] = vv.w[j] | newb.w[j];
                anynew |= newb.w[j] != 0;
            }
            mstore<W>(Fn, v, newb);
            if (anynew) {
                mstore<W>(V, v, nv);
                fe += (u64)(row[v + 1] - row[v]);
            }
        }
        found_any |= anynew ? 1ull : 0ull;
        if (PJ_MS_FZ) {
            const u64 zb = __ballot(anynew);
            if (lane == 0) Zn[base >> 6] = zb;
        }
        if (PJ_MS_UF)
#pragma unroll
            for (int j = 0; j < W; ++j) ufl[j] |= newb.w[j];
        ms_write_dist<W>(newb, dist, n, v, L + 1);
    }
    if (PJ_MS_UF) ms_uf_add<W>(ctl, L % 3, ufl, ured);
    fe = block_sum<MB / WAVE>(fe, red);
    if (threadIdx.x == 0 && fe) ms_add_fedges(ctl, L % 3, fe);
    if (__ballot(found_any != 0) && lane == 0) ctl->active[L % 3] = 1;
}

template <typename Off, int W>
__global__ __launch_bounds__(MB) void ms_level_k(i64 n, const Off* __restrict__ crow, const u32* __restrict__ ccol,
                                                 const Off* __restrict__ row, u64* __restrict__ V,
                                                 const u64* __restrict__ F, u64* __restrict__ Fn,
                                                 int32_t* __restrict__ dist, int32_t L, Mask<W> smask,
                                                 u64 push_max, MsCtl* ctl, const u64* __restrict__ Z,
                                                 u64* __restrict__ Zn) {
    // level L computes distance L+1 from the frontier of level L-1 (pull form)
    if (!ms_live(ctl, L) || ms_is_push(ctl, L, push_max)) return;
    __shared__ u64 red[MB / WAVE];
    __shared__ u64 ured[MB / WAVE][MS_WMAX];
    const int lane = lane_id();
    u64 found_any = 0, fe = 0;
    u64 ufl[W] = {}, act[W];
    if (PJ_MS_UF) ms_uf_read<W>(ctl, (L + 2) % 3, act);
    const i64 nwaves = (i64)gridDim.x * (MB / WAVE);
    for (i64 base = ((i64)blockIdx.x * (MB / WAVE) + wave_id()) * 64; base < n; base += nwaves * 64) {
        const i64 v = base + lane;
        const bool inr = v < n;
        Mask<W> vv, need;
        if (inr) vv = mload<W>(V, v);
#pragma unroll
        for (int j = 0; j < W; ++j) {
            if (!inr) vv.w[j] = ~0ull;
            need.w[j] = ~vv.w[j] & smask.w[j];  // sources of this batch that have not reached v
            if (PJ_MS_UF) need.w[j] &= act[j];  // ... and whose search is still running
        }
        const bool hasneed = many<W>(need);
        if (__ballot(hasneed) == 0) {
            if (PJ_MS_FZ) {
                if (lane == 0) Zn[base >> 6] = 0;
            } else if (inr) {
                mstore<W>(Fn, v, Mask<W>{});
            }
            continue;
        }
        Off b = 0, e = 0;
        if (hasneed) {
            b = crow[v];
            e = crow[v + 1];
        }
        Mask<W> acc{};
        Off k = b;
        const Off lim = (e - b > (Off)MS_SERIAL) ? b + (Off)MS_SERIAL : e;
        bool go = hasneed && k < lim;
        while (__ballot(go)) {
            if (go) {
                // MS_U in-edges per step: their ids, then their masks, as independent loads
                u32 u[MS_U];
#pragma unroll
                for (int q = 0; q < MS_U; ++q) u[q] = (k + (Off)q < lim) ? ccol[k + q] : 0u;
                bool z[MS_U];
#pragma unroll
                for (int q = 0; q < MS_U; ++q) z[q] = (k + (Off)q < lim) && (!PJ_MS_FZ || zbit(Z, u[q]));
                Mask<W> f[MS_U];
#pragma unroll
                for (int q = 0; q < MS_U; ++q) {
                    if (z[q]) f[q] = mload<W>(F, u[q]);
                    else f[q] = Mask<W>{};
                }
#pragma unroll
                for (int q = 0; q < MS_U; ++q)
#pragma unroll
                    for (int j = 0; j < W; ++j) acc.w[j] |= f[q].w[j];
                k = (lim - k > (Off)MS_U) ? k + (Off)MS_U : lim;
                go = mopen<W>(need, acc) && k < lim;
            }
        }
        u64 open = __ballot(mopen<W>(need, acc) && k < e);
        while (open) {
            const int l = __ffsll((long long)open) - 1;
            open &= open - 1;
            const Off kb = __shfl(k, l, 64), ke = __shfl(e, l, 64);
            Mask<W> want, got;
#pragma unroll
            for (int j = 0; j < W; ++j) {
                want.w[j] = __shfl(need.w[j], l, 64);
                got.w[j] = __shfl(acc.w[j], l, 64);
            }
            // two 64-edge chunks per step (independent loads), one wave reduction
            for (Off kk = kb; kk < ke && mopen<W>(want, got); kk += 2 * WAVE) {
                const Off k0 = kk + lane, k1 = kk + WAVE + lane;
                const u32 u0 = k0 < ke ? ccol[k0] : 0u, u1 = k1 < ke ? ccol[k1] : 0u;
                const bool z0 = k0 < ke && (!PJ_MS_FZ || zbit(Z, u0)), z1 = k1 < ke && (!PJ_MS_FZ || zbit(Z, u1));
                Mask<W> x{}, y{};
                if (z0) x = mload<W>(F, u0);
                if (z1) y = mload<W>(F, u1);
#pragma unroll
                for (int j = 0; j < W; ++j) got.w[j] |= wave_or(x.w[j] | y.w[j]);
            }
            if (lane == l) acc = got;
        }
        Mask<W> newb;
        bool anynew = false;
#pragma unroll
        for (int j = 0; j < W; ++j) {
            newb.w[j] = acc.w[j] & need.w[j];
            anynew |= newb.w[j] != 0;
        }
        if (inr) {
            if (!PJ_MS_FZ || anynew) mstore<W>(Fn, v, newb);
            if (anynew) {
                Mask<W> nv;
#pragma unroll
                for (int j = 0; j < W; ++j) nv.w[j] = vv.w[j] | newb.w[j];
                mstore<W>(V, v, nv);
            }
        }
        found_any |= anynew ? 1ull : 0ull;
        if (PJ_MS_FZ) {
            const u64 zb = __ballot(anynew);
            if (lane == 0) Zn[base >> 6] = zb;
        }
        if (PJ_MS_UF)
#pragma unroll
            for (int j = 0; j < W; ++j) ufl[j] |= newb.w[j];
        if (anynew) fe += (u64)(row[v + 1] - row[v]);
        ms_write_dist<W>(newb, dist, n, v, L + 1);
    }
    if (PJ_MS_UF) ms_uf_add<W>(ctl, L % 3, ufl, ured);
    fe = block_sum<MB / WAVE>(fe, red);
    if (threadIdx.x == 0 && fe) ms_add_fedges(ctl, L % 3, fe);
    if (__ballot(found_any != 0) && lane == 0) ctl->active[L % 3] = 1;
}

}  // namespace

// The distance block from the level archive: entries [0, nlev), entry a holding at row v
// the sources that reached v at level a (valid where bit v of its row bitmap is set). A
// wave takes 64 consecutive vertices; per chunk of up to 8 mask words (one 64-byte line of
// a row) it ORs each lane's entries into the five bit planes of the level number
// (MS_LCAP <= 32), then stores source by source 64 consecutive distances (INT_INF where no
// entry holds the bit), streaming (nontemporal) stores. (A word at a time re-fetched a
// row's line for every word once the distance stores had pushed it out of L2: 5.4 GB of
// traffic per 512-source pass against ~2.3 GB of rows and distances, profiles/r05/ms1024_pmc_w8_r5q.txt.)
constexpr int MS_LCAP = 32;  // archive entries at most (the level number in 5 bit planes)
#ifndef PJ_MS_JC
#define PJ_MS_JC 8  // mask words per expansion chunk
#endif
template <int W>
__global__ __launch_bounds__(MB) void ms_expand_k(i64 n, const u64* __restrict__ arch, const u64* __restrict__ zarch,
                                                  i64 nzw, int nlev, int ns, int32_t* __restrict__ dist) {
    const int lane = lane_id();
    const i64 nwaves = (i64)gridDim.x * (MB / WAVE);
    for (i64 base = ((i64)blockIdx.x * (MB / WAVE) + wave_id()) * 64; base < n; base += nwaves * 64) {
        const i64 v = base + lane;
        const bool inr = v < n;
        u32 zm = 0;  // the entries holding a row for v
        for (int a = 0; a < nlev; ++a)
            if ((zarch[(i64)a * nzw + (base >> 6)] >> lane) & 1ull) zm |= 1u << a;
        constexpr int JC = W < PJ_MS_JC ? W : PJ_MS_JC;
#pragma unroll
        for (int j0 = 0; j0 < W; j0 += JC) {
            if (64 * j0 >= ns) break;
            u64 any[JC], p0[JC], p1[JC], p2[JC], p3[JC], p4[JC];
#pragma unroll
            for (int j = 0; j < JC; ++j) any[j] = p0[j] = p1[j] = p2[j] = p3[j] = p4[j] = 0;
            for (u32 m = zm; m; m &= m - 1) {
                const int a = __ffs((int)m) - 1;
                u64 x[JC];
#pragma unroll
                for (int j = 0; j < JC; ++j) x[j] = arch[((i64)a * n + v) * W + j0 + j];
#pragma unroll
                for (int j = 0; j < JC; ++j) {
                    any[j] |= x[j];
                    if (a & 1) p0[j] |= x[j];
                    if (a & 2) p1[j] |= x[j];
                    if (a & 4) p2[j] |= x[j];
                    if (a & 8) p3[j] |= x[j];
                    if (a & 16) p4[j] |= x[j];
                }
            }
#pragma unroll
            for (int j = 0; j < JC; ++j) {
                const int nb = min(64, ns - 64 * (j0 + j));
                for (int b = 0; b < nb; ++b) {
                    const int32_t lv =
                        (int32_t)(((p0[j] >> b) & 1ull) | (((p1[j] >> b) & 1ull) << 1) | (((p2[j] >> b) & 1ull) << 2) |
                                  (((p3[j] >> b) & 1ull) << 3) | (((p4[j] >> b) & 1ull) << 4));
                    if (inr)
                        __builtin_nontemporal_store(((any[j] >> b) & 1ull) ? lv : INT_INF,
                                                    dist + (i64)(64 * (j0 + j) + b) * n + v);
                }
            }
        }
    }
}

// One pass in flight: its masks, distance block, control block, stream and events.
// Slot 0 runs on the ctx stream; further slots (option ms_streams) own a stream, and
// passes of one batch run on the slots at once, one host thread each: a pass is a chain
// of latency-bound levels, so two of them interleave on the CUs.
struct MsSlot {
    DevBuf<u64> V;
    DevBuf<u64> arch;   // level archive: lcap entries of n x W words (the frontier masks F, Fn of
                        // each level are two of its entries)
    DevBuf<u64> zarch;  // (PJ_MS_FZ) each entry's nonzero-row bitmap, nzw words
    int lcap = 0;
    DevBuf<int32_t> dist;
    DevBuf<int64_t> src;
    DevBuf<MsCtl> ctl;
    int64_t* host = nullptr;
    int32_t last_levels = 0;  // level iterations the previous pass used: sizes the first batch
    hipStream_t s = nullptr;
    bool own_stream = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    ~MsSlot() {
        if (host) (void)hipHostFree(host);
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (own_stream && s) (void)hipStreamDestroy(s);
    }
};

struct MsWork {
    int W = 0;  // words per vertex mask of the allocation
    std::vector<std::unique_ptr<MsSlot>> slots;
};

void delete_ms_work(MsWork* p) { delete p; }

template <typename Off, int W>
static void ms_pass(Graph& g, MsSlot& w, const int64_t* sources, int ns, double* kernel_ms, i64* levels) {
    hipStream_t s = w.s;
    const i64 n = g.n;
    const Off* crow = static_cast<const Off*>(g.crow_ptr());
    const u32* ccol = pull_ccol(g);
    PJ_HIP(hipMemcpyAsync(w.src.p, sources, sizeof(int64_t) * (size_t)ns, hipMemcpyHostToDevice, s));
    int64_t* host_dev = nullptr;
    PJ_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&host_dev), w.host, 0));
    Mask<W> smask{};  // bits of the valid sources of this batch
    bool any = false;
    for (int i = 0; i < ns; ++i)
        if (sources[i] >= 0 && sources[i] < n) {
            smask.w[i >> 6] |= 1ull << (i & 63);
            any = true;
        }
    const unsigned grid = (unsigned)g.ctx->cu_count * (unsigned)PJ_MS_GPC;
    const Off* row = static_cast<const Off*>(g.row_ptr());
    const u32* col = g.col.p;
    // push while the frontier's out-edges are below nnz / ms_alpha (0: never)
    const u64 push_max = g.ms_alpha > 0 ? (u64)((double)g.nnz / g.ms_alpha) : 0ull;
    const i64 nzw = (n + 63) / 64 + 1;
    auto entry = [&](int a) { return w.arch.p + (size_t)a * (size_t)n * W; };
    auto zentry = [&](int a) { return w.zarch.p + (size_t)a * (size_t)nzw; };
    // archive mode while level L's output entry L + 1 exists; then (a pass deeper than the
    // archive, or no archive) the levels store their distances and F / Fn alternate between
    // the last two entries
    bool archive = PJ_MS_FZ && w.lcap > 2;
    PJ_HIP(hipEventRecord(w.ev0, s));
    ms_init_k<<<grid_for(std::max<i64>(n * W, archive ? 0 : (i64)ns * n / 4), MB, (unsigned)g.ctx->cu_count * 8u), MB,
                0, s>>>(w.V.p, entry(0), n * W, archive ? nullptr : w.dist.p, (i64)ns * n, w.ctl.p, host_dev, zentry(0),
                        (n + 63) / 64);
    PJ_LAUNCH_CHECK();
    ms_sources_k<Off><<<(ns + 255) / 256, 256, 0, s>>>(w.src.p, ns, W, n, row, w.V.p, entry(0),
                                                    archive ? nullptr : w.dist.p, w.ctl.p, zentry(0));
    PJ_LAUNCH_CHECK();
    int32_t L = 0;
    // first batch: the previous pass's levels (passes over one graph need about as many);
    // then 2, 4, 8, ... (each idle level costs its 2-4 launches inside the timed region)
    int batch = w.last_levels > 0 ? w.last_levels : 16;
    int next = 2;
    int fa = 0, fb = 1;  // entries of F and Fn (direct mode: alternating)
    for (;;) {
        for (int i = 0; i < batch && L < INT_INF; ++i, ++L) {
            if (archive) {
                if (L + 1 >= w.lcap) break;  // (the archive is full: the host decides below)
                fa = L;
                fb = L + 1;
            }
            u64 *F = entry(fa), *Fn = entry(fb), *Z = zentry(fa), *Zn = zentry(fb);
            int32_t* dst = archive ? nullptr : w.dist.p;
            ms_prep_k<W><<<grid, MB, 0, s>>>(n, Fn, L, push_max, w.ctl.p, host_dev);
            PJ_LAUNCH_CHECK();
            ms_level_k<Off, W><<<grid, MB, 0, s>>>(n, crow, ccol, row, w.V.p, F, Fn, dst, L, smask, push_max,
                                                   w.ctl.p, Z, Zn);
            PJ_LAUNCH_CHECK();
            if (push_max) {
                ms_push_k<Off, W><<<grid, MB, 0, s>>>(n, row, col, F, Fn, L, push_max, w.ctl.p, Z);
                PJ_LAUNCH_CHECK();
                ms_fin_k<Off, W><<<grid, MB, 0, s>>>(n, row, w.V.p, Fn, dst, L, smask, push_max, w.ctl.p, Zn);
                PJ_LAUNCH_CHECK();
            }
            if (!archive) std::swap(fa, fb);
        }
        PJ_HIP(hipStreamSynchronize(s));
        const int64_t done = *(volatile int64_t*)w.host;
        if (archive && (done >= 0 || !any)) {
            // level done - 1 found nothing: entries [0, done] hold every arrival
            const int nlev = any ? (int)done + 1 : 1;
            ms_expand_k<W><<<grid, MB, 0, s>>>(n, w.arch.p, w.zarch.p, nzw, nlev, ns, w.dist.p);
            PJ_LAUNCH_CHECK();
            break;
        }
        if (done >= 0 || L >= INT_INF || !any) break;
        if (archive && L + 1 >= w.lcap) {
            // the archive is full and the pass goes on: expand it (every distance, INT_INF for
            // the pairs not reached yet), then store the later levels' distances directly
            ms_expand_k<W><<<grid, MB, 0, s>>>(n, w.arch.p, w.zarch.p, nzw, w.lcap, ns, w.dist.p);
            PJ_LAUNCH_CHECK();
            archive = false;
            fa = L;      // level L reads entry L (= lcap - 1) ...
            fb = L - 1;  // ... and writes over entry L - 1, already expanded
        }
        batch = next;
        next = next < 1024 ? next * 2 : next;
    }
    PJ_HIP(hipEventRecord(w.ev1, s));
    PJ_HIP(hipEventSynchronize(w.ev1));
    float ms = 0.f;
    PJ_HIP(hipEventElapsedTime(&ms, w.ev0, w.ev1));
    *kernel_ms += ms;
    const i64 lv = (i64)*(volatile int64_t*)w.host;
    if (any && lv >= 0) w.last_levels = (int32_t)lv + 1;
    *levels = std::max<i64>(*levels, lv);
}

template <typename Off>
static void ms_pass_w(int W, Graph& g, MsSlot& w, const int64_t* sources, int ns, double* kernel_ms, i64* levels) {
    if (W == 16) ms_pass<Off, 16>(g, w, sources, ns, kernel_ms, levels);
    else if (W == 8) ms_pass<Off, 8>(g, w, sources, ns, kernel_ms, levels);
    else if (W == 4) ms_pass<Off, 4>(g, w, sources, ns, kernel_ms, levels);
    else if (W == 2) ms_pass<Off, 2>(g, w, sources, ns, kernel_ms, levels);
    else ms_pass<Off, 1>(g, w, sources, ns, kernel_ms, levels);
}

// Device bytes of one pass slot: the distance block (64 W x n int32), the masks V (W words
// per vertex) and the level archive (lcap entries of W words per vertex and a row bitmap).
static double ms_slot_bytes(i64 n, int W, int lcap) {
    return (double)n * (64.0 * W * 4.0 + (1.0 + lcap) * W * 8.0) + lcap * ((double)n / 8.0 + 16.0);
}
// Archive entries of a slot: MS_LCAP, fewer when the slot would exceed MS_BUDGET / 2 (the
// later levels of a deeper pass store their distances directly); 2 = no archive.
static int ms_lcap(i64 n, int W);
constexpr double MS_BUDGET = 16e9;  // device bytes all slots of a batch may hold
// Pass width: the fewest words that hold the batch, at most MS_WMAX (g.ms_width
// caps it), with one slot's buffers within the budget.
static int ms_words(const Graph& g, int n_src) {
    int W = 1;
    const int cap = g.ms_width > 0 ? std::min(g.ms_width, MS_WMAX) : MS_WDEF;
    while (W < cap && 64 * W < n_src && ms_slot_bytes(g.n, 2 * W, 2) <= MS_BUDGET) W *= 2;
    return W;
}
static int ms_lcap(i64 n, int W) {
    if (!PJ_MS_FZ) return 2;  // (the archive needs the row bitmaps)
    int lc = MS_LCAP;
    while (lc > 2 && ms_slot_bytes(n, W, lc) > MS_BUDGET / 2) --lc;
    return lc;
}

static void ms_slot_alloc(Graph& g, MsSlot& sl, int W, int lcap, bool own_stream) {
    const size_t n = (size_t)g.n;
    sl.V.alloc(n ? n * W : 1);
    sl.lcap = lcap;
    sl.arch.alloc(n ? (size_t)lcap * n * W : 1);
    sl.zarch.alloc((size_t)lcap * ((n + 63) / 64 + 1));
    sl.dist.alloc(n ? 64 * W * n : 1);
    sl.src.alloc(64 * W);
    sl.ctl.alloc(1);
    PJ_HIP(hipHostMalloc(reinterpret_cast<void**>(&sl.host), sizeof(int64_t), hipHostMallocMapped));
    PJ_HIP(hipEventCreate(&sl.ev0));
    PJ_HIP(hipEventCreate(&sl.ev1));
    if (own_stream) {
        PJ_HIP(hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking));
        sl.own_stream = true;
    }
}

void msbfs_each(Graph& g, const int64_t* sources, int n_src, const MsPassFn& on_pass) {
    (void)pull_ccol(g);  // (built here, once, before the slots' host threads read it)
    const int W = ms_words(g, n_src);
    const int per = 64 * W;
    const int npass = (n_src + per - 1) / per;
    int nslots = std::max(1, std::min(g.ms_streams, npass));
    if (!g.ms_work || g.ms_work->W < W) {
        g.ms_work.reset(new MsWork());
        g.ms_work->W = W;
    }
    MsWork& mw = *g.ms_work;
    // Every slot holds a whole pass (ms_slot_bytes: ~3.8 GB at n = 916K, W = 8, with a
    // 32-entry archive): the slots in flight stay within MS_BUDGET, and a slot beyond the
    // first is only added while it takes at most half the free device memory; if its
    // allocation still fails, the batch runs on the slots it has.
    const int lcap = ms_lcap(g.n, mw.W);
    const double sb = ms_slot_bytes(g.n, mw.W, lcap);
    while (nslots > 1 && (double)nslots * sb > MS_BUDGET) --nslots;
    if (mw.slots.empty()) {
        std::unique_ptr<MsSlot> sl(new MsSlot());
        ms_slot_alloc(g, *sl, mw.W, lcap, false);
        mw.slots.push_back(std::move(sl));
    }
    while ((int)mw.slots.size() < nslots) {
        const size_t fr = dev_free_bytes();  // (libpj's idle cached blocks count as free)
        if (sb > 0.5 * (double)fr) break;
        std::unique_ptr<MsSlot> sl(new MsSlot());
        try {
            ms_slot_alloc(g, *sl, mw.W, lcap, true);
        } catch (const Error&) {
            (void)hipGetLastError();
            break;
        }
        mw.slots.push_back(std::move(sl));
    }
    nslots = std::min(nslots, (int)mw.slots.size());
    mw.slots[0]->s = g.ctx->stream;  // (pj_set_stream may change it)
    auto t0 = std::chrono::steady_clock::now();
    pj_stats st{};
    double kms = 0;
    i64 levels = 0;
    auto run = [&](MsSlot& sl, int off, double* k, i64* lv) {
        const int ns = std::min(per, n_src - off);
        if (g.off64) ms_pass_w<u64>(W, g, sl, sources + off, ns, k, lv);
        else ms_pass_w<u32>(W, g, sl, sources + off, ns, k, lv);
        return ns;
    };
    if (nslots == 1) {
        for (int off = 0; off < n_src; off += per) {
            const int ns = run(*mw.slots[0], off, &kms, &levels);
            if (on_pass) on_pass(off, ns, mw.slots[0]->dist.p);
        }
    } else {
        PJ_HIP(hipStreamSynchronize(g.ctx->stream));
        std::atomic<int> next{0};
        std::mutex mu;
        std::vector<std::exception_ptr> errs((size_t)nslots);
        auto work = [&](int k) {
            try {
                PJ_HIP(hipSetDevice(g.ctx->device));
                MsSlot& sl = *mw.slots[(size_t)k];
                for (int p; (p = next.fetch_add(1)) < npass;) {
                    double km = 0;
                    i64 lv = 0;
                    const int off = p * per;
                    const int ns = run(sl, off, &km, &lv);
                    std::lock_guard<std::mutex> lk(mu);
                    kms += km;
                    levels = std::max(levels, lv);
                    if (on_pass) on_pass(off, ns, sl.dist.p);
                }
            } catch (...) {
                errs[(size_t)k] = std::current_exception();
                next.store(npass);
            }
        };
        std::vector<std::thread> th;
        for (int k = 1; k < nslots; ++k) th.emplace_back(work, k);
        work(0);
        for (auto& t : th) t.join();
        for (auto& e : errs)
            if (e) std::rethrow_exception(e);
    }
    st.kernel_ms = kms;
    st.levels = levels;
    st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    g.stats = st;
    // the per-source result of the last pass's final source is not kept in g.dist
}

void msbfs_solve(Graph& g, const int64_t* sources, int n_src, int32_t* dist_out) {
    const size_t n = (size_t)g.n;
    MsPassFn copy;
    if (dist_out && n)
        copy = [&](int off, int ns, const int32_t* rows) {
            PJ_HIP(hipMemcpy(dist_out + (size_t)off * n, rows, sizeof(int32_t) * (size_t)ns * n, hipMemcpyDeviceToHost));
        };
    msbfs_each(g, sources, n_src, copy);
}

}  // namespace pj
