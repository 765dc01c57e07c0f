// delta.hip — weighted SSSP: direction-optimizing delta-stepping over bitmap
// frontiers.
//
// Generalises the reference's label-correcting relaxation (extract_local_pq
// :226-278, apply loop :557-573) to integer weights >= 0, keeping its output
// contract: candidates >= INT_INF are discarded and the
// result is the true distance when it is < INT_INF. The reference settles one
// vertex per heap pop; here a whole distance band [lo, hi = lo + delta) is
// settled at once (Meyer & Sanders' delta-stepping). The solver runs on the
// degree-ordered relabeled copy of the graph (relabel.hip); rows are sorted by
// weight, so the light edges (w < delta) of v are the prefix of its row, packed
// per delta into a light CSR, and the heavy ones the rest of the row.
//
// Per band: light rounds (push, tile-dense push or pull, decided on the device
// per round) until the band's frontier is empty, then one heavy step (push of the
// members' heavy suffixes, or a pull by the unsettled vertices fused with the next
// band's selection). The host reads the counters once per batch of light rounds and
// once per band (the analogue of the reference's termination allreduce, :579-593).
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <functional>
#include <mutex>
#include <thread>

#include "lb.h"

namespace pj {

namespace {

constexpr int DB = 256;             // relax workgroup
#ifndef PJ_COHERENT_CHECK
#define PJ_COHERENT_CHECK 1
#endif
// The pre-check of dist[t] before the atomicMin: per-XCD L2s are not coherent
// with each other, so a plain load can return a stale (higher) value for a hot
// target and let every relaxation into it through to the atomic, which then
// serialises at ~88 per us per address. An agent-scope load (sc1) sees the
// value the atomics left.
__device__ __forceinline__ int32_t dist_now(const int32_t* p) {
    if (PJ_COHERENT_CHECK) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return *p;
}

__global__ void d_source_k(i64 s, int32_t* __restrict__ dist) { dist[s] = 0; }

#ifndef PJ_V2_GPC
#define PJ_V2_GPC 24  // swept 4..48 on s26w: 8 -> 24 is ~+4% (profiles/r01/v2_grid_sweep.txt)
#endif
#ifndef PJ_V2_GPC_PULL
#define PJ_V2_GPC_PULL PJ_V2_GPC
#endif
// distances back to input ids: out[v] = dist'[inv[v]] (INT_INF past n_scan)
__global__ void unlabel_k(const u32* __restrict__ inv, const int32_t* __restrict__ dl, i64 n, i64 n_scan,
                          int32_t* __restrict__ out) {
    // (bound by the gathered distance lines: 8 ids per thread step measured 192.5 against
    // 200.6 us at s26, profiles/r03/experiments_r3ab_select.txt)
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x) {
        const u32 x = inv[v];
        out[v] = (i64)x < n_scan ? dl[x] : INT_INF;
    }
}

// Serial probes of a weight-sorted row, PU edges per step with independent
// loads (the probes are latency-bound; one edge per step leaves the memory
// system idle). Weights ascend along the row, so once lo + w >= cur for an
// edge, that edge and every later one are useless: the step returns true.
#ifndef PJ_PU
#define PJ_PU 2  // swept 1..8 with the 24-per-CU grid: 2 is ~+3% over 4 (profiles/r01/v2_unroll_sweep.txt)
#endif
constexpr int PU = PJ_PU;
// Edge records read as u64 (col | w << 32): the interleaved CSR (cw), or the
// light CSR packed in 32 bits (col | w << cb, when every light weight fits 32 - cb
// bits and every id cb bits: half the bytes per light edge).
// Or split: u32 ids (e32) beside u8 weights (w8), 5 bytes per edge, when every
// weight fits 8 bits (the heavy pull and the tail read the whole CSR this way).
struct ESrc {
    const u64* e64;
    const u32* e32;  // non-null: packed records, or the ids when w8 is set
    u32 cb;
    const uint8_t* w8;
};
__device__ __forceinline__ u64 eat(const ESrc& s, u64 k) {
    if (s.w8) return (u64)s.e32[k] | ((u64)s.w8[k] << 32);
    if (s.e32) {
        const u32 x = s.e32[k];
        return (u64)(x & ((1u << s.cb) - 1u)) | ((u64)(x >> s.cb) << 32);
    }
    return s.e64[k];
}

// A pull takes its candidate from every in-neighbour u with dist[u] < hi, one dist probe
// (round 5), instead of first testing u's bit in the round's frontier (light) or the band's
// members (heavy) and reading dist[u] only for a set bit. Exact: every u with dist[u] < hi
// outside that set has already relaxed its edges of this kind at its current distance (a
// lowered vertex re-enters the frontier), so dist[u] + w >= dist[v] and it never lowers v's
// running best. k26w 450.6 -> 487.0 GTEPS interleaved (profiles/r05/nofin_ab_r5a.txt); the
// bits probed first on sparse rounds only measured 1-2% slower (ab_fbits_r5i.txt), and a
// per-round byte map of the frontier's distances 7% slower (its build launches cost more
// than the pulls gained, ab_fmap_r5h.txt).
// the candidate distance u offers through a pulled edge (INT_INF = none)
__device__ __forceinline__ int32_t pull_src(const int32_t* __restrict__ dist, u32 u, int32_t hi) {
    const int32_t d = dist[u];
    return d < hi ? d : INT_INF;
}
template <typename Off, typename E>
__device__ __forceinline__ bool pull_step_dist(const E ed, const int32_t* __restrict__ dist, Off& k, Off lim,
                                               int32_t lo, int32_t hi, int32_t& cur) {
    u32 w[PU], u[PU];
    bool ok[PU];
#pragma unroll
    for (int j = 0; j < PU; ++j) {
        ok[j] = k + (Off)j < lim;
        const u64 x = ok[j] ? eat(ed, (u64)(k + j)) : 0ull;
        w[j] = (u32)(x >> 32);
        u[j] = (u32)x;
    }
    bool stop = false;
    int nv = 0;
#pragma unroll
    for (int j = 0; j < PU; ++j) {
        if (ok[j] && (long long)lo + w[j] >= (long long)cur) stop = true;
        ok[j] = ok[j] && !stop;
        nv += ok[j];
    }
    int32_t du[PU];
#pragma unroll
    for (int j = 0; j < PU; ++j) du[j] = ok[j] ? dist[u[j]] : INT_INF;
#pragma unroll
    for (int j = 0; j < PU; ++j) du[j] = du[j] < hi ? du[j] : INT_INF;
#pragma unroll
    for (int j = 0; j < PU; ++j)
        if (du[j] < INT_INF) {
            const long long nd = (long long)du[j] + w[j];
            if (nd < cur) cur = (int32_t)nd;
        }
    k += (Off)nv;
    return stop;
}

// the same step probing a byte map (dist - lo of the probed set, 0xFF = not in it): the heavy
// pull's map is 1/4 of dist and stays in the Infinity Cache (v2_hmap_k)
template <typename Off, typename E>
__device__ __forceinline__ bool pull_step_map(const E ed, const uint8_t* __restrict__ map, Off& k, Off lim,
                                              int32_t lo, int32_t& cur) {
    u32 w[PU], u[PU];
    bool ok[PU];
#pragma unroll
    for (int j = 0; j < PU; ++j) {
        ok[j] = k + (Off)j < lim;
        const u64 x = ok[j] ? eat(ed, (u64)(k + j)) : 0ull;
        w[j] = (u32)(x >> 32);
        u[j] = (u32)x;
    }
    bool stop = false;
    int nv = 0;
#pragma unroll
    for (int j = 0; j < PU; ++j) {
        if (ok[j] && (long long)lo + w[j] >= (long long)cur) stop = true;
        ok[j] = ok[j] && !stop;
        nv += ok[j];
    }
    uint32_t m[PU];
#pragma unroll
    for (int j = 0; j < PU; ++j) m[j] = ok[j] ? map[u[j]] : 0xFFu;
#pragma unroll
    for (int j = 0; j < PU; ++j)
        if (m[j] != 0xFFu) {
            const long long nd = (long long)lo + m[j] + w[j];
            if (nd < cur) cur = (int32_t)nd;
        }
    k += (Off)nv;
    return stop;
}

// Pull screening (v2_pull_k, v2_pull_light_body): a wave reads the dists of PSC
// groups of 64 vertices, compacts the candidates into lanes, probes PSERIAL edges
// per lane (wave-uniform loop), then scans the long rows with the whole wave.
#ifndef PJ_PSC
#define PJ_PSC 16
#endif
constexpr int PSC = PJ_PSC;
#ifndef PJ_PSERIAL
#define PJ_PSERIAL 32
#endif
constexpr int PSERIAL = PJ_PSERIAL;
// lsplit[v] = number of edges of v with weight < delta (rows are weight-sorted)
template <typename Off, typename WT>
__global__ void light_split_k(const Off* __restrict__ row, const WT* __restrict__ w, i64 n, u32 delta,
                              u32* __restrict__ lsplit) {
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x) {
        Off lo = row[v], hi = row[v + 1];
        const Off b = lo;
        while (lo < hi) {
            const Off mid = lo + (hi - lo) / 2;
            if (w[mid] < delta) lo = mid + 1;
            else hi = mid;
        }
        lsplit[v] = (u32)(lo - b);
    }
}

// sum (out[0]) and max (out[1]) of the edge weights in one pass: the auto delta's mean
// weight and the v2 tail's "every edge is light" test (two passes over the 2^31 weights
// of s26 cost 2.2 + 1.5 ms of the solver preparation)
__global__ __launch_bounds__(DB) void wsummax_k(const u32* __restrict__ w, i64 n, u64* __restrict__ out) {
    __shared__ u64 red[DB / WAVE];
    u64 acc = 0;
    u32 mx = 0;
    for (i64 i = (i64)blockIdx.x * DB + threadIdx.x; i < n; i += (i64)gridDim.x * DB) {
        const u32 x = w[i];
        acc += x;
        mx = max(mx, x);
    }
    acc = block_sum<DB / WAVE>(acc, red);
    mx = wave_max(mx);
    if (lane_id() == 0) red[wave_id()] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 0; k < DB / WAVE; ++k) mx = max(mx, (u32)red[k]);
        if (acc) atomicAdd(&out[0], acc);
        if (mx) atomicMax(&out[1], (u64)mx);
    }
}

__global__ __launch_bounds__(DB) void wsum_k(const u32* __restrict__ w, i64 n, u64* __restrict__ out) {
    u64 acc = 0;
    for (i64 i = (i64)blockIdx.x * DB + threadIdx.x; i < n; i += (i64)gridDim.x * DB) acc += w[i];
    acc = wave_sum(acc);
    if (lane_id() == 0 && acc) atomicAdd(out, acc);
}


// ---------------------------------------------------------------------------
// v2 band loop: bitmap frontiers, no per-band list building.
//
//   light round : the band's frontier bitmap F_in (members whose light edges are
//                 not relaxed yet) is screened wave by wave; a lane relaxes the
//                 light prefix of its vertex's row (<= V2_LS edges alone, then the
//                 whole wave for segments <= V2_HT, longer segments go to a hub
//                 queue relaxed edge-balanced by v2_hub_k). A target lowered below
//                 hi is marked in F_out: the next round's frontier. Every frontier
//                 vertex joins the band's member bitmap mb; new members add their
//                 heavy-edge count to ctl.mh (the push cost of the heavy step).
//   heavy step  : pull (d_pull-style, fused with the next band's selection) when
//                 the heavy edges left on unsettled vertices are few, else a push
//                 over mb's heavy segments (same kernel, heavy mode) and a select.
//   counts      : frontier sizes live in a ring of 4 slots (a light round reads
//                 slot c, adds to c+1, zeroes c+2), each slot sharded over 8
//                 64-B lines; hub queues in a ring of 3. The host reads the ring
//                 once per batch of light rounds and once per band.
// ---------------------------------------------------------------------------
constexpr int V2_SC = 16;     // frontier words a wave screens at once
// a light relaxation's dist update (no return value: nothing waits for it) and
// frontier mark (true = newly marked)
__device__ __forceinline__ void v2_dmin(int32_t* p, int32_t v) { atomicMin(p, v); }
__device__ __forceinline__ bool v2_mark(u64* __restrict__ fout, u32 t) {
    const u64 bit = 1ull << (t & 63);
    return !(atomicOr(fout + (t >> 6), bit) & bit);
}
#ifndef PJ_V2_LS
#define PJ_V2_LS 2  // swept 1, 2, 4 (round 2 end): 1 ~ 2, 4 is ~1% slower
#endif
constexpr int V2_LS = PJ_V2_LS;  // segment edges a lane relaxes alone
#ifndef PJ_V2_HT
#define PJ_V2_HT 64  // swept 32 / 128 (round 4, row filters on): 1% / 3.5% slower
#endif
constexpr u64 V2_HT = PJ_V2_HT;  // longer segments: hub queue (edge-balanced). The low ids hold the
                                 // high-degree vertices, so a wave that relaxed mid-size rows itself
                                 // would carry a whole dense chunk of them alone (load imbalance).
constexpr int V2_EB = 40;     // hub counter: (slots << V2_EB) | edges
constexpr int V2_NSH = 8;     // shards of a count slot
#ifndef PJ_V2_HTM
#define PJ_V2_HTM 2  // swept 1, 2, 4, 8 (round 2 end): 1-2 best, +0.7% over 4, 8 is 4% slower
#endif
constexpr int V2_HTILE = DB * PJ_V2_HTM;  // hub-queue tile: edges per workgroup step (PJ_V2_HTM per thread)
#ifndef PJ_V2_PLMAX
// swept 32 / 128 in round 4 (1% / 14% slower than 64); late round 5, with the frontier-minimum
// bound and the 7-wave light-round kernel, 96-160 with 512- or 1024-edge chunks are 4% faster
// than 64 / 256 (profiles/r05/pull_rows_r5h27.txt)
#define PJ_V2_PLMAX 128
#endif
#ifndef PJ_V2_PCH
#define PJ_V2_PCH 1024
#endif
constexpr u32 V2_PLMAX = PJ_V2_PLMAX;  // pull rounds: longer light rows go to v2_pull_long_body
constexpr u32 V2_PCH = PJ_V2_PCH;      // light edges per v2_pull_long_body work item

struct alignas(64) V2Line {
    u64 v;
    u64 pad[7];
};
// The work of a solve, always counted (SURVEY.md §8d's byte model counts every reached edge; a
// pull stops a row at its first useless weight and most of a push's targets are probed once):
// per kernel class, the edge records its relaxations read (.v), the probes of the edges' other
// ends they issued (.pad[0]: dist, the heavy pull's byte map, or the tail's settled bitmap) and
// the bytes of both as stored (.pad[1]: records of 4, 5 or 8 bytes, probes of 4 or 1). Each
// wave sums its counts in wave-uniform registers; one atomic per workgroup and counter at the
// end of a launch (v2_flush_work).
enum { V2W_ROUND = 0, V2W_HUB = 1, V2W_HPULL = 2, V2W_HPUSH = 3, V2W_N = 4 };
struct V2Ctl {
    V2Line cnt[4][V2_NSH];  // frontier vertices marked per light round (ring)
    V2Line hub[3];          // hub queue packed counters (ring)
    V2Line mh[V2_NSH];      // heavy edges of this band's members
    V2Line minv[V2_NSH];    // min dist >= lo of the last select / pull (next band search), per shard
    V2Line aux;             // v2_heavy_left_k's sum (the tail switch's heavy_left)
    V2Line work[V2W_N][V2_NSH];
};
// Waves per SIMD the compiler must fit the register budget to (0 = its own choice): the light
// round kernel took 81-91 VGPRs (5 waves per SIMD); at 7 (72 VGPRs, 16 bytes of scratch per lane)
// its latency-bound pulls keep more loads in flight: k26w 596 -> 643 GTEPS interleaved (6: 634,
// 8: 627 with 92 bytes of scratch; profiles/r05/occupancy_r5h17.txt). The heavy pull (65-73
// VGPRs) at 8 measured equal. Round 6 (the speculative round, one round per check at a band's
// start, 3 hub workgroups per CU): 6 beats 7 by 0.7% over 6 interleaved passes
// (profiles/r06/delta_variants_r6ba.txt).
#ifndef PJ_V2_WPE_R
#define PJ_V2_WPE_R 6
#endif
#ifndef PJ_V2_WPE_H
#define PJ_V2_WPE_H 8  // the heavy pull: 0 (the compiler's choice) until round 6; 8 +1.0% over 7 interleaved
                       // passes once the round kernel ran at 6 (profiles/r06/delta_variants_r6be.txt)
#endif
#if PJ_V2_WPE_R
#define V2_WPE_R __attribute__((amdgpu_waves_per_eu(PJ_V2_WPE_R)))
#else
#define V2_WPE_R
#endif
#if PJ_V2_WPE_H
#define V2_WPE_H __attribute__((amdgpu_waves_per_eu(PJ_V2_WPE_H)))
#else
#define V2_WPE_H
#endif

struct V2Args {
    i64 n, nwords;
    int32_t lo, hi;
    int32_t* dist;
    const u32* lsplit;
    const u64* cw;    // edges interleaved: col | w << 32 (the relabeled CSR)
    const u64* lrow;  // light CSR: the light prefixes of the rows, packed
    const u64* lcw;
    const u32* lcw32; // packed light CSR (col | w << lcb), or null
    u32 lcb;
    const u32* col;   // relabeled ids beside w8 (split records of the whole CSR), when w8 is set
    const uint8_t* w8;
    const u64* hl;    // bit v: v has a light edge (lsplit[v] > 0) for this delta; null in the tail
    const uint8_t* w1;  // the lightest weight of v's row (capped at 255): the light pull's candidate filter
    const uint8_t* hw;  // weight of v's first heavy edge for the current threshold (capped at 255; 0 = no
                        // heavy edge): the heavy pull's candidate filter
    int ltail;        // tail mode: light prefixes are row[v] + [0, lsplit[v]) of cw (no light CSR)
    const u64* sbits; // tail mode: settled-before-the-tail bitmap; relaxations skip its targets
    u64* swrite;      // the heavy step entering the tail writes that bitmap (pull / select)
    const u32* fesplit;  // the heavy step entering the tail counts the next frontier's edges with the
                         // tail's light prefixes (lsplit2), so its first round sees its true push cost
    u64* mb;
    V2Ctl* ctl;
    u32* hv;     // [3][hcap]
    u64* hbeg;   // [3][hcap]
    u64* hoff;   // [3][hcap]
    u64 hcap;
    u64* rlog;   // round_log option: [0] = rounds logged, then (kind, frontier, its light edges) per round
    int32_t hz;  // heavy push: relax only the edges with du + w < hz (INT_INF = all; defer_heavy)
    const uint8_t* hmap;  // heavy pull: dist - lo of every vertex with dist in [lo, hi), 0xFF otherwise
                          // (null = probe dist: bands wider than 255)
    u64* dsave;  // heavy push: the member words are OR-ed in here (their far edges are deferred), or null
};
// the light edges of a band round (light CSR, or the light prefixes of cw in the tail)
__device__ __forceinline__ ESrc v2_cw_src(const V2Args& a) {
    if (a.w8) return ESrc{a.cw, a.col, 0, a.w8};
    return ESrc{a.cw, nullptr, 0, nullptr};
}
__device__ __forceinline__ ESrc v2_light_src(const V2Args& a) {
    if (a.ltail) return v2_cw_src(a);
    return ESrc{a.lcw, a.lcw32, a.lcb, nullptr};
}
// bytes of one edge record as stored: u32 id + u8 weight, a packed 32-bit record, or u64
__device__ __forceinline__ u32 esrc_bytes(const ESrc& s) { return s.w8 ? 5u : s.e32 ? 4u : 8u; }

// A wave's work counts, flushed once per launch into ctl->work[kind] (one atomic per
// workgroup and counter). The increments are taken from lane 0 (readfirstlane), so the
// counters live in scalar registers and cost the latency-bound kernels no VGPR; every
// increment is made in wave-uniform control flow.
__device__ __forceinline__ u32 v2_uni(u32 x) { return (u32)__builtin_amdgcn_readfirstlane((int)x); }
struct V2Work {
    u32 rec = 0, prb = 0;
    __device__ __forceinline__ void add(u32 r, u32 p) {
#ifdef PJ_V2_NOCOUNT  // (measurement build only: the counters' own cost, A/B)
        return;
#endif
        rec += v2_uni(r);
        prb += v2_uni(p);
    }
};
// div: every wave of the block added the same block-uniform counts (tile-wide work), so the
// block's sum is divided by the waves
__device__ __forceinline__ void v2_flush_work(const V2Args& a, int kind, const V2Work& wk, u32 rec_bytes,
                                              u32 prb_bytes, u64* red, u32 div = 1) {
    __syncthreads();
    if (lane_id() == 0) {
        red[wave_id()] = wk.rec;
        red[DB / WAVE + wave_id()] = wk.prb;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        u64 r = 0, p = 0;
        for (int w = 0; w < DB / WAVE; ++w) {
            r += red[w];
            p += red[DB / WAVE + w];
        }
        r /= div;
        p /= div;
        V2Line& l = a.ctl->work[kind][blockIdx.x % V2_NSH];
        if (r) atomicAdd(&l.v, r);
        if (p) atomicAdd(&l.pad[0], p);
        if (r | p) atomicAdd(&l.pad[1], r * rec_bytes + p * prb_bytes);
    }
    __syncthreads();
}


__device__ __forceinline__ u64 v2_slot_sum(const V2Line* sl) {
    u64 t = 0;
#pragma unroll
    for (int i = 0; i < V2_NSH; ++i) t += sl[i].v;
    return t;
}

// (vertices, their light edges) into a count slot: .v and .pad[0]
__device__ __forceinline__ void v2_flush2(u64 x, u64 e, V2Line* sl, u64* red) {
    x = block_sum<DB / WAVE>(x, red);
    e = block_sum<DB / WAVE>(e, red);
    if (threadIdx.x == 0) {
        if (x) atomicAdd(&sl[blockIdx.x % V2_NSH].v, x);
        if (e) atomicAdd(&sl[blockIdx.x % V2_NSH].pad[0], e);
    }
}
// min{mn} of the block into a minv shard: one atomic per workgroup (the heavy pull's
// 24K waves taking one atomicMin each on one word serialized behind its ~88 per us)
__device__ __forceinline__ void v2_flush_min(int32_t mn, V2Ctl* ctl, u64* red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const int32_t y = __shfl_xor(mn, off, 64);
        mn = y < mn ? y : mn;
    }
    if (lane_id() == 0) red[wave_id()] = (u64)(u32)mn;
    __syncthreads();
    if (threadIdx.x == 0) {
        int32_t m = INT_INF;
        for (int w = 0; w < DB / WAVE; ++w) m = min(m, (int32_t)(u32)red[w]);
        if (m < INT_INF) atomicMin(&ctl->minv[blockIdx.x % V2_NSH].v, (u64)m);
    }
    __syncthreads();
}
// The least distance the frontier of a count slot holds (.pad[1]): every write that lowers
// a vertex into the band is folded in (a relaxation that marks, a pull's store, the selection
// of a band's first frontier), so it bounds the frontier from below and a pull round can stop
// a row at fmin + w >= its best instead of lo + w (round 5: the first band's big pull scanned
// ~19M light edges instead of ~100M, +8%, profiles/r05/ab_fmin_r5h2.txt).
__device__ __forceinline__ void v2_flush_fmin(int32_t m, V2Line* sl, u64* red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const int32_t y = __shfl_xor(m, off, 64);
        m = y < m ? y : m;
    }
    if (lane_id() == 0) red[wave_id()] = (u64)(u32)m;
    __syncthreads();
    if (threadIdx.x == 0) {
        int32_t b = INT_INF;
        for (int w = 0; w < DB / WAVE; ++w) b = min(b, (int32_t)(u32)red[w]);
        if (b < INT_INF) atomicMin(&sl[blockIdx.x % V2_NSH].pad[1], (u64)b);
    }
    __syncthreads();
}
__device__ __forceinline__ int32_t v2_slot_fmin(const V2Line* sl) {
    u64 m = ~0ull;
#pragma unroll
    for (int i = 0; i < V2_NSH; ++i) m = sl[i].pad[1] < m ? sl[i].pad[1] : m;
    return m < (u64)INT_INF ? (int32_t)m : INT_INF;
}
// the frontier bound of a pull round over slot c: max(lo, fmin), or lo without one
__device__ __forceinline__ int32_t v2_pull_lo(const V2Args& a, int c) {
    const int32_t f = v2_slot_fmin(a.ctl->cnt[c]);
    return (f > a.lo && f < a.hi) ? f : a.lo;
}
__device__ __forceinline__ u64 v2_slot_edges(const V2Line* sl) {
    u64 t = 0;
#pragma unroll
    for (int i = 0; i < V2_NSH; ++i) t += sl[i].pad[0];
    return t;
}

// N independent edges (any positions, own source distances) with the loads
// issued together: edge words, then target distances, then the atomics. The
// atomicMin is issued without a return value (nothing waits for it): a target
// whose read distance was above nd has been lowered to <= nd this round, by
// this lane or another, so it belongs in the next frontier either way. The
// frontier mark counts the new frontier vertex and its light edges (the next
// round's push cost): a returning atomicOr, then the lsplit read of a newly marked
// target. (Round 4: the lsplit read issued beside the atomicOr measured equal, a plain
// read of the mark word plus a returnless atomicOr 5% slower; both removed.)
template <bool LIGHT, int N>
__device__ __forceinline__ u32 v2_relax_g(const V2Args& a, const ESrc ed, const u64 (&idx)[N],
                                          const int32_t (&du)[N], const bool (&val)[N], u64* __restrict__ fout,
                                          u64& fe, int32_t& fm) {
    u32 t[N];
    long long nd[N];
    bool ok[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const u64 x = val[j] ? eat(ed, idx[j]) : 0ull;
        t[j] = (u32)x;
        nd[j] = (long long)du[j] + (long long)(x >> 32);
        ok[j] = val[j] && nd[j] < INT_INF;
    }
    if (a.sbits) {  // tail: skip targets settled before the tail (a cache-resident bit, not dist)
        u64 sw[N];
#pragma unroll
        for (int j = 0; j < N; ++j) sw[j] = ok[j] ? a.sbits[t[j] >> 6] : 0ull;
#pragma unroll
        for (int j = 0; j < N; ++j) ok[j] = ok[j] && !((sw[j] >> (t[j] & 63)) & 1ull);
    }
    int32_t cd[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        cd[j] = ok[j] ? dist_now(a.dist + t[j]) : 0;
    }
    bool mk[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const bool imp = ok[j] && (int32_t)nd[j] < cd[j];
        if (imp) v2_dmin(a.dist + t[j], (int32_t)nd[j]);
        mk[j] = LIGHT && imp && (int32_t)nd[j] < a.hi;
        if (mk[j] && (int32_t)nd[j] < fm) fm = (int32_t)nd[j];
    }
    if (!LIGHT) return 0u;
    u32 newc = 0;
#pragma unroll
    for (int j = 0; j < N; ++j)
        if (mk[j]) {
            if (v2_mark(fout, t[j])) {
                ++newc;
                fe += a.lsplit[t[j]];
            }
        }
    return newc;
}

// PU consecutive edges [k, min(k + PU, lim)) of one source in one step
template <bool LIGHT>
__device__ __forceinline__ u32 v2_relax_n(const V2Args& a, const ESrc ed, u64 k, u64 lim, int32_t du,
                                          u64* __restrict__ fout, u64& fe, int32_t& fm) {
    u64 idx[PU];
    int32_t d[PU];
    bool val[PU];
#pragma unroll
    for (int j = 0; j < PU; ++j) {
        idx[j] = k + j;
        d[j] = du;
        val[j] = k + j < lim;
    }
    return v2_relax_g<LIGHT, PU>(a, ed, idx, d, val, fout, fe, fm);
}

// one relaxation
template <bool LIGHT>
__device__ __forceinline__ u32 v2_relax(const V2Args& a, const ESrc ed, u64 k, int32_t du, u64* __restrict__ fout,
                                        u64& fe, int32_t& fm) {
    const u64 idx[1] = {k};
    const int32_t d[1] = {du};
    const bool val[1] = {true};
    return v2_relax_g<LIGHT, 1>(a, ed, idx, d, val, fout, fe, fm);
}

// Hub queue appends (whole wave; lanes with hub = true hand their segment [b, e) to the
// queue of ring slot hs and get e = b back).
// One slot per segment, (source, row position, edge offset) from ONE packed atomic,
// relaxed by v2_hub_body in edge-balanced block tiles (an LDS binary search per edge, the
// tile's slot offsets and source distances staged in LDS). (Round 4: 256- or 128-edge chunk
// descriptors, one wave each, measured 2-3% slower; a slot carrying the source's distance
// instead of its id 1% slower; removed.)
__device__ __forceinline__ void v2_hub_append(const V2Args& a, int hs, bool hub, u32 v, int32_t du, u64 b, u64& e) {
    const int lane = lane_id();
    const u64 hm = __ballot(hub);
    if (!hm) return;
    const u64 mask = (1ull << V2_EB) - 1ull;
    const u64 seg = hub ? e - b : 0;
    const u64 ie = wave_incl_scan(seg);
    const u64 tot = __shfl(ie, 63, 64);
    const int leader = __ffsll((long long)hm) - 1;
    u64 base = 0;
    if (lane == leader) base = atomicAdd(&a.ctl->hub[hs].v, ((u64)__popcll(hm) << V2_EB) | tot);
    base = __shfl(base, leader, 64);
    if (hub) {
        const u64 slot = (base >> V2_EB) + (u64)__popcll(hm & lanemask_lt());
        const u64 q = (u64)hs * a.hcap + slot;
        a.hv[q] = v;
        a.hbeg[q] = b;
        a.hoff[q] = (base & mask) + ie - seg;
        e = b;
    }
}

// Dense light round (the frontier holds more than dense_min vertices): the
// workgroup takes a tile of V2_DT consecutive vertices, reads their frontier
// words, row offsets and distances with coalesced loads (4 consecutive vertices
// per thread), compacts the frontier vertices' light segments into LDS with one
// block scan and relaxes the tile's edges edge-balanced, 4 independent edges per
// thread (v2_relax_g), instead of one vertex per lane with a dependent chain of
// loads per vertex. Segments longer than V2_DHT go to the hub queue.
#ifndef PJ_V2_DV
#define PJ_V2_DV 4  // swept 2, 4, 8 (round 2 end): 2 ~ 4, 8 is 8% slower
#endif
constexpr int V2_DV = PJ_V2_DV;   // dense tiles: consecutive vertices per thread
constexpr int V2_DT = DB * V2_DV; // vertices per dense tile (V2_DV * 4 frontier words)
constexpr u32 V2_DVM = (1u << V2_DV) - 1u;
#ifndef PJ_V2_DHT
#define PJ_V2_DHT 4096  // swept 1024, 4096, 16384 (round 2 end): within the +-1% noise
#endif
constexpr u64 V2_DHT = PJ_V2_DHT; // dense mode: longer segments -> hub queue
#ifndef PJ_V2_DNJ
#define PJ_V2_DNJ 4
#endif
constexpr int V2_DNJ = PJ_V2_DNJ; // dense mode: independent edges per thread per relax step
template <typename Off>
struct V2Dense {
    Off b[V2_DT];                 // segment begin (edge index into lcw, or cw in the tail)
    u32 off[V2_DT];               // segment start inside the tile's edge range
    int32_t du[V2_DT];
    u64 f[V2_DT / 64], fnew[V2_DT / 64];
    u64 red[DB / WAVE];
};

__device__ __forceinline__ u32 v2_dense_find(const u32* off, u32 ns, u32 e) {
    u32 lo = 0, hi = ns - 1;
    while (lo < hi) {
        const u32 mid = (lo + hi + 1) >> 1;
        if (off[mid] <= e) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

template <typename Off>
__device__ __forceinline__ void v2_dense_body(const V2Args& a, const Off* __restrict__ row, u64* __restrict__ fin,
                                              u64* __restrict__ fout, int hs, u32& newc, u64& fe, u64& mh, u64& ml,
                                              int32_t& fm, V2Work& wk, V2Dense<Off>& sh) {
    const int tid = threadIdx.x;
    const u64 mask = (1ull << V2_EB) - 1ull;
    const ESrc ed = v2_light_src(a);
    const i64 ntiles = (a.n + V2_DT - 1) / V2_DT;
    for (i64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const i64 w0 = tile * (V2_DT / 64);
        if (tid < V2_DT / 64) {
            u64 f = 0, nw = 0;
            if (w0 + tid < a.nwords) {
                f = fin[w0 + tid];
                if (f) {
                    fin[w0 + tid] = 0;
                    const u64 old = a.mb[w0 + tid];  // the block owns these words of mb
                    nw = f & ~old;
                    if (nw) a.mb[w0 + tid] = old | f;
                }
            }
            sh.f[tid] = f;
            sh.fnew[tid] = nw;
        }
        __syncthreads();
        u64 anyf = 0;
#pragma unroll
        for (int k = 0; k < V2_DT / 64; ++k) anyf |= sh.f[k];
        if (!anyf) {  // block-uniform
            __syncthreads();
            continue;
        }
        const int i0 = tid * V2_DV;
        const i64 v0 = tile * V2_DT + i0;
        const u32 nib = (u32)(sh.f[i0 >> 6] >> (i0 & 63)) & V2_DVM;
        const u32 nnew = (u32)(sh.fnew[i0 >> 6] >> (i0 & 63)) & V2_DVM;
        u64 b[V2_DV], e[V2_DV];
        int32_t du[V2_DV];
#pragma unroll
        for (int j = 0; j < V2_DV; ++j) {
            b[j] = e[j] = 0;
            du[j] = 0;
            if ((nib >> j) & 1u) {
                const i64 v = v0 + j;
                du[j] = a.dist[v];
                if (a.ltail) {
                    b[j] = (u64)row[v];
                    e[j] = b[j] + a.lsplit[v];
                } else {
                    b[j] = a.lrow[v];
                    e[j] = a.lrow[v + 1];
                }
                if ((nnew >> j) & 1u) {
                    mh += (u64)row[v + 1] - (u64)row[v] - (e[j] - b[j]);
                    ml += e[j] - b[j];
                }
            }
        }
        // long segments -> hub queue (wave-aggregated append, v2_hub_append)
#pragma unroll
        for (int j = 0; j < V2_DV; ++j) v2_hub_append(a, hs, e[j] - b[j] > V2_DHT, (u32)(v0 + j), du[j], b[j], e[j]);
        u64 cnt = 0, edges = 0;
#pragma unroll
        for (int j = 0; j < V2_DV; ++j)
            if (e[j] > b[j]) {
                ++cnt;
                edges += e[j] - b[j];
            }
        u64 tot;
        const u64 ex = block_excl_scan<DB / WAVE>((cnt << V2_EB) | edges, sh.red, tot);
        u32 slot = (u32)(ex >> V2_EB);
        u32 eo = (u32)(ex & mask);
#pragma unroll
        for (int j = 0; j < V2_DV; ++j)
            if (e[j] > b[j]) {
                sh.b[slot] = (Off)b[j];
                sh.du[slot] = du[j];
                sh.off[slot] = eo;
                ++slot;
                eo += (u32)(e[j] - b[j]);
            }
        const u32 ns = (u32)(tot >> V2_EB), te = (u32)(tot & mask);
        wk.add(te, te);  // (block-uniform: flushed with div = waves)
        __syncthreads();
        for (u32 e0 = 0; e0 < te; e0 += DB * V2_DNJ) {
            u64 idx[V2_DNJ];
            int32_t dj[V2_DNJ];
            bool val[V2_DNJ];
#pragma unroll
            for (int j = 0; j < V2_DNJ; ++j) {
                const u32 x = e0 + (u32)j * DB + (u32)tid;
                val[j] = x < te;
                const u32 sl = val[j] ? v2_dense_find(sh.off, ns, x) : 0u;
                idx[j] = val[j] ? (u64)sh.b[sl] + (x - sh.off[sl]) : 0ull;
                dj[j] = val[j] ? sh.du[sl] : 0;
            }
            newc += v2_relax_g<true, V2_DNJ>(a, ed, idx, dj, val, fout, fe, fm);
        }
        __syncthreads();
    }
}

// LIGHT: relax the light prefixes of fin's vertices (a band round); HEAVY: the
// heavy segments of fin = mb (push heavy step). fin words are cleared as read.
// Light rounds use a ring of three frontier bitmaps: round r reads f[r], writes
// f[r+1] and clears f[r+2] (read by round r-1, written by nobody until round r+1),
// so a pull round, whose probes read its input from every wave, never has to clear it.
__device__ __forceinline__ void v2_clear_words(u64* __restrict__ f, i64 nwords) {
    if (f)
        for (i64 wi = (i64)blockIdx.x * DB + threadIdx.x; wi < nwords; wi += (i64)gridDim.x * DB) f[wi] = 0;
}
__device__ __forceinline__ void v2_zero_slot(const V2Args& a, int c) {
    if (blockIdx.x == 0 && threadIdx.x < V2_NSH) {
        a.ctl->cnt[c][threadIdx.x].v = 0;
        a.ctl->cnt[c][threadIdx.x].pad[0] = 0;
        a.ctl->cnt[c][threadIdx.x].pad[1] = (u64)INT_INF;
    }
}

template <typename Off, bool LIGHT>
__device__ __forceinline__ void v2_expand_body(const V2Args& a, const Off* __restrict__ row, u64* __restrict__ fin,
                                               u64* __restrict__ fout, int cin, int hs, u64* red);

// first position in [b, e) of a weight-sorted row whose weight is >= lim (binary search)
__device__ __forceinline__ u64 v2_first_w_ge(const V2Args& a, u64 b, u64 e, long long lim) {
    while (b < e) {
        const u64 m = (b + e) >> 1;
        const u32 w = a.w8 ? (u32)a.w8[m] : (u32)(a.cw[m] >> 32);
        if ((long long)w >= lim) e = m;
        else b = m + 1;
    }
    return b;
}

// Heavy push step: the heavy segments of the band's members (fin = mb; hub queue hs).
// With a.hz < INT_INF only the edges landing below hz (the next band) are relaxed and
// the member words are saved in a.dsave: the rest is left to the next heavy step.
template <typename Off>
__global__ __launch_bounds__(DB) void v2_heavy_push_k(V2Args a, const Off* __restrict__ row, u64* __restrict__ fin,
                                                      int hs) {
    __shared__ u64 red[2 * DB / WAVE];
    v2_expand_body<Off, false>(a, row, fin, nullptr, 0, hs, red);
}

template <typename Off, bool LIGHT>
__device__ __forceinline__ void v2_expand_body(const V2Args& a, const Off* __restrict__ row, u64* __restrict__ fin,
                                               u64* __restrict__ fout, int cin, int hs, u64* red) {
    constexpr int NWV = DB / WAVE;
    const int lane = lane_id();
    u32 newc = 0;
    u64 mh = 0, ml = 0, fe = 0;
    int32_t fm = INT_INF;
    V2Work wk;
    const ESrc esrc = LIGHT ? v2_light_src(a) : v2_cw_src(a);
    const i64 nsc = (a.nwords + V2_SC - 1) / V2_SC;
    for (i64 sc = (i64)blockIdx.x * NWV + wave_id(); sc < nsc; sc += (i64)gridDim.x * NWV) {
        const i64 wbase = sc * V2_SC;
        u64 mytodo = 0, mynew = 0;
        if (lane < V2_SC && wbase + lane < a.nwords) {
            mytodo = fin[wbase + lane];
            if (mytodo) {
                fin[wbase + lane] = 0;
                if (!LIGHT && a.dsave) a.dsave[wbase + lane] |= mytodo;  // (the wave owns the word)
                if (LIGHT) {  // the wave owns these words of mb: plain read-modify-write
                    const u64 old = a.mb[wbase + lane];
                    mynew = mytodo & ~old;
                    if (mynew) a.mb[wbase + lane] = old | mytodo;
                }
            }
        }
        if (!__ballot(mytodo != 0)) continue;
        if (LIGHT && a.hl) {
            // frontier vertices without light edges have nothing to relax: only a new
            // member's heavy-edge count (its whole row) is accounted
            const u64 hw = mytodo ? a.hl[wbase + lane] : 0ull;
            const u64 nl = mynew & ~hw;
            mytodo &= hw;
            const u32 c2 = (u32)__popcll(nl);
            const u32 i2 = wave_incl_scan(c2);
            const u32 x2 = i2 - c2;
            const u32 T2 = __shfl(i2, 63, 64);
            for (u32 r0 = 0; r0 < T2; r0 += WAVE) {
                const u32 c = r0 + lane;
                u32 jw = 0;
#pragma unroll
                for (u32 step = V2_SC / 2; step > 0; step >>= 1) {
                    const u32 x = __shfl(x2, jw + step, 64);
                    if (x <= c) jw += step;
                }
                const u32 ex = __shfl(x2, jw, 64);
                const u64 tw = __shfl(nl, jw, 64);
                if (c < T2) {
                    const u32 v = (u32)((wbase + jw) * 64 + select_bit(tw, c - ex));
                    mh += (u64)row[v + 1] - (u64)row[v];
                }
            }
        }
        const u32 cnt = (u32)__popcll(mytodo);
        const u32 incl = wave_incl_scan(cnt);
        const u32 myex = incl - cnt;
        const u32 T = __shfl(incl, 63, 64);
        for (u32 r0 = 0; r0 < T; r0 += WAVE) {
            const u32 c = r0 + lane;
            const bool act = c < T;
            u32 jw = 0;
#pragma unroll
            for (u32 step = V2_SC / 2; step > 0; step >>= 1) {
                const u32 x = __shfl(myex, jw + step, 64);
                if (x <= c) jw += step;
            }
            const u32 ex = __shfl(myex, jw, 64);
            const u64 tw = __shfl(mytodo, jw, 64);
            const u64 tn = __shfl(mynew, jw, 64);
            int32_t du = 0;
            u64 b = 0, e = 0;
            u32 v = 0;
            if (act) {
                const u32 bit = select_bit(tw, c - ex);
                v = (u32)((wbase + jw) * 64 + bit);
                du = a.dist[v];
                if (LIGHT) {  // light CSR (tail mode: the light prefix in cw)
                    b = a.ltail ? (u64)row[v] : a.lrow[v];
                    e = a.ltail ? b + a.lsplit[v] : a.lrow[v + 1];
                    if ((tn >> bit) & 1ull) {
                        mh += (u64)row[v + 1] - (u64)row[v] - (e - b);
                        ml += e - b;
                    }
                } else {      // heavy suffix of the row (up to the horizon: defer_heavy)
                    b = (u64)row[v] + a.lsplit[v];
                    e = (u64)row[v + 1];
                    if (a.hz < INT_INF) e = v2_first_w_ge(a, b, e, (long long)a.hz - du);
                }
            }
            // long segment -> hub queue (wave-aggregated append; all lanes here)
            v2_hub_append(a, hs, e - b > V2_HT, v, du, b, e);
            {  // the wave relaxes the rest of every segment: one record and one probe per edge
                const u32 se = wave_sum((u32)(e - b));
                wk.add(se, se);
            }
            // lane-serial part
            u64 k = b;
            const u64 lim = (e - b > (u64)V2_LS) ? b + V2_LS : e;
            bool go = k < lim;
            while (__ballot(go)) {
                if (go) {
                    newc += v2_relax_n<LIGHT>(a, esrc, k, lim, du, fout, fe, fm);
                    k = k + PU < lim ? k + PU : lim;
                    go = k < lim;
                }
            }
            // the rest of the segments (<= V2_HT): edge-balanced over the wave, 64
            // edges per step (a lane finds its segment by binary search over the
            // lanes' inclusive edge counts)
            if (__ballot(k < e)) {
                const u64 rem = k < e ? e - k : 0;
                const u64 inc = wave_incl_scan(rem);
                const u64 exc = inc - rem;
                const u64 tot = __shfl(inc, 63, 64);
                for (u64 r0 = 0; r0 < tot; r0 += WAVE) {
                    const u64 gi = r0 + lane;
                    int l = 0;
#pragma unroll
                    for (int step = 32; step > 0; step >>= 1)
                        if (__shfl(inc, l + step - 1, 64) <= gi) l += step;
                    const u64 kl = __shfl(k, l, 64), xl = __shfl(exc, l, 64);
                    const int32_t dl = __shfl(du, l, 64);
                    if (gi < tot) newc += v2_relax<LIGHT>(a, esrc, kl + (gi - xl), dl, fout, fe, fm);
                }
            }
        }
    }
    if (LIGHT) {
        v2_flush2(newc, fe, a.ctl->cnt[(cin + 1) & 3], red);
        v2_flush_fmin(fm, a.ctl->cnt[(cin + 1) & 3], red);
        v2_flush2(mh, ml, a.ctl->mh, red);
    }
    v2_flush_work(a, LIGHT ? V2W_ROUND : V2W_HPUSH, wk, esrc_bytes(esrc), 4u, red);
}

// Edge-balanced relaxation of hub queue hs (slots' edge offsets are monotonic:
// one packed atomic gave both), over the whole grid (block-uniform).
struct V2HubLds {
    LbShared<V2_HTILE> sh;
    int32_t s_du[V2_HTILE];
    u64 s_b[V2_HTILE];
};
template <bool LIGHT>
__device__ __forceinline__ void v2_hub_body(const V2Args& a, u64* __restrict__ fout, int hs, u64 packed, u32& newc,
                                            u64& fe, int32_t& fm, V2Work& wk, V2HubLds& L) {
    const u64 nq = packed >> V2_EB, total = packed & ((1ull << V2_EB) - 1ull);
    const u32* hv = a.hv + (u64)hs * a.hcap;
    const u64* hb = a.hbeg + (u64)hs * a.hcap;
    const u64* ho = a.hoff + (u64)hs * a.hcap;
    for (u64 e0 = (u64)blockIdx.x * V2_HTILE; e0 < total; e0 += (u64)gridDim.x * V2_HTILE) {
        const u32 te = (u32)min((u64)V2_HTILE, total - e0);
        wk.add(te, te);  // (block-uniform: flushed with div = waves)
        u64 s0;
        u32 ns;
        lb_tile_load<V2_HTILE>(ho, nq, e0, L.sh, s0, ns);
        for (u32 i = threadIdx.x; i < ns; i += DB) {
            L.s_du[i] = a.dist[hv[s0 + i]];
            L.s_b[i] = hb[s0 + i];
        }
        __syncthreads();
        constexpr int NJ = V2_HTILE / DB;
        u64 idx[NJ];
        int32_t du[NJ];
        bool val[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const u64 e = e0 + (u64)j * DB + threadIdx.x;
            val[j] = e < total;
            const u32 sl = val[j] ? lb_find<V2_HTILE>(L.sh, ns, e) : 0u;
            idx[j] = val[j] ? L.s_b[sl] + (e - L.sh.off[sl]) : 0ull;
            du[j] = val[j] ? L.s_du[sl] : 0;
        }
        newc += v2_relax_g<LIGHT, NJ>(a, LIGHT ? v2_light_src(a) : v2_cw_src(a), idx, du, val, fout, fe, fm);
        __syncthreads();
    }
}

// The hub queue hs of one round in its own launch. Zeroes the next ring slot hz for
// later appends.
template <bool LIGHT>
__global__ __launch_bounds__(DB) void v2_hub_k(V2Args a, u64* __restrict__ fout, int cin, int hs, int hz) {
    __shared__ V2HubLds L;
    __shared__ u64 red[2 * DB / WAVE];
    const u64 packed = a.ctl->hub[hs].v;
    if (blockIdx.x == 0 && threadIdx.x == 0) a.ctl->hub[hz].v = 0;
    if ((packed >> V2_EB) == 0) return;
    u32 newc = 0;
    u64 fe = 0;
    int32_t fm = INT_INF;
    V2Work wk;
    v2_hub_body<LIGHT>(a, fout, hs, packed, newc, fe, fm, wk, L);
    if (LIGHT) {
        v2_flush2(newc, fe, a.ctl->cnt[(cin + 1) & 3], red);
        v2_flush_fmin(fm, a.ctl->cnt[(cin + 1) & 3], red);
    }
    v2_flush_work(a, LIGHT ? V2W_HUB : V2W_HPUSH, wk, esrc_bytes(LIGHT ? v2_light_src(a) : v2_cw_src(a)), 4u, red,
                  DB / WAVE);
}

// Next band [lo, hi): fout words = members, count into slot cout, min dist >= lo.
// A wave takes V2_SELW consecutive words per step with their distance loads issued
// together (one 256-byte load per step and wave left each wave one load in flight:
// 42.5 us for the 134 MB of s26 distances; 28 us with 4, profiles/r03/experiments_r3ab_select.txt).
#ifndef PJ_V2_SELW
#define PJ_V2_SELW 4
#endif
constexpr int V2_SELW = PJ_V2_SELW;
template <typename Off>
__global__ __launch_bounds__(DB) void v2_select_k(V2Args a, const Off* __restrict__ row, u64* __restrict__ fout,
                                                  int cout) {
    __shared__ u64 red[DB / WAVE];
    const int lane = lane_id();
    u32 c = 0;
    u64 fe = 0, mh = 0, ml = 0;
    int32_t mn = INT_INF;
    for (i64 w0 = ((i64)blockIdx.x * (DB / WAVE) + wave_id()) * V2_SELW; w0 < a.nwords;
         w0 += (i64)gridDim.x * (DB / WAVE) * V2_SELW) {
        int32_t dd[V2_SELW];
#pragma unroll
        for (int j = 0; j < V2_SELW; ++j) {
            const i64 v = (w0 + j) * 64 + lane;
            dd[j] = v < a.n ? a.dist[v] : INT_INF;
        }
#pragma unroll
        for (int j = 0; j < V2_SELW; ++j) {
            const i64 wi = w0 + j;
            if (wi >= a.nwords) break;
            const i64 v = wi * 64 + lane;
            const int32_t d = dd[j];
            const bool mem = d >= a.lo && d < a.hi;
            const u64 m = __ballot(mem);
            if (a.swrite) {
                const u64 sm = __ballot(v < a.n && d < a.lo);
                if (lane == 0) a.swrite[wi] = sm;
            }
            if (d >= a.lo && d < mn) mn = d;
            if (mem) {
                const u32 ls = (a.fesplit ? a.fesplit : a.lsplit)[v];
                fe += ls;
                mh += (u64)row[v + 1] - (u64)row[v] - ls;
                ml += ls;
            }
            if (lane == 0) {
                fout[wi] = m;
                a.mb[wi] = m;  // (mb is clear here: the heavy step consumed it)
            }
            c += lane == 0 ? (u32)__popcll(m) : 0u;
        }
    }
    v2_flush2(c, fe, a.ctl->cnt[cout], red);
    v2_flush2(mh, ml, a.ctl->mh, red);
    v2_flush_fmin(mn, a.ctl->cnt[cout], red);  // (min over dist >= lo: below every member)
    v2_flush_min(mn, a.ctl, red);
}

// The heavy pull's probe map: dist - lo for dist in [lo, hi), 0xFF otherwise (hi - lo <= 255)
__global__ __launch_bounds__(256) void v2_hmap_k(const int32_t* __restrict__ dist, i64 n, int32_t lo, int32_t hi,
                                                 uint8_t* __restrict__ map) {
    const i64 n4 = n / 4;
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (i64)gridDim.x * blockDim.x) {
        const int4 d = reinterpret_cast<const int4*>(dist)[i];
        const int32_t dd[4] = {d.x, d.y, d.z, d.w};
        u32 m = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) m |= (u32)((dd[j] >= lo && dd[j] < hi) ? dd[j] - lo : 0xFF) << (8 * j);
        reinterpret_cast<u32*>(map)[i] = m;
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        const i64 v = n4 * 4 + threadIdx.x;
        map[v] = (uint8_t)((dist[v] >= lo && dist[v] < hi) ? dist[v] - lo : 0xFF);
    }
}

// Pull step of the heavy edges of band [lo, hi) fused with the selection of the
// next band [hi, nhi) -- symmetric graphs only, where a row is also the vertex's
// in-edges with the same weights. Every vertex with dist >= hi looks through the
// heavy part of its own row (weights ascending) for in-neighbours in the band and
// stops as soon as lo + w >= the best value it has, since no band member can then
// offer less. This replaces pushing the members' heavy edges when few edges remain
// unsettled: most of a late band's heavy pushes hit vertices that are already
// settled (measured on Kronecker s20: 94% of all heavy relaxations), while the
// unsettled rows are short and cut early. A lane writes only its own vertex's
// dist, with a plain store; the old and new values are both >= hi, so the band
// tests of other lanes do not change. The wave owns its
// PSC words: it writes the next band's member words of fout whole (and so clears
// them), counts them into slot cout and folds min{new dist >= hi} into minv.
template <typename Off>
__global__ __launch_bounds__(DB) V2_WPE_H void v2_pull_k(V2Args a, const Off* __restrict__ row, u64* __restrict__ fout,
                                                int32_t nhi, int cout) {
    constexpr int NWV = DB / WAVE;
    __shared__ u32 s_new[NWV][2 * PSC];
    __shared__ u64 red[2 * NWV];
    const int lane = lane_id();
    const int32_t lo = a.lo, hi = a.hi;
    u32* newb = s_new[wave_id()];
    u32 ccount = 0;
    u64 fe = 0, mh = 0, ml = 0;  // (the next band's members' degrees)
    int32_t mn = INT_INF;
    V2Work wk;
    const i64 ngroups = a.nwords;
    const i64 nsc = (ngroups + PSC - 1) / PSC;
    for (i64 sc = (i64)blockIdx.x * NWV + wave_id(); sc < nsc; sc += (i64)gridDim.x * NWV) {
        const i64 gbase = sc * PSC;
        u64 mytodo = 0;
#pragma unroll
        for (int k = 0; k < PSC; ++k) {
            const i64 v = (gbase + k) * 64 + lane;
            const int32_t d = v < a.n ? a.dist[v] : 0;
            const bool up = v < a.n && d >= hi;
            // heavy-head filter: no band member can lower d below lo + (the row's lightest
            // heavy weight); such vertices (and those without heavy edges) are not scanned,
            // but still join the next band / its minimum (round 4: +0.5%, profiles/r04/ab_r4c.txt)
            // (the form with a.hw tested, although it is never null, compiles to 68 VGPRs where
            // the unconditional one takes 84)
            const int h = (a.hw && up) ? (int)a.hw[v] : 1;
            const bool cand = up && (!a.hw || (h != 0 && (long long)lo + h < (long long)d));
            const u64 m = __ballot(cand);
            u64 nm = 0;
            if (a.hw) {
                const bool sk = up && !cand;
                if (sk && d < mn) mn = d;
                nm = __ballot(sk && d < nhi);
                if (sk && d < nhi) {
                    const u32 ls = (a.fesplit ? a.fesplit : a.lsplit)[v];
                    fe += ls;
                    mh += (u64)row[v + 1] - (u64)row[v] - ls;
                    ml += ls;
                }
            }
            if (lane == k) {
                mytodo = m;
                newb[2 * k] = (u32)nm;
                newb[2 * k + 1] = (u32)(nm >> 32);
            }
            if (a.swrite) {
                const u64 sm = __ballot(v < a.n && d < hi);
                if (lane == k && gbase + k < a.nwords) a.swrite[gbase + k] = sm;
            }
        }
        const u32 cnt = (u32)__popcll(mytodo);
        const u32 incl = wave_incl_scan(cnt);
        const u32 myex = incl - cnt;
        const u32 T = __shfl(incl, 63, 64);
        for (u32 r0 = 0; r0 < T; r0 += WAVE) {
            const u32 c = r0 + lane;
            const bool act = c < T;
            u32 jw = 0;
#pragma unroll
            for (u32 step = PSC / 2; step > 0; step >>= 1) {
                const u32 x = __shfl(myex, jw + step, 64);
                if (x <= c) jw += step;
            }
            const u32 ex = __shfl(myex, jw, 64);
            const u64 tw = __shfl(mytodo, jw, 64);
            const i64 v = act ? (gbase + jw) * 64 + select_bit(tw, c - ex) : 0;
            int32_t d0 = INT_INF, cur = INT_INF;
            Off k = 0, e = 0;
            if (act) {
                d0 = a.dist[v];
                cur = d0;
                k = row[v] + (Off)a.lsplit[v];
                e = row[v + 1];
            }  // (edges in a.cw)
            const Off lim = (e - k > (Off)PSERIAL) ? k + (Off)PSERIAL : e;
            bool go = act && k < lim, done = !act || k >= e;
            const Off kst = k;
            while (__ballot(go)) {
                if (go) {
                    // the band's byte map (cache-resident), else dist itself
                    if (a.hmap ? pull_step_map<Off>(v2_cw_src(a), a.hmap, k, lim, lo, cur)
                               : pull_step_dist<Off>(v2_cw_src(a), a.dist, k, lim, lo, hi, cur)) {
                        done = true;
                        go = false;
                    } else {
                        go = k < lim;
                        done = k >= e;
                    }
                }
            }
            {  // a lane probed k - kst records; one more was read when its weight stopped the row
                const u32 p = (u32)(k - kst);
                wk.add(wave_sum(p + (u32)(act && done && k < e)), wave_sum(p));
            }
            u64 open = __ballot(!done);
            while (open) {
                const int l = __ffsll((long long)open) - 1;
                open &= open - 1;
                const Off kb = __shfl(k, l, 64), ke = __shfl(e, l, 64);
                int32_t cl = __shfl(cur, l, 64);
                for (Off kk = kb; kk < ke; kk += WAVE) {
                    const Off k0 = kk + lane;
                    const bool valid = k0 < ke;
                    const u64 x = valid ? eat(v2_cw_src(a), (u64)k0) : 0ull;
                    const u32 w = (u32)(x >> 32);
                    const bool stop = !valid || (long long)lo + w >= (long long)cl;
                    wk.add((u32)__popcll(__ballot(valid)), (u32)__popcll(__ballot(!stop)));
                    int32_t cand = INT_INF;
                    if (!stop) {
                        int32_t du;
                        if (a.hmap) {
                            const u32 m = a.hmap[(u32)x];
                            du = m != 0xFFu ? lo + (int32_t)m : INT_INF;
                        } else {
                            du = pull_src(a.dist, (u32)x, hi);
                        }
                        if (du < INT_INF) {
                            const long long nd = (long long)du + w;
                            cand = nd < INT_INF ? (int32_t)nd : INT_INF;
                        }
                    }
#pragma unroll
                    for (int off = 32; off > 0; off >>= 1) {
                        const int32_t y = __shfl_xor(cand, off, 64);
                        cand = y < cand ? y : cand;
                    }
                    cl = cand < cl ? cand : cl;
                    if (__ballot(stop)) break;
                }
                if (lane == l) cur = cl;
            }
            if (act) {
                if (cur < d0) a.dist[v] = cur;
                if (cur < mn) mn = cur;
                if (cur < nhi) {  // cur >= hi always here
                    const i64 wl = (v >> 6) - gbase;
                    atomicOr(&newb[2 * wl + ((v >> 5) & 1)], 1u << (v & 31));
                    const u32 ls = (a.fesplit ? a.fesplit : a.lsplit)[v];
                    fe += ls;
                    mh += (u64)row[v + 1] - (u64)row[v] - ls;
                    ml += ls;
                }
            }
        }
        if (lane < PSC && gbase + lane < a.nwords) {
            const u64 word = (u64)newb[2 * lane] | ((u64)newb[2 * lane + 1] << 32);
            fout[gbase + lane] = word;
            a.mb[gbase + lane] = word;  // (no wave reads mb here: the probes read the map or dist)
            ccount += (u32)__popcll(word);
        }
    }
    v2_flush2(ccount, fe, a.ctl->cnt[cout], red);
    v2_flush2(mh, ml, a.ctl->mh, red);
    v2_flush_fmin(mn, a.ctl->cnt[cout], red);  // (min over every dist >= hi: below the next band's members)
    v2_flush_min(mn, a.ctl, red);
    v2_flush_work(a, V2W_HPULL, wk, esrc_bytes(v2_cw_src(a)), a.hmap ? 1u : 4u, red);
}

// Pull form of a light round (symmetric graphs): every vertex that can still
// improve (dist > lo) scans the light prefix of its own row (= its light
// in-edges) for in-neighbours in the round's frontier fin — a bitmap probe, fin
// being 1/32 of dist and mostly L2-resident — and stops once lo + w >= its best
// value. Run instead of the push when the frontier's light edges exceed
// pull_thresh (the big rounds of the first bands). No atomics: a lane writes only
// its own vertex. The wave owns its PSC words of fout (written whole) and of mb
// (new members add their heavy / light degrees to ctl.mh).
template <typename Off>
__device__ __forceinline__ void v2_pull_light_body(const V2Args& a, const Off* __restrict__ row,
                                                   const u64* __restrict__ fin, u64* __restrict__ fout, u32* newb,
                                                   int32_t flo, u32& newc, u64& fe, u64& mh, u64& ml, int32_t& fm,
                                                   V2Work& wk) {
    constexpr int NWV = DB / WAVE;
    const int lane = lane_id();
    const int32_t lo = a.lo, hi = a.hi;  // flo: the frontier's least distance (v2_pull_lo), >= lo
    const i64 nsc = (a.nwords + PSC - 1) / PSC;
    for (i64 sc = (i64)blockIdx.x * NWV + wave_id(); sc < nsc; sc += (i64)gridDim.x * NWV) {
        const i64 gbase = sc * PSC;
        // the frontier joins the members; new members add their heavy / light degrees (a
        // lane walks the bits of its word; a lane per vertex of the PSC words with the loads
        // issued together, PJ_V2_MBPAR in round 4, made the k26w solve 1.5x slower, r4a)
        u64 nmw = 0;
        if (lane < PSC && gbase + lane < a.nwords) {
            const u64 f = fin[gbase + lane];
            if (f) {
                const u64 old = a.mb[gbase + lane];
                nmw = f & ~old;
                if (nmw) a.mb[gbase + lane] = old | f;
            }
        }
        // (compacted: 64 new members per wave step, a lane each; one lane walking the bits of
        // its word serialized a frontier of millions of new members in 16 lanes of the wave:
        // +0.6%, profiles/r05/mbc_r5h10.txt)
        {
            const u32 mc = (u32)__popcll(nmw);
            const u32 mincl = wave_incl_scan(mc);
            const u32 mex = mincl - mc;
            const u32 MT = __shfl(mincl, 63, 64);
            for (u32 r0 = 0; r0 < MT; r0 += WAVE) {
                const u32 c = r0 + lane;
                u32 jw = 0;
#pragma unroll
                for (u32 step = PSC / 2; step > 0; step >>= 1) {
                    const u32 x = __shfl(mex, jw + step, 64);
                    if (x <= c) jw += step;
                }
                const u32 ex = __shfl(mex, jw, 64);
                const u64 tw = __shfl(nmw, jw, 64);
                if (c < MT) {
                    const i64 v = (gbase + jw) * 64 + select_bit(tw, c - ex);
                    const u64 rb = (u64)row[v], ls = a.lsplit[v];
                    mh += (u64)row[v + 1] - rb - ls;
                    ml += ls;
                }
            }
        }
        u64 mytodo = 0;
#pragma unroll
        for (int k = 0; k < PSC; ++k) {
            const i64 v = (gbase + k) * 64 + lane;
            const int32_t d = v < a.n ? a.dist[v] : 0;
            // (w1 filter: a frontier in-neighbour offers at least lo + the row's lightest weight;
            // round 4: +2.5%, profiles/r04/ab_r4a.txt)
            const int w1 = (v < a.n && d > lo) ? (int)a.w1[v] : 0;
            const u64 m = __ballot(v < a.n && d > lo && (long long)flo + w1 < (long long)d);
            if (lane == k) mytodo = m;
        }
        // a vertex without light edges has no light in-edge (symmetric graph): not a candidate
        if (a.hl && mytodo) mytodo &= a.hl[gbase + lane];
        if (lane < 2 * PSC) newb[lane] = 0;
        const u32 cnt = (u32)__popcll(mytodo);
        const u32 incl = wave_incl_scan(cnt);
        const u32 myex = incl - cnt;
        const u32 T = __shfl(incl, 63, 64);
        // candidate c of the wave's list: its vertex, dist and light-row bounds
        auto fetch = [&](u32 c, bool& act, i64& v, int32_t& d0, Off& k, u32& ls) {
            act = c < T;
            u32 jw = 0;
#pragma unroll
            for (u32 step = PSC / 2; step > 0; step >>= 1) {
                const u32 x = __shfl(myex, jw + step, 64);
                if (x <= c) jw += step;
            }
            const u32 ex = __shfl(myex, jw, 64);
            const u64 tw = __shfl(mytodo, jw, 64);
            v = act ? (gbase + jw) * 64 + select_bit(tw, c - ex) : 0;
            d0 = INT_INF;
            k = 0;
            ls = 0;
            if (act) {
                d0 = a.dist[v];
                if (a.ltail) {  // the tail: the light prefix of the row in the whole CSR, no long-row list
                    k = row[v];
                    ls = a.lsplit[v];
                } else {
                    k = (Off)a.lrow[v];
                    ls = (u32)(a.lrow[v + 1] - a.lrow[v]);
                }
            }
        };
        // (round 5: issuing the next 64 candidates' loads before this batch's scan measured
        // 0.5% slower, profiles/r05/ab_pfx_r5n.txt)
        for (u32 r0 = 0; r0 < T; r0 += WAVE) {
            bool act;
            i64 v;
            int32_t d0;
            Off k;
            u32 ls;
            fetch(r0 + lane, act, v, d0, k, ls);
            int32_t cur = d0;
            Off e = k;
            if (act) e = (a.ltail || ls <= V2_PLMAX) ? k + (Off)ls : k;  // long rows: v2_pull_long_body
            // (round 6: rows above 32 or 64 light edges sent wave-wide at once instead of walked
            // PSERIAL edges by their lane first measured 23% slower, profiles/r06/pwide_ab_r6g.txt)
            const Off lim = (e - k > (Off)PSERIAL) ? k + (Off)PSERIAL : e;
            bool go = act && k < lim, done = !act || k >= e;
            while (__ballot(go)) {
                // (counted with ballots in the wave-uniform loop: a start-of-row register held
                // over the loop spilled in this 72-VGPR kernel) records the step reads; each
                // row the step stops probes one fewer (PU - 1 fewer at most, when its first
                // record stops it)
                u32 r = 0;
#pragma unroll
                for (int j = 0; j < PU; ++j) r += (u32)__popcll(__ballot(go && k + (Off)j < lim));
                bool stp = false;
                if (go) {
                    if (pull_step_dist<Off>(v2_light_src(a), a.dist, k, lim, flo, hi, cur)) {
                        done = true;
                        go = false;
                        stp = true;
                    } else {
                        go = k < lim;
                        done = k >= e;
                    }
                }
                wk.add(r, r - (u32)__popcll(__ballot(stp)));
            }
            u64 open = __ballot(!done);
            while (open) {
                const int l = __ffsll((long long)open) - 1;
                open &= open - 1;
                const Off kb = __shfl(k, l, 64), ke = __shfl(e, l, 64);
                int32_t cl = __shfl(cur, l, 64);
                for (Off kk = kb; kk < ke; kk += WAVE) {
                    const Off k0 = kk + lane;
                    const bool valid = k0 < ke;
                    const u64 x = valid ? eat(v2_light_src(a), (u64)k0) : 0ull;
                    const u32 w = (u32)(x >> 32);
                    const bool stop = !valid || (long long)flo + w >= (long long)cl;
                    wk.add((u32)__popcll(__ballot(valid)), (u32)__popcll(__ballot(!stop)));
                    int32_t cand = INT_INF;
                    if (!stop) {
                        const int32_t du = pull_src(a.dist, (u32)x, hi);
                        if (du < INT_INF) {
                            const long long nd = (long long)du + w;
                            cand = nd < INT_INF ? (int32_t)nd : INT_INF;
                        }
                    }
#pragma unroll
                    for (int off = 32; off > 0; off >>= 1) {
                        const int32_t y = __shfl_xor(cand, off, 64);
                        cand = y < cand ? y : cand;
                    }
                    cl = cand < cl ? cand : cl;
                    if (__ballot(stop)) break;
                }
                if (lane == l) cur = cl;
            }
            if (act && cur < d0) {
                a.dist[v] = cur;
                if (cur < hi) {
                    if (cur < fm) fm = cur;
                    const i64 wl = (v >> 6) - gbase;
                    atomicOr(&newb[2 * wl + ((v >> 5) & 1)], 1u << (v & 31));
                    ++newc;
                    fe += ls;
                }
            }
        }
        // fout is zero at the start of a round and v2_pull_long_body may set bits of
        // the same words (long-row vertices) concurrently: OR the word in
        if (lane < PSC && gbase + lane < a.nwords) {
            const u64 word = (u64)newb[2 * lane] | ((u64)newb[2 * lane + 1] << 32);
            if (word) atomicOr(fout + gbase + lane, word);
        }
    }
}

// Long light rows (lsplit > V2_PLMAX, the high-degree vertices) are left out of
// v2_pull_light_body (round 5: chunks that published an improvement at once and re-read
// the row's distance every 64 edges scanned as many edges -- the hubs' rows hold their
// first frontier neighbour late -- and measured 0.5% slower, profiles/r05/ab_lpub_r5t.txt): one lane scanning tens of thousands of edges would hold up
// its wave. Their pull runs here instead, over a static list of (vertex, chunk
// of V2_PCH light edges) built once per delta; a wave takes a chunk, skips it
// when even its lightest edge cannot help, and folds the result in with
// atomicMin (the vertex's chunks run in different waves).
__device__ __forceinline__ void v2_pull_long_body(const V2Args& a, const u64* __restrict__ fin, u64* __restrict__ fout,
                                                  const u32* __restrict__ lcv, const u32* __restrict__ lcc, u64 nlc,
                                                  int32_t flo, u32& newc, u64& fe, int32_t& fm, V2Work& wk) {
    const int lane = lane_id();
    const int32_t lo = a.lo, hi = a.hi;
    for (u64 it = (u64)blockIdx.x * (DB / WAVE) + wave_id(); it < nlc; it += (u64)gridDim.x * (DB / WAVE)) {
        const u32 v = lcv[it];
        const int32_t d0 = dist_now(a.dist + v);
        if (d0 <= lo) continue;
        const u64 rb = a.lrow[v];
        const u32 ls = (u32)(a.lrow[v + 1] - rb);
        const u64 kb = rb + (u64)lcc[it] * V2_PCH;
        const u64 ke = min(rb + ls, kb + V2_PCH);
        wk.add(1u, 0u);  // (the chunk's first record, read by every lane for the skip test)
        if ((long long)flo + (eat(v2_light_src(a), kb) >> 32) >= (long long)d0) continue;
        int32_t cur = d0;
        for (u64 kk = kb; kk < ke; kk += WAVE) {
            const u64 k0 = kk + lane;
            const bool valid = k0 < ke;
            const u64 x = valid ? eat(v2_light_src(a), k0) : 0ull;
            const u32 w = (u32)(x >> 32);
            const bool stop = !valid || (long long)flo + w >= (long long)cur;
            wk.add((u32)__popcll(__ballot(valid)), (u32)__popcll(__ballot(!stop)));
            int32_t cand = INT_INF;
            if (!stop) {
                const int32_t du = pull_src(a.dist, (u32)x, hi);
                if (du < INT_INF) {
                    const long long nd = (long long)du + w;
                    cand = nd < INT_INF ? (int32_t)nd : INT_INF;
                }
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const int32_t y = __shfl_xor(cand, off, 64);
                cand = y < cand ? y : cand;
            }
            cur = cand < cur ? cand : cur;
            if (__ballot(stop)) break;
        }
        if (lane == 0 && cur < d0) {
            const int32_t old = atomicMin(a.dist + v, cur);
            if (cur < old && cur < hi) {
                if (cur < fm) fm = cur;
                const u64 bit = 1ull << (v & 63);
                if (!(atomicOr(fout + (v >> 6), bit) & bit)) {
                    ++newc;
                    fe += ls;
                }
            }
        }
    }
}

template <typename Off>
union V2RoundLds {  // the round kernel's LDS: a tile-dense push
    V2Dense<Off> push;
};

// One light round in one launch, decided on the device from the previous round's
// counters: a pull (the chunks of the long light rows, v2_pull_long_body, and the
// short rows, v2_pull_light_body, over the whole grid; the two touch disjoint
// vertices, frontier words are OR-ed in), a tile-dense push, or a sparse push.
template <typename Off>
__global__ __launch_bounds__(DB) V2_WPE_R void v2_pull_round_k(V2Args a, const Off* __restrict__ row, u64* __restrict__ fin,
                                                      u64* __restrict__ fout, int cin, u64 pull_thresh,
                                                      const u32* __restrict__ lcv, const u32* __restrict__ lcc, u64 nlc,
                                                      int hs, u64 dense_min, u64* __restrict__ fclr) {
    constexpr int NWV = DB / WAVE;
    __shared__ u32 s_new[NWV][2 * PSC];
    __shared__ u64 red[2 * NWV];
    __shared__ V2RoundLds<Off> lds;
    v2_zero_slot(a, (cin + 2) & 3);
    v2_clear_words(fclr, a.nwords);
    const u64 fcount = v2_slot_sum(a.ctl->cnt[cin]);
    if (a.rlog && blockIdx.x == 0 && threadIdx.x == 0) {  // (debug: round_log; one entry per launch)
        const u64 fe0 = v2_slot_edges(a.ctl->cnt[cin]);
        const u64 i = atomicAdd(a.rlog, 1ull);
        if (i < 255) {
            a.rlog[1 + 3 * i] = !fcount ? 3ull : fe0 > pull_thresh ? 2ull : (fcount > dense_min ? 1ull : 0ull);
            a.rlog[2 + 3 * i] = fcount;
            a.rlog[3 + 3 * i] = fe0 | ((u64)a.lo << 40);
        }
    }
    if (fcount == 0) return;
    if (v2_slot_edges(a.ctl->cnt[cin]) <= pull_thresh) {
        if (fcount <= dense_min) {  // a sparse push round
            v2_expand_body<Off, true>(a, row, fin, fout, cin, hs, red);
            return;
        }
        u32 newc = 0;
        u64 mh = 0, ml = 0, fe = 0;
        int32_t fm = INT_INF;
        V2Work wk;
        v2_dense_body<Off>(a, row, fin, fout, hs, newc, fe, mh, ml, fm, wk, lds.push);
        v2_flush2(newc, fe, a.ctl->cnt[(cin + 1) & 3], red);
        v2_flush_fmin(fm, a.ctl->cnt[(cin + 1) & 3], red);
        v2_flush2(mh, ml, a.ctl->mh, red);
        v2_flush_work(a, V2W_ROUND, wk, esrc_bytes(v2_light_src(a)), 4u, red, NWV);
        return;
    }
    u32 newc = 0;
    u64 fe = 0, mh = 0, ml = 0;
    int32_t fm = INT_INF;
    V2Work wk;
    const int32_t flo = v2_pull_lo(a, cin);
    if (nlc && !a.ltail) v2_pull_long_body(a, fin, fout, lcv, lcc, nlc, flo, newc, fe, fm, wk);
    v2_pull_light_body<Off>(a, row, fin, fout, s_new[wave_id()], flo, newc, fe, mh, ml, fm, wk);
    v2_flush2(newc, fe, a.ctl->cnt[(cin + 1) & 3], red);
    v2_flush_fmin(fm, a.ctl->cnt[(cin + 1) & 3], red);
    v2_flush2(mh, ml, a.ctl->mh, red);
    v2_flush_work(a, V2W_ROUND, wk, esrc_bytes(v2_light_src(a)), 4u, red);
}

// static chunk list of the long light rows: count, then append (order is irrelevant)
__global__ void v2_long_count_k(const u32* __restrict__ lsplit, i64 n, u64* __restrict__ cnt) {
    u64 c = 0;
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x)
        if (lsplit[v] > V2_PLMAX) c += (lsplit[v] + V2_PCH - 1) / V2_PCH;
    c = wave_sum(c);
    if (lane_id() == 0 && c) atomicAdd(cnt, c);
}
__global__ void v2_long_fill_k(const u32* __restrict__ lsplit, i64 n, u64* __restrict__ cnt, u32* __restrict__ lcv,
                               u32* __restrict__ lcc) {
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x)
        if (lsplit[v] > V2_PLMAX) {
            const u32 nc = (lsplit[v] + V2_PCH - 1) / V2_PCH;
            const u64 b = atomicAdd(cnt, (u64)nc);
            for (u32 c = 0; c < nc; ++c) {
                lcv[b + c] = (u32)v;
                lcc[b + c] = c;
            }
        }
}

// Interleaved copy of the relabeled CSR edges: cw[k] = col[k] | w[k] << 32.
__global__ void v2_interleave_k(const u32* __restrict__ col, const u32* __restrict__ w, i64 m, u64* __restrict__ cw) {
    for (i64 k = (i64)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (i64)gridDim.x * blockDim.x)
        cw[k] = (u64)col[k] | ((u64)w[k] << 32);
}
__global__ void widen_k(const uint8_t* __restrict__ w8, i64 m, u32* __restrict__ w) {
    for (i64 k = (i64)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (i64)gridDim.x * blockDim.x) w[k] = w8[k];
}
// Light CSR: lcw[lrow[v] + j] = the record of row[v] + j for j < lsplit[v], packed
// (col | w << cb) in 32 bits when it fits.
__device__ __forceinline__ void v2_lput(u64* __restrict__ o, u64 k, u64 x, u32) { o[k] = x; }
__device__ __forceinline__ void v2_lput(u32* __restrict__ o, u64 k, u64 x, u32 cb) {
    o[k] = (u32)x | ((u32)(x >> 32) << cb);
}
// (the edge records come from cw, or from the relabeled col / w arrays when cw is null)
template <typename WT>
__device__ __forceinline__ u64 v2_rec(const u64* __restrict__ cw, const u32* __restrict__ col,
                                      const WT* __restrict__ wt, u64 k) {
    return cw ? cw[k] : (u64)col[k] | ((u64)wt[k] << 32);
}
// Edge-tiled light CSR build (a lane-per-vertex form stored each lane's prefix to
// its own place: uncoalesced, 11 ms at s26): a block takes LT_E consecutive
// light-CSR positions, stages the light-row starts of the vertices they belong to in
// LDS (tile table lt_row, like relabel.hip's copy tiles) and copies LT_E / 256 entries
// per thread with coalesced stores, each row found by a binary search in LDS.
constexpr int LT_E = 1024;   // light-CSR positions per tile
constexpr int LT_R = 4096;   // light-row starts staged per tile (most vertices have no light edge)
__global__ void v2_light_tiles_k(const u64* __restrict__ lrow, i64 n, u64 light, u32* __restrict__ trow) {
    const i64 ntiles = (i64)((light + LT_E - 1) / LT_E);
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x) {
        const i64 b = (i64)lrow[v], e = (i64)lrow[v + 1];
        if (e <= b) continue;
        for (i64 t = (b + LT_E - 1) / LT_E; t * LT_E < e; ++t) trow[t] = (u32)v;
        if (e == (i64)light) trow[ntiles] = (u32)v;
    }
}
template <typename Off, typename OutT, typename WT>
__global__ __launch_bounds__(256) void v2_light_csr_tiled_k(const Off* __restrict__ row, const u64* __restrict__ lrow,
                                                            const u64* __restrict__ cw, const u32* __restrict__ col,
                                                            const WT* __restrict__ wt, u64 light,
                                                            const u32* __restrict__ trow, OutT* __restrict__ lcw,
                                                            u32 cb) {
    __shared__ u64 s_lb[LT_R + 1];
    const i64 ntiles = (i64)((light + LT_E - 1) / LT_E);
    for (i64 t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const u64 e0 = (u64)t * LT_E, e1 = min(e0 + (u64)LT_E, light);
        const u32 r0 = trow[t], r1 = trow[t + 1];
        const u32 nr = r1 - r0 + 1;
        const bool staged = nr <= (u32)LT_R + 1;
        if (staged)
            for (u32 j = threadIdx.x; j < nr; j += 256) s_lb[j] = lrow[r0 + j];
        __syncthreads();
#pragma unroll 4
        for (u64 k = e0 + threadIdx.x; k < e1; k += 256) {
            u32 a = 0, b = nr - 1;  // largest j with lrow[r0 + j] <= k
            while (a < b) {
                const u32 mid = (a + b + 1) >> 1;
                if ((staged ? s_lb[mid] : lrow[r0 + mid]) <= k) a = mid;
                else b = mid - 1;
            }
            const u64 lb = staged ? s_lb[a] : lrow[r0 + a];
            const u64 rb = (u64)row[r0 + a];
            v2_lput(lcw, k, v2_rec(cw, col, wt, rb + (k - lb)), cb);
        }
        __syncthreads();
    }
}

// heavy edges (w >= the current light threshold) of the vertices not settled
// below lo: the pull decision's heavy_left after a switch of the threshold
template <typename Off>
__global__ __launch_bounds__(DB) void v2_heavy_left_k(const Off* __restrict__ row, const u32* __restrict__ lsplit,
                                                      const int32_t* __restrict__ dist, i64 n, int32_t lo,
                                                      u64* __restrict__ out) {
    u64 acc = 0;
    for (i64 v = (i64)blockIdx.x * DB + threadIdx.x; v < n; v += (i64)gridDim.x * DB)
        if (dist[v] >= lo) acc += (u64)(row[v + 1] - row[v]) - lsplit[v];
    acc = wave_sum(acc);
    if (lane_id() == 0 && acc) atomicAdd(out, acc);
}



// hw[v] = the weight of v's first heavy edge (row[v] + lsplit[v]; rows are weight-sorted),
// capped at 255, or 0 when v has no heavy edge (heavy weights are >= the threshold >= 1)
// w1[v] = the lightest weight of v's row (its first: rows are weight-sorted), capped at 255
template <typename Off, typename WT>
__global__ void v2_w1_k(const Off* __restrict__ row, const WT* __restrict__ w, i64 n, uint8_t* __restrict__ w1) {
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x) {
        const u64 b = (u64)row[v], e = (u64)row[v + 1];
        w1[v] = b < e ? (uint8_t)min(255u, (u32)w[b]) : (uint8_t)255;
    }
}

template <typename Off, typename WT>
__global__ void v2_hw_k(const Off* __restrict__ row, const u32* __restrict__ lsplit, const WT* __restrict__ w, i64 n,
                        uint8_t* __restrict__ hw) {
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x) {
        const u64 b = (u64)row[v] + lsplit[v], e = (u64)row[v + 1];
        hw[v] = b < e ? (uint8_t)max(1u, min(255u, (u32)w[b])) : (uint8_t)0;
    }
}

// hl bit v = (lsplit[v] > 0): the vertices that have light edges for this delta
__global__ void v2_haslight_k(const u32* __restrict__ lsplit, i64 n, u64* __restrict__ hl) {
    const i64 nw = (n + 63) / 64;
    for (i64 wi = ((i64)blockIdx.x * blockDim.x + threadIdx.x) / WAVE; wi < nw;
         wi += (i64)gridDim.x * blockDim.x / WAVE) {
        const i64 v = wi * 64 + lane_id();
        const u64 m = __ballot(v < n && lsplit[v] > 0);
        if (lane_id() == 0) hl[wi] = m;
    }
}

}  // namespace

// The state of one solve in flight: its stream, distances (relabeled ids), frontier
// ring, member bitmap, counters and hub queues. DeltaWork owns one for single-source
// solves (on the ctx stream) and more for concurrent batches (delta_batch).
struct DeltaSolve {
    hipStream_t s = nullptr;
    bool own_stream = false;
    int32_t* dist = nullptr;   // relabeled distances (R.dist for the main solve)
    DevBuf<int32_t> dist_own;  // (extra solves)
    int32_t* out = nullptr;    // distances in input ids (g.dist for the main solve)
    DevBuf<int32_t> out_own;
    DevBuf<u64> f[3], mb;      // light-round frontier ring (v2_clear_words), band members
    DevBuf<u64> sb;            // settled-before-the-tail bitmap
    DevBuf<uint8_t> hmap;      // the heavy pull's probe map (v2_hmap_k)
    DevBuf<u64> db;            // members whose far heavy edges are deferred (defer_heavy); all zero
    bool db_dirty = true;      // unless a solve stopped with a deferral pending (an error)
    DevBuf<V2Ctl> ctl;
    V2Ctl* hctl = nullptr;     // mapped pinned host copy, written by v2_publish_k
    V2Ctl* hctl_dev = nullptr;
    u64* hseq = nullptr;       // mapped pinned sequence word of v2_publish_k
    u64* hseq_dev = nullptr;
    u64 seq = 0;
    DevBuf<u32> hv;
    DevBuf<u64> hbeg, hoff;
    u64 hcap = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    pj_stats st{};
    ~DeltaSolve() {
        if (hctl) (void)hipHostFree(hctl);
        if (hseq) (void)hipHostFree(hseq);
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (own_stream && s) (void)hipStreamDestroy(s);
    }
};

// Per graph and light threshold: the light prefixes, the light CSR, the has-light
// bitmap, the long-row chunk list and the edge records (shared read-only by every
// solve in flight), plus the main solve.
struct DeltaWork {
    DevBuf<u32> lsplit;
    DevBuf<u32> lsplit2;   // light prefixes for the tail threshold (g.tail_delta)
    u32 lsplit2_delta = 0;
    long long maxw = -1;   // largest edge weight (-1: not computed)
    u32 lsplit_delta = 0;  // delta lsplit was computed for (0 = none)
    u64 heavy_total = 0;   // edges with w >= delta (for the pull decision)
    u64 light_total = 0;   // edges with w < delta
    DevBuf<u32> lcv, lcc;  // long light rows: (vertex, chunk) work items
    u64 nlc = 0;
    DevBuf<u64> cw;        // interleaved relabeled edges
    ScanWs lscan;
    DevBuf<u64> lrow, lcw; // light CSR (per delta)
    DevBuf<u32> lcw32;     // the light CSR packed (col | w << lcb), when it fits
    u32 lcb = 0;
    int packed_for = -1;   // g.light_pack the light CSR was built for
    DevBuf<u64> hl;        // has-light-edges bitmap (per delta)
    DevBuf<uint8_t> hw, hw2;  // first heavy weight per vertex for delta / the tail threshold (v2_hw_k)
    DevBuf<uint8_t> w1;       // lightest weight per vertex (any threshold, v2_w1_k)
    DeltaSolve main;
    std::vector<std::unique_ptr<DeltaSolve>> extra;  // concurrent batch solves
};

void delete_delta_work(DeltaWork* p) { delete p; }

// device bytes of a weighted graph's solver state: the relabeled copy and the delta
// workspace with its solve slots (what delta_solve / delta_batch added to the graph's CSR)
i64 delta_device_bytes(const Graph& g) {
    size_t b = 0;
    if (g.rl) {
        const Relabeled& R = *g.rl;
        b += R.perm.bytes() + R.inv.bytes() + R.row32.bytes() + R.row64.bytes() + R.col.bytes() + R.w8.bytes() +
             R.w.bytes() + R.dist.bytes();
    }
    if (g.delta_work) {
        const DeltaWork& w = *g.delta_work;
        b += w.lsplit.bytes() + w.lsplit2.bytes() + w.lcv.bytes() + w.lcc.bytes() + w.cw.bytes() + w.lrow.bytes() +
             w.lcw.bytes() + w.lcw32.bytes() + w.hl.bytes() + w.hw.bytes() + w.hw2.bytes() + w.w1.bytes();
        auto slot = [&](const DeltaSolve& v) {
            b += v.dist_own.bytes() + v.out_own.bytes() + v.f[0].bytes() + v.f[1].bytes() + v.f[2].bytes() +
                 v.mb.bytes() + v.sb.bytes() + v.hmap.bytes() + v.db.bytes() + v.ctl.bytes() + v.hv.bytes() +
                 v.hbeg.bytes() + v.hoff.bytes();
        };
        slot(w.main);
        for (const auto& x : w.extra) slot(*x);
    }
    return (i64)b;
}

void preload_delta_module() {
    hipFuncAttributes fa;
    (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&light_split_k<u32, uint8_t>));
}

namespace {

// u32 relabeled weights, widened from the relabel copy's u8 weights on first use
// (the v1 band loop and the interleaved records read u32)
void ensure_w32(Graph& g) {
    Relabeled& R = *g.rl;
    if (R.w.p || !R.w8.p || g.nnz == 0) return;
    R.w.alloc((size_t)g.nnz);
    widen_k<<<grid_for(g.nnz, 256, (unsigned)g.ctx->cu_count * 8u), 256, 0, g.ctx->stream>>>(R.w8.p, g.nnz, R.w.p);
    PJ_LAUNCH_CHECK();
}

template <typename Off>
void launch_light_split(const Relabeled& R, const Off* row, i64 n, u32 delta, u32* out, unsigned maxgrid,
                        hipStream_t s) {
    if (R.w8.p) light_split_k<Off, uint8_t><<<grid_for(n, 256, maxgrid), 256, 0, s>>>(row, R.w8.p, n, delta, out);
    else light_split_k<Off, u32><<<grid_for(n, 256, maxgrid), 256, 0, s>>>(row, R.w.p, n, delta, out);
    PJ_LAUNCH_CHECK();
}

template <typename Off>
void launch_hw(const Relabeled& R, const Off* row, const u32* lsplit, i64 n, DevBuf<uint8_t>& out, unsigned maxgrid,
               hipStream_t s) {
    out.ensure((size_t)std::max<i64>(n, 1));
    if (R.w8.p) v2_hw_k<Off, uint8_t><<<grid_for(n, 256, maxgrid), 256, 0, s>>>(row, lsplit, R.w8.p, n, out.p);
    else v2_hw_k<Off, u32><<<grid_for(n, 256, maxgrid), 256, 0, s>>>(row, lsplit, R.w.p, n, out.p);
    PJ_LAUNCH_CHECK();
}

template <typename Off, typename OutT>
void light_csr_tiled(const Relabeled& R, const Off* row, const DeltaWork& w, u64 light, const u32* ltrow, OutT* out,
                     u32 cb, unsigned grid, hipStream_t s) {
    if (R.w8.p)
        v2_light_csr_tiled_k<Off, OutT, uint8_t><<<grid, 256, 0, s>>>(row, w.lrow.p, w.cw.p, R.col.p, R.w8.p, light,
                                                                      ltrow, out, cb);
    else
        v2_light_csr_tiled_k<Off, OutT, u32><<<grid, 256, 0, s>>>(row, w.lrow.p, w.cw.p, R.col.p, R.w.p, light,
                                                                  ltrow, out, cb);
}

// delta (explicit option, else auto_delta: c(n) x mean weight / mean out-degree over all
// input ids, internal.h; light edges are then ~4-5% of a row) and, once per delta, the
// light prefix length of every row and the number of heavy edges.
int32_t tail_delta_of(const Graph& g, int32_t delta) {
    return (int32_t)std::min(65536.0, g.tail_delta < 0 ? 64.0 * delta : g.tail_delta);
}

template <typename Off>
int32_t prepare_delta(Graph& g, DeltaWork& w) {
    Ctx& ctx = *g.ctx;
    hipStream_t s = ctx.stream;
    Relabeled& R = *g.rl;
    const i64 n = R.n_scan;
    const Off* row = static_cast<const Off*>(R.row_ptr(g.off64));
    const unsigned maxgrid = (unsigned)ctx.cu_count * 8u;
    int32_t delta = (int32_t)g.delta;
    if (delta <= 0) delta = (int32_t)auto_delta((double)g.n, (double)g.nnz, g.mean_weight);
    w.maxw = std::max(0ll, g.max_weight);  // (the relabel copy's reduction; the relabeled weights are the same)
    // whole-CSR records: u32 ids + u8 weights (split) when every weight fits 8 bits (the
    // relabel copy then wrote them as u8), else the interleaved u64 copy
    const bool split = g.split_w && R.w8.p;
    if (!split && !w.cw.p && g.nnz > 0) {
        ensure_w32(g);
        w.cw.alloc((size_t)g.nnz);
        v2_interleave_k<<<grid_for(g.nnz, 256, maxgrid), 256, 0, s>>>(R.col.p, R.w.p, g.nnz, w.cw.p);
        PJ_LAUNCH_CHECK();
    }
    if ((w.lsplit_delta != (u32)delta || w.packed_for != g.light_pack) && n > 0) {
        w.packed_for = g.light_pack;
        launch_light_split<Off>(R, row, n, (u32)delta, w.lsplit.p, maxgrid, s);
        w.lsplit_delta = (u32)delta;
        DevBuf<u64> acc(1);
        PJ_HIP(hipMemsetAsync(acc.p, 0, sizeof(u64), s));
        wsum_k<<<grid_for(n, DB, maxgrid), DB, 0, s>>>(w.lsplit.p, n, acc.p);
        PJ_LAUNCH_CHECK();
        u64 light = 0;
        PJ_HIP(hipMemcpyAsync(&light, acc.p, sizeof(u64), hipMemcpyDeviceToHost, s));
        PJ_HIP(hipStreamSynchronize(s));
        w.heavy_total = (u64)g.nnz - light;
        w.light_total = light;
        PJ_HIP(hipMemsetAsync(acc.p, 0, sizeof(u64), s));
        v2_long_count_k<<<grid_for(n, 256, maxgrid), 256, 0, s>>>(w.lsplit.p, n, acc.p);
        PJ_LAUNCH_CHECK();
        PJ_HIP(hipMemcpyAsync(&w.nlc, acc.p, sizeof(u64), hipMemcpyDeviceToHost, s));
        PJ_HIP(hipStreamSynchronize(s));
        launch_hw<Off>(R, row, w.lsplit.p, n, w.hw, maxgrid, s);
        if (!w.w1.p) {
            w.w1.alloc((size_t)std::max<i64>(n, 1));
            if (R.w8.p) v2_w1_k<Off, uint8_t><<<grid_for(n, 256, maxgrid), 256, 0, s>>>(row, R.w8.p, n, w.w1.p);
            else v2_w1_k<Off, u32><<<grid_for(n, 256, maxgrid), 256, 0, s>>>(row, R.w.p, n, w.w1.p);
            PJ_LAUNCH_CHECK();
        }
        // the light CSR of this delta
        w.hl.alloc((size_t)(n + 63) / 64);
        v2_haslight_k<<<grid_for(n, 256, maxgrid), 256, 0, s>>>(w.lsplit.p, n, w.hl.p);
        PJ_LAUNCH_CHECK();
        w.lrow.alloc((size_t)n + 1);
        exclusive_scan_u32(w.lsplit.p, w.lrow.p, n, w.lscan, s);
        // packed light records when every light weight (< delta) fits the bits above the ids
        int wb = 1;
        while ((1ll << wb) < (long long)delta) ++wb;
        const u32 cb = (u32)(32 - wb);
        w.lcb = (g.light_pack && wb < 32 && (u64)n <= (1ull << cb)) ? cb : 0u;
        w.lcw.release();
        w.lcw32.release();
        const i64 lt = (i64)((light + LT_E - 1) / LT_E);
        DevBuf<u32> ltrow((size_t)lt + 1);
        if (light) {
            v2_light_tiles_k<<<grid_for(n, 256, maxgrid), 256, 0, s>>>(w.lrow.p, n, light, ltrow.p);
            PJ_LAUNCH_CHECK();
        }
        const unsigned ltgrid = (unsigned)std::max<i64>(1, std::min<i64>(lt, (i64)ctx.cu_count * 8));
        if (w.lcb) {
            w.lcw32.alloc(std::max<u64>(light, 1));
            if (light) light_csr_tiled<Off, u32>(R, row, w, light, ltrow.p, w.lcw32.p, w.lcb, ltgrid, s);
        } else {
            w.lcw.alloc(std::max<u64>(light, 1));
            if (light) light_csr_tiled<Off, u64>(R, row, w, light, ltrow.p, w.lcw.p, 0u, ltgrid, s);
        }
        PJ_LAUNCH_CHECK();
        PJ_HIP(hipStreamSynchronize(s));  // (ltrow is freed on return)
        w.lcv.alloc(std::max<u64>(w.nlc, 1));
        w.lcc.alloc(std::max<u64>(w.nlc, 1));
        PJ_HIP(hipMemsetAsync(acc.p, 0, sizeof(u64), s));
        if (w.nlc) {
            v2_long_fill_k<<<grid_for(n, 256, maxgrid), 256, 0, s>>>(w.lsplit.p, n, acc.p, w.lcv.p, w.lcc.p);
            PJ_LAUNCH_CHECK();
        }
        PJ_HIP(hipStreamSynchronize(s));
    }
    // the tail's light prefixes (lsplit2), prepared here so that concurrent solves only read
    const int32_t tdelta = tail_delta_of(g, delta);
    if (tdelta > delta && w.lsplit2_delta != (u32)tdelta && n > 0) {
        w.lsplit2.ensure((size_t)n);
        launch_light_split<Off>(R, row, n, (u32)tdelta, w.lsplit2.p, maxgrid, s);
        launch_hw<Off>(R, row, w.lsplit2.p, n, w.hw2, maxgrid, s);
        w.lsplit2_delta = (u32)tdelta;
        PJ_HIP(hipStreamSynchronize(s));
    }
    return delta;
}

// copies the counter block to mapped host memory, then (system-scope release) the
// sequence number the host spins on; then resets the counters the host consumes
// per check (the members' degree sums mh, which the host accumulates over a band's
// checks, and minv), so no memset launch precedes the next band or heavy step
__global__ __launch_bounds__(256) void v2_publish_k(V2Ctl* __restrict__ ctl, u64* __restrict__ host, u64* seqp,
                                                    u64 seq) {
    const u64* c = reinterpret_cast<const u64*>(ctl);
    constexpr int nw = sizeof(V2Ctl) / sizeof(u64);
    for (int i = threadIdx.x; i < nw; i += 256) host[i] = c[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(seqp, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (threadIdx.x < V2_NSH) {
        ctl->mh[threadIdx.x].v = 0;
        ctl->mh[threadIdx.x].pad[0] = 0;
    }
    if (threadIdx.x < V2_NSH) ctl->minv[threadIdx.x].v = ~0ull;
}

// solve start in one launch: dist := INF (the source 0), frontier 0 := {source},
// frontier 1 and the member bitmap := 0, counters := 0 with the source counted
__global__ void v2_init_k(int32_t* __restrict__ dist, i64 n, i64 nwords, i64 src, u64* __restrict__ f0,
                          u64* __restrict__ f1, u64* __restrict__ mb, V2Ctl* __restrict__ ctl) {
    const i64 stride = (i64)gridDim.x * blockDim.x;
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += stride) dist[v] = v == src ? 0 : INT_INF;
    for (i64 wi = (i64)blockIdx.x * blockDim.x + threadIdx.x; wi < nwords; wi += stride) {
        f0[wi] = (src >= 0 && wi == (src >> 6)) ? 1ull << (src & 63) : 0ull;
        f1[wi] = 0;
        mb[wi] = 0;
    }
    if (blockIdx.x == 0) {
        u64* c = reinterpret_cast<u64*>(ctl);
        for (int i = threadIdx.x; i < (int)(sizeof(V2Ctl) / sizeof(u64)); i += blockDim.x) c[i] = 0;
        __syncthreads();
        if (threadIdx.x < V2_NSH) ctl->minv[threadIdx.x].v = ~0ull;
        // frontier minimum of the ring's slots: the source's 0 in slot 0, none elsewhere
        if (threadIdx.x < 3 * V2_NSH) ctl->cnt[1 + threadIdx.x / V2_NSH][threadIdx.x % V2_NSH].pad[1] = (u64)INT_INF;
        if (threadIdx.x == 0 && src >= 0) ctl->cnt[0][0].v = 1;
    }
}

// Buffers of a solve (allocated once per solve slot).
void ensure_solve(Graph& g, DeltaSolve& v) {
    if (v.hctl) return;
    Relabeled& R = *g.rl;
    const i64 n = R.n_scan;
    const size_t nw = n ? (size_t)((n + 63) / 64) : 1;
    v.f[0].alloc(nw);
    v.f[1].alloc(nw);
    v.f[2].alloc(nw);
    v.mb.alloc(nw);
    v.sb.alloc(nw);
    v.db.alloc(nw);
    v.hmap.alloc((size_t)(n ? n : 1) + 16);
    v.ctl.alloc(1);
    v.hcap = (u64)std::max<i64>(1, std::min<i64>(n, g.nnz / (i64)V2_HT + 1));
    v.hv.alloc(3 * v.hcap);  // the hub queue's ring of three slots
    v.hbeg.alloc(3 * v.hcap);
    v.hoff.alloc(3 * v.hcap);
    PJ_HIP(hipHostMalloc(reinterpret_cast<void**>(&v.hctl), sizeof(V2Ctl), hipHostMallocMapped));
    PJ_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&v.hctl_dev), v.hctl, 0));
    PJ_HIP(hipHostMalloc(reinterpret_cast<void**>(&v.hseq), 64, hipHostMallocMapped | hipHostMallocCoherent));
    PJ_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&v.hseq_dev), v.hseq, 0));
    *v.hseq = 0;
    v.seq = 0;
    if (!v.ev0) PJ_HIP(hipEventCreate(&v.ev0));
    if (!v.ev1) PJ_HIP(hipEventCreate(&v.ev1));
}

// One single-source solve on v's stream into v.dist (relabeled ids), and with unlabel set
// into v.out (input ids) as well; the preparation of delta (prepare_delta) has run. Reads
// only the shared graph and DeltaWork arrays, so solves of different DeltaSolve slots may
// run concurrently from different host threads. Returns the source's relabeled id (>= n_scan:
// a source without edges, -1: out of range).
template <typename Off>
i64 delta2_run(Graph& g, DeltaWork& w, DeltaSolve& v, int32_t delta, i64 source, bool unlabel) {
    Ctx& ctx = *g.ctx;
    hipStream_t s = v.s;
    Relabeled& R = *g.rl;
    const i64 n = R.n_scan;
    const i64 nwords = (n + 63) / 64;
    const Off* row = static_cast<const Off*>(R.row_ptr(g.off64));
    // host check of the buffers every band kernel dereferences (a missing allocation is an
    // error here, not a device fault)
    if (n > 0 && (!row || !v.dist || !v.out || !v.f[0].p || !v.f[1].p || !v.f[2].p || !v.mb.p || !v.sb.p ||
                  !v.ctl.p || !v.hv.p || !v.hbeg.p || !v.hoff.p || v.hv.n < 3 * v.hcap || !w.lsplit.p ||
                  !w.lrow.p || (!w.lcw.p && !w.lcw32.p) || !w.w1.p || !w.hw.p || !v.hmap.p))
        throw Error(PJ_ERR_HIP, "delta-stepping: a solver buffer is missing (internal error)");
    const unsigned maxgrid = (unsigned)ctx.cu_count * (unsigned)PJ_V2_GPC;  // workgroups per CU of the v2 kernels (grid-stride)
    const unsigned pullgrid = (unsigned)ctx.cu_count * (unsigned)PJ_V2_GPC_PULL;
    // light-round grids (grid-stride kernels): a launch that finds its round empty costs
    // in proportion to its workgroups, so these may be sized to the resident capacity
    const unsigned roundgrid = g.round_gpc > 0 ? (unsigned)ctx.cu_count * (unsigned)g.round_gpc : pullgrid;
    const unsigned hubgrid = g.hub_gpc > 0 ? (unsigned)ctx.cu_count * (unsigned)g.hub_gpc : maxgrid;
    const unsigned heavygrid = g.heavy_gpc > 0 ? (unsigned)ctx.cu_count * (unsigned)g.heavy_gpc : pullgrid;
    // band width: at most the light threshold (an edge that can stay inside its
    // band must be light, so the band's light rounds see it)
    int32_t bw = g.band_width > 0 ? std::min<int32_t>(delta, (int32_t)g.band_width) : delta;
    ensure_solve(g, v);
    V2Args a{};
    a.n = n;
    a.nwords = nwords;
    a.dist = v.dist;
    a.lsplit = w.lsplit.p;
    a.cw = w.cw.p;
    a.lrow = w.lrow.p;
    a.lcw = w.lcw.p;
    a.lcw32 = w.lcb ? w.lcw32.p : nullptr;
    a.lcb = w.lcb;
    a.col = R.col.p;
    a.w8 = g.split_w ? R.w8.p : nullptr;
    a.hl = g.light_filter ? w.hl.p : nullptr;
    a.hw = w.hw.p;
    a.w1 = w.w1.p;
    // light rounds whose frontier holds more than dense_frac x n vertices run tile-dense
    const u64 dense_min = g.dense_frac > 0.0 ? (u64)(g.dense_frac * (double)n) : ~0ull;
    a.mb = v.mb.p;
    a.ctl = v.ctl.p;
    a.hv = v.hv.p;
    a.hbeg = v.hbeg.p;
    a.hoff = v.hoff.p;
    a.hcap = v.hcap;
    DevBuf<u64> rlog;
    if (g.round_log) {
        rlog.alloc(1 + 3 * 255);
        PJ_HIP(hipMemsetAsync(rlog.p, 0, sizeof(u64), s));
        a.rlog = rlog.p;
    }
    a.hz = INT_INF;
    a.dsave = nullptr;
    a.hmap = nullptr;
    // the heavy pull's probe map over [mlo, mhi) when its values fit a byte (else dist is
    // probed): v2_pull_k 853 -> 789 us per k26w solve for 34 us of map building (round 5,
    // profiles/r05/hmap_r5h23.txt)
    auto set_hmap = [&](int32_t mlo, int32_t mhi) {
        a.hmap = nullptr;
        if (n == 0 || (long long)mhi - (long long)mlo > 255) return;
        v2_hmap_k<<<grid_for((n + 3) / 4, 256, maxgrid), 256, 0, s>>>(v.dist, n, mlo, mhi, v.hmap.p);
        PJ_LAUNCH_CHECK();
        a.hmap = v.hmap.p;
    };
    // the host's view of the counters: one block copies them into mapped host memory
    // (a D2H hipMemcpyAsync of the same 3.3 KB ran as a ~30 us blit per sync)
    // The host spins on the sequence number (wakes within ~1 us of the copy instead of
    // the stream synchronization's latency); after 0.2 s of spinning it synchronizes the
    // stream, which surfaces a failed kernel instead of spinning forever.
    auto publish_ctl = [&]() {
        const u64 seq = ++v.seq;
        v2_publish_k<<<1, 256, 0, s>>>(v.ctl.p, reinterpret_cast<u64*>(v.hctl_dev), v.hseq_dev, seq);
        PJ_LAUNCH_CHECK();
        return seq;
    };
    auto wait_ctl = [&](u64 seq) {
        if (g.spin_sync) {
            const auto t0 = std::chrono::steady_clock::now();
            while (__atomic_load_n(v.hseq, __ATOMIC_ACQUIRE) != seq) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
                    PJ_HIP(hipStreamSynchronize(s));
                    break;
                }
            }
        } else {
            PJ_HIP(hipStreamSynchronize(s));
        }
    };
    auto sync_ctl = [&]() { wait_ctl(publish_ctl()); };
    auto slot = [&](int c) {
        u64 t = 0;
        for (int i = 0; i < V2_NSH; ++i) t += v.hctl->cnt[c][i].v;
        return t;
    };
    auto hminv = [&]() {
        u64 m = ~0ull;
        for (int i = 0; i < V2_NSH; ++i) m = std::min<u64>(m, v.hctl->minv[i].v);
        return m;
    };

    pj_stats st{};
    const bool valid = source >= 0 && source < g.n;
    const i64 ls = valid ? relabeled_id(R, source, s) : -1;  // the source's new id (before the timed region)
    auto t_host0 = std::chrono::steady_clock::now();
    PJ_HIP(hipEventRecord(v.ev0, s));
    if (n > 0) {
        v2_init_k<<<grid_for(n, 256, maxgrid), 256, 0, s>>>(v.dist, n, nwords, (valid && ls < n) ? ls : -1,
                                                            v.f[0].p, v.f[1].p, v.mb.p, v.ctl.p);
        PJ_LAUNCH_CHECK();
    }
    if (valid && ls < n) {
        if (v.db_dirty) {
            PJ_HIP(hipMemsetAsync(v.db.p, 0, sizeof(u64) * (size_t)nwords, s));
            v.db_dirty = false;
        }
        int cs = 0, hr = 0, fi = 0;
        long long lo = 0;
        u64 heavy_left = w.heavy_total, light_left = w.light_total;
        const bool can_pull = g.symmetric && g.pull_factor > 0.0;
        bool can_pull_light = g.symmetric && g.light_pull > 0.0;
        double light_pull = g.light_pull;  // (tail_light_pull once in the tail)
        bool tail = false;
        u64 tail_unsettled = 0;
        const int32_t tdelta = tail_delta_of(g, delta);
        // Deferred band check: after a heavy step the host does not wait for its
        // counters; it enqueues the next band's first rounds at once and learns at their
        // check whether that band had any vertex (its start slot survives the first two
        // rounds of the counter ring) and, if not, the next occupied band (minv of the
        // heavy step, copied by the same publish before it resets minv).
        const bool defer_ok = g.defer_check && g.round_batch <= 2;
        bool deferred = false;
        bool finished = false;
        // Deferred far heavy edges (defer_heavy): a heavy push of a band whose members hold
        // many heavy edges relaxes only those landing in the next band; the members stay in db
        // and their other heavy edges go with the next heavy step -- a pull that takes its stop
        // rule from their band (lo_def), or a push of db's whole heavy rows first. Before an
        // empty band's jump or the end, db is pushed whole (flush_def).
        u64 mh_carry = 0, ml_carry = 0;  // (the next band's members' degrees, counted by its selection and published early)
        bool dpend = false;
        long long lo_def = 0;
        u64 mh_def = 0;
        auto push_heavy = [&](u64* members, int32_t hz, u64* dsave) {
            a.hz = hz;
            a.dsave = dsave;
            v2_heavy_push_k<Off><<<maxgrid, DB, 0, s>>>(a, row, members, hr);
            PJ_LAUNCH_CHECK();
            v2_hub_k<false><<<maxgrid, DB, 0, s>>>(a, nullptr, cs, hr, (hr + 1) % 3);
            PJ_LAUNCH_CHECK();
            a.hz = INT_INF;
            a.dsave = nullptr;
            hr = (hr + 1) % 3;
            st.td_levels++;
        };
        // push db whole, then select the band from nlo (the bands below it are settled)
        // (or, by the heavy-pull rule, a pull from lo_def that selects that band itself)
        auto flush_def = [&](long long nlo) {
            const int32_t nhi = (int32_t)std::min<long long>(nlo + bw, INT_INF);
            if (can_pull && (double)heavy_left < g.pull_factor * (double)mh_def) {
                a.lo = (int32_t)lo_def;
                a.hi = (int32_t)nlo;
                set_hmap(a.lo, a.hi);
                v2_pull_k<Off><<<heavygrid, DB, 0, s>>>(a, row, v.f[fi].p, nhi, cs);
                a.hmap = nullptr;
                PJ_LAUNCH_CHECK();
                PJ_HIP(hipMemsetAsync(v.db.p, 0, sizeof(u64) * (size_t)nwords, s));
                st.bu_levels++;
            } else {
                push_heavy(v.db.p, INT_INF, nullptr);
                a.lo = (int32_t)nlo;
                a.hi = nhi;
                v2_select_k<Off><<<maxgrid, DB, 0, s>>>(a, row, v.f[fi].p, cs);
                PJ_LAUNCH_CHECK();
            }
            a.lo = (int32_t)nlo;
            a.hi = nhi;
            dpend = false;
            v.db_dirty = false;
            mh_def = 0;
        };
        while (lo < INT_INF && !finished) {
            const int32_t hi = (int32_t)std::min<long long>(lo + bw, INT_INF);
            a.lo = (int32_t)lo;
            a.hi = hi;
            st.levels++;
            // members' heavy / light degree sums (reset by every publish; the band's first
            // members were counted by its selection, read by a publish after the heavy step)
            u64 mh = mh_carry, ml = ml_carry;
            mh_carry = ml_carry = 0;
            const int cs_start = cs;
            bool jumped = false;
            // light rounds until the band's frontier is empty, launched round_batch per
            // host check, doubling (starting each band at the previous band's round count,
            // or at 4 or 8, measured slower: idle rounds cost more than the checks they save)
            int K = g.round_batch;
            for (;;) {
                const u64 pull_thresh = can_pull_light ? (u64)((double)light_left / light_pull) : ~0ull;
                auto round = [&]() {
                    u64* fin = v.f[fi].p;
                    u64* fout = v.f[(fi + 1) % 3].p;
                    u64* fclr = v.f[(fi + 2) % 3].p;
                    // one launch decides pull / tile-dense push / sparse push on the device
                    v2_pull_round_k<Off><<<roundgrid, DB, 0, s>>>(a, row, fin, fout, cs, pull_thresh, w.lcv.p,
                                                                 w.lcc.p, w.nlc, hr, dense_min, fclr);
                    PJ_LAUNCH_CHECK();
                    v2_hub_k<true><<<hubgrid, DB, 0, s>>>(a, fout, cs, hr, (hr + 1) % 3);
                    PJ_LAUNCH_CHECK();
                    fi = (fi + 1) % 3;
                    cs = (cs + 1) & 3;
                    hr = (hr + 1) % 3;
                    st.relax_rounds++;
                };
                for (int q = 0; q < K; ++q) round();
                // spec_round: one more round enqueued behind the publish runs while the host waits
                // for it -- the next round of the band, or an empty one (a launch that reads a zero
                // count) when the band has ended; the ring state stays consistent either way, since
                // every later step writes its frontier words whole and counts into a slot the rounds
                // before zeroed
                const int cpub = cs;
                const u64 pseq = publish_ctl();
                for (int q = 0; q < g.spec_round; ++q) round();
                wait_ctl(pseq);
                if (deferred) {
                    deferred = false;
                    if (slot(cs_start) == 0 && dpend) {  // empty, but deferred edges may land past it
                        st.levels--;
                        lo = hi;
                        flush_def(lo);
                        deferred = true;
                        jumped = true;
                        break;
                    }
                    if (slot(cs_start) == 0) {  // the band was empty: its rounds were idle
                        st.levels--;
                        const u64 mv = hminv();
                        if (mv >= (u64)INT_INF) {  // nothing reached beyond the settled bands
                            finished = true;
                            break;
                        }
                        lo = (long long)mv / bw * bw;  // jump to the next occupied band
                        a.lo = (int32_t)lo;
                        a.hi = (int32_t)std::min<long long>(lo + bw, INT_INF);
                        v2_select_k<Off><<<maxgrid, DB, 0, s>>>(a, row, v.f[fi].p, cs);
                        PJ_LAUNCH_CHECK();
                        jumped = true;
                        break;
                    }
                }
                for (int i = 0; i < V2_NSH; ++i) {
                    mh += v.hctl->mh[i].v;
                    ml += v.hctl->mh[i].pad[0];
                }
                if (slot(cpub) == 0) break;
                K = std::max(1, std::min(2 * K, 16) - g.spec_round);
            }
            if (finished) break;
            if (jumped) continue;  // (the select of the jumped-to band is enqueued)
            heavy_left = heavy_left > mh ? heavy_left - mh : 0;
            light_left = light_left > ml ? light_left - ml : 0;
            // Tail: past the dense first bands the remaining rows are short and the
            // bands sparse, so wide bands (few band steps) pay off. Once the edges of
            // the unsettled vertices drop below tail_frac x nnz, the bands after this
            // one use the light threshold tdelta (light prefixes from lsplit2; the
            // packed light CSR belongs to delta) and width tdelta. Decided here, before
            // the heavy step, so that its fused selection already picks the first tail
            // band and writes the settled bitmap the tail's relaxations filter their
            // targets with. Exact at any band boundary: everything below hi is settled
            // and relaxed after this heavy step.
            const bool enter_tail = !tail && tdelta > delta && (int)st.levels >= g.tail_after &&
                                    (double)(heavy_left + light_left) < g.tail_frac * (double)g.nnz;
            const int32_t nbw = enter_tail ? tdelta : bw;
            const int32_t nhi_t = (int32_t)std::min<long long>((long long)hi + nbw, INT_INF);
            if (enter_tail) {
                a.swrite = v.sb.p;
                a.fesplit = w.lsplit2.p;
            }
            const u64 mh_all = mh + mh_def;  // (a push would relax the deferred edges too)
            const bool dfr_ok = can_pull && g.defer_heavy > 0.0 && !enter_tail && nhi_t < INT_INF &&
                                (double)mh >= g.defer_heavy * (double)g.nnz;
            // (round 5: deferring heavy pulls the same way, the next heavy step pulling both
            // bands, measured 1.5% slower: profiles/r05/defer_heavy_r5h7.txt)
            const bool pull_now = can_pull && mh_all > 0 && (double)heavy_left < g.pull_factor * (double)mh_all;
            if (pull_now) {
                // deferred members (dist >= lo_def) are probed like this band's (dist < hi): the
                // map, when built, covers [lo_def, hi), and a dist probe takes every dist < hi
                if (dpend) a.lo = (int32_t)lo_def;
                set_hmap(a.lo, a.hi);
                v2_pull_k<Off><<<heavygrid, DB, 0, s>>>(a, row, v.f[fi].p, nhi_t, cs);
                a.hmap = nullptr;
                PJ_LAUNCH_CHECK();
                a.lo = (int32_t)lo;
                if (dpend) PJ_HIP(hipMemsetAsync(v.db.p, 0, sizeof(u64) * (size_t)nwords, s));
                if (dpend) v.db_dirty = false;
                dpend = false;
                mh_def = 0;
                st.bu_levels++;
            } else {
                if (dpend) {  // the deferred edges first, whole (db is cleared as read)
                    push_heavy(v.db.p, INT_INF, nullptr);
                    dpend = false;
                    v.db_dirty = false;
                    mh_def = 0;
                }
                if (mh > 0) {
                    const bool dfr = dfr_ok;
                    if (dfr) v.db_dirty = true;
                    push_heavy(v.mb.p, dfr ? nhi_t : INT_INF, dfr ? v.db.p : nullptr);
                    if (dfr) {
                        dpend = true;
                        lo_def = lo;
                        mh_def = mh;
                    }
                }  // (the select below writes every mb word)
                a.lo = hi;
                a.hi = nhi_t;
                v2_select_k<Off><<<maxgrid, DB, 0, s>>>(a, row, v.f[fi].p, cs);
                PJ_LAUNCH_CHECK();
            }
            if (enter_tail) {
                tail = true;
                a.hl = nullptr;  // the tail's light prefixes come from lsplit2
                a.swrite = nullptr;
                a.fesplit = nullptr;
                a.sbits = v.sb.p;
                a.lsplit = w.lsplit2.p;
                a.hw = w.hw2.p;
                a.ltail = 1;
                bw = tdelta;
                // light pulls in the tail (tail_pull): rows are scanned in weight order and
                // stop at the first w with lo + w >= the vertex's distance; light_pull = 0
                // ("never") covers the tail too
                can_pull_light = g.symmetric && g.tail_pull && g.light_pull > 0.0;
                light_pull = g.tail_light_pull;
                tail_unsettled = heavy_left + light_left;
                if ((long long)tdelta > w.maxw) {
                    heavy_left = 0;  // every edge is light in the tail
                    light_left = tail_unsettled;
                } else {
                    PJ_HIP(hipMemsetAsync(&v.ctl.p->aux, 0, sizeof(V2Line), s));
                    v2_heavy_left_k<Off><<<maxgrid, DB, 0, s>>>(row, a.lsplit, v.dist, n, hi, &v.ctl.p->aux.v);
                    PJ_LAUNCH_CHECK();
                }
            }
            if (defer_ok && !(enter_tail && (long long)tdelta <= w.maxw)) {
                deferred = true;  // checked at the next band's first publish
                lo = hi;
                continue;
            }
            sync_ctl();
            if (enter_tail && (long long)tdelta <= w.maxw) {
                heavy_left = v.hctl->aux.v;
                light_left = tail_unsettled > heavy_left ? tail_unsettled - heavy_left : 0;
            }
            if (slot(cs) == 0 && dpend) {  // the next band is empty; deferred edges land past it
                lo = nhi_t;
                flush_def(lo);
                deferred = true;
                continue;
            }
            if (slot(cs) == 0) {
                const u64 mv = hminv();
                if (mv >= (u64)INT_INF) break;  // nothing reached beyond the settled bands
                lo = (long long)mv / bw * bw;  // jump to the next occupied band
                a.lo = (int32_t)lo;
                a.hi = (int32_t)std::min<long long>(lo + bw, INT_INF);
                v2_select_k<Off><<<maxgrid, DB, 0, s>>>(a, row, v.f[fi].p, cs);
                PJ_LAUNCH_CHECK();
                continue;
            }
            for (int i = 0; i < V2_NSH; ++i) {  // (the next band's members, counted by its selection)
                mh_carry += v.hctl->mh[i].v;
                ml_carry += v.hctl->mh[i].pad[0];
            }
            lo = hi;
        }
        if (dpend) throw Error(PJ_ERR_HIP, "delta-stepping: deferred heavy edges left (internal error)");
        // every exit of the band loop but the last band's end (lo reaching INT_INF) follows a
        // publish of the counters after the solve's last relaxation kernel
        if (lo >= INT_INF) sync_ctl();
        for (int k = 0; k < V2W_N; ++k) {
            for (int i = 0; i < V2_NSH; ++i) {
                const V2Line& l = v.hctl->work[k][i];
                st.work_by_kernel[k][0] += (int64_t)l.v;
                st.work_by_kernel[k][1] += (int64_t)l.pad[0];
                st.work_by_kernel[k][2] += (int64_t)l.pad[1];
            }
            st.scanned_edges += st.work_by_kernel[k][0];
            st.probes += st.work_by_kernel[k][1];
            st.work_bytes += st.work_by_kernel[k][2];
        }
    }
    if (unlabel && g.n > 0) {
        unlabel_k<<<grid_for(g.n, 256, maxgrid), 256, 0, s>>>(R.inv.p, v.dist, g.n, n, v.out);
        PJ_LAUNCH_CHECK();
        if (valid && ls >= n) d_source_k<<<1, 1, 0, s>>>(source, v.out);  // a source without edges
    }
    PJ_HIP(hipEventRecord(v.ev1, s));
    PJ_HIP(hipEventSynchronize(v.ev1));
    float ms = 0.f;
    PJ_HIP(hipEventElapsedTime(&ms, v.ev0, v.ev1));
    st.kernel_ms = ms;
    st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_host0).count();
    v.st = st;
    if (g.round_log) {  // debug: one stderr line per non-empty light round
        std::vector<u64> h(1 + 3 * 255);
        PJ_HIP(hipMemcpy(h.data(), rlog.p, sizeof(u64) * h.size(), hipMemcpyDeviceToHost));
        static const char* kind[4] = {"push", "dense", "pull", "empty"};
        for (u64 i = 0; i < std::min<u64>(h[0], 255); ++i)
            fprintf(stderr, "round %llu lo %llu %s frontier %llu light_edges %llu\n", (unsigned long long)i,
                    (unsigned long long)(h[3 + 3 * i] >> 40), kind[h[1 + 3 * i] % 4], (unsigned long long)h[2 + 3 * i],
                    (unsigned long long)(h[3 + 3 * i] & ((1ull << 40) - 1)));
    }
    return valid ? ls : -1;
}

}  // namespace

namespace {

// The graph's DeltaWork (relabeled copy, weight statistics) and the preparation of
// the current light threshold; returns delta.
int32_t delta_setup(Graph& g) {
    const size_t n = (size_t)g.n;
    g.dist.ensure(n ? n : 1);
    if (!g.rl) {
        build_relabeled(g);
        g.delta_work.reset();
    }
    if (!g.delta_work) {
        g.delta_work.reset(new DeltaWork());
        g.delta_work->lsplit.alloc(n ? n : 1);
    }
    if (g.mean_weight < 0.0) {
        u64 h[2] = {0, 0};
        if (g.nnz > 0) {
            DevBuf<u64> acc;
            acc.alloc(2);
            PJ_HIP(hipMemsetAsync(acc.p, 0, 2 * sizeof(u64), g.ctx->stream));
            wsummax_k<<<grid_for(g.nnz, DB, (unsigned)g.ctx->cu_count * 8u), DB, 0, g.ctx->stream>>>(g.w.p, g.nnz,
                                                                                                     acc.p);
            PJ_LAUNCH_CHECK();
            PJ_HIP(hipMemcpyAsync(h, acc.p, 2 * sizeof(u64), hipMemcpyDeviceToHost, g.ctx->stream));
            PJ_HIP(hipStreamSynchronize(g.ctx->stream));
        }
        g.mean_weight = g.nnz > 0 ? (double)h[0] / (double)g.nnz : 1.0;
        g.max_weight = (long long)h[1];
    }
    DeltaWork& w = *g.delta_work;
    const int32_t delta = g.off64 ? prepare_delta<u64>(g, w) : prepare_delta<u32>(g, w);
    // the main solve slot: the ctx stream (pj_set_stream may change it), R.dist, g.dist
    w.main.s = g.ctx->stream;
    w.main.dist = g.rl->dist.p;
    w.main.out = g.dist.p;
    ensure_solve(g, w.main);
    return delta;
}

i64 run_solve(Graph& g, DeltaSolve& v, int32_t delta, i64 source, bool unlabel) {
    if (g.off64) return delta2_run<u64>(g, *g.delta_work, v, delta, source, unlabel);
    return delta2_run<u32>(g, *g.delta_work, v, delta, source, unlabel);
}

}  // namespace

// The solve ends with the distances in the solver's degree-ordered ids (R.dist); the input-id
// vector g.dist is materialized by its first consumer (delta_materialize: the D2H copy, the
// sol_file writer, pj_dist_device, the tree and reach passes), one gather over inv[] of
// 8 bytes per vertex (0.19 ms at s26) that the solve itself no longer carries.
void delta_solve(Graph& g, i64 source) {
    const int32_t delta = delta_setup(g);
    DeltaSolve& v = g.delta_work->main;
    g.dist_pending = false;
    const i64 ls = run_solve(g, v, delta, source, false);
    g.stats = v.st;
    g.dist_pending = true;
    g.pending_source = (ls >= g.rl->n_scan) ? source : -1;  // (a source without edges: 0 after the gather)
    g.have_result = true;
}

void delta_materialize(Graph& g) {
    if (!g.dist_pending) return;
    g.dist_pending = false;
    if (g.n == 0) return;
    hipStream_t s = g.ctx->stream;
    unlabel_k<<<grid_for(g.n, 256, (unsigned)g.ctx->cu_count * (unsigned)PJ_V2_GPC), 256, 0, s>>>(
        g.rl->inv.p, g.rl->dist.p, g.n, g.rl->n_scan, g.dist.p);
    PJ_LAUNCH_CHECK();
    if (g.pending_source >= 0) d_source_k<<<1, 1, 0, s>>>(g.pending_source, g.dist.p);
    PJ_LAUNCH_CHECK();
    PJ_HIP(hipStreamSynchronize(s));  // (readers may copy on other streams, e.g. small hipMemcpy)
}

// Johnson-style weighted batch: `slots` solves in flight at once, each on its own
// stream with its own frontiers, counters, hub queues and distance rows, driven by
// one host thread per slot that takes the next source from a shared counter. The
// solves share the graph and the light CSR (read-only). Their light rounds are
// latency-bound, so two solves interleave on the CUs (round 3's N = 2 rehearsal:
// +10% throughput over one at a time). on_row(i, device row, stream) is called once
// per source, serialised, with the row complete and valid until it returns.
void delta_batch(Graph& g, const i64* sources, int n_src, int slots,
                 const std::function<void(int, const int32_t*, hipStream_t)>& on_row) {
    const int32_t delta = delta_setup(g);
    g.dist_pending = false;  // (the main slot's rows overwrite R.dist and g.dist)
    DeltaWork& w = *g.delta_work;
    slots = std::max(1, std::min(slots, n_src));
    const i64 n_scan = g.rl->n_scan;
    // A slot beyond the main one holds its own rows (relabeled and input-id distances), five
    // n-bit bitmaps and the hub queue ring (3 x hcap x 20 bytes, hcap ~ nnz / 64: ~2 GB at
    // s26). One is added only while it takes at most half the free device memory, and if its
    // allocation still fails the batch runs on the slots it has.
    const double slot_bytes = 4.0 * (double)(n_scan + g.n) + 5.0 * 8.0 * (double)((n_scan + 63) / 64) +
                              60.0 * (double)std::max<i64>(1, std::min<i64>(n_scan, g.nnz / (i64)V2_HT + 1));
    while ((int)w.extra.size() < slots - 1) {
        const size_t fr = dev_free_bytes();  // (libpj's idle cached blocks count as free)
        if (slot_bytes > 0.5 * (double)fr) break;
        std::unique_ptr<DeltaSolve> v(new DeltaSolve());
        try {
            PJ_HIP(hipStreamCreateWithFlags(&v->s, hipStreamNonBlocking));
            v->own_stream = true;
            v->dist_own.alloc((size_t)std::max<i64>(n_scan, 1));
            v->out_own.alloc((size_t)std::max<i64>(g.n, 1));
            v->dist = v->dist_own.p;
            v->out = v->out_own.p;
            ensure_solve(g, *v);
        } catch (const Error&) {
            (void)hipGetLastError();
            break;
        }
        w.extra.push_back(std::move(v));
    }
    slots = std::min(slots, (int)w.extra.size() + 1);
    std::vector<DeltaSolve*> slot{&w.main};
    for (int k = 0; k + 1 < slots; ++k) slot.push_back(w.extra[(size_t)k].get());
    PJ_HIP(hipDeviceSynchronize());  // (the preparation ran on the ctx stream)
    auto t0 = std::chrono::steady_clock::now();
    std::atomic<int> next{0};
    std::mutex mu;
    pj_stats sum{};
    std::vector<std::exception_ptr> errs((size_t)slots);
    auto work = [&](int k) {
        try {
            PJ_HIP(hipSetDevice(g.ctx->device));
            DeltaSolve& v = *slot[(size_t)k];
            for (int i; (i = next.fetch_add(1)) < n_src;) {
                run_solve(g, v, delta, sources[i], true);  // (rows in input ids for on_row)
                std::lock_guard<std::mutex> lk(mu);
                sum.kernel_ms += v.st.kernel_ms;
                sum.levels += v.st.levels;
                sum.relax_rounds += v.st.relax_rounds;
                sum.td_levels += v.st.td_levels;
                sum.bu_levels += v.st.bu_levels;
                sum.scanned_edges += v.st.scanned_edges;
                sum.probes += v.st.probes;
                sum.work_bytes += v.st.work_bytes;
                for (int k = 0; k < V2W_N; ++k)
                    for (int j = 0; j < 3; ++j) sum.work_by_kernel[k][j] += v.st.work_by_kernel[k][j];
                on_row(i, v.out, v.s);
            }
        } catch (...) {
            errs[(size_t)k] = std::current_exception();
            next.store(n_src);  // the other slots stop after their current row
        }
    };
    std::vector<std::thread> th;
    for (int k = 1; k < slots; ++k) th.emplace_back(work, k);
    work(0);
    for (auto& t : th) t.join();
    for (auto& e : errs)
        if (e) std::rethrow_exception(e);
    sum.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    g.stats = sum;
}

}  // namespace pj
