// wpart.hip — weighted SSSP (delta-stepping) over a 1D vertex partition, one
// process per GPU ("Δ-stepping variant").
//
// Same block geometry as part.hip (the reference's nn2rank / get_start_nn,
// ParallelJohnson.cpp:169-200, with 64-aligned blocks): rank r owns vertices
// [lo, hi) and their out-rows (weights kept, rows weight-sorted as graph.hip
// stores them). The band loop runs in the caller (paralleljohnson_amd/
// partition.py, torch.distributed over RCCL), the analogue of the reference's
// round loop :488-594:
//
//   select(lo, hi)     : frontier := owned vertices with dist in [lo, hi);
//                        all_reduce(sum) of its size, all_reduce(min) of the
//                        smallest owned dist >= lo (the next occupied band when
//                        this one is empty; INF everywhere = the end, cf. :579-593)
//   light rounds       : relax the frontier's light edges (w < delta). An owned
//                        target is lowered with atomicMin and joins the next
//                        frontier when it lands below hi; a remote target's
//                        (id, candidate) pair is appended by the relax itself to
//                        the rank's claim queue (64 shards, one counter each).
//                        count: the queued pairs per owner; pack (into a send
//                        buffer sized to that count): the pairs owner-major —
//                        the per-owner send buffers of :537-542 — exchanged with
//                        all_to_all_single (:522-554); apply: the owner folds the
//                        received candidates in the same way (duplicates fold
//                        into the same atomicMin: the dedup is the owner's).
//                        A round ends with all_reduce(sum) of the new frontier sizes.
//   heavy step         : the band's members relax their heavy edges once (same
//                        relax / pack / exchange / apply).
//
// A direct-mapped cache of the (id, best value) pairs this rank has sent during the
// solve (block entries: O(block) like the rest of the rank's vertex state) drops a
// remote relaxation that cannot beat what was already sent for that id. It may forget
// (a colliding id evicts the entry), which costs only a redundant pair, never a lost
// one. A round whose pairs overflow a queue shard is run again after the queue grows
// (the band's members as its frontier, the cache cleared: see wpart_relax); the queue
// keeps its size for the later rounds and solves.
// Row segments longer than WP_LONG edges go to a queue relaxed edge-balanced
// over the whole grid (1024-edge tiles, lb.h).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <thread>

#include "kron.h"
#include "lb.h"
#include "engine.h"

namespace pj {

namespace {

// current value of a distance that atomics may have lowered (agent-scope load:
// the L2 of this XCD may hold a stale line; see delta.hip dist_now)
__device__ __forceinline__ int32_t wp_now(const int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int WB = 256;
constexpr int WSC = 16;        // frontier words a wave screens at once
constexpr int WP_SERIAL = 8;   // edges a lane relaxes alone
#ifndef PJ_WP_LONG
#define PJ_WP_LONG 64  // with the per-block degree order (below); 1024 before it (r4c: 64 without it ~6% slower)
#endif
constexpr u64 WP_LONG = PJ_WP_LONG;  // longer row segments: the grid-wide queue
constexpr int WP_MAXW = 64;    // largest world size
constexpr int WP_EB = 40;      // long queue counter: (slots << WP_EB) | edges
constexpr int WP_TILE = WB * 4;

// stat slots (u64): [0, 64) per-owner region counts, then:
constexpr int ST_LONGQ = 64;   // long-row queue length
constexpr int ST_NF = 65;      // vertices marked in the next frontier
constexpr int ST_MIN = 66;     // min owned dist >= lo (select)
constexpr int ST_CNT = 67;     // selected frontier size
constexpr int ST_REACH = 68;   // reached vertices, [69] their out-edges
constexpr int ST_ACC = 72;     // [72, 75): the per-band counts (heavy / light / unsettled edges)
constexpr int ST_CUR = 75;     // [75, 75 + 64): pack cursors per owner
constexpr int ST_QTOT = 75 + WP_MAXW;  // pairs the round tried to queue (all shards)
constexpr int ST_QSP = ST_QTOT + 1;     // of them, pairs that went to the spill region (> its capacity: overflow)
constexpr int ST_N = ST_QSP + 1;
constexpr int WQ_S = 64;       // claim-queue shards (blockIdx % WQ_S), each counter on its own 64-byte line

struct WArgs {
    i64 n, lo, nl, block, bw;
    int rank;
    int32_t dlo, dhi;  // band [dlo, dhi)
    const u64* row;    // nl + 1
    const u32* col;
    const u32* w;
    const u32* lsplit;
    int32_t* dist;     // nl
    u64* rc;           // (world > 1) sent-pair cache: (id << 32 | best), 2^rcb entries, ~0 = empty
    u32 rcb;
    u64* q;            // (world > 1) claim queue: WQ_S shards of qsh pairs (id | cand << 32), then
    u64 qsh, qsp;      // the spill region of qsp pairs
    u64* qctr;         // WQ_S + 1 counters (the shards', the spill's), 8 words apart
    u64* fr;           // bw
    u64* frn;          // bw
    u64* mb;           // bw
    u32* lq_v;         // long-row queue: local vertex, row position, edge offset of the slot
    u64* lq_b;
    u64* lq_e;
    u64* stat;
    const u64* sbits;  // the tail's settled filter (global ids; null before the tail switch)
};

// A relaxation: an owned target is lowered with atomicMin and, in a light step below hi,
// marked in the next frontier (returning 1 when this relaxation set the mark: the callers
// count the marks per thread and add the block's sum to ST_NF once -- an atomicAdd per
// marked vertex on that one word serialized the light rounds behind its atomic rate); a
// remote target's (id, candidate) goes to the claim queue unless the sent-pair cache
// shows a value at least as good already sent for that id.

// the cache slot of id t (multiplicative hash) and its entry (id << 32 | value)
__device__ __forceinline__ u64* wp_rc_slot(const WArgs& a, u32 t) {
    return a.rc + (((u32)(t * 0x9E3779B1u)) >> (32 - a.rcb));
}
// the best value the cache shows as sent for t (INT_INF: none). Agent-scope accesses: the
// entries written during the round by other XCDs' lanes are seen (a stale hit is still a
// value that was sent, so no pair is ever lost; a miss costs one redundant pair).
__device__ __forceinline__ int32_t wp_rc_get(const WArgs& a, u32 t) {
    const u64 c = __hip_atomic_load(wp_rc_slot(a, t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (u32)(c >> 32) == t ? (int32_t)(u32)c : INT_INF;
}
__device__ __forceinline__ void wp_rc_put(const WArgs& a, u32 t, int32_t v) {
    __hip_atomic_store(wp_rc_slot(a, t), ((u64)t << 32) | (u32)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Appends the pairs (t[j], nd[j]) with app[j] set to the claim queue: one atomic per call
// for all active lanes (positions from the ballots), in shard blockIdx % WQ_S. Pairs past
// the shard's capacity go to the spill region (a second atomic, only then), so the queue is
// sized by the round's total pairs, not by its fullest shard. A pair past the spill's
// capacity is not written; the spill counter still counts it, which is how the host sees the
// overflow (ST_QSP > qsp).
template <int N>
__device__ __forceinline__ void wp_append(const WArgs& a, const bool (&app)[N], const u32 (&t)[N],
                                          const long long (&nd)[N]) {
    u32 off[N], tot = 0;
    const u64 lt = lanemask_lt();
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const u64 m = __ballot(app[j]);
        off[j] = tot + (u32)__popcll(m & lt);
        tot += (u32)__popcll(m);
    }
    if (tot == 0) return;
    const int leader = __ffsll((long long)__ballot(true)) - 1;
    u64* ctr = a.qctr + (size_t)(blockIdx.x % WQ_S) * 8;
    u64 base = 0;
    if (lane_id() == leader) base = atomicAdd(ctr, (u64)tot);
    base = __shfl(base, leader, 64);
    u64* qs = a.q + (size_t)(blockIdx.x % WQ_S) * a.qsh;
    if (base + tot <= a.qsh) {  // (wave-uniform: the usual case)
#pragma unroll
        for (int j = 0; j < N; ++j)
            if (app[j]) qs[base + off[j]] = (u64)t[j] | ((u64)(u32)(int32_t)nd[j] << 32);
        return;
    }
    u32 soff[N], stot = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const bool sp = app[j] && base + off[j] >= a.qsh;
        const u64 m = __ballot(sp);
        soff[j] = stot + (u32)__popcll(m & lt);
        stot += (u32)__popcll(m);
    }
    u64 sbase = 0;
    if (stot && lane_id() == leader) sbase = atomicAdd(a.qctr + (size_t)WQ_S * 8, (u64)stot);
    sbase = __shfl(sbase, leader, 64);
    u64* qp = a.q + (size_t)WQ_S * a.qsh;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        if (!app[j]) continue;
        const u64 x = (u64)t[j] | ((u64)(u32)(int32_t)nd[j] << 32);
        const u64 pos = base + off[j];
        if (pos < a.qsh) qs[pos] = x;
        else if (sbase + soff[j] < a.qsp) qp[sbase + soff[j]] = x;
    }
}
// region r of the claim queue (r < WQ_S: a shard, r == WQ_S: the spill): its pairs and count
__device__ __forceinline__ const u64* wp_qregion(const WArgs& a, u32 r, u64& cnt) {
    const u64 c = a.qctr[(size_t)r * 8];
    cnt = r < (u32)WQ_S ? min(c, a.qsh) : min(c, a.qsp);
    return a.q + (size_t)r * a.qsh;
}

// WP_PU edges of one source in one step: the target reads of all of them issued before
// any atomic (one edge at a time is a dependent chain of read, atomicMin and atomicOr per
// edge); returns the number of newly marked frontier vertices
#ifndef PJ_WP_PU
#define PJ_WP_PU 2
#endif
constexpr int WP_PU = PJ_WP_PU;
__device__ __forceinline__ u32 wp_edges(const WArgs& a, bool light, u64 k, u64 lim, int32_t du) {
    u32 t[WP_PU];
    long long nd[WP_PU];
    bool ok[WP_PU], loc[WP_PU];
    int32_t cur[WP_PU];
#pragma unroll
    for (int j = 0; j < WP_PU; ++j) {
        ok[j] = k + j < lim;
        t[j] = ok[j] ? a.col[k + j] : 0u;
        nd[j] = (long long)du + (ok[j] ? a.w[k + j] : 0u);
        ok[j] = ok[j] && nd[j] < INT_INF;
    }
    if (a.sbits) {  // the tail: settled targets are skipped before their distance is read
        u64 sw[WP_PU];
#pragma unroll
        for (int j = 0; j < WP_PU; ++j) sw[j] = ok[j] ? a.sbits[t[j] >> 6] : 0ull;
#pragma unroll
        for (int j = 0; j < WP_PU; ++j) ok[j] = ok[j] && !((sw[j] >> (t[j] & 63)) & 1ull);
    }
#pragma unroll
    for (int j = 0; j < WP_PU; ++j) {
        const i64 tl = (i64)t[j] - a.lo;
        loc[j] = tl >= 0 && tl < a.nl;
        cur[j] = !ok[j] ? 0 : (loc[j] ? wp_now(a.dist + tl) : wp_rc_get(a, t[j]));
    }
    u32 nf = 0;
    bool app[WP_PU];
#pragma unroll
    for (int j = 0; j < WP_PU; ++j) {
        app[j] = false;
        if (!ok[j] || (int32_t)nd[j] >= cur[j]) continue;
        if (loc[j]) {
            const i64 tl = (i64)t[j] - a.lo;
            atomicMin(a.dist + tl, (int32_t)nd[j]);
            if (light && (int32_t)nd[j] < a.dhi) {
                const u64 bit = 1ull << (tl & 63);
                if (!(atomicOr(a.frn + (tl >> 6), bit) & bit)) ++nf;
            }
        } else {
            wp_rc_put(a, t[j], (int32_t)nd[j]);
            app[j] = true;
        }
    }
    if (a.q) wp_append<WP_PU>(a, app, t, nd);
    return nf;
}

// N independent edges (any sources: target t, offer nd, valid ok) relaxed with the loads
// issued together -- the settled bits, then the target distances / candidates, then the
// atomics -- instead of one dependent chain per edge (wp_edge); returns the marks
template <int N>
__device__ __forceinline__ u32 wp_edges_g(const WArgs& a, bool light, const u32 (&t)[N], const long long (&nd)[N],
                                          bool (&ok)[N]) {
#pragma unroll
    for (int j = 0; j < N; ++j) ok[j] = ok[j] && nd[j] < INT_INF;
    if (a.sbits) {
        u64 sw[N];
#pragma unroll
        for (int j = 0; j < N; ++j) sw[j] = ok[j] ? a.sbits[t[j] >> 6] : 0ull;
#pragma unroll
        for (int j = 0; j < N; ++j) ok[j] = ok[j] && !((sw[j] >> (t[j] & 63)) & 1ull);
    }
    bool loc[N];
    int32_t cur[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const i64 tl = (i64)t[j] - a.lo;
        loc[j] = tl >= 0 && tl < a.nl;
        cur[j] = !ok[j] ? 0 : (loc[j] ? wp_now(a.dist + tl) : wp_rc_get(a, t[j]));
    }
    u32 nf = 0;
    bool app[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        app[j] = false;
        if (!ok[j] || (int32_t)nd[j] >= cur[j]) continue;
        if (loc[j]) {
            const i64 tl = (i64)t[j] - a.lo;
            atomicMin(a.dist + tl, (int32_t)nd[j]);
            if (light && (int32_t)nd[j] < a.dhi) {
                const u64 bit = 1ull << (tl & 63);
                if (!(atomicOr(a.frn + (tl >> 6), bit) & bit)) ++nf;
            }
        } else {
            wp_rc_put(a, t[j], (int32_t)nd[j]);
            app[j] = true;
        }
    }
    if (a.q) wp_append<N>(a, app, t, nd);
    return nf;
}

// the block's newly marked frontier vertices into ST_NF (one atomic per block)
__device__ __forceinline__ void wp_flush_nf(const WArgs& a, u32 nf, u64* red) {
    const u64 t = block_sum<WB / WAVE>((u64)nf, red);
    if (threadIdx.x == 0 && t) atomicAdd(&a.stat[ST_NF], t);
}

__global__ void wp_seed_k(WArgs a, i64 s) {
    const i64 sl = s - a.lo;
    if (sl >= 0 && sl < a.nl) a.dist[sl] = 0;
}

// frontier := owned vertices with dist in [dlo, dhi); frn := 0; mb := 0 (new band)
__global__ __launch_bounds__(WB) void wp_select_k(WArgs a) {
    __shared__ u64 red[WB / WAVE];
    const int lane = lane_id();
    u64 c = 0;
    int32_t mn = INT_INF;
    // (8 words per wave step, loads issued together; lane j then stores word j of the step,
    // so the three bitmaps take one 64-byte store each instead of eight single-lane stores)
    constexpr int SELW = 8;
    for (i64 w0 = ((i64)blockIdx.x * (WB / WAVE) + wave_id()) * SELW; w0 < a.bw;
         w0 += (i64)gridDim.x * (WB / WAVE) * SELW) {
        int32_t dd[SELW];
#pragma unroll
        for (int j = 0; j < SELW; ++j) {
            const i64 v = (w0 + j) * 64 + lane;
            dd[j] = v < a.nl ? a.dist[v] : INT_INF;
        }
        u64 mine = 0;
#pragma unroll
        for (int j = 0; j < SELW; ++j) {
            const int32_t d = dd[j];
            const u64 m = __ballot(d >= a.dlo && d < a.dhi);
            if (d >= a.dlo && d < mn) mn = d;
            if (lane == j) mine = m;
        }
        if (lane < SELW && w0 + lane < a.bw) {
            a.fr[w0 + lane] = mine;
            a.frn[w0 + lane] = 0;
            a.mb[w0 + lane] = 0;
            c += (u64)__popcll(mine);
        }
    }
    c = block_sum<WB / WAVE>(c, red);
    if (threadIdx.x == 0 && c) atomicAdd(&a.stat[ST_CNT], c);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const int32_t y = __shfl_xor(mn, off, 64);
        mn = y < mn ? y : mn;
    }
    // one atomicMin per block, not per wave
    if (lane == 0) red[wave_id()] = (u64)(u32)mn;
    __syncthreads();
    if (threadIdx.x == 0) {
        int32_t m = INT_INF;
        for (int k = 0; k < WB / WAVE; ++k) m = min(m, (int32_t)(u32)red[k]);
        if (m < INT_INF) atomicMin(&a.stat[ST_MIN], (u64)m);
    }
}

// LIGHT: the frontier fr relaxes its light prefixes (fr words are cleared as
// read, members join mb); HEAVY: mb relaxes its heavy suffixes.
template <bool LIGHT>
__global__ __launch_bounds__(WB) void wp_relax_k(WArgs a) {
    __shared__ u64 red[WB / WAVE];
    const int lane = lane_id();
    u32 nf = 0;
    const i64 nsc = (a.bw + WSC - 1) / WSC;
    for (i64 sc = (i64)blockIdx.x * (WB / WAVE) + wave_id(); sc < nsc; sc += (i64)gridDim.x * (WB / WAVE)) {
        const i64 wbase = sc * WSC;
        u64 mytodo = 0;
        if (lane < WSC && wbase + lane < a.bw) {
            if (LIGHT) {
                mytodo = a.fr[wbase + lane];
                if (mytodo) {
                    a.fr[wbase + lane] = 0;
                    a.mb[wbase + lane] |= mytodo;  // the wave owns these words
                }
            } else {
                mytodo = a.mb[wbase + lane];
            }
        }
        if (!__ballot(mytodo != 0)) continue;
        const u32 cnt = (u32)__popcll(mytodo);
        const u32 incl = wave_incl_scan(cnt);
        const u32 myex = incl - cnt;
        const u32 T = __shfl(incl, 63, 64);
        for (u32 r0 = 0; r0 < T; r0 += WAVE) {
            const u32 c = r0 + lane;
            const bool act = c < T;
            u32 jw = 0;
#pragma unroll
            for (u32 step = WSC / 2; step > 0; step >>= 1) {
                const u32 x = __shfl(myex, jw + step, 64);
                if (x <= c) jw += step;
            }
            const u32 ex = __shfl(myex, jw, 64);
            const u64 tw = __shfl(mytodo, jw, 64);
            u64 b = 0, e = 0;
            int32_t du = 0;
            u32 v = 0;
            if (act) {
                v = (u32)((wbase + jw) * 64 + select_bit(tw, c - ex));
                du = a.dist[v];
                const u64 r0v = a.row[v], sp = r0v + a.lsplit[v];
                b = LIGHT ? r0v : sp;
                e = LIGHT ? sp : a.row[v + 1];
            }
            // long segments: the edge-balanced queue (one packed atomic per wave
            // gives slots and edge offsets, monotonic in the slot)
            const bool lng = act && e - b > WP_LONG;
            const u64 hm = __ballot(lng);
            if (hm) {
                const u64 seg = lng ? e - b : 0;
                const u64 ie = wave_incl_scan(seg);
                const u64 tot = __shfl(ie, 63, 64);
                const int leader = __ffsll((long long)hm) - 1;
                u64 base = 0;
                if (lane == leader) base = atomicAdd(&a.stat[ST_LONGQ], ((u64)__popcll(hm) << WP_EB) | tot);
                base = __shfl(base, leader, 64);
                if (lng) {
                    const u64 q = (base >> WP_EB) + (u64)__popcll(hm & lanemask_lt());
                    a.lq_v[q] = v;
                    a.lq_b[q] = b;
                    a.lq_e[q] = (base & ((1ull << WP_EB) - 1ull)) + ie - seg;  // edge offset of the slot
                    e = b;
                }
            }
            u64 k = b;
            const u64 lim = (e - b > (u64)WP_SERIAL) ? b + WP_SERIAL : e;
            for (; k < lim; k += WP_PU) nf += wp_edges(a, LIGHT, k, lim, du);
            k = k < lim ? k : lim;
            // the rest, edge-balanced over the wave
            if (__ballot(k < e)) {
                const u64 rem = k < e ? e - k : 0;
                const u64 inc = wave_incl_scan(rem);
                const u64 exc = inc - rem;
                const u64 tot = __shfl(inc, 63, 64);
                constexpr int NJ = 4;  // edges per lane and step, relaxed together (wp_edges_g)
                for (u64 g0 = 0; g0 < tot; g0 += NJ * WAVE) {
                    u32 t[NJ];
                    long long nd[NJ];
                    bool ok[NJ];
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        const u64 gi = g0 + (u64)j * WAVE + lane;
                        int l = 0;
#pragma unroll
                        for (int step = 32; step > 0; step >>= 1)
                            if (__shfl(inc, l + step - 1, 64) <= gi) l += step;
                        const u64 kl = __shfl(k, l, 64), xl = __shfl(exc, l, 64);
                        const int32_t dl = __shfl(du, l, 64);
                        ok[j] = gi < tot;
                        const u64 kk = kl + (gi - xl);
                        t[j] = ok[j] ? a.col[kk] : 0u;
                        nd[j] = (long long)dl + (ok[j] ? a.w[kk] : 0u);
                    }
                    nf += wp_edges_g<NJ>(a, LIGHT, t, nd, ok);
                }
            }
        }
    }
    if (LIGHT) wp_flush_nf(a, nf, red);
}

// the long segments queued by wp_relax_k, edge-balanced: 1024-edge tiles over
// the slots' monotonic edge offsets (lb.h), the source distances staged in LDS
template <bool LIGHT>
__global__ __launch_bounds__(WB) void wp_long_k(WArgs a) {
    __shared__ LbShared<WP_TILE> sh;
    __shared__ int32_t s_du[WP_TILE];
    __shared__ u64 s_b[WP_TILE];
    __shared__ u64 red[WB / WAVE];
    u32 nf = 0;
    const u64 packed = a.stat[ST_LONGQ];
    const u64 nq = packed >> WP_EB, total = packed & ((1ull << WP_EB) - 1ull);
    if (nq == 0) return;
    for (u64 e0 = (u64)blockIdx.x * WP_TILE; e0 < total; e0 += (u64)gridDim.x * WP_TILE) {
        u64 s0;
        u32 ns;
        lb_tile_load<WP_TILE>(a.lq_e, nq, e0, sh, s0, ns);
        for (u32 i = threadIdx.x; i < ns; i += WB) {
            s_du[i] = a.dist[a.lq_v[s0 + i]];
            s_b[i] = a.lq_b[s0 + i];
        }
        __syncthreads();
        constexpr int NJ = WP_TILE / WB;  // the thread's edges, relaxed together (wp_edges_g)
        u32 t[NJ];
        long long nd[NJ];
        bool ok[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const u64 e = e0 + (u64)j * WB + threadIdx.x;
            ok[j] = e < total;
            u64 k = 0;
            int32_t du = 0;
            if (ok[j]) {
                const u32 sl = lb_find<WP_TILE>(sh, ns, e);
                k = s_b[sl] + (e - sh.off[sl]);
                du = s_du[sl];
            }
            t[j] = ok[j] ? a.col[k] : 0u;
            nd[j] = (long long)du + (ok[j] ? a.w[k] : 0u);
        }
        nf += wp_edges_g<NJ>(a, LIGHT, t, nd, ok);
        __syncthreads();
    }
    if (LIGHT) wp_flush_nf(a, nf, red);
}

// The claim queue's pairs per owner -> stat[o]; the pairs tried (ST_QTOT) and spilled
// (ST_QSP, above the spill's capacity: the round overflowed). Block b reads region
// b % (WQ_S + 1) (the shards, then the spill), the blocks of a region stride over its pairs;
// per wave one LDS add per owner present.
__device__ __forceinline__ void wp_owner_rank(u32 o, bool ok, u32* cnt, u32* rank_out) {
    // (wave) lanes with ok grouped by owner o: cnt[o] += group size (LDS), *rank_out = the
    // lane's rank in its group plus the LDS count before the group's add
    u64 pending = __ballot(ok);
    const int lane = lane_id();
    while (pending) {
        const int l = __ffsll((long long)pending) - 1;
        const u32 ol = __shfl(o, l, 64);
        const u64 grp = __ballot(ok && o == ol);
        pending &= ~grp;
        u32 b = 0;
        if (lane == l) b = atomicAdd(&cnt[ol], (u32)__popcll(grp));
        b = __shfl(b, l, 64);
        if (ok && o == ol && rank_out) *rank_out = b + (u32)__popcll(grp & lanemask_lt());
    }
}
__global__ __launch_bounds__(WB) void wp_qcount_k(WArgs a, int world) {
    __shared__ u32 h[WP_MAXW];
    for (int o = threadIdx.x; o < world; o += WB) h[o] = 0;
    __syncthreads();
    const u32 sh = blockIdx.x % (WQ_S + 1), per = gridDim.x / (WQ_S + 1), c = blockIdx.x / (WQ_S + 1);
    const u64 att = a.qctr[(size_t)sh * 8];
    u64 cnt;
    const u64* qs = wp_qregion(a, sh, cnt);
    for (u64 i0 = (u64)c * WB; i0 < cnt; i0 += (u64)per * WB) {
        const u64 i = i0 + threadIdx.x;
        const bool ok = i < cnt;
        const u32 o = ok ? (u32)((u64)(u32)qs[i] / (u64)a.block) : 0u;
        wp_owner_rank(o, ok, h, nullptr);
    }
    __syncthreads();
    for (int o = threadIdx.x; o < world; o += WB)
        if (h[o]) atomicAdd(&a.stat[o], (u64)h[o]);
    if (c == 0 && threadIdx.x == 0 && att) atomicAdd(&a.stat[sh < (u32)WQ_S ? ST_QTOT : ST_QSP], att);
}

// Pack: the queued pairs at their owner's segment of send (segments owner-major, sizes
// stat[o] from wp_qcount_k; a cursor per owner, one atomic per block tile and owner).
// Order inside a segment is free: the owner folds the pairs with atomicMin.
__global__ __launch_bounds__(WB) void wp_qpack_k(WArgs a, int world, u64* __restrict__ send) {
    __shared__ u32 h[WP_MAXW];
    __shared__ u64 base[WP_MAXW];
    const u32 sh = blockIdx.x % (WQ_S + 1), per = gridDim.x / (WQ_S + 1), c = blockIdx.x / (WQ_S + 1);
    u64 cnt;
    const u64* qs = wp_qregion(a, sh, cnt);
    for (u64 i0 = (u64)c * WB; i0 < cnt; i0 += (u64)per * WB) {  // (block-uniform)
        for (int o = threadIdx.x; o < world; o += WB) h[o] = 0;
        __syncthreads();
        const u64 i = i0 + threadIdx.x;
        const bool ok = i < cnt;
        const u64 x = ok ? qs[i] : 0ull;
        const u32 o = ok ? (u32)((u64)(u32)x / (u64)a.block) : 0u;
        u32 r = 0;
        wp_owner_rank(o, ok, h, &r);
        __syncthreads();
        for (int q = threadIdx.x; q < world; q += WB) {
            u64 b = 0;
            if (h[q]) {
                b = atomicAdd(&a.stat[ST_CUR + q], (u64)h[q]);
                for (int k = 0; k < q; ++k) b += a.stat[k];  // the segment's start
            }
            base[q] = b;
        }
        __syncthreads();
        if (ok) send[base[o] + r] = x;
        __syncthreads();
    }
}

// World 2: every queued pair is the one peer's, so the counts are the regions' fills (one
// wave: no pass over the pairs) and the pack is a copy of each region's pairs behind the
// fills of the regions before it (no owner ranking). (round 5: the two general passes took
// ~0.6 ms per s26w solve and rank, profiles/r05/wpart_timeline_r5m.txt)
__global__ void wp_qsum2_k(WArgs a, int peer) {
    const int lane = lane_id();
    u64 fill = 0, att_sh = 0, att_sp = 0;
    for (int r = lane; r <= WQ_S; r += WAVE) {
        const u64 att = a.qctr[(size_t)r * 8];
        fill += r < WQ_S ? min(att, a.qsh) : min(att, a.qsp);
        if (r < WQ_S) att_sh += att;
        else att_sp += att;
    }
    fill = wave_sum(fill);
    att_sh = wave_sum(att_sh);
    att_sp = wave_sum(att_sp);
    if (lane == 0) {
        a.stat[peer] = fill;
        a.stat[ST_QTOT] = att_sh;
        a.stat[ST_QSP] = att_sp;
    }
}
// (host != null: block 0 also publishes the counts -- the peer's fill and the overflow
// counters -- into the host copy of the stat block and bumps its sequence word, so the
// relax step needs no publish launch: the pack's own consumers are stream-ordered)
__global__ __launch_bounds__(WB) void wp_qcopy2_k(WArgs a, u64* __restrict__ send, int rank, u64* __restrict__ host,
                                                  u64* seqp, u64 seq) {
    __shared__ u64 s_off;
    const u32 sh = blockIdx.x % (WQ_S + 1), per = gridDim.x / (WQ_S + 1), c = blockIdx.x / (WQ_S + 1);
    if (host && blockIdx.x == 0 && threadIdx.x < WAVE) {
        u64 fill = 0, att_sh = 0, att_sp = 0;
        for (int r = (int)threadIdx.x; r <= WQ_S; r += WAVE) {
            const u64 att = a.qctr[(size_t)r * 8];
            fill += r < WQ_S ? min(att, a.qsh) : min(att, a.qsp);
            if (r < WQ_S) att_sh += att;
            else att_sp += att;
        }
        fill = wave_sum(fill);
        att_sh = wave_sum(att_sh);
        att_sp = wave_sum(att_sp);
        if (threadIdx.x == 0) {
            a.stat[1 - rank] = fill;
            a.stat[ST_QTOT] = att_sh;
            a.stat[ST_QSP] = att_sp;
            host[rank] = 0;
            host[1 - rank] = fill;
            host[ST_QTOT] = att_sh;
            host[ST_QSP] = att_sp;
            __threadfence_system();
            __hip_atomic_store(seqp, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (threadIdx.x < WAVE) {  // the fills of the regions before this one
        u64 f = 0;
        for (u32 r = threadIdx.x; r < sh; r += WAVE) {
            const u64 att = a.qctr[(size_t)r * 8];
            f += r < (u32)WQ_S ? min(att, a.qsh) : min(att, a.qsp);
        }
        f = wave_sum(f);
        if (threadIdx.x == 0) s_off = f;
    }
    __syncthreads();
    u64 cnt;
    const u64* qs = wp_qregion(a, sh, cnt);
    u64* dst = send + s_off;
    for (u64 i = (u64)c * WB + threadIdx.x; i < cnt; i += (u64)per * WB) dst[i] = qs[i];
}

// received (id | cand << 32) for this rank
__global__ __launch_bounds__(WB) void wp_apply_k(WArgs a, const u64* __restrict__ recv, i64 nr, int light) {
    __shared__ u64 red[WB / WAVE];
    u32 nf = 0;
    constexpr int NJ = 4;  // received pairs per thread and step, relaxed together
    const i64 stride = (i64)gridDim.x * WB;
    for (i64 i0 = (i64)blockIdx.x * WB + threadIdx.x; i0 < nr; i0 += NJ * stride) {
        u32 t[NJ];
        long long nd[NJ];
        bool ok[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const i64 i = i0 + (i64)j * stride;
            ok[j] = i < nr;
            const u64 x = ok[j] ? recv[i] : 0ull;
            t[j] = (u32)x;
            nd[j] = (long long)(int32_t)(u32)(x >> 32);
        }
        nf += wp_edges_g<NJ>(a, light != 0, t, nd, ok);
    }
    if (light) wp_flush_nf(a, nf, red);
}


__global__ void wp_rebase_k(const void* row, bool off64, i64 lo, i64 nl, u64* __restrict__ out) {
    const u64 base = off64 ? ((const u64*)row)[lo] : (u64)((const u32*)row)[lo];
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i <= nl; i += (i64)gridDim.x * blockDim.x)
        out[i] = (off64 ? ((const u64*)row)[lo + i] : (u64)((const u32*)row)[lo + i]) - base;
}

__global__ void wp_lsplit_k(const u64* __restrict__ row, const u32* __restrict__ w, i64 nl, u32 delta,
                            u32* __restrict__ out) {
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < nl; v += (i64)gridDim.x * blockDim.x) {
        u64 lo = row[v], hi = row[v + 1];
        const u64 b = lo;
        while (lo < hi) {  // rows are weight-sorted
            const u64 mid = lo + (hi - lo) / 2;
            if (w[mid] < delta) lo = mid + 1;
            else hi = mid;
        }
        out[v] = (u32)(lo - b);
    }
}

// Heavy pull (engine.h DeltaSteps): (members' heavy edges, unsettled vertices' heavy edges,
// and all out-edges of the vertices >= hi: the tail switch's count, which the heavy step
// does not change -- its offers are >= lo + delta = hi -- so wpart_unsettled reuses it)
// It also writes this rank's slice of the member map (as wp_member_slice_k) when `own` is
// set: the heavy pull that may follow then needs no pass of its own.
__global__ __launch_bounds__(WB) void wp_heavy_counts_k(WArgs a, int32_t hi, u64* __restrict__ out,
                                                       uint8_t* __restrict__ own) {
    __shared__ u64 red[WB / WAVE];
    u64 m = 0, u = 0, ua = 0;
    // (one vertex per thread step: 4 per step with the loads issued together measured 37%
    // slower here, r4i)
    for (i64 v = (i64)blockIdx.x * WB + threadIdx.x; v < a.block; v += (i64)gridDim.x * WB) {
        uint8_t x = 0xFF;
        if (v < a.nl) {
            const u64 deg = a.row[v + 1] - a.row[v], hd = deg - a.lsplit[v];
            const int32_t d = a.dist[v];
            if ((a.mb[v >> 6] >> (v & 63)) & 1ull) {
                m += hd;
                x = (uint8_t)(d - a.dlo);
            } else if (d >= hi) {
                u += hd;
                ua += deg;
            }
        }
        if (own) own[v] = x;
    }
    m = block_sum<WB / WAVE>(m, red);
    u = block_sum<WB / WAVE>(u, red);
    ua = block_sum<WB / WAVE>(ua, red);
    if (threadIdx.x == 0) {
        if (m) atomicAdd(&out[0], m);
        if (u) atomicAdd(&out[1], u);
        if (ua) atomicAdd(&out[2], ua);
    }
}

// bit v of the rank's words of the settled map: dist[v] < lo (v past nl: 0)
__global__ void wp_settled_k(WArgs a, int32_t lo, u64* __restrict__ words) {
    constexpr int SW = 8;  // words per wave step (loads together, one 8-lane store)
    const int lane = lane_id();
    const i64 nwaves = (i64)gridDim.x * (blockDim.x / WAVE);
    for (i64 w0 = ((i64)blockIdx.x * (blockDim.x / WAVE) + wave_id()) * SW; w0 < a.bw; w0 += nwaves * SW) {
        int32_t dd[SW];
#pragma unroll
        for (int j = 0; j < SW; ++j) {
            const i64 v = (w0 + j) * 64 + lane;
            dd[j] = v < a.nl ? a.dist[v] : INT_INF;
        }
        u64 mine = 0;
#pragma unroll
        for (int j = 0; j < SW; ++j) {
            const u64 m = __ballot(dd[j] < lo);
            if (lane == j) mine = m;
        }
        if (lane < SW && w0 + lane < a.bw) words[w0 + lane] = mine;
    }
}
// this rank's slice of the member map: dist - lo of a band member, 0xFF otherwise
__global__ void wp_member_slice_k(WArgs a, uint8_t* __restrict__ own) {
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < a.block; v += (i64)gridDim.x * blockDim.x) {
        uint8_t x = 0xFF;
        if (v < a.nl && ((a.mb[v >> 6] >> (v & 63)) & 1ull)) x = (uint8_t)(a.dist[v] - a.dlo);
        own[v] = x;
    }
}
// every unsettled owned vertex scans its heavy row (ascending weight) for band members
// (any rank's, through the replicated map) and stops once lo + w >= its best value; the
// first WP_PSERIAL edges by the lane alone, the rest of a long row by the whole wave
constexpr int WP_PSERIAL = 16;
#ifndef PJ_WP_HPU
#define PJ_WP_HPU 1  // 2 and 4 measured no faster at s26w (13.0-13.5 against 12.8-13.2 ms at world 1, r3ai)
#endif
constexpr int WP_HPU = PJ_WP_HPU;
// It also selects the next band [hi, nhi) as wp_select_k would (frontier words, frn and mb
// cleared, ST_CNT and ST_MIN): a vertex's distance is final for this step once its lane is
// done, and the wave owns its word.
__global__ __launch_bounds__(WB) void wp_pull_heavy_k(WArgs a, const uint8_t* __restrict__ mmap, int32_t nhi) {
    __shared__ u64 red[WB / WAVE];
    const int lane = lane_id();
    const int32_t lo = a.dlo, hi = a.dhi;
    const i64 nwaves = (i64)gridDim.x * (WB / WAVE);
    u64 c = 0;
    int32_t mn = INT_INF;
    for (i64 b0 = ((i64)blockIdx.x * (WB / WAVE) + wave_id()) * 64; b0 < a.bw * 64; b0 += nwaves * 64) {
        const i64 v = b0 + lane;
        int32_t d0 = INT_INF, cur = INT_INF;
        u64 k = 0, e = 0;
        bool act = false;
        if (v < a.nl) {
            d0 = a.dist[v];
            act = d0 >= hi;
            if (act) {
                cur = d0;
                k = a.row[v] + a.lsplit[v];
                e = a.row[v + 1];
            }
        }
        const u64 lim = e - k > (u64)WP_PSERIAL ? k + WP_PSERIAL : e;
        bool done = !act || k >= e;
        // WP_HPU edges per step: their weight, id and map loads issued together, then taken
        // in row order with the same early stop (the probes past a stop are wasted only)
        while (act && k < lim) {
            u32 w[WP_HPU], c[WP_HPU];
            uint8_t m[WP_HPU];
#pragma unroll
            for (int j = 0; j < WP_HPU; ++j) {
                const bool in = k + j < lim;
                w[j] = in ? a.w[k + j] : 0u;
                c[j] = in ? a.col[k + j] : 0u;
            }
#pragma unroll
            for (int j = 0; j < WP_HPU; ++j)
                m[j] = (k + j < lim && (long long)lo + w[j] < (long long)cur) ? mmap[c[j]] : (uint8_t)0xFF;
            bool stop = false;
#pragma unroll
            for (int j = 0; j < WP_HPU; ++j) {
                if (stop || k >= lim) continue;
                if ((long long)lo + w[j] >= (long long)cur) {
                    stop = true;
                    continue;
                }
                if (m[j] != 0xFF) cur = min(cur, lo + (int32_t)m[j] + (int32_t)w[j]);
                ++k;
            }
            if (stop) {
                done = true;
                break;
            }
        }
        if (k >= e) done = true;
        u64 open = __ballot(!done);
        while (open) {  // long rows: 64 edges per wave step, early stop when any lane may
            const int l = __ffsll((long long)open) - 1;
            open &= open - 1;
            const u64 kb = __shfl(k, l, 64), ke = __shfl(e, l, 64);
            int32_t cl = __shfl(cur, l, 64);
            for (u64 kk = kb; kk < ke; kk += WAVE) {
                const u64 k0 = kk + lane;
                const bool valid = k0 < ke;
                const u32 w = valid ? a.w[k0] : 0u;
                const bool stop = !valid || (long long)lo + w >= (long long)cl;
                int32_t cand = INT_INF;
                if (!stop) {
                    const uint8_t m = mmap[a.col[k0]];
                    if (m != 0xFF) cand = lo + (int32_t)m + (int32_t)w;
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
        if (act && cur < d0) a.dist[v] = cur;  // (the vertex's own rank is its only writer here)
        const int32_t dn = act ? cur : d0;  // (d0 = INT_INF past nl)
        const u64 m = __ballot(dn >= hi && dn < nhi);
        if (dn >= hi && dn < mn) mn = dn;
        if (lane == 0) {
            a.fr[b0 >> 6] = m;
            a.frn[b0 >> 6] = 0;
            a.mb[b0 >> 6] = 0;
            c += (u64)__popcll(m);
        }
    }
    c = block_sum<WB / WAVE>(c, red);
    if (threadIdx.x == 0 && c) atomicAdd(&a.stat[ST_CNT], c);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const int32_t y = __shfl_xor(mn, off, 64);
        mn = y < mn ? y : mn;
    }
    __syncthreads();
    if (lane == 0) red[wave_id()] = (u64)(u32)mn;
    __syncthreads();
    if (threadIdx.x == 0) {
        int32_t m = INT_INF;
        for (int k = 0; k < WB / WAVE; ++k) m = min(m, (int32_t)(u32)red[k]);
        if (m < INT_INF) atomicMin(&a.stat[ST_MIN], (u64)m);
    }
}

// Light pull rounds (engine.h DeltaSteps): (frontier light edges, light edges of vertices above lo)
__global__ __launch_bounds__(WB) void wp_light_counts_k(WArgs a, u64* __restrict__ out) {
    __shared__ u64 red[WB / WAVE];
    u64 f = 0, u = 0;
    int32_t fm = INT_INF;  // (out[2]: the least distance of this rank's frontier, the pulls' bound)
    constexpr int LU = 4;  // vertices per thread step, loads issued together
    const i64 stride = (i64)gridDim.x * WB;
    for (i64 v0 = (i64)blockIdx.x * WB + threadIdx.x; v0 < a.nl; v0 += LU * stride) {
        u64 ls[LU], fw[LU];
        int32_t d[LU];
#pragma unroll
        for (int j = 0; j < LU; ++j) {
            const i64 v = v0 + (i64)j * stride;
            const bool in = v < a.nl;
            ls[j] = in ? a.lsplit[v] : 0;
            fw[j] = in ? a.fr[v >> 6] : 0;
            d[j] = in ? a.dist[v] : 0;
        }
#pragma unroll
        for (int j = 0; j < LU; ++j) {
            const i64 v = v0 + (i64)j * stride;
            if ((fw[j] >> (v & 63)) & 1ull) {
                f += ls[j];
                fm = d[j] < fm ? d[j] : fm;
            }
            if (v < a.nl && d[j] > a.dlo) u += ls[j];
        }
    }
    f = block_sum<WB / WAVE>(f, red);
    u = block_sum<WB / WAVE>(u, red);
    if (threadIdx.x == 0) {
        if (f) atomicAdd(&out[0], f);
        if (u) atomicAdd(&out[1], u);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const int32_t y = __shfl_xor(fm, off, 64);
        fm = y < fm ? y : fm;
    }
    if (lane_id() == 0 && fm < INT_INF) atomicMin(&out[2], (u64)fm);
}
// this rank's slice of the frontier map: dist - lo of a frontier vertex, all ones otherwise
// (MT = u8 for bands up to 255 wide, u16 for the tail's wide bands)
template <typename MT>
__global__ void wp_frontier_slice_k(WArgs a, MT* __restrict__ own) {
    constexpr MT NONE = (MT)~(MT)0;
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < a.block; v += (i64)gridDim.x * blockDim.x) {
        MT x = NONE;
        if (v < a.nl && ((a.fr[v >> 6] >> (v & 63)) & 1ull)) x = (MT)(a.dist[v] - a.dlo);
        own[v] = x;
    }
}
// Light rows longer than WP_PLMAX (the hubs, at the lowest ids of the degree order) are
// pulled by wp_pull_long_k from a static list of (vertex, chunk of WP_PCH light edges),
// built once per light threshold, in the bands before the tail (in the tail the hubs are
// settled and such a list, of most of the graph's rows at the tail's threshold, cost
// ~1 ms per solve in skipped chunks): scanned inside wp_pull_light_k, one wave walked a hub's
// whole light row alone while the rest of the grid idled (an s26w solve whose hubs were
// unsettled at a light pull took 20-25 ms instead of 10, profiles/r05/wpart_sweep_r5k.txt).
constexpr u32 WP_PLMAX = 64;
constexpr u32 WP_PCH = 256;
__global__ void wp_plong_count_k(const u32* __restrict__ lsplit, i64 nl, u64* __restrict__ cnt) {
    u64 c = 0;
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < nl; v += (i64)gridDim.x * blockDim.x)
        if (lsplit[v] > WP_PLMAX) c += (lsplit[v] + WP_PCH - 1) / WP_PCH;
    c = wave_sum(c);
    if (lane_id() == 0 && c) atomicAdd(cnt, c);
}
__global__ void wp_plong_fill_k(const u32* __restrict__ lsplit, i64 nl, u64* __restrict__ cnt, u32* __restrict__ lv,
                                u32* __restrict__ lc) {
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < nl; v += (i64)gridDim.x * blockDim.x)
        if (lsplit[v] > WP_PLMAX) {
            const u32 nc = (lsplit[v] + WP_PCH - 1) / WP_PCH;
            const u64 b = atomicAdd(cnt, (u64)nc);
            for (u32 c = 0; c < nc; ++c) {
                lv[b + c] = (u32)v;
                lc[b + c] = c;
            }
        }
}
// A light pull stops a row at flo + w >= its best, flo = the least distance of every rank's
// frontier (the ranks' wp_light_counts_k minima, min-all-reduced by the engine), instead of
// lo + w: no frontier in-neighbour offers less than flo + w (v2's frontier-minimum bound,
// delta.hip v2_pull_lo).

// a wave per chunk: skipped when even its lightest edge cannot help, else scanned with the
// early stop; the result goes in with atomicMin (a vertex's chunks run in different waves)
// and the vertex's next-frontier bit with a returning atomicOr (counted once)
template <typename MT>
__global__ __launch_bounds__(WB) void wp_pull_long_k(WArgs a, const MT* __restrict__ fmap, const u32* __restrict__ lv,
                                                     const u32* __restrict__ lc, u64 nlc, int32_t flo) {
    constexpr MT NONE = (MT)~(MT)0;
    __shared__ u64 red[WB / WAVE];
    const int lane = lane_id();
    const int32_t lo = a.dlo, hi = a.dhi;
    u64 marks = 0;
    for (u64 it = (u64)blockIdx.x * (WB / WAVE) + wave_id(); it < nlc; it += (u64)gridDim.x * (WB / WAVE)) {
        const u32 v = lv[it];
        const int32_t d0 = __hip_atomic_load(a.dist + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d0 <= lo) continue;
        const u64 rb = a.row[v];
        const u64 kb = rb + (u64)lc[it] * WP_PCH;
        const u64 ke = min(rb + (u64)a.lsplit[v], kb + WP_PCH);
        if ((long long)flo + a.w[kb] >= (long long)d0) continue;
        int32_t cur = d0;
        for (u64 kk = kb; kk < ke; kk += WAVE) {
            const u64 k0 = kk + lane;
            const bool valid = k0 < ke;
            const u32 w = valid ? a.w[k0] : 0u;
            const bool stop = !valid || (long long)flo + w >= (long long)cur;
            int32_t cand = INT_INF;
            if (!stop) {
                const MT m = fmap[a.col[k0]];
                if (m != NONE) cand = lo + (int32_t)m + (int32_t)w;
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
                const u64 bit = 1ull << (v & 63);
                if (!(atomicOr(a.frn + (v >> 6), bit) & bit)) ++marks;
            }
        }
    }
    marks = block_sum<WB / WAVE>(marks, red);
    if (threadIdx.x == 0 && marks) atomicAdd(&a.stat[ST_NF], marks);
}

// every owned vertex above lo scans its light row (ascending weight) for frontier vertices
// (any rank's, through the map; frozen at the slice: a label-correcting round) and stops
// once lo + w >= its best value; improved vertices below hi join the next frontier. The
// wave owns its 64 vertices' words: the frontier word moves into mb (the round consumed
// it) and the next-frontier word is OR-ed in (wp_pull_long_k, launched before, may have
// set bits of it). Rows longer than plmax are wp_pull_long_k's.
template <typename MT>
__global__ __launch_bounds__(WB) void wp_pull_light_k(WArgs a, const MT* __restrict__ fmap, u32 plmax,
                                                      int32_t flo) {
    constexpr MT NONE = (MT)~(MT)0;
    __shared__ u64 red[WB / WAVE];
    const int lane = lane_id();
    const int32_t lo = a.dlo, hi = a.dhi;
    const i64 nwaves = (i64)gridDim.x * (WB / WAVE);
    u64 marks = 0;
    for (i64 b0 = ((i64)blockIdx.x * (WB / WAVE) + wave_id()) * 64; b0 < a.nl; b0 += nwaves * 64) {
        const i64 v = b0 + lane;
        if (lane == 0) {  // (cleared as consumed: end_round swaps fr and frn)
            const u64 f = a.fr[b0 >> 6];
            if (f) {
                a.mb[b0 >> 6] |= f;
                a.fr[b0 >> 6] = 0;
            }
        }
        int32_t d0 = INT_INF, cur = INT_INF;
        u64 k = 0, e = 0;
        bool act = false;
        if (v < a.nl) {
            d0 = a.dist[v];
            act = d0 > lo;
            if (act) {
                cur = d0;
                k = a.row[v];
                const u32 ls = a.lsplit[v];
                e = ls > plmax ? k : k + ls;
            }
        }
        const u64 lim = e - k > (u64)WP_PSERIAL ? k + WP_PSERIAL : e;
        bool done = !act || k >= e;
        while (act && k < lim) {
            const u32 w = a.w[k];
            if ((long long)flo + w >= (long long)cur) {
                done = true;
                break;
            }
            const MT m = fmap[a.col[k]];
            if (m != NONE) cur = min(cur, lo + (int32_t)m + (int32_t)w);
            ++k;
        }
        if (k >= e) done = true;
        u64 open = __ballot(!done);
        while (open) {
            const int l = __ffsll((long long)open) - 1;
            open &= open - 1;
            const u64 kb = __shfl(k, l, 64), ke = __shfl(e, l, 64);
            int32_t cl = __shfl(cur, l, 64);
            for (u64 kk = kb; kk < ke; kk += WAVE) {
                const u64 k0 = kk + lane;
                const bool valid = k0 < ke;
                const u32 w = valid ? a.w[k0] : 0u;
                const bool stop = !valid || (long long)flo + w >= (long long)cl;
                int32_t cand = INT_INF;
                if (!stop) {
                    const MT m = fmap[a.col[k0]];
                    if (m != NONE) cand = lo + (int32_t)m + (int32_t)w;
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
        const bool imp = act && cur < d0;
        if (imp) a.dist[v] = cur;
        const u64 nb = __ballot(imp && cur < hi);
        if (lane == 0 && nb) {
            a.frn[b0 >> 6] |= nb;
            marks += (u64)__popcll(nb);
        }
    }
    marks = block_sum<WB / WAVE>(marks, red);
    if (threadIdx.x == 0 && marks) atomicAdd(&a.stat[ST_NF], marks);
}

// out-edges of the owned vertices not settled below hi (dist >= hi, unreached included)
__global__ __launch_bounds__(WB) void wp_unsettled_k(WArgs a, int32_t hi, u64* __restrict__ out) {
    __shared__ u64 red[WB / WAVE];
    u64 acc = 0;
    for (i64 v = (i64)blockIdx.x * WB + threadIdx.x; v < a.nl; v += (i64)gridDim.x * WB)
        if (a.dist[v] >= hi) acc += a.row[v + 1] - a.row[v];
    acc = block_sum<WB / WAVE>(acc, red);
    if (threadIdx.x == 0 && acc) atomicAdd(out, acc);
}

__global__ __launch_bounds__(WB) void wp_reach_k(WArgs a) {
    __shared__ u64 red[WB / WAVE];
    u64 c = 0, m = 0;
    for (i64 v = (i64)blockIdx.x * WB + threadIdx.x; v < a.nl; v += (i64)gridDim.x * WB)
        if (a.dist[v] < INT_INF) {
            ++c;
            m += a.row[v + 1] - a.row[v];
        }
    c = block_sum<WB / WAVE>(c, red);
    m = block_sum<WB / WAVE>(m, red);
    if (threadIdx.x == 0) {
        if (c) atomicAdd(&a.stat[ST_REACH], c);
        if (m) atomicAdd(&a.stat[ST_REACH + 1], m);
    }
}

__global__ void wsum_all_k(const u32* __restrict__ w, i64 m, u64* __restrict__ out) {
    u64 s = 0;
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (i64)gridDim.x * blockDim.x) s += w[i];
    s = wave_sum(s);
    if (lane_id() == 0 && s) atomicAdd(out, s);
}

// stat[k0, k1) and [k2, k3) into the host copy, then the sequence word the host spins on
// (as delta.hip's v2_publish_k)
__global__ __launch_bounds__(256) void wp_publish_k(const u64* __restrict__ stat, u64* __restrict__ host, int k0,
                                                    int k1, int k2, int k3, u64* seqp, u64 seq) {
    for (int i = k0 + (int)threadIdx.x; i < k1; i += 256) host[i] = stat[i];
    for (int i = k2 + (int)threadIdx.x; i < k3; i += 256) host[i] = stat[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(seqp, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace

// The stat block's host copy: mapped pinned memory written by wp_publish_k, with a sequence
// word the host spins on. (A D2H hipMemcpyAsync of the block ran as a ~12 us blit per read
// plus the stream synchronization's wake-up, ~100 reads per world-2 s26w solve,
// profiles/r05/wpart_timeline_r5i.txt.)
struct PinnedStat {
    u64* p = nullptr;
    u64* dev = nullptr;
    u64* seqw = nullptr;
    u64* seq_dev = nullptr;
    u64 seq = 0;
    PinnedStat() {
        PJ_HIP(hipHostMalloc(reinterpret_cast<void**>(&p), sizeof(u64) * ST_N, hipHostMallocMapped));
        PJ_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev), p, 0));
        PJ_HIP(hipHostMalloc(reinterpret_cast<void**>(&seqw), 64, hipHostMallocMapped | hipHostMallocCoherent));
        PJ_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&seq_dev), seqw, 0));
        __atomic_store_n(seqw, 0ull, __ATOMIC_RELEASE);
    }
    ~PinnedStat() {
        if (p) (void)hipHostFree(p);
        if (seqw) (void)hipHostFree(seqw);
    }
    u64& operator[](size_t i) { return p[i]; }
    // stat[k0, k1) of the device block once the stream's earlier work is done: the host
    // spins on the sequence word (after 0.2 s it synchronizes the stream instead, which
    // surfaces a failed kernel rather than spinning forever)
    void read(const u64* stat, int k0, int k1, hipStream_t s, int k2 = 0, int k3 = 0) {
        const u64 q = next();
        wp_publish_k<<<1, 256, 0, s>>>(stat, dev, k0, k1, k2, k3, seq_dev, q);
        PJ_LAUNCH_CHECK();
        wait(q, s);
    }
    u64 next() { return ++seq; }  // the sequence value the next publication writes
    void wait(u64 q, hipStream_t s) {
        const auto t0 = std::chrono::steady_clock::now();
        while (__atomic_load_n(seqw, __ATOMIC_ACQUIRE) != q) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
                PJ_HIP(hipStreamSynchronize(s));
                break;
            }
        }
    }
    PinnedStat(const PinnedStat&) = delete;
    PinnedStat& operator=(const PinnedStat&) = delete;
};

struct WPart {
    Ctx* ctx = nullptr;
    i64 n = 0, lo = 0, hi = 0, nl = 0, block = 64, bw = 1, nnz_local = 0, nnz = 0;
    int rank = 0, world = 1;
    double mean_w = 1.0;
    int32_t delta = 0;
    int32_t delta_alt = 0;         // the light threshold lsplit_alt was computed for (0 = none)
    double tail[2] = {0.3, 64.0};  // tail switch (engine.h DeltaSteps): tail_frac (0 = off), threshold / delta
                                   // (tail_frac 0.1 until round 5: 0.3 measured best at s24w / s26w,
                                   // worlds 1 and 2, profiles/r05/wpart_sweep_r5o.txt)
    double pull_factor = 4.0;      // heavy pull when unsettled heavy edges < pull_factor x members' (0 = push)
    double tail_light_pull = 3.0;  // the same rule after the tail switch (independent of light_pull; 0 =
                                   // push), with a 16-bit frontier map for the tail's wide bands
    double light_pull = 3.0;       // light pull round when the frontier's light edges > the light edges
                                   // of the vertices above lo / light_pull (0 = push). 0 from round 3
                                   // (r3ad) until round 6: with the pulls' frontier-minimum bound, 3
                                   // measured 9.57-9.81 against 10.02-10.03 ms at world 2 (s26w,
                                   // interleaved, profiles/r06/wpart_light_pull_r6l.txt)
    bool symmetric = false;        // rows are also the in-edges (Kronecker graphs): the heavy pull applies
    DevBuf<uint8_t> mmap;          // replicated member map of the heavy pull (world x block bytes)
    DevBuf<uint16_t> fmap16;       // replicated frontier map of a light pull in a band wider than 255
    bool map16 = false;            // the last slice went to fmap16 (member_map() hands it out)
    DevBuf<u64> row;
    DevBuf<u32> col, w, lsplit;
    struct PullLong {              // the light pull's long-row chunk list of one light threshold
        DevBuf<u32> v, c;
        u64 n = 0;
        bool built = false;
    } pl, pl_alt;                  // (of delta and delta_alt)
    DevBuf<u32> lsplit_alt;        // the other light threshold's prefixes (delta and the tail's are
                                   // used in turn by every solve: each was recomputed per solve)
    DevBuf<int32_t> dist;
    DevBuf<u64> fr, frn, mb, stat;
    DevBuf<u64> rc;                // (world > 1) sent-pair cache, 2^rcb entries (>= block)
    u32 rcb = 1;
    DevBuf<u64> q, qctr;           // (world > 1) claim queue: WQ_S shards of qsh pairs + a spill of qsp, and
    u64 qsh = 0, qsp = 0;          // the counters
    i64 qsh_min = -1;              // option "queue_shard": smallest shard capacity (-1 = automatic)
    bool pending_pack = false;     // the last relax's pairs are queued and not packed yet
    DevBuf<u32> rl_inv;   // (relabeled blocks) old local id -> new local id; empty: input ids
    DevBuf<u64> sb;       // the tail's settled map, world x block bits (engine all-gathers the slices)
    bool sb_on = false;   // sb holds this solve's map (set at the tail switch)
    int32_t ua_hi = INT_MIN;  // wp_heavy_counts_k's third count is for this hi (this band)
    i64 ua = 0;
    int32_t ms_lo = INT_MIN;  // wp_heavy_counts_k wrote the member slice of the band starting here
    int32_t fs_lo = INT_MIN, fs_hi = INT_MIN;  // wp_pull_heavy_k selected [fs_lo, fs_hi) (stat, fr, frn, mb)
    i64 exch_bytes = 0;  // the engine view's send + recv buffers (sized to the largest round)
    DevBuf<u32> lq_v;
    DevBuf<u64> lq_b, lq_e;
    PinnedStat hstat;
    std::unique_ptr<DeltaSteps> steps;  // engine view with its own exchange buffers (lazy)
    int single_gpu = 1;                 // world 1: solve with delta.hip's v2 (wpart_solve_single)
    int pull_fmin = 1;                  // light pulls stop rows at the frontier's least distance
    i64 fmin_own = INT_INF;             // this rank's frontier minimum (wpart_light_counts)
    i64 fmin_all = INT_INF;             // every rank's (DeltaSteps::set_frontier_min), or -1: none
    std::unique_ptr<Graph> g1;          // (its Graph over copies of the rows, built at the first solve)
    int gpc = 8;                        // workgroups per CU of the grid-stride kernels (option grid_per_cu)
    unsigned grid() const { return (unsigned)ctx->cu_count * (unsigned)gpc; }
    unsigned qgrid() const {  // (region-major: the shards and the spill)
        return (unsigned)(WQ_S + 1) * std::max(1u, grid() / (unsigned)(WQ_S + 1));
    }
    u64 qcap() const { return (u64)WQ_S * qsh + qsp; }
    WArgs args(int32_t dlo = 0, int32_t dhi = 0) {
        WArgs a{};
        a.n = n;
        a.lo = lo;
        a.nl = nl;
        a.block = block;
        a.bw = bw;
        a.rank = rank;
        a.dlo = dlo;
        a.dhi = dhi;
        a.row = row.p;
        a.col = col.p;
        a.w = w.p;
        a.lsplit = lsplit.p;
        a.dist = dist.p;
        a.rc = rc.p;
        a.rcb = rcb;
        a.q = world > 1 ? q.p : nullptr;
        a.qsh = qsh;
        a.qsp = qsp;
        a.qctr = qctr.p;
        a.fr = fr.p;
        a.frn = frn.p;
        a.mb = mb.p;
        a.lq_v = lq_v.p;
        a.lq_b = lq_b.p;
        a.lq_e = lq_e.p;
        a.stat = stat.p;
        a.sbits = sb_on ? sb.p : nullptr;
        return a;
    }
    // (the pack cursors ST_CUR.. are the device's own: every other word)
    void read_stat() { hstat.read(stat.p, 0, ST_CUR, ctx->stream, ST_QTOT, ST_N); }
    void read_acc(u64* out, int k) {  // stat[ST_ACC, ST_ACC + k) through the host copy
        hstat.read(stat.p, ST_ACC, ST_ACC + k, ctx->stream);
        for (int i = 0; i < k; ++i) out[i] = hstat.p[ST_ACC + i];
    }
    void clear_stat() { PJ_HIP(hipMemsetAsync(stat.p, 0, sizeof(u64) * ST_N, ctx->stream)); }
};

void delete_wpart(WPart* p) { delete p; }

namespace {

// the claim queue at shard capacity qsh and spill capacity qsp (pairs), counters cleared
void wpart_queue(WPart& p, u64 qsh, u64 qsp) {
    p.qsh = std::max<u64>(qsh, 1ull);
    p.qsp = std::max<u64>(qsp, 1ull);
    p.q.alloc((size_t)p.qcap());
    PJ_HIP(hipMemsetAsync(p.qctr.p, 0, p.qctr.bytes(), p.ctx->stream));
}

u64 weight_sum(const u32* w, i64 m, unsigned grid, hipStream_t s) {
    u64 wsum = 0;
    if (m > 0) {
        DevBuf<u64> acc(1);
        PJ_HIP(hipMemsetAsync(acc.p, 0, sizeof(u64), s));
        wsum_all_k<<<grid_for(m, 256, grid), 256, 0, s>>>(w, m, acc.p);
        PJ_LAUNCH_CHECK();
        PJ_HIP(hipMemcpyAsync(&wsum, acc.p, sizeof(u64), hipMemcpyDeviceToHost, s));
        PJ_HIP(hipStreamSynchronize(s));
    }
    return wsum;
}

// Block geometry of rank / world over n vertices (the pj_part_* rule).
std::unique_ptr<WPart> wpart_geometry(Ctx* ctx, i64 n, i64 nnz, int rank, int world) {
    if (world < 1 || world > WP_MAXW || rank < 0 || rank >= world) throw Error(PJ_ERR_ARG, "rank/world out of range");
    std::unique_ptr<WPart> p(new WPart());
    p->ctx = ctx;
    p->n = n;
    p->nnz = nnz;
    p->rank = rank;
    p->world = world;
    const i64 per = (n + world - 1) / world;
    p->block = std::max<i64>(64, (per + 63) / 64 * 64);
    p->bw = p->block / 64;
    p->lo = std::min<i64>((i64)rank * p->block, n);
    p->hi = std::min<i64>(p->lo + p->block, n);
    p->nl = p->hi - p->lo;
    return p;
}

// The block's weighted rows = rows [first, first + nl) of g (weight-sorted CSR, global
// column ids): offsets rebased, edges and weights copied; then the per-solve state.
void wpart_cut(WPart* p, const Graph& g, i64 first, double mean_w) {
    hipStream_t s = p->ctx->stream;
    u64 eb = 0, ee = 0;
    if (g.n > 0) {
        if (g.off64) {
            PJ_HIP(hipMemcpyAsync(&eb, g.row64.p + first, sizeof(u64), hipMemcpyDeviceToHost, s));
            PJ_HIP(hipMemcpyAsync(&ee, g.row64.p + first + p->nl, sizeof(u64), hipMemcpyDeviceToHost, s));
        } else {
            u32 b32 = 0, e32 = 0;
            PJ_HIP(hipMemcpyAsync(&b32, g.row32.p + first, sizeof(u32), hipMemcpyDeviceToHost, s));
            PJ_HIP(hipMemcpyAsync(&e32, g.row32.p + first + p->nl, sizeof(u32), hipMemcpyDeviceToHost, s));
            PJ_HIP(hipStreamSynchronize(s));
            eb = b32;
            ee = e32;
        }
        PJ_HIP(hipStreamSynchronize(s));
    }
    p->nnz_local = (i64)(ee - eb);
    p->row.alloc((size_t)p->nl + 1);
    if (g.n > 0) {
        wp_rebase_k<<<grid_for(p->nl + 1, 256, p->grid()), 256, 0, s>>>(g.row_ptr(), g.off64, first, p->nl, p->row.p);
        PJ_LAUNCH_CHECK();
    } else {
        PJ_HIP(hipMemsetAsync(p->row.p, 0, sizeof(u64), s));
    }
    p->col.alloc((size_t)std::max<i64>(p->nnz_local, 1));
    p->w.alloc((size_t)std::max<i64>(p->nnz_local, 1));
    if (p->nnz_local) {
        PJ_HIP(hipMemcpyAsync(p->col.p, g.col.p + eb, sizeof(u32) * (size_t)p->nnz_local, hipMemcpyDeviceToDevice, s));
        PJ_HIP(hipMemcpyAsync(p->w.p, g.w.p + eb, sizeof(u32) * (size_t)p->nnz_local, hipMemcpyDeviceToDevice, s));
    }
    p->mean_w = mean_w;
    const size_t nl1 = (size_t)std::max<i64>(p->nl, 1);
    p->lsplit.alloc(nl1);
    p->dist.alloc(nl1);
    p->fr.alloc((size_t)p->bw);
    p->frn.alloc((size_t)p->bw);
    p->mb.alloc((size_t)p->bw);
    p->lq_v.alloc(nl1);
    p->lq_b.alloc(nl1);
    p->lq_e.alloc(nl1);
    p->stat.alloc(ST_N);
    std::fill(p->hstat.p, p->hstat.p + ST_N, 0ull);
    if (p->world > 1) {
        while (p->rcb < 31 && ((i64)1 << p->rcb) < std::max<i64>(p->block, 4096)) ++p->rcb;
        p->rc.alloc((size_t)1 << p->rcb);
        p->qctr.alloc((size_t)(WQ_S + 1) * 8);
        // (grows with the rounds' pairs; a rerun costs a round, so start at block / 4 pairs over
        // the shards and block / 8 as spill)
        const u64 q0 = (u64)std::max<i64>(16, p->block / 256);
        wpart_queue(*p, q0, WQ_S * q0 / 2);
    }
    PJ_HIP(hipStreamSynchronize(s));
}

// keep the edges whose source lies in [lo, hi): count per block, scan, write (file order)
__global__ void wp_filter_count_k(const u32* __restrict__ src, i64 m, u32 lo, u32 hi, u32* __restrict__ bcnt) {
    __shared__ u32 red[4];
    u32 c = 0;
    const i64 b0 = (i64)blockIdx.x * 4096;
    for (i64 i = b0 + threadIdx.x; i < min(b0 + 4096, m); i += 256) c += (src[i] >= lo && src[i] < hi) ? 1u : 0u;
    c = block_sum<4>(c, red);
    if (threadIdx.x == 0) bcnt[blockIdx.x] = c;
}
__global__ void wp_filter_write_k(const u32* __restrict__ src, const u32* __restrict__ dst, const u32* __restrict__ w,
                                  i64 m, u32 lo, u32 hi, const u64* __restrict__ boff, u32* __restrict__ os,
                                  u32* __restrict__ od, u32* __restrict__ ow) {
    __shared__ u64 red[4];
    const i64 b0 = (i64)blockIdx.x * 4096;
    u64 base = boff[blockIdx.x];
    for (i64 i0 = b0; i0 < min(b0 + 4096, m); i0 += 256) {
        const i64 i = i0 + threadIdx.x;
        const bool keep = i < m && src[i] >= lo && src[i] < hi;
        u64 tot;
        const u64 ex = block_excl_scan<4>((u64)(keep ? 1 : 0), red, tot);
        if (keep) {
            os[base + ex] = src[i] - lo;
            od[base + ex] = dst[i];
            ow[base + ex] = w[i];
        }
        base += tot;
    }
}


// ---- per-block degree order (PJ_WP_RELABEL) --------------------------------------
// delta.hip's relabel (hot distances share lines) restated for the partition: inside
// every block, vertices by out-degree descending (ties by input id). A vertex keeps its
// block, so the owner of a new id is the owner of the old one and the block geometry,
// the exchange and the pulls' byte map are unchanged; every rank derives the same map
// from the degrees of ALL vertices (each builder sees every entry: the generator's
// tuples, the parsed file, the full graph) and keeps only its block's inverse. The
// source is mapped on entry, distances are mapped back on the way out. With it, the rows
// longer than WP_LONG = 64 edges go to the edge-balanced queue: the order puts the long
// rows into the first waves of the block, and one wave per 64 of them relaxed 3x slower
// (r4a, at 1024). s26w 11.1-12.7 -> 8.9-10.5 ms at world 1, 17.1-18.6 -> 13.4-15.6 ms at
// world 2 (r4c, profiles/r04/wpart_r4c.txt).
#ifndef PJ_WP_RELABEL
#define PJ_WP_RELABEL 1
#endif
__global__ void wp_deg_key_k(const u32* __restrict__ deg, i64 n, u32 maxdeg, u32* __restrict__ key,
                             u32* __restrict__ ids) {
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x) {
        key[v] = maxdeg - deg[v];
        ids[v] = (u32)v;
    }
}
// block q's part of the global map: its vertex lo_q + order[i] becomes lo_q + i
__global__ void wp_inv_blk_k(const u32* __restrict__ order, i64 nq, i64 lo_q, u32* __restrict__ inv) {
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < nq; i += (i64)gridDim.x * blockDim.x)
        inv[lo_q + order[i]] = (u32)(lo_q + i);
}
// new local row l = old local row order[l]: its degree, and the old local -> new local map
__global__ void wp_newdeg_k(const u32* __restrict__ order, const u32* __restrict__ inv, const u64* __restrict__ row,
                            i64 lo, i64 nl, u32* __restrict__ ndeg, u32* __restrict__ linv) {
    for (i64 l = (i64)blockIdx.x * blockDim.x + threadIdx.x; l < nl; l += (i64)gridDim.x * blockDim.x) {
        const i64 o = (i64)order[l];
        ndeg[l] = (u32)(row[o + 1] - row[o]);
        linv[l] = (u32)((i64)inv[lo + l] - lo);
    }
}
// copy the rows in the new order, columns through the global map (a wave per row)
__global__ __launch_bounds__(256) void wp_copy_rows_k(const u32* __restrict__ order, const u32* __restrict__ inv,
                                                      const u64* __restrict__ row, const u32* __restrict__ col,
                                                      const u32* __restrict__ w, const u64* __restrict__ nrow, i64 lo,
                                                      i64 nl, u32* __restrict__ ncol, u32* __restrict__ nw) {
    const int lane = lane_id();
    for (i64 l = ((i64)blockIdx.x * blockDim.x + threadIdx.x) / WAVE; l < nl;
         l += (i64)gridDim.x * blockDim.x / WAVE) {
        const i64 o = (i64)order[l];
        const u64 b = row[o], e = row[o + 1], nb = nrow[l];
        for (u64 k = b + (u64)lane; k < e; k += WAVE) {
            ncol[nb + (k - b)] = inv[col[k]];
            nw[nb + (k - b)] = w[k];
        }
    }
}
__global__ void wp_deg_coo_k(const u32* __restrict__ src, i64 m, u32* __restrict__ deg) {
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (i64)gridDim.x * blockDim.x)
        atomicAdd(&deg[src[i]], 1u);
}
__global__ void wp_deg_row_k(const void* row, bool off64, i64 n, u32* __restrict__ deg) {
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x)
        deg[v] = off64 ? (u32)(((const u64*)row)[v + 1] - ((const u64*)row)[v])
                       : ((const u32*)row)[v + 1] - ((const u32*)row)[v];
}
__global__ void wp_max_k(const u32* __restrict__ in, i64 n, u32* __restrict__ out) {
    u32 m = 0;
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) m = max(m, in[i]);
    m = wave_max(m);
    if (lane_id() == 0 && m) atomicMax(out, m);
}
__global__ void wp_unlabel_k(const int32_t* __restrict__ dist, const u32* __restrict__ linv, i64 nl,
                             int32_t* __restrict__ out) {
    for (i64 l = (i64)blockIdx.x * blockDim.x + threadIdx.x; l < nl; l += (i64)gridDim.x * blockDim.x)
        out[l] = dist[linv[l]];
}

// Per-block weighted Kronecker build: every rank enumerates the tuples of the
// generator spec (kron.h, both directions, the tuple's weight on each), keeps the
// entries whose source lies in its block, in enumeration order (= the single-GPU
// generator's file order, so the rows sort to the same weight-sorted rows), and sums
// every entry's weight for the whole graph's mean (each rank sees all tuples, so every
// rank derives the same automatic delta). 2048 tuples per block.
constexpr int WK_IPT = 8;
__global__ __launch_bounds__(256) void wp_kron_count_k(int scale, u64 seed, PermKeys pk, u64 M, u32 lo, u32 hi,
                                                       u32* __restrict__ bcnt, u64* __restrict__ wsum) {
    __shared__ u64 red[4];
    const u64 base = (u64)blockIdx.x * 256 * WK_IPT;
    u32 c = 0;
    u64 ws = 0;
    for (int k = 0; k < WK_IPT; ++k) {
        const u64 i = base + (u64)k * 256 + threadIdx.x;
        if (i < M) {
            u32 pu, pv;
            kron_tuple(scale, seed, pk, i, pu, pv);
            c += (pu >= lo && pu < hi) + (pv >= lo && pv < hi);
            ws += 2ull * kron_weight(seed, i, true);
        }
    }
    c = (u32)block_sum<4>((u64)c, red);
    ws = block_sum<4>(ws, red);
    if (threadIdx.x == 0) {
        bcnt[blockIdx.x] = c;
        atomicAdd(wsum, ws);
    }
}
__global__ __launch_bounds__(256) void wp_kron_deg_k(int scale, u64 seed, PermKeys pk, u64 M, u32* __restrict__ deg) {
    const u64 base = (u64)blockIdx.x * 256 * WK_IPT;
    for (int k = 0; k < WK_IPT; ++k) {
        const u64 i = base + (u64)k * 256 + threadIdx.x;
        if (i < M) {
            u32 pu, pv;
            kron_tuple(scale, seed, pk, i, pu, pv);
            atomicAdd(&deg[pu], 1u);
            atomicAdd(&deg[pv], 1u);
        }
    }
}
__global__ __launch_bounds__(256) void wp_kron_write_k(int scale, u64 seed, PermKeys pk, u64 M, u32 lo, u32 hi,
                                                       const u64* __restrict__ boff, u32* __restrict__ os,
                                                       u32* __restrict__ od, u32* __restrict__ ow) {
    __shared__ u64 red[4];
    const u64 b0 = (u64)blockIdx.x * 256 * WK_IPT;
    u64 pos = boff[blockIdx.x];
    for (int k = 0; k < WK_IPT; ++k) {
        const u64 i = b0 + (u64)k * 256 + threadIdx.x;
        u32 pu = 0, pv = 0, w = 0;
        bool k0 = false, k1 = false;
        if (i < M) {
            kron_tuple(scale, seed, pk, i, pu, pv);
            w = kron_weight(seed, i, true);
            k0 = pu >= lo && pu < hi;  // entry 2i: pu -> pv
            k1 = pv >= lo && pv < hi;  // entry 2i + 1: pv -> pu
        }
        u64 tot;
        u64 p = pos + block_excl_scan<4>((u64)k0 + (u64)k1, red, tot);
        if (k0) {
            os[p] = pu - lo;
            od[p] = pv;
            ow[p] = w;
            ++p;
        }
        if (k1) {
            os[p] = pv - lo;
            od[p] = pu;
            ow[p] = w;
        }
        pos += tot;
    }
}

}  // namespace

namespace {
// Relabel a built block (rows, col, w in input ids) given the degrees of every vertex:
// within every block the vertices in descending degree (ties by id), so the new ids stay in
// their block. The blocks are ordered one at a time (block-sized sort buffers), so the
// transient device memory is the degrees and the global map, 8 N bytes, plus 16 x block
// (round 4 sorted all N vertices at once: 20 N bytes); the graph's col ids go through the
// map, which is why it is global.
void wpart_relabel(WPart& p, DevBuf<u32>& deg) {
    hipStream_t s = p.ctx->stream;
    const i64 n = p.n;
    if (n == 0) return;
    const unsigned grid = p.grid();
    DevBuf<u32> mx(1);
    PJ_HIP(hipMemsetAsync(mx.p, 0, sizeof(u32), s));
    wp_max_k<<<grid_for(n, 256, grid), 256, 0, s>>>(deg.p, n, mx.p);
    PJ_LAUNCH_CHECK();
    u32 maxdeg = 0;
    PJ_HIP(hipMemcpyAsync(&maxdeg, mx.p, sizeof(u32), hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
    const i64 nl = p.nl;
    const size_t bsz = (size_t)std::max<i64>(1, std::min<i64>(p.block, n));
    DevBuf<u32> inv((size_t)n), own((size_t)std::max<i64>(nl, 1));  // the global map, this block's order
    {
        DevBuf<u32> key(bsz), kalt(bsz), ids(bsz), valt(bsz);
        SortWs ws;
        int bits = 1;
        while (bits < 32 && ((u64)1 << bits) <= (u64)maxdeg) ++bits;
        for (int q = 0; q < p.world; ++q) {
            const i64 lo_q = (i64)q * p.block, nq = std::min<i64>(p.block, n - lo_q);
            if (nq <= 0) break;
            wp_deg_key_k<<<grid_for(nq, 256, grid), 256, 0, s>>>(deg.p + lo_q, nq, maxdeg, key.p, ids.p);
            PJ_LAUNCH_CHECK();
            u32 *kr, *vr;  // (stable: ties keep ascending ids)
            radix_sort_pairs<u32>(key.p, kalt.p, ids.p, valt.p, nq, bits, ws, s, &kr, &vr);
            wp_inv_blk_k<<<grid_for(nq, 256, grid), 256, 0, s>>>(vr, nq, lo_q, inv.p);
            PJ_LAUNCH_CHECK();
            if (q == p.rank && nl > 0)
                PJ_HIP(hipMemcpyAsync(own.p, vr, sizeof(u32) * (size_t)nl, hipMemcpyDeviceToDevice, s));
        }
        PJ_HIP(hipStreamSynchronize(s));
    }
    deg.release();
    const u32* order = own.p;
    DevBuf<u32> ndeg((size_t)std::max<i64>(nl, 1));
    p.rl_inv.alloc((size_t)std::max<i64>(nl, 1));
    DevBuf<u64> nrow((size_t)nl + 1);
    if (nl > 0) {
        wp_newdeg_k<<<grid_for(nl, 256, grid), 256, 0, s>>>(order, inv.p, p.row.p, p.lo, nl, ndeg.p, p.rl_inv.p);
        PJ_LAUNCH_CHECK();
        ScanWs sw;
        exclusive_scan_u32(ndeg.p, nrow.p, nl, sw, s);
        DevBuf<u32> ncol((size_t)std::max<i64>(p.nnz_local, 1)), nw((size_t)std::max<i64>(p.nnz_local, 1));
        wp_copy_rows_k<<<grid_for(nl * WAVE, 256, grid), 256, 0, s>>>(order, inv.p, p.row.p, p.col.p, p.w.p, nrow.p,
                                                                      p.lo, nl, ncol.p, nw.p);
        PJ_LAUNCH_CHECK();
        PJ_HIP(hipStreamSynchronize(s));
        p.row = std::move(nrow);
        p.col = std::move(ncol);
        p.w = std::move(nw);
    }
    PJ_HIP(hipStreamSynchronize(s));
}
}  // namespace

WPart* wpart_from_kronecker(Ctx& ctx, int scale, int edgefactor, uint64_t seed, int rank, int world) {
    hipStream_t s = ctx.stream;
    const u64 M = (u64)edgefactor << scale;
    std::unique_ptr<WPart> p = wpart_geometry(&ctx, (i64)1 << scale, (i64)(2 * M), rank, world);
    const PermKeys pk = make_perm_keys(scale, seed);
    const i64 nb = (i64)((M + 256 * WK_IPT - 1) / (256 * WK_IPT));
    i64 m = 0;
    u64 wsum = 0;
    DevBuf<u32> ls, ld, lw;
    if (nb > 0) {
        DevBuf<u32> bcnt((size_t)nb);
        DevBuf<u64> boff((size_t)nb + 1), acc(1);
        ScanWs ws;
        PJ_HIP(hipMemsetAsync(acc.p, 0, sizeof(u64), s));
        wp_kron_count_k<<<(unsigned)nb, 256, 0, s>>>(scale, seed, pk, M, (u32)p->lo, (u32)p->hi, bcnt.p, acc.p);
        PJ_LAUNCH_CHECK();
        exclusive_scan_u32(bcnt.p, boff.p, nb, ws, s);
        u64 tot = 0;
        PJ_HIP(hipMemcpyAsync(&tot, boff.p + nb, sizeof(u64), hipMemcpyDeviceToHost, s));
        PJ_HIP(hipMemcpyAsync(&wsum, acc.p, sizeof(u64), hipMemcpyDeviceToHost, s));
        PJ_HIP(hipStreamSynchronize(s));
        m = (i64)tot;
        ls.alloc((size_t)std::max<i64>(m, 1));
        ld.alloc((size_t)std::max<i64>(m, 1));
        lw.alloc((size_t)std::max<i64>(m, 1));
        wp_kron_write_k<<<(unsigned)nb, 256, 0, s>>>(scale, seed, pk, M, (u32)p->lo, (u32)p->hi, boff.p, ls.p, ld.p,
                                                     lw.p);
        PJ_LAUNCH_CHECK();
        PJ_HIP(hipStreamSynchronize(s));
    }
    Graph local;  // the block's rows, local ids, global columns, weight-sorted
    local.ctx = &ctx;
    build_graph_from_coo(local, ls, ld, &lw, m, p->nl, false);
    wpart_cut(p.get(), local, 0, M > 0 ? (double)wsum / (double)(2 * M) : 1.0);
    p->symmetric = true;  // both directions of every tuple, same weight
    if (PJ_WP_RELABEL && nb > 0) {  // every vertex's degree: both entries of every tuple
        DevBuf<u32> deg((size_t)p->n);
        PJ_HIP(hipMemsetAsync(deg.p, 0, deg.bytes(), s));
        wp_kron_deg_k<<<(unsigned)nb, 256, 0, s>>>(scale, seed, pk, M, deg.p);
        PJ_LAUNCH_CHECK();
        wpart_relabel(*p, deg);
    }
    return p.release();
}

WPart* wpart_from_graph(Graph& g, int rank, int world) {
    if (!g.weighted) throw Error(PJ_ERR_ARG, "pj_wpart_from_graph: the graph has no weights");
    std::unique_ptr<WPart> p = wpart_geometry(g.ctx, g.n, g.nnz, rank, world);
    const u64 wsum = weight_sum(g.w.p, g.nnz, p->grid(), g.ctx->stream);
    wpart_cut(p.get(), g, p->lo, g.nnz > 0 ? (double)wsum / (double)g.nnz : 1.0);
    p->symmetric = g.symmetric;
    if (PJ_WP_RELABEL && g.n > 0) {
        DevBuf<u32> deg((size_t)g.n);
        wp_deg_row_k<<<grid_for(g.n, 256, p->grid()), 256, 0, g.ctx->stream>>>(g.row_ptr(), g.off64, g.n, deg.p);
        PJ_LAUNCH_CHECK();
        wpart_relabel(*p, deg);
    }
    return p.release();
}

namespace {
// The COO entries whose source lies in [lo, hi), as (source - lo, target, weight) in file
// order, on ctx's stream; returns their count.
i64 wp_filter(Ctx& ctx, const DevBuf<u32>& src, const DevBuf<u32>& dst, const DevBuf<u32>& w, i64 nnz, i64 lo,
              i64 hi, DevBuf<u32>& ls, DevBuf<u32>& ld, DevBuf<u32>& lw) {
    hipStream_t s = ctx.stream;
    const i64 nb = (nnz + 4095) / 4096;
    i64 m = 0;
    if (nb > 0) {
        DevBuf<u32> bcnt((size_t)nb);
        DevBuf<u64> boff((size_t)nb + 1);
        ScanWs ws;
        wp_filter_count_k<<<(unsigned)nb, 256, 0, s>>>(src.p, nnz, (u32)lo, (u32)hi, bcnt.p);
        PJ_LAUNCH_CHECK();
        exclusive_scan_u32(bcnt.p, boff.p, nb, ws, s);
        u64 tot = 0;
        PJ_HIP(hipMemcpyAsync(&tot, boff.p + nb, sizeof(u64), hipMemcpyDeviceToHost, s));
        PJ_HIP(hipStreamSynchronize(s));
        m = (i64)tot;
        ls.alloc((size_t)std::max<i64>(m, 1));
        ld.alloc((size_t)std::max<i64>(m, 1));
        lw.alloc((size_t)std::max<i64>(m, 1));
        wp_filter_write_k<<<(unsigned)nb, 256, 0, s>>>(src.p, dst.p, w.p, nnz, (u32)lo, (u32)hi, boff.p, ls.p, ld.p,
                                                       lw.p);
        PJ_LAUNCH_CHECK();
        PJ_HIP(hipStreamSynchronize(s));
    }
    return m;
}

// every vertex's out-degree from the whole COO (the per-block degree order's keys)
DevBuf<u32> wp_coo_degrees(Ctx& ctx, const DevBuf<u32>& src, i64 nnz, i64 n, unsigned grid) {
    DevBuf<u32> deg;
    if (PJ_WP_RELABEL && n > 0) {
        deg.alloc((size_t)n);
        PJ_HIP(hipMemsetAsync(deg.p, 0, deg.bytes(), ctx.stream));
        if (nnz > 0) {
            wp_deg_coo_k<<<grid_for(nnz, 256, grid), 256, 0, ctx.stream>>>(src.p, nnz, deg.p);
            PJ_LAUNCH_CHECK();
        }
    }
    return deg;
}

// the block's rows from its filtered COO (consumed), then the relabel
void wp_build_block(WPart& p, DevBuf<u32>& ls, DevBuf<u32>& ld, DevBuf<u32>& lw, i64 m, double mean_w,
                    DevBuf<u32>& deg) {
    Graph local;  // the block's rows, local ids, global columns, weight-sorted
    local.ctx = p.ctx;
    build_graph_from_coo(local, ls, ld, &lw, m, p.nl, false);
    wpart_cut(&p, local, 0, mean_w);
    if (deg.p) wpart_relabel(p, deg);
}
}  // namespace

// The rank's block from device COO (consumed): only the block's rows are sorted and
// kept, so a rank holds its share of the graph plus the parsed COO while building.
WPart* wpart_from_coo(Ctx& ctx, DevBuf<u32>& src, DevBuf<u32>& dst, DevBuf<u32>& w, i64 nnz, i64 n, int rank,
                      int world) {
    hipStream_t s = ctx.stream;
    std::unique_ptr<WPart> p = wpart_geometry(&ctx, n, nnz, rank, world);
    const u64 wsum = weight_sum(w.p, nnz, p->grid(), s);
    DevBuf<u32> ls, ld, lw;
    const i64 m = wp_filter(ctx, src, dst, w, nnz, p->lo, p->hi, ls, ld, lw);
    DevBuf<u32> deg = wp_coo_degrees(ctx, src, nnz, n, p->grid());
    src.release();
    dst.release();
    w.release();
    wp_build_block(*p, ls, ld, lw, m, nnz > 0 ? (double)wsum / (double)nnz : 1.0, deg);
    return p.release();
}

// Parse once, scatter (the reference's rank 0 reads and scatters, :313-338, :344-410): the
// device COO on ctxs[0] (consumed) is filtered into every rank's piece there, the pieces and
// the degree keys of the per-block order are copied to the ranks' GPUs, and every rank builds
// its block from its piece alone, the ranks in parallel (one host thread each).
std::vector<WPart*> wparts_from_coo_group(const std::vector<Ctx*>& ctxs, DevBuf<u32>& src, DevBuf<u32>& dst,
                                          DevBuf<u32>& w, i64 nnz, i64 n) {
    const int world = (int)ctxs.size();
    Ctx& c0 = *ctxs[0];
    PJ_HIP(hipSetDevice(c0.device));
    std::vector<std::unique_ptr<WPart>> parts((size_t)world);
    for (int r = 0; r < world; ++r) parts[(size_t)r] = wpart_geometry(ctxs[(size_t)r], n, nnz, r, world);
    const u64 wsum = weight_sum(w.p, nnz, parts[0]->grid(), c0.stream);
    const double mean_w = nnz > 0 ? (double)wsum / (double)nnz : 1.0;
    struct Piece {
        DevBuf<u32> ls, ld, lw, deg;
        i64 m = 0;
    };
    std::vector<Piece> pc((size_t)world);
    DevBuf<u32> deg0 = wp_coo_degrees(c0, src, nnz, n, parts[0]->grid());
    for (int r = 0; r < world; ++r) {
        WPart& p = *parts[(size_t)r];
        Piece& q = pc[(size_t)r];
        PJ_HIP(hipSetDevice(c0.device));
        DevBuf<u32> ls, ld, lw;
        q.m = wp_filter(c0, src, dst, w, nnz, p.lo, p.hi, ls, ld, lw);
        if (p.ctx == &c0) {
            q.ls = std::move(ls);
            q.ld = std::move(ld);
            q.lw = std::move(lw);
            continue;
        }
        PJ_HIP(hipSetDevice(p.ctx->device));
        auto ship = [&](const DevBuf<u32>& from, DevBuf<u32>& to, i64 cnt) {
            to.alloc((size_t)std::max<i64>(cnt, 1));
            if (cnt)
                PJ_HIP(hipMemcpyPeerAsync(to.p, p.ctx->device, from.p, c0.device, sizeof(u32) * (size_t)cnt,
                                          c0.stream));
        };
        ship(ls, q.ls, q.m);
        ship(ld, q.ld, q.m);
        ship(lw, q.lw, q.m);
        if (deg0.p) ship(deg0, q.deg, n);
        PJ_HIP(hipSetDevice(c0.device));
        PJ_HIP(hipStreamSynchronize(c0.stream));
    }
    if (deg0.p) pc[0].deg = std::move(deg0);  // (rank 0's context keeps the original)
    src.release();
    dst.release();
    w.release();
    std::vector<std::exception_ptr> errs((size_t)world);
    std::vector<std::thread> th;
    for (int r = 0; r < world; ++r)
        th.emplace_back([&, r] {
            try {
                WPart& p = *parts[(size_t)r];
                PJ_HIP(hipSetDevice(p.ctx->device));
                Piece& q = pc[(size_t)r];
                wp_build_block(p, q.ls, q.ld, q.lw, q.m, mean_w, q.deg);
            } catch (...) {
                errs[(size_t)r] = std::current_exception();
            }
        });
    for (auto& t : th) t.join();
    for (auto& e : errs)
        if (e) std::rethrow_exception(e);
    std::vector<WPart*> out;
    for (auto& p : parts) out.push_back(p.release());
    return out;
}

void wpart_info(const WPart& p, i64* out) {
    out[0] = p.n;
    out[1] = p.lo;
    out[2] = p.hi;
    out[3] = p.block;
    out[4] = p.nnz_local;
    out[5] = p.world;
    out[6] = p.rank;
    out[7] = p.nnz;
}

// device bytes of this rank: [0] rows; [1] O(block) vertex state, the sent-pair cache
// (2 x block entries) included; [2] the replicated maps the pulls and the tail all-gather
// (member / frontier byte maps: N bytes, 2N for the tail's 16-bit map; the settled map:
// N bits -- the analogue of the BFS pull's replicated visited bitmap); [3] the claim queue
// and the exchange buffers (sized to the largest round's pairs)
void wpart_device_bytes(const WPart& p, i64* out4) {
    out4[0] = (i64)(p.row.bytes() + p.col.bytes() + p.w.bytes());
    if (p.g1)  // (world 1: the single-GPU solver's copy of the rows, its relabeled copy and workspace)
        out4[0] += (i64)(p.g1->row32.bytes() + p.g1->row64.bytes() + p.g1->col.bytes() + p.g1->w.bytes() +
                         p.g1->dist.bytes()) + delta_device_bytes(*p.g1);
    out4[1] = (i64)(p.lsplit.bytes() + p.lsplit_alt.bytes() + p.dist.bytes() + p.fr.bytes() + p.frn.bytes() +
                    p.mb.bytes() + p.lq_v.bytes() + p.lq_b.bytes() + p.lq_e.bytes() + p.stat.bytes() +
                    p.rc.bytes() + p.qctr.bytes() + p.rl_inv.bytes() + p.pl.v.bytes() + p.pl.c.bytes() +
                    p.pl_alt.v.bytes() + p.pl_alt.c.bytes());
    out4[2] = (i64)(p.mmap.bytes() + p.fmap16.bytes() + p.sb.bytes());
    out4[3] = p.exch_bytes + (i64)p.q.bytes();
}

void wpart_heavy_counts(WPart& p, int32_t lo, int32_t hi, i64* out2) {
    hipStream_t s = p.ctx->stream;
    u64 h[3] = {0, 0, 0};
    if (p.nl > 0) {
        u64* acc = p.stat.p + ST_ACC;  // (a temporary buffer here cost a hipFree per band)
        PJ_HIP(hipMemsetAsync(acc, 0, 3 * sizeof(u64), s));
        if (!p.mmap.p) p.mmap.alloc((size_t)p.world * (size_t)p.block);
        wp_heavy_counts_k<<<grid_for(p.block, WB, p.grid()), WB, 0, s>>>(
            p.args(lo, hi), hi, acc, hi - lo <= 255 ? p.mmap.p + (size_t)p.rank * (size_t)p.block : nullptr);
        PJ_LAUNCH_CHECK();
        p.read_acc(h, 3);
    }
    out2[0] = (i64)h[0];
    out2[1] = (i64)h[1];
    p.map16 = false;  // (the member map is the u8 one)
    p.ua_hi = hi;  // (wpart_unsettled(hi) of this band)
    p.ua = (i64)h[2];
    p.ms_lo = hi - lo <= 255 && p.nl > 0 ? lo : INT_MIN;  // (the member slice of this band is written)
}

void wpart_light_counts(WPart& p, int32_t lo, int32_t hi, i64* out2) {
    hipStream_t s = p.ctx->stream;
    u64 h[3] = {0, 0, ~0ull};
    if (p.nl > 0) {
        u64* acc = p.stat.p + ST_ACC;
        PJ_HIP(hipMemsetAsync(acc, 0, 2 * sizeof(u64), s));
        PJ_HIP(hipMemsetAsync(acc + 2, 0xFF, sizeof(u64), s));
        wp_light_counts_k<<<grid_for(p.nl, WB, p.grid()), WB, 0, s>>>(p.args(lo, hi), acc);
        PJ_LAUNCH_CHECK();
        p.read_acc(h, 3);
    }
    out2[0] = (i64)h[0];
    out2[1] = (i64)h[1];
    p.fmin_own = h[2] < (u64)INT_INF ? (i64)h[2] : (i64)INT_INF;
    p.fmin_all = -1;  // (until the engine hands over every rank's minimum)
}

void wpart_frontier_slice(WPart& p, int32_t lo, int32_t hi) {
    p.map16 = hi - lo > 255;  // (the tail's bands: 16-bit offsets; member_map() follows)
    if (p.map16) {
        if (!p.fmap16.p) p.fmap16.alloc((size_t)p.world * (size_t)p.block);
        wp_frontier_slice_k<uint16_t><<<grid_for(p.block, 256, p.grid()), 256, 0, p.ctx->stream>>>(
            p.args(lo, hi), p.fmap16.p + (size_t)p.rank * (size_t)p.block);
    } else {
        if (!p.mmap.p) p.mmap.alloc((size_t)p.world * (size_t)p.block);
        wp_frontier_slice_k<uint8_t><<<grid_for(p.block, 256, p.grid()), 256, 0, p.ctx->stream>>>(
            p.args(lo, hi), p.mmap.p + (size_t)p.rank * (size_t)p.block);
    }
    PJ_LAUNCH_CHECK();
}

// one light round by pull (the counters ST_NF as a push round leaves them)
void wpart_light_pull(WPart& p, int32_t lo, int32_t hi) {
    hipStream_t s = p.ctx->stream;
    p.clear_stat();
    // the frontier-minimum bound (every rank's frontier; the engine's min-all-reduce of the
    // ranks' light-count minima): flo in [lo, hi), else lo
    const int32_t flo = (p.pull_fmin && p.fmin_all > lo && p.fmin_all < hi) ? (int32_t)p.fmin_all : lo;
    if (p.nl > 0 && p.map16) {  // the tail's bands (hubs settled; a list would mostly hold settled rows)
        wp_pull_light_k<uint16_t><<<p.grid(), WB, 0, s>>>(p.args(lo, hi), p.fmap16.p, ~0u, flo);
        PJ_LAUNCH_CHECK();
    } else if (p.nl > 0) {
        WPart::PullLong& L = p.pl;
        if (!L.built) {  // the long-row chunk list of this light threshold: count, then fill
            u64* acc = p.stat.p + ST_ACC;
            PJ_HIP(hipMemsetAsync(acc, 0, sizeof(u64), s));
            wp_plong_count_k<<<grid_for(p.nl, 256, p.grid()), 256, 0, s>>>(p.lsplit.p, p.nl, acc);
            PJ_LAUNCH_CHECK();
            u64 nc = 0;
            p.read_acc(&nc, 1);
            L.v.alloc((size_t)std::max<u64>(nc, 1));
            L.c.alloc((size_t)std::max<u64>(nc, 1));
            PJ_HIP(hipMemsetAsync(acc, 0, sizeof(u64), s));
            if (nc) {
                wp_plong_fill_k<<<grid_for(p.nl, 256, p.grid()), 256, 0, s>>>(p.lsplit.p, p.nl, acc, L.v.p, L.c.p);
                PJ_LAUNCH_CHECK();
            }
            PJ_HIP(hipMemsetAsync(acc, 0, sizeof(u64), s));
            L.n = nc;
            L.built = true;
        }
        const WArgs a = p.args(lo, hi);
        if (L.n) {
            wp_pull_long_k<uint8_t><<<p.grid(), WB, 0, s>>>(a, p.mmap.p, L.v.p, L.c.p, L.n, flo);
            PJ_LAUNCH_CHECK();
        }
        wp_pull_light_k<uint8_t><<<p.grid(), WB, 0, s>>>(a, p.mmap.p, WP_PLMAX, flo);
        PJ_LAUNCH_CHECK();
    }
}

void wpart_member_slice(WPart& p, int32_t lo, int32_t hi) {
    p.map16 = false;
    if (p.ms_lo == lo) {  // written by this band's wp_heavy_counts_k
        p.ms_lo = INT_MIN;
        return;
    }
    if (!p.mmap.p) p.mmap.alloc((size_t)p.world * (size_t)p.block);
    wp_member_slice_k<<<grid_for(p.block, 256, p.grid()), 256, 0, p.ctx->stream>>>(
        p.args(lo, hi), p.mmap.p + (size_t)p.rank * (size_t)p.block);
    PJ_LAUNCH_CHECK();
}

void wpart_heavy_pull(WPart& p, int32_t lo, int32_t hi) {
    hipStream_t s = p.ctx->stream;
    if (p.nl > 0) {
        // the next band's select rides along (wpart_select_async of [hi, nhi) then reads it)
        const int32_t nhi = (int32_t)std::min<i64>((i64)hi + p.delta, INT_INF);
        PJ_HIP(hipMemsetAsync(p.stat.p + ST_MIN, 0xFF, sizeof(u64), s));
        PJ_HIP(hipMemsetAsync(p.stat.p + ST_CNT, 0, sizeof(u64), s));
        wp_pull_heavy_k<<<p.grid(), WB, 0, s>>>(p.args(lo, hi), p.mmap.p, nhi);
        p.fs_lo = hi;
        p.fs_hi = nhi;
        PJ_LAUNCH_CHECK();
    }
    // (no wait: the band's next host step -- the tail count or the select -- waits on the stream)
}

i64 wpart_unsettled(WPart& p, int32_t hi) {
    hipStream_t s = p.ctx->stream;
    if (p.ua_hi == hi) {  // counted by this band's wp_heavy_counts_k
        p.ua_hi = INT_MIN;
        return p.ua;
    }
    u64 h = 0;
    if (p.nl > 0) {
        u64* acc = p.stat.p + ST_ACC;
        PJ_HIP(hipMemsetAsync(acc, 0, sizeof(u64), s));
        wp_unsettled_k<<<grid_for(p.nl, WB, p.grid()), WB, 0, s>>>(p.args(), hi, acc);
        PJ_LAUNCH_CHECK();
        p.read_acc(&h, 1);
    }
    return (i64)h;
}

// the tail's settled map: this rank's words (bit v: dist[v] < lo), enabled for the rest of the solve
static u64* wpart_settled_map(WPart& p) {
    if (!p.sb.p) p.sb.alloc((size_t)p.world * (size_t)p.bw);
    return p.sb.p;
}
static void wpart_settled_slice(WPart& p, int32_t lo) {
    u64* words = wpart_settled_map(p) + (size_t)p.rank * (size_t)p.bw;
    wp_settled_k<<<grid_for(p.bw * 64, 256, p.grid()), 256, 0, p.ctx->stream>>>(p.args(), lo, words);
    PJ_LAUNCH_CHECK();
    p.sb_on = true;
}

// the light prefixes of light threshold delta in p.lsplit: the current buffer, the other
// cached one (swapped in), or computed into the buffer of the older threshold
void wpart_use_delta(WPart& p, int32_t delta) {
    if (delta == p.delta || p.nl <= 0) {
        p.delta = delta;
        return;
    }
    std::swap(p.lsplit, p.lsplit_alt);
    std::swap(p.pl, p.pl_alt);
    std::swap(p.delta, p.delta_alt);
    if (delta == p.delta) return;
    if (!p.lsplit.p) p.lsplit.alloc((size_t)p.nl);
    wp_lsplit_k<<<grid_for(p.nl, 256, p.grid()), 256, 0, p.ctx->stream>>>(p.row.p, p.w.p, p.nl, (u32)delta,
                                                                          p.lsplit.p);
    PJ_LAUNCH_CHECK();
    p.pl.built = false;
    p.delta = delta;
}

// a new light threshold at a band boundary (the tail switch): the light prefixes follow it
void wpart_set_delta(WPart& p, int32_t delta) { wpart_use_delta(p, delta); }

int32_t wpart_begin(WPart& p, i64 source, int32_t delta) {
    hipStream_t s = p.ctx->stream;
    if (delta <= 0) {
        delta = (int32_t)auto_delta((double)p.n, (double)p.nnz, p.mean_w);  // (the single-GPU rule)
    }
    wpart_use_delta(p, delta);
    p.sb_on = false;
    p.ua_hi = INT_MIN;
    p.ms_lo = INT_MIN;
    p.fs_lo = p.fs_hi = INT_MIN;
    if (p.nl > 0) PJ_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(p.dist.p), INT_INF, (size_t)p.nl, s));
    if (p.world > 1) PJ_HIP(hipMemsetAsync(p.rc.p, 0xFF, p.rc.bytes(), s));  // (the sent-pair cache: empty)
    p.pending_pack = false;
    if (source >= 0 && source < p.n) {
        i64 src = source;
        if (p.rl_inv.p && source >= p.lo && source < p.hi) {  // relabeled block: the source's new id
            u32 x = 0;
            PJ_HIP(hipMemcpyAsync(&x, p.rl_inv.p + (source - p.lo), sizeof(u32), hipMemcpyDeviceToHost, s));
            PJ_HIP(hipStreamSynchronize(s));
            src = p.lo + (i64)x;
        }
        wp_seed_k<<<1, 1, 0, s>>>(p.args(), src);
        PJ_LAUNCH_CHECK();
    }
    PJ_HIP(hipStreamSynchronize(s));
    return delta;
}

static void wpart_select_async(WPart& p, int32_t lo, int32_t hi) {
    hipStream_t s = p.ctx->stream;
    if (p.pending_pack) throw Error(PJ_ERR_STATE, "wpart select: the last relax's pairs were not packed");
    if (p.fs_lo == lo && p.fs_hi == hi) {  // selected by the heavy pull that ended the last band
        p.fs_lo = p.fs_hi = INT_MIN;
        return;
    }
    p.fs_lo = p.fs_hi = INT_MIN;
    p.clear_stat();
    PJ_HIP(hipMemsetAsync(p.stat.p + ST_MIN, 0xFF, sizeof(u64), s));
    wp_select_k<<<grid_for(p.bw * 64, WB, p.grid()), WB, 0, s>>>(p.args(lo, hi));
    PJ_LAUNCH_CHECK();
}

void wpart_select(WPart& p, int32_t lo, int32_t hi, i64* out2) {
    wpart_select_async(p, lo, hi);
    p.read_stat();
    out2[0] = (i64)p.hstat[ST_CNT];
    out2[1] = p.hstat[ST_MIN] >= (u64)INT_INF ? (i64)INT_INF : (i64)p.hstat[ST_MIN];
}

// Relax the frontier's light (or the members' heavy) edges; counts[o] = the pairs queued
// for owner o. send != NULL (room for their sum) also packs them (wpart_pack); else the
// caller packs once it has sized its buffer, before the next step.
//
// Overflow: a round whose pairs exceed a queue shard is run again with the queue grown to
// twice the largest shard count seen. Everything the first run did stays valid (owned
// targets lowered and marked, ST_NF counting each new mark once); its lost pairs are
// recovered by relaxing again all of the band's members (light) or again the members'
// heavy edges, with the sent-pair cache cleared so that no pair is skipped for having
// been "sent" by the run whose queue was dropped. Redundant work, but only until the
// queue has grown: it keeps its size.
static void wpart_relax_impl(WPart& p, int light, int32_t lo, int32_t hi, i64* counts,
                             DevBuf<u64>* pre);
void wpart_relax(WPart& p, int light, int32_t lo, int32_t hi, i64* counts) {
    wpart_relax_impl(p, light, lo, hi, counts, nullptr);
}
// pre != NULL (the engine's send buffer): grown to the queue's capacity and packed right
// behind the count kernel, before the one host wait of the step (no second wait to pack)
static void wpart_relax_impl(WPart& p, int light, int32_t lo, int32_t hi, i64* counts, DevBuf<u64>* pre) {
    hipStream_t s = p.ctx->stream;
    if (p.pending_pack) throw Error(PJ_ERR_STATE, "wpart relax: the last relax's pairs were not packed");
    p.clear_stat();
    for (int attempt = 0;; ++attempt) {
        if (p.world > 1) PJ_HIP(hipMemsetAsync(p.qctr.p, 0, p.qctr.bytes(), s));
        const WArgs a = p.args(lo, hi);
        if (light) wp_relax_k<true><<<p.grid(), WB, 0, s>>>(a);
        else wp_relax_k<false><<<p.grid(), WB, 0, s>>>(a);
        PJ_LAUNCH_CHECK();
        if (light) wp_long_k<true><<<p.grid(), WB, 0, s>>>(a);
        else wp_long_k<false><<<p.grid(), WB, 0, s>>>(a);
        PJ_LAUNCH_CHECK();
        if (p.world < 2) break;  // (world 1 sends nothing: no host wait here)
        if (p.world == 2 && pre) {  // count, pack and publish in one launch
            pre->ensure((size_t)p.qcap());
            const u64 q = p.hstat.next();
            wp_qcopy2_k<<<p.qgrid(), WB, 0, s>>>(a, pre->p, p.rank, p.hstat.dev, p.hstat.seq_dev, q);
            PJ_LAUNCH_CHECK();
            p.hstat.wait(q, s);
        } else {
            if (p.world == 2) wp_qsum2_k<<<1, WAVE, 0, s>>>(a, 1 - p.rank);
            else wp_qcount_k<<<p.qgrid(), WB, 0, s>>>(a, p.world);
            PJ_LAUNCH_CHECK();
            if (pre) {  // (pairs past a shard's capacity are not packed: an overflow reruns anyway)
                pre->ensure((size_t)p.qcap());
                wp_qpack_k<<<p.qgrid(), WB, 0, s>>>(a, p.world, pre->p);
                PJ_LAUNCH_CHECK();
            }
            p.read_stat();
        }
        if (p.hstat[ST_QSP] <= p.qsp) break;
        if (attempt > 8) throw Error(PJ_ERR_HIP, "wpart relax: the claim queue keeps overflowing (internal error)");
        // shards at twice the round's average, the spill at the round's pairs (a rerun tries more
        // pairs than the run it repeats: it may overflow once more)
        const u64 tot = p.hstat[ST_QTOT];
        wpart_queue(p, std::max<u64>(p.qsh, 2 * (tot / WQ_S) + 16), std::max<u64>(p.qsp, tot + 4096));
        PJ_HIP(hipMemsetAsync(p.rc.p, 0xFF, p.rc.bytes(), s));
        if (light)  // (the run consumed the frontier into the members: relax all of them again)
            PJ_HIP(hipMemcpyAsync(p.fr.p, p.mb.p, p.fr.bytes(), hipMemcpyDeviceToDevice, s));
        // every counter but the marks of the first run (ST_NF)
        PJ_HIP(hipMemsetAsync(p.stat.p, 0, sizeof(u64) * ST_NF, s));
        PJ_HIP(hipMemsetAsync(p.stat.p + ST_NF + 1, 0, sizeof(u64) * (ST_N - ST_NF - 1), s));
    }
    for (int o = 0; o < p.world; ++o) counts[o] = p.world > 1 ? (i64)p.hstat[o] : 0;
    p.pending_pack = p.world > 1 && !pre;
}

// The queued pairs (id | cand << 32), owner-major, into send (room for the sum of the
// last relax's counts).
void wpart_pack(WPart& p, u64* send) {
    if (p.world < 2) return;
    hipStream_t s = p.ctx->stream;
    if (p.world == 2) wp_qcopy2_k<<<p.qgrid(), WB, 0, s>>>(p.args(), send, p.rank, nullptr, nullptr, 0);
    else wp_qpack_k<<<p.qgrid(), WB, 0, s>>>(p.args(), p.world, send);
    PJ_LAUNCH_CHECK();
    PJ_HIP(hipStreamSynchronize(s));
    p.pending_pack = false;
}

void wpart_apply(WPart& p, const u64* recv, i64 nr, int light, int32_t lo, int32_t hi) {
    hipStream_t s = p.ctx->stream;
    if (p.pending_pack) throw Error(PJ_ERR_STATE, "wpart apply: the last relax's pairs were not packed");
    if (nr > 0) {
        wp_apply_k<<<grid_for(nr, WB, p.grid()), WB, 0, s>>>(p.args(lo, hi), recv, nr, light);
        PJ_LAUNCH_CHECK();
    }
    // (no wait: the next step that needs the host -- end_round's counters or the
    // transport's row gather -- waits for the stream after this kernel)
}

// The round's new frontier becomes current; returns its size on this rank (the
// marks counted by the round's relax and apply: each vertex once, by the
// atomicOr's old bit). The round's kernels cleared fr's words as they consumed them,
// so the two bitmaps trade places with no kernel (wp_swap_k copied and cleared them).
static void wpart_end_round_async(WPart& p) {
    if (p.pending_pack) throw Error(PJ_ERR_STATE, "wpart end_round: the last relax's pairs were not packed");
    std::swap(p.fr, p.frn);
}

i64 wpart_end_round(WPart& p) {
    wpart_end_round_async(p);
    p.read_stat();
    return (i64)p.hstat[ST_NF];
}

void wpart_reach(WPart& p, i64* out2) {
    p.clear_stat();
    wp_reach_k<<<grid_for(std::max<i64>(p.nl, 1), WB, p.grid()), WB, 0, p.ctx->stream>>>(p.args());
    PJ_LAUNCH_CHECK();
    p.read_stat();
    out2[0] = (i64)p.hstat[ST_REACH];
    out2[1] = (i64)p.hstat[ST_REACH + 1];
}

void wpart_copy_dist(WPart& p, int32_t* host) {
    if (p.nl <= 0) return;
    if (p.rl_inv.p) {  // back to input ids
        DevBuf<int32_t> o((size_t)p.nl);
        wp_unlabel_k<<<grid_for(p.nl, 256, p.grid()), 256, 0, p.ctx->stream>>>(p.dist.p, p.rl_inv.p, p.nl, o.p);
        PJ_LAUNCH_CHECK();
        PJ_HIP(hipMemcpyAsync(host, o.p, sizeof(int32_t) * (size_t)p.nl, hipMemcpyDeviceToHost, p.ctx->stream));
        PJ_HIP(hipStreamSynchronize(p.ctx->stream));
        return;
    }
    PJ_HIP(hipMemcpy(host, p.dist.p, sizeof(int32_t) * (size_t)p.nl, hipMemcpyDeviceToHost));
}

// ---- world 1: the single-GPU solver --------------------------------------------------
// A one-rank partition holds the whole graph, and its rows (in the block's degree order,
// columns mapped through the same order) are a complete weight-sorted CSR. Its solve is
// therefore delta.hip's v2 -- the single-GPU path's band and round kernels -- on a Graph over
// copies of those rows (built at the first solve: 2 x 4 bytes per entry), and the distances
// come back into p.dist, so the step API, the gather and the reach pass see them as the band
// loop's. Option "single_gpu" 0 keeps the band loop of engine.cpp over this file's kernels
// (what every rank runs at world > 1).
__global__ void wp_narrow_k(const u64* __restrict__ in, i64 m, u32* __restrict__ out) {
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (i64)gridDim.x * blockDim.x) out[i] = (u32)in[i];
}

void wpart_solve_single(WPart& p, i64 source, int32_t delta, pj_part_stats* st) {
    const auto t0 = std::chrono::steady_clock::now();
    hipStream_t s = p.ctx->stream;
    if (!p.g1) {
        auto g = std::make_unique<Graph>();
        g->ctx = p.ctx;
        g->n = p.n;
        g->nnz = p.nnz_local;
        g->weighted = true;
        g->symmetric = p.symmetric;
        g->off64 = (u64)g->nnz > 0xFFFFFFFFull;
        const size_t nr = (size_t)p.n + 1, m = (size_t)std::max<i64>(g->nnz, 1);
        if (g->off64) {
            g->row64.alloc(nr);
            PJ_HIP(hipMemcpyAsync(g->row64.p, p.row.p, 8 * nr, hipMemcpyDeviceToDevice, s));
        } else {
            g->row32.alloc(nr);
            wp_narrow_k<<<grid_for((i64)nr, 256, p.grid()), 256, 0, s>>>(p.row.p, (i64)nr, g->row32.p);
            PJ_LAUNCH_CHECK();
        }
        g->col.alloc(m);
        g->w.alloc(m);
        if (g->nnz) {
            PJ_HIP(hipMemcpyAsync(g->col.p, p.col.p, 4 * (size_t)g->nnz, hipMemcpyDeviceToDevice, s));
            PJ_HIP(hipMemcpyAsync(g->w.p, p.w.p, 4 * (size_t)g->nnz, hipMemcpyDeviceToDevice, s));
        }
        PJ_HIP(hipStreamSynchronize(s));
        p.g1 = std::move(g);
    }
    Graph& g = *p.g1;
    g.delta = delta > 0 ? (double)delta : 0.0;
    i64 src = source;
    if (source >= 0 && source < p.n && p.rl_inv.p) {  // the block's degree order: the source's new id
        u32 x = 0;
        PJ_HIP(hipMemcpyAsync(&x, p.rl_inv.p + source, sizeof(u32), hipMemcpyDeviceToHost, s));
        PJ_HIP(hipStreamSynchronize(s));
        src = (i64)x;
    }
    delta_solve(g, src);
    delta_materialize(g);  // (g.dist in the block's ids, complete on return)
    if (p.nl) PJ_HIP(hipMemcpyAsync(p.dist.p, g.dist.p, 4 * (size_t)p.nl, hipMemcpyDeviceToDevice, s));
    i64 rc[2] = {0, 0};
    wpart_reach(p, rc);  // (synchronizes the stream)
    if (st) {
        *st = pj_part_stats{};
        st->solve_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        st->levels = st->bands = g.stats.levels;
        st->rounds = g.stats.relax_rounds;
        st->td_levels = g.stats.td_levels;
        st->bu_levels = g.stats.bu_levels;
        st->reached = rc[0];
        st->reached_edges = rc[1];
        st->delta = delta > 0 ? delta : (int32_t)auto_delta((double)g.n, (double)g.nnz, g.mean_weight);
    }
}
bool wpart_single(const WPart& p) { return p.world == 1 && p.single_gpu; }
int& wpart_single_gpu(WPart& p) { return p.single_gpu; }
int& wpart_pull_fmin(WPart& p) { return p.pull_fmin; }
int& wpart_grid_per_cu(WPart& p) { return p.gpc; }

// ------------------------------------------------------------ engine view ---
namespace {

// The exchange buffers follow the traffic: relax leaves the improved remote targets in
// `touched` and their per-owner counts on the host; exchange_buffers grows send / recv
// to the largest round seen so far and packs.
struct WPartGpuSteps final : DeltaSteps {
    WPart& p;
    DevBuf<u64> send_b, recv_b;
    explicit WPartGpuSteps(WPart& part) : p(part) {
        n = p.n;
        rank = p.rank;
        world = p.world;
        send_b.alloc(1);
        recv_b.alloc(1);
        send = send_b.p;
        recv = recv_b.p;
    }
    void exchange_buffers(i64 nsend, i64 nrecv) override {
        (void)nsend;  // (relax packed the pairs into send_b already)
        if ((size_t)nrecv > recv_b.n) {
            recv_b.ensure((size_t)nrecv + (size_t)nrecv / 4);
            recv = recv_b.p;
        }
        p.exch_bytes = (i64)(send_b.bytes() + recv_b.bytes());
    }
    hipStream_t stream() override { return p.ctx->stream; }
    int32_t begin(i64 source, int32_t delta) override { return wpart_begin(p, source, delta); }
    void select(int32_t lo, int32_t hi, i64* out2) override { wpart_select(p, lo, hi, out2); }
    void relax(int light, int32_t lo, int32_t hi, i64* counts) override {
        wpart_relax_impl(p, light, lo, hi, counts, p.world > 1 ? &send_b : nullptr);
        send = send_b.p;
    }
    void apply(i64 nr, int light, int32_t lo, int32_t hi) override { wpart_apply(p, recv_b.p, nr, light, lo, hi); }
    i64 end_round() override { return wpart_end_round(p); }
    void reach(i64* out2) override { wpart_reach(p, out2); }
    // device rows: [ST_MIN, ST_CNT] and ST_NF of the stat block
    const i64* select_dev() override { return reinterpret_cast<const i64*>(p.stat.p + ST_MIN); }
    const i64* nf_dev() override { return reinterpret_cast<const i64*>(p.stat.p + ST_NF); }
    void select_async(int32_t lo, int32_t hi) override { wpart_select_async(p, lo, hi); }
    void end_round_async() override { wpart_end_round_async(p); }
    double tail_frac() override { return p.tail[0]; }
    int32_t tail_delta(int32_t delta) override {
        return (int32_t)std::min(65536.0, std::max((double)delta, std::round(p.tail[1] * delta)));
    }
    i64 unsettled_edges(int32_t hi) override { return wpart_unsettled(p, hi); }
    i64 local_edges() override { return p.nnz_local; }
    void set_delta(int32_t delta) override { wpart_set_delta(p, delta); }
    void* settled_map() override { return wpart_settled_map(p); }
    size_t settled_bytes() override { return (size_t)p.bw * sizeof(u64); }
    void settled_slice(int32_t lo) override { wpart_settled_slice(p, lo); }
    double pull_factor() override { return p.symmetric ? p.pull_factor : 0.0; }  // (0: this rank vetoes)
    void heavy_counts(int32_t lo, int32_t hi, i64* out2) override { wpart_heavy_counts(p, lo, hi, out2); }
    void member_slice(int32_t lo, int32_t hi) override { wpart_member_slice(p, lo, hi); }
    void* member_map() override { return p.map16 ? (void*)p.fmap16.p : (void*)p.mmap.p; }
    size_t member_bytes() override { return (size_t)p.block * (p.map16 ? 2 : 1); }
    void heavy_pull(int32_t lo, int32_t hi) override { wpart_heavy_pull(p, lo, hi); }
    double light_pull_factor() override { return p.symmetric ? p.light_pull : 0.0; }
    double tail_light_pull_factor() override { return p.symmetric ? p.tail_light_pull : 0.0; }
    int32_t pull_map_width() override { return 65534; }
    void light_counts(int32_t lo, int32_t hi, i64* out2) override { wpart_light_counts(p, lo, hi, out2); }
    i64 frontier_min() override { return p.fmin_own; }
    void set_frontier_min(i64 m) override { p.fmin_all = m; }
    void frontier_slice(int32_t lo, int32_t hi) override { wpart_frontier_slice(p, lo, hi); }
    void light_pull(int32_t lo, int32_t hi) override { wpart_light_pull(p, lo, hi); }
};

}  // namespace

const Ctx& wpart_ctx(const WPart& p) { return *p.ctx; }
int wpart_world(const WPart& p) { return p.world; }
bool wpart_pending(const WPart& p) { return p.pending_pack; }
// option "queue_shard": the claim queue's shard capacity in pairs from now on (it grows again
// when a round overflows it; tests use small values to run the overflow path)
void wpart_set_queue_shard(WPart& p, i64 pairs) {
    p.qsh_min = pairs;
    if (p.world > 1) {
        p.qsh = p.qsp = 0;
        wpart_queue(p, (u64)pairs, (u64)pairs);
        PJ_HIP(hipStreamSynchronize(p.ctx->stream));
    }
}

double* wpart_tail_params(WPart& p) { return p.tail; }
double& wpart_pull_factor(WPart& p) { return p.pull_factor; }
double& wpart_light_pull(WPart& p) { return p.light_pull; }
double& wpart_tail_light_pull(WPart& p) { return p.tail_light_pull; }

DeltaSteps& wpart_steps(WPart& p) {
    if (!p.steps) p.steps.reset(new WPartGpuSteps(p));
    return *p.steps;
}

void wpart_gather_dist(WPart& p, Comm& comm, int32_t* out) {
    hipStream_t s = p.ctx->stream;
    DevBuf<int32_t> own((size_t)p.block), all((size_t)p.world * (size_t)p.block);
    PJ_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(own.p), INT_INF, (size_t)p.block, s));
    if (p.nl && p.rl_inv.p) {  // relabeled block: back to input ids
        wp_unlabel_k<<<grid_for(p.nl, 256, p.grid()), 256, 0, s>>>(p.dist.p, p.rl_inv.p, p.nl, own.p);
        PJ_LAUNCH_CHECK();
    } else if (p.nl) {
        PJ_HIP(hipMemcpyAsync(own.p, p.dist.p, sizeof(int32_t) * (size_t)p.nl, hipMemcpyDeviceToDevice, s));
    }
    comm.allgather(own.p, all.p, sizeof(int32_t) * (size_t)p.block, s);
    if (out && p.n) PJ_HIP(hipMemcpyAsync(out, all.p, sizeof(int32_t) * (size_t)p.n, hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
}

}  // namespace pj
