// delta.hip — weighted SSSP: delta-stepping with light/heavy edges and
// in-workgroup recursion for the near phase.
//
// Generalises the reference's label-correcting relaxation (extract_local_pq
// :226-278, apply loop :557-573) to integer weights >= 0, keeping its output
// contract: candidates >= INT_INF are discarded and the
// result is the true distance when it is < INT_INF. The reference settles one
// vertex per heap pop; here a whole distance band [lo, hi = lo + delta) is
// settled at once (Meyer & Sanders' delta-stepping). Rows are sorted by weight
// (graph.hip), so the light edges (w < delta) of v are the prefix
// row[v] .. row[v] + lsplit[v] and the heavy ones the rest of the row.
//
// Per band:
//   select(DIST) : one streaming pass over dist lists the band's members
//                  (lo <= dist < hi) with their light and heavy edge ranges and
//                  yields min{dist >= lo}, so an empty band jumps straight to the
//                  next occupied one. No far pile is kept: far vertices are simply
//                  those with dist >= hi.
//   light pass   : edge-balanced (lb.h) over the members' light edges, atomicMin
//                  on dist. A vertex lowered below hi joins the band: the
//                  workgroup that lowered it pushes it on an LDS worklist and
//                  relaxes its whole row itself, recursively, before it exits, so
//                  the band's near phase is ONE launch instead of one launch per
//                  Bellman-Ford round. Worklist overflow and rows longer than
//                  LOCAL_MAX go to the `chg` bitmap instead, and select(BITS)
//                  turns that into a follow-up round (rare).
//   heavy pass   : edge-balanced over the members' heavy edges; their targets
//                  land at >= hi, so nothing joins the band.
// Frontier lists are built without atomics: pass 1 counts per wave (64 bitmap
// words each), a one-block scan turns the counts into offsets, pass 2 writes the
// entries in vertex order. The host reads the band totals from mapped memory
// once per band (the analogue of the reference's termination allreduce,
// :579-593).
#include <chrono>
#include <cmath>
#include <cstdio>

#include "lb.h"

namespace pj {

namespace {

#ifndef PJ_D_IPT
#define PJ_D_IPT 4
#endif
#ifndef PJ_D_SETTLED
#define PJ_D_SETTLED 0
#endif
#ifndef PJ_D_STAGE_IB
#define PJ_D_STAGE_IB 0
#endif
constexpr int DB = 256;             // relax workgroup
constexpr int D_IPT = PJ_D_IPT;
constexpr int D_TILE = DB * D_IPT;  // edges per relax tile
#ifndef PJ_WL_CAP
#define PJ_WL_CAP 2048
#endif
#ifndef PJ_LOCAL_BUDGET
#define PJ_LOCAL_BUDGET 512
#endif
constexpr int WL_CAP = PJ_WL_CAP;   // LDS worklist of a relax workgroup
constexpr u32 LOCAL_BUDGET = PJ_LOCAL_BUDGET;  // worklist vertices a workgroup relaxes itself
constexpr int WL_BATCH = DB;        // worklist entries expanded per step
constexpr u64 LOCAL_MAX = 4096;     // longest row a workgroup relaxes alone
constexpr int SB = 256;             // select workgroup
constexpr int SNW = SB / WAVE;
constexpr int WPW = 64;             // bitmap words per select wave (one per lane in pass 2)
constexpr int SU = 8;               // words whose loads a select wave issues together
#ifndef PJ_SCAN_T
#define PJ_SCAN_T 1024
#endif
#ifndef PJ_SCAN_HOSTCOPY
#define PJ_SCAN_HOSTCOPY 0
#endif
constexpr int SCAN_T = PJ_SCAN_T;   // threads of the one-block scan

// DIST_L / DIST_H: band members (lo <= dist < hi) with their light / heavy edges;
// BITS: the deferred vertices of `chg` with their light edges.
enum SelMode : int { SEL_DIST_L = 0, SEL_BITS = 1, SEL_DIST_H = 2 };

// Totals of one selection, written by sel_scan_k (device + mapped host copy).
struct DTot {
    u64 nl, ml;    // light list: entries with light edges, their light edges (BITS: whole rows)
    u64 nh, mh;    // heavy list: entries with heavy edges, their heavy edges (BITS: none)
    u64 members;   // DIST: vertices with lo <= dist < hi
    u64 minv;      // DIST: min{dist : lo <= dist < INT_INF} (INT_INF if none)
    u64 overflow;  // a relax since the previous selection deferred vertices to `chg`
};

struct SelArgs {
    i64 n, nwords;
    i64 nwaves;  // select waves (WPW words each)
    int32_t lo, hi;
    const int32_t* dist;
    const u32* lsplit;
    u64* chg;   // vertices deferred by a relax workgroup (worklist overflow / long rows)
    u64* settled;  // DIST_L selections write it: bit v = dist[v] < lo (final, never improved again)
    u64* sel;   // the frontier being built
    u64* part;  // [6][nwaves]: light count/edges, heavy count/edges, members, min per wave
    u64* boff;  // [4][nwaves]: exclusive light count/edges, heavy count/edges per wave
    // two frontier lists (every entry has >= 1 edge in its range, as lb.h requires)
    u32 *qvl, *qvh;
    u64 *qbl, *qbh;  // range begin: row[v] / row[v] + lsplit[v]
    u64 *qol, *qoh;  // [n + 1] exclusive edge offsets
    u32* flag;  // set by relax workgroups that wrote `chg`
    DTot* tot;
    DTot* host;  // mapped pinned copy of *tot
};

// Light / heavy edge counts of v for the list MODE builds.
template <typename Off, int MODE>
__device__ __forceinline__ void edge_split(const SelArgs& a, const Off* __restrict__ row, i64 v, u64& lc,
                                           u64& hc, u64& hskip) {
    if (MODE == SEL_DIST_H) {
        hskip = a.lsplit[v];  // the heavy range starts after the light prefix
        lc = 0;
        hc = (u64)(row[v + 1] - row[v]) - hskip;
    } else {
        lc = a.lsplit[v];
        hc = 0;
        hskip = 0;
    }
}

// Pass 1: each wave classifies its WPW bitmap words (lane = vertex of a word,
// SU words' loads in flight at once), writes the `sel` words and publishes
// (count, light edges, heavy edges, members, min) for the wave.
template <typename Off, int MODE>
__global__ __launch_bounds__(SB) void sel_count_k(SelArgs a, const Off* __restrict__ row) {
    const int lane = lane_id();
    const i64 wave = (i64)blockIdx.x * SNW + wave_id();
    if (wave >= a.nwaves) return;
    const i64 wb = wave * WPW;
    u64 cl = 0, chh = 0, el = 0, eh = 0, members = 0;
    long long mn = INT_INF;
    for (int k0 = 0; k0 < WPW; k0 += SU) {
        bool s[SU];
        if (MODE != SEL_BITS) {
            int32_t d[SU];
#pragma unroll
            for (int k = 0; k < SU; ++k) {
                const i64 v = ((wb + k0 + k) << 6) + lane;
                d[k] = v < a.n ? a.dist[v] : INT_INF;
            }
#pragma unroll
            for (int k = 0; k < SU; ++k) {
                s[k] = d[k] >= a.lo && d[k] < a.hi;
                if (d[k] >= a.lo && d[k] < mn) mn = d[k];
            }
            if (MODE == SEL_DIST_L) {
#pragma unroll
                for (int k = 0; k < SU; ++k) {
                    const u64 fin = __ballot(d[k] < a.lo);
                    const i64 wi = wb + k0 + k;
                    if (lane == 0 && wi < a.nwords) a.settled[wi] = fin;
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < SU; ++k) {
                const i64 wi = wb + k0 + k;
                const u64 word = wi < a.nwords ? a.chg[wi] : 0ull;  // wave-uniform
                s[k] = (word >> lane) & 1ull;
                if (word && lane == 0) a.chg[wi] = 0;
            }
        }
        u64 lc[SU], hc[SU];
#pragma unroll
        for (int k = 0; k < SU; ++k) {
            u64 skip = 0;
            lc[k] = hc[k] = 0;
            if (s[k]) edge_split<Off, MODE>(a, row, ((wb + k0 + k) << 6) + lane, lc[k], hc[k], skip);
        }
#pragma unroll
        for (int k = 0; k < SU; ++k) {
            const i64 wi = wb + k0 + k;
            if (MODE != SEL_BITS) members += __popcll(__ballot(s[k]));
            const u64 sb = __ballot(lc[k] + hc[k] > 0);
            cl += __popcll(__ballot(lc[k] > 0));
            chh += __popcll(__ballot(hc[k] > 0));
            el += lc[k];
            eh += hc[k];
            if (lane == 0 && wi < a.nwords) a.sel[wi] = sb;
        }
    }
    el = wave_sum(el);
    eh = wave_sum(eh);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const long long y = __shfl_xor(mn, off, 64);
        mn = y < mn ? y : mn;
    }
    if (lane == 0) {
        const i64 nw = a.nwaves;
        a.part[wave] = cl;
        a.part[nw + wave] = el;
        a.part[2 * nw + wave] = chh;
        a.part[3 * nw + wave] = eh;
        a.part[4 * nw + wave] = members;
        a.part[5 * nw + wave] = (u64)mn;
    }
}

// One block: exclusive scans of the per-wave partials, the totals, and the
// relax overflow flag. Thread t owns SPT consecutive partials of each pass, so
// all of its loads are issued before the block scan (one barrier pair per pass).
constexpr int SPT = 8;
__global__ __launch_bounds__(SCAN_T) void sel_scan_k(SelArgs a) {
    __shared__ u64 lds[4][SCAN_T / WAVE];
    const i64 nw = a.nwaves;
    const int lane = lane_id(), wid = wave_id();
    u64 run[4] = {0, 0, 0, 0}, m = 0, mi = INT_INF;
    for (i64 base = 0; base < nw; base += (i64)SCAN_T * SPT) {
        const i64 i0 = base + (i64)threadIdx.x * SPT;
        u64 x[4][SPT], sum[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < SPT; ++k) {
            const i64 i = i0 + k;
            const bool ok = i < nw;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                x[j][k] = ok ? a.part[j * nw + i] : 0;
                sum[j] += x[j][k];
            }
            if (ok) {
                m += a.part[4 * nw + i];
                const u64 y = a.part[5 * nw + i];
                mi = y < mi ? y : mi;
            }
        }
        u64 inc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            inc[j] = wave_incl_scan(sum[j]);
            if (lane == 63) lds[j][wid] = inc[j];
        }
        __syncthreads();
        u64 wp[4] = {0, 0, 0, 0}, tot[4] = {0, 0, 0, 0};
#pragma unroll 2
        for (int w = 0; w < SCAN_T / WAVE; ++w) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const u64 v = lds[j][w];
                wp[j] += w < wid ? v : 0;
                tot[j] += v;
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            u64 o = run[j] + wp[j] + inc[j] - sum[j];
#pragma unroll
            for (int k = 0; k < SPT; ++k) {
                if (i0 + k < nw) a.boff[j * nw + i0 + k] = o;
                o += x[j][k];
            }
            run[j] += tot[j];
        }
        __syncthreads();
    }
    m = block_sum<SCAN_T / WAVE>(m, lds[0]);
    mi = ~wave_max(~mi);  // wave min via max of complements
    if (lane_id() == 0) lds[1][wave_id()] = mi;
    __syncthreads();
    if (threadIdx.x == 0) {
        u64 y = INT_INF;
        for (int w = 0; w < SCAN_T / WAVE; ++w) y = lds[1][w] < y ? lds[1][w] : y;
        const u64 ov = *a.flag;
        *a.flag = 0;
        DTot t{run[0], run[1], run[2], run[3], m, y, ov};
        *a.tot = t;
        if (!PJ_SCAN_HOSTCOPY) {
            a.host->nl = t.nl;
            a.host->ml = t.ml;
            a.host->nh = t.nh;
            a.host->mh = t.mh;
            a.host->members = t.members;
            a.host->minv = t.minv;
            a.host->overflow = t.overflow;
        }
        a.qol[t.nl] = t.ml;
        a.qoh[t.nh] = t.mh;
    }
}

// Pass 2: each wave writes the entries of its WPW `sel` words in vertex order at
// its offsets (lane = word to find the non-empty words, then lane = vertex),
// and clears the words.
template <typename Off, int MODE>
__global__ __launch_bounds__(SB) void sel_write_k(SelArgs a, const Off* __restrict__ row) {
    const int lane = lane_id();
    const i64 wave = (i64)blockIdx.x * SNW + wave_id();
    if (wave >= a.nwaves) return;
    const i64 nw = a.nwaves;
    const i64 wb = wave * WPW;
    const i64 my = wb + lane;
    const u64 myword = my < a.nwords ? a.sel[my] : 0ull;
    if (myword) a.sel[my] = 0;
    u64 nz = __ballot(myword != 0);
    u64 pl = a.boff[wave], el = a.boff[nw + wave], ph = a.boff[2 * nw + wave], eh = a.boff[3 * nw + wave];
    while (nz) {
        int kw[SU];
        u64 word[SU];
#pragma unroll
        for (int k = 0; k < SU; ++k) {
            kw[k] = nz ? __ffsll((long long)nz) - 1 : -1;
            if (nz) nz &= nz - 1;
            word[k] = kw[k] >= 0 ? __shfl(myword, kw[k], 64) : 0ull;
        }
        u64 lc[SU], hc[SU], b[SU], hb[SU];
#pragma unroll
        for (int k = 0; k < SU; ++k) {
            lc[k] = hc[k] = b[k] = hb[k] = 0;
            if ((word[k] >> lane) & 1ull) {
                const i64 v = ((wb + kw[k]) << 6) + lane;
                u64 skip = 0;
                b[k] = (u64)row[v];
                edge_split<Off, MODE>(a, row, v, lc[k], hc[k], skip);
                hb[k] = b[k] + skip;
            }
        }
#pragma unroll
        for (int k = 0; k < SU; ++k) {
            if (!word[k]) continue;  // wave-uniform
            const u32 v = (u32)(((wb + kw[k]) << 6) + lane);
            const u64 ml = __ballot(lc[k] > 0), mh = __ballot(hc[k] > 0);
            const u64 il = wave_incl_scan(lc[k]);
            const u64 ih = wave_incl_scan(hc[k]);
            if (lc[k] > 0) {
                const u64 slot = pl + (u64)__popcll(ml & lanemask_lt());
                a.qvl[slot] = v;
                a.qbl[slot] = b[k];
                a.qol[slot] = el + il - lc[k];
            }
            if (hc[k] > 0) {
                const u64 slot = ph + (u64)__popcll(mh & lanemask_lt());
                a.qvh[slot] = v;
                a.qbh[slot] = hb[k];
                a.qoh[slot] = eh + ih - hc[k];
            }
            pl += __popcll(ml);
            ph += __popcll(mh);
            el += __shfl(il, 63, 64);
            eh += __shfl(ih, 63, 64);
        }
    }
}

struct Wl {
    u32 n;  // entries pushed (may exceed WL_CAP: the excess went to chg)
    u32 v[WL_CAP];
    int32_t bdu[WL_BATCH];
    u64 bbeg[WL_BATCH];
    u64 boff[WL_BATCH + 1];
    u64 scan[DB / WAVE];
};

__device__ __forceinline__ void defer_vertex(u32 v, u64* __restrict__ chg, u32* __restrict__ flag) {
    atomicOr(chg + (v >> 6), 1ull << (v & 63));
    *flag = 1u;
}

// Push the lanes' newly in-band vertices on the workgroup's worklist.
__device__ __forceinline__ void wl_push(bool p, u32 v, Wl& wl, u64* __restrict__ chg, u32* __restrict__ flag) {
    const u64 m = __ballot(p);
    if (!m) return;
    const int leader = __ffsll((long long)m) - 1;
    u32 base = 0;
    if (lane_id() == leader) base = atomicAdd(&wl.n, (u32)__popcll(m));
    base = __shfl(base, leader, 64);
    if (p) {
        const u32 slot = base + (u32)__popcll(m & lanemask_lt());
        if (slot < WL_CAP) wl.v[slot] = v;
        else defer_vertex(v, chg, flag);
    }
}

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

// One edge: relax u -> col[idx]; true if the target was lowered into the band.
__device__ __forceinline__ bool relax_edge(u64 idx, int32_t du, const u32* __restrict__ col,
                                           const u32* __restrict__ wt, int32_t* __restrict__ dist, int32_t hi,
                                           const u64* __restrict__ settled, u32& v) {
    v = col[idx];
    const long long nd = (long long)du + (long long)wt[idx];
    // a target settled in an earlier band cannot improve: skip its dist probe (the
    // settled bitmap is 1/32 of dist and mostly L2-resident; dist lines are not)
    if (PJ_D_SETTLED && ((settled[v >> 6] >> (v & 63)) & 1ull)) return false;
    if (nd < INT_INF && (int32_t)nd < dist_now(dist + v)) {
        const int32_t old = atomicMin(dist + v, (int32_t)nd);
        return (int32_t)nd < old && (int32_t)nd < hi;
    }
    return false;
}

// Relax the edges [ib[i], ib[i] + deg_i) of the frontier, edge-balanced.
// LIGHT: targets lowered below hi are relaxed (whole rows) by this workgroup
// before it exits; HEAVY targets cannot land below hi.
template <typename Off, bool LIGHT>
__global__ __launch_bounds__(DB) void d_relax_k(const u32* __restrict__ iv, const u64* __restrict__ ib,
                                                const u64* __restrict__ io, const DTot* __restrict__ tot,
                                                const Off* __restrict__ row, const u32* __restrict__ lsplit,
                                                const u32* __restrict__ col, const u32* __restrict__ wt,
                                                int32_t* __restrict__ dist, int32_t hi, u64* __restrict__ chg,
                                                u32* __restrict__ flag, const u64* __restrict__ settled) {
    __shared__ LbShared<D_TILE> sh;
    __shared__ int32_t s_du[D_TILE];
    __shared__ u64 s_ib[PJ_D_STAGE_IB ? D_TILE : 1];
    __shared__ Wl wl;
    if (LIGHT && threadIdx.x == 0) wl.n = 0;
    const u64 nq = LIGHT ? tot->nl : tot->nh, total = LIGHT ? tot->ml : tot->mh;
    const u64 ntiles = (total + D_TILE - 1) / D_TILE;
    for (u64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const u64 e0 = tile * D_TILE;
        const u64 e1 = min(e0 + (u64)D_TILE, total);
        u64 s0;
        u32 ns;
        lb_tile_load<D_TILE>(io, nq, e0, sh, s0, ns);
        for (u32 i = threadIdx.x; i < ns; i += DB) {
            s_du[i] = dist[iv[s0 + i]];
            if (PJ_D_STAGE_IB) s_ib[i] = ib[s0 + i];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < D_IPT; ++k) {
            const u64 e = e0 + (u64)k * DB + threadIdx.x;
            bool p = false;
            u32 v = 0;
            if (e < e1) {
                const u32 j = lb_find<D_TILE>(sh, ns, e);
                const u64 rb = PJ_D_STAGE_IB ? s_ib[j] : ib[s0 + j];
                p = relax_edge(rb + (e - sh.off[j]), s_du[j], col, wt, dist, hi, settled, v);
            }
            if (LIGHT) wl_push(p, v, wl, chg, flag);
        }
        __syncthreads();
    }
    if (!LIGHT) return;
    // ---- drain the worklist FIFO: relax the light edges of the vertices this
    // workgroup lowered into the band (their heavy edges wait for the heavy pass), WL_BATCH per step, at most LOCAL_BUDGET in
    // all (a cascade larger than that is spread over the grid by a BITS round)
    u32 head = 0;
    for (;;) {
        __syncthreads();
        const u32 n = min(wl.n, (u32)WL_CAP);
        if (head >= n) break;
        const u32 t = threadIdx.x;
        if (head >= LOCAL_BUDGET) {
            for (u32 i = head + t; i < n; i += DB) defer_vertex(wl.v[i], chg, flag);
            break;
        }
        const u32 take = min(n - head, (u32)WL_BATCH);
        u64 deg = 0;
        if (t < take) {
            const u32 v = wl.v[head + t];
            const Off b = row[v];
            deg = lsplit[v];
            if (deg > LOCAL_MAX) {
                defer_vertex(v, chg, flag);
                deg = 0;
            }
            wl.bdu[t] = dist[v];
            wl.bbeg[t] = (u64)b;
        }
        u64 total_e;
        const u64 ex = block_excl_scan<DB / WAVE>(deg, wl.scan, total_e);
        if (t < take) wl.boff[t] = ex;
        head += take;
        __syncthreads();
        for (u64 f0 = 0; f0 < total_e; f0 += DB) {
            const u64 f = f0 + t;
            bool p = false;
            u32 v = 0;
            if (f < total_e) {
                u32 lo = 0, hi2 = take - 1;  // last entry with boff <= f
                while (lo < hi2) {
                    const u32 mid = (lo + hi2 + 1) >> 1;
                    if (wl.boff[mid] <= f) lo = mid;
                    else hi2 = mid - 1;
                }
                p = relax_edge(wl.bbeg[lo] + (f - wl.boff[lo]), wl.bdu[lo], col, wt, dist, hi, settled, v);
            }
            wl_push(p, v, wl, chg, flag);
        }
    }
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

// lsplit[v] = number of edges of v with weight < delta (rows are weight-sorted)
// Serial probes of a weight-sorted row, PU edges per step with independent
// loads (the probes are latency-bound; one edge per step leaves the memory
// system idle). Weights ascend along the row, so once lo + w >= cur for an
// edge, that edge and every later one are useless: the step returns true.
#ifndef PJ_PU
#define PJ_PU 2  // swept 1..8 with the 24-per-CU grid: 2 is ~+3% over 4 (profiles/r01/v2_unroll_sweep.txt)
#endif
constexpr int PU = PJ_PU;
// pull from band members [lo, hi)
template <typename Off>
__device__ __forceinline__ bool pull_step_band(const u32* __restrict__ wt, const u32* __restrict__ col,
                                               const int32_t* __restrict__ dist, Off& k, Off lim, int32_t lo,
                                               int32_t hi, int32_t& cur) {
    u32 w[PU], u[PU];
    bool ok[PU];
#pragma unroll
    for (int j = 0; j < PU; ++j) {
        ok[j] = k + (Off)j < lim;
        w[j] = ok[j] ? wt[k + j] : 0u;
        u[j] = ok[j] ? col[k + j] : 0u;
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
    for (int j = 0; j < PU; ++j)
        if (ok[j] && du[j] >= lo && du[j] < hi) {
            const long long nd = (long long)du[j] + w[j];
            if (nd < cur) cur = (int32_t)nd;
        }
    k += (Off)nv;
    return stop;
}
// pull from the frontier bitmap fin (members of the band's last round)
template <typename Off>
__device__ __forceinline__ bool pull_step_fin(const u32* __restrict__ wt, const u32* __restrict__ col,
                                              const int32_t* __restrict__ dist, const u64* __restrict__ fin, Off& k,
                                              Off lim, int32_t lo, int32_t& cur) {
    u32 w[PU], u[PU];
    bool ok[PU];
#pragma unroll
    for (int j = 0; j < PU; ++j) {
        ok[j] = k + (Off)j < lim;
        w[j] = ok[j] ? wt[k + j] : 0u;
        u[j] = ok[j] ? col[k + j] : 0u;
    }
    bool stop = false;
    int nv = 0;
#pragma unroll
    for (int j = 0; j < PU; ++j) {
        if (ok[j] && (long long)lo + w[j] >= (long long)cur) stop = true;
        ok[j] = ok[j] && !stop;
        nv += ok[j];
    }
    u64 fw[PU];
#pragma unroll
    for (int j = 0; j < PU; ++j) fw[j] = ok[j] ? fin[u[j] >> 6] : 0ull;
    int32_t du[PU];
#pragma unroll
    for (int j = 0; j < PU; ++j) du[j] = (ok[j] && ((fw[j] >> (u[j] & 63)) & 1ull)) ? dist[u[j]] : INT_INF;
#pragma unroll
    for (int j = 0; j < PU; ++j)
        if (du[j] < INT_INF) {
            const long long nd = (long long)du[j] + w[j];
            if (nd < cur) cur = (int32_t)nd;
        }
    k += (Off)nv;
    return stop;
}

// the same over interleaved edges (col | w << 32)
template <typename Off>
__device__ __forceinline__ bool pull_step_band_cw(const u64* __restrict__ ed, const int32_t* __restrict__ dist, Off& k,
                                                  Off lim, int32_t lo, int32_t hi, int32_t& cur) {
    u32 w[PU], u[PU];
    bool ok[PU];
#pragma unroll
    for (int j = 0; j < PU; ++j) {
        ok[j] = k + (Off)j < lim;
        const u64 x = ok[j] ? ed[k + j] : 0ull;
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
    for (int j = 0; j < PU; ++j)
        if (ok[j] && du[j] >= lo && du[j] < hi) {
            const long long nd = (long long)du[j] + w[j];
            if (nd < cur) cur = (int32_t)nd;
        }
    k += (Off)nv;
    return stop;
}
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

template <typename Off, typename E>
__device__ __forceinline__ bool pull_step_fin_cw(const E ed, const int32_t* __restrict__ dist,
                                                 const u64* __restrict__ fin, Off& k, Off lim, int32_t lo,
                                                 int32_t& cur) {
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
    u64 fw[PU];
#pragma unroll
    for (int j = 0; j < PU; ++j) fw[j] = ok[j] ? fin[u[j] >> 6] : 0ull;
    int32_t du[PU];
#pragma unroll
    for (int j = 0; j < PU; ++j) du[j] = (ok[j] && ((fw[j] >> (u[j] & 63)) & 1ull)) ? dist[u[j]] : INT_INF;
#pragma unroll
    for (int j = 0; j < PU; ++j)
        if (du[j] < INT_INF) {
            const long long nd = (long long)du[j] + w[j];
            if (nd < cur) cur = (int32_t)nd;
        }
    k += (Off)nv;
    return stop;
}

// Pull step for the heavy edges of band [lo, hi) — symmetric graphs only, where
// a row is also the vertex's in-edges with the same weights. Every vertex with
// dist >= hi looks through the heavy part of its own row (weights ascending)
// for in-neighbours in the band and stops as soon as lo + w >= the best value
// it has, since no band member can then offer less. This replaces pushing the
// members' heavy edges when few edges remain unsettled: most of a late band's
// heavy pushes hit vertices that are already settled (measured on Kronecker
// s20: 94% of all heavy relaxations), while the unsettled rows are short and
// cut early. A lane writes only its own vertex's dist, with a plain store; the
// old and new values are both >= hi, so the band tests of other lanes do not
// change. Screening as in the BFS pull: a wave reads the dists of PSC groups of
// 64 vertices, compacts the candidates into lanes, probes PSERIAL edges per lane
// (wave-uniform loop), then scans the long rows with the whole wave.
constexpr int PSC = 16;
#ifndef PJ_PSERIAL
#define PJ_PSERIAL 32
#endif
constexpr int PSERIAL = PJ_PSERIAL;
template <typename Off>
__global__ __launch_bounds__(DB) void d_pull_heavy_k(const Off* __restrict__ row, const u32* __restrict__ lsplit,
                                                     const u32* __restrict__ col, const u32* __restrict__ wt,
                                                     int32_t* __restrict__ dist, i64 n, int32_t lo, int32_t hi) {
    constexpr int NWV = DB / WAVE;
    const int lane = lane_id();
    const i64 ngroups = (n + 63) / 64;
    const i64 nsc = (ngroups + PSC - 1) / PSC;
    for (i64 sc = (i64)blockIdx.x * NWV + wave_id(); sc < nsc; sc += (i64)gridDim.x * NWV) {
        const i64 gbase = sc * PSC;
        u64 mytodo = 0;
#pragma unroll
        for (int k = 0; k < PSC; ++k) {
            const i64 v = (gbase + k) * 64 + lane;
            const int32_t d = v < n ? dist[v] : 0;
            const u64 m = __ballot(v < n && d >= hi);
            if (lane == k) mytodo = m;
        }
        const u32 cnt = (u32)__popcll(mytodo);
        const u32 incl = wave_incl_scan(cnt);
        const u32 myex = incl - cnt;
        const u32 T = __shfl(incl, 63, 64);
        for (u32 r0 = 0; r0 < T; r0 += WAVE) {
            const u32 c = r0 + lane;
            const bool act = c < T;
            u32 jw = 0;  // group of candidate c: largest lane jw < PSC with ex[jw] <= c
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
                d0 = dist[v];
                cur = d0;
                k = row[v] + (Off)lsplit[v];
                e = row[v + 1];
            }
            const Off lim = (e - k > (Off)PSERIAL) ? k + (Off)PSERIAL : e;
            bool go = act && k < lim, done = !act || k >= e;
            while (__ballot(go)) {
                if (go) {
                    if (pull_step_band<Off>(wt, col, dist, k, lim, lo, hi, cur)) {
                        done = true;
                        go = false;
                    } else {
                        go = k < lim;
                        done = k >= e;
                    }
                }
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
                    const u32 w = valid ? wt[k0] : 0u;
                    const bool stop = !valid || (long long)lo + w >= (long long)cl;
                    int32_t cand = INT_INF;
                    if (!stop) {
                        const int32_t du = dist[col[k0]];
                        if (du >= lo && du < hi) {
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
                    if (__ballot(stop)) break;  // weights ascend: every later edge stops too
                }
                if (lane == l) cur = cl;
            }
            if (act && cur < d0) dist[v] = cur;
        }
    }
}

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
#ifndef PJ_V2_ORPRE
#define PJ_V2_ORPRE 0  // frontier marks: read the word first, atomicOr only when the bit is clear
#endif
#ifndef PJ_V2_NOATOM
#define PJ_V2_NOATOM 0  // TIMING EXPERIMENT ONLY (wrong results): plain stores instead of atomicMin
#endif
// a light relaxation's dist update and frontier mark (1 = newly marked)
__device__ __forceinline__ void v2_dmin(int32_t* p, int32_t v) {
    if (PJ_V2_NOATOM) *p = v;
    else atomicMin(p, v);
}
__device__ __forceinline__ bool v2_mark(u64* __restrict__ fout, u32 t) {
    const u64 bit = 1ull << (t & 63);
    if (PJ_V2_ORPRE && (__hip_atomic_load(fout + (t >> 6), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit))
        return false;
    return !(atomicOr(fout + (t >> 6), bit) & bit);
}
#ifndef PJ_V2_LS
#define PJ_V2_LS 2  // swept 1, 2, 4 (round 2 end): 1 ~ 2, 4 is ~1% slower
#endif
constexpr int V2_LS = PJ_V2_LS;  // segment edges a lane relaxes alone
#ifndef PJ_V2_HT
#define PJ_V2_HT 64
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
#define PJ_V2_PLMAX 64
#endif
#ifndef PJ_V2_PCH
#define PJ_V2_PCH 256
#endif
constexpr u32 V2_PLMAX = PJ_V2_PLMAX;  // pull rounds: longer light rows go to v2_pull_long_body
constexpr u32 V2_PCH = PJ_V2_PCH;      // light edges per v2_pull_long_body work item

struct alignas(64) V2Line {
    u64 v;
    u64 pad[7];
};
struct V2Ctl {
    V2Line cnt[4][V2_NSH];  // frontier vertices marked per light round (ring)
    V2Line hub[3];          // hub queue packed counters (ring)
    V2Line mh[V2_NSH];      // heavy edges of this band's members
    V2Line minv[V2_NSH];    // min dist >= lo of the last select / pull (next band search), per shard
    V2Line dbg[8];          // PJ_V2_STATS builds: vertices, edges, atomics, marks, hub edges
};
#ifndef PJ_V2_PSTATS
#define PJ_V2_PSTATS 0  // debug build: heavy-pull scan-length counters (printed per solve)
#endif
#ifndef PJ_V2_STATS
#define PJ_V2_STATS 0
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
    int ltail;
    int dense_pull;   // light pulls in tile-dense form (v2_dense_pull_body)        // tail mode: light prefixes are row[v] + [0, lsplit[v]) of cw (no light CSR)
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


__device__ __forceinline__ u64 v2_slot_sum(const V2Line* sl) {
    u64 t = 0;
#pragma unroll
    for (int i = 0; i < V2_NSH; ++i) t += sl[i].v;
    return t;
}

// one relaxation; LIGHT: a target lowered below hi is marked in fout (returns 1 if newly marked)
template <bool LIGHT>
__device__ __forceinline__ u32 v2_relax(const V2Args& a, const ESrc ed, u64 k, int32_t du,
                                        u64* __restrict__ fout, u64& fe) {
    const u64 x = eat(ed, k);
    const u32 t = (u32)x;
    const long long nd = (long long)du + (long long)(x >> 32);
    if (PJ_V2_STATS) atomicAdd(&a.ctl->dbg[1].v, 1ull);
    if (a.sbits && ((a.sbits[t >> 6] >> (t & 63)) & 1ull)) return 0u;
    if (nd < INT_INF && (int32_t)nd < dist_now(a.dist + t)) {
        if (PJ_V2_STATS) atomicAdd(&a.ctl->dbg[2].v, 1ull);
        v2_dmin(a.dist + t, (int32_t)nd);  // no return: see v2_relax_g
        if (LIGHT && (int32_t)nd < a.hi) {
            if (PJ_V2_STATS) atomicAdd(&a.ctl->dbg[4].v, 1ull);
            const u32 nw = v2_mark(fout, t) ? 1u : 0u;
            if (PJ_V2_STATS && nw) atomicAdd(&a.ctl->dbg[3].v, 1ull);
            if (nw) fe += a.lsplit[t];  // the next round's push cost
            return nw;
        }
    }
    return 0u;
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
__device__ __forceinline__ u64 v2_slot_edges(const V2Line* sl) {
    u64 t = 0;
#pragma unroll
    for (int i = 0; i < V2_NSH; ++i) t += sl[i].pad[0];
    return t;
}

// PU consecutive edges [k, min(k + PU, lim)) of one source in one step (independent loads).
template <bool LIGHT>
__device__ __forceinline__ u32 v2_relax_n(const V2Args& a, const ESrc ed, u64 k, u64 lim, int32_t du,
                                          u64* __restrict__ fout, u64& fe) {
    u32 t[PU];
    long long nd[PU];
    bool ok[PU];
#pragma unroll
    for (int j = 0; j < PU; ++j) {
        ok[j] = k + j < lim;
        const u64 x = ok[j] ? eat(ed, k + j) : 0ull;
        t[j] = (u32)x;
        nd[j] = (long long)du + (long long)(x >> 32);
        ok[j] = ok[j] && nd[j] < INT_INF;
    }
    if (a.sbits) {  // tail: skip targets settled before the tail (a cache-resident bit, not dist)
        u64 sw[PU];
#pragma unroll
        for (int j = 0; j < PU; ++j) sw[j] = ok[j] ? a.sbits[t[j] >> 6] : 0ull;
#pragma unroll
        for (int j = 0; j < PU; ++j) ok[j] = ok[j] && !((sw[j] >> (t[j] & 63)) & 1ull);
    }
    int32_t cd[PU];
#pragma unroll
    for (int j = 0; j < PU; ++j) cd[j] = ok[j] ? dist_now(a.dist + t[j]) : 0;
    if (PJ_V2_STATS)
        for (int j = 0; j < PU; ++j)
            if (ok[j]) atomicAdd(&a.ctl->dbg[1].v, 1ull);
    u32 newc = 0;
#pragma unroll
    for (int j = 0; j < PU; ++j) {
        if (ok[j] && (int32_t)nd[j] < cd[j]) {
            v2_dmin(a.dist + t[j], (int32_t)nd[j]);
            if (PJ_V2_STATS) atomicAdd(&a.ctl->dbg[2].v, 1ull);
            if (LIGHT && (int32_t)nd[j] < a.hi) {
                if (PJ_V2_STATS) atomicAdd(&a.ctl->dbg[4].v, 1ull);
                if (v2_mark(fout, t[j])) {
                    if (PJ_V2_STATS) atomicAdd(&a.ctl->dbg[3].v, 1ull);
                    ++newc;
                    fe += a.lsplit[t[j]];
                }
            }
        }
    }
    return newc;
}

// N independent edges (any positions, own source distances) with the loads
// issued together: edge words, then target distances, then the atomics. The
// atomicMin is issued without a return value (nothing waits for it): a target
// whose read distance was above nd has been lowered to <= nd this round, by
// this lane or another, so it belongs in the next frontier either way; the
// atomicOr's old bit keeps the count of new frontier vertices exact.
template <bool LIGHT, int N>
__device__ __forceinline__ u32 v2_relax_g(const V2Args& a, const ESrc ed, const u64 (&idx)[N],
                                          const int32_t (&du)[N], const bool (&val)[N], u64* __restrict__ fout,
                                          u64& fe) {
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
    if (a.sbits) {
        u64 sw[N];
#pragma unroll
        for (int j = 0; j < N; ++j) sw[j] = ok[j] ? a.sbits[t[j] >> 6] : 0ull;
#pragma unroll
        for (int j = 0; j < N; ++j) ok[j] = ok[j] && !((sw[j] >> (t[j] & 63)) & 1ull);
    }
    int32_t cd[N];
#pragma unroll
    for (int j = 0; j < N; ++j) cd[j] = ok[j] ? dist_now(a.dist + t[j]) : 0;
    if (PJ_V2_STATS)
        for (int j = 0; j < N; ++j)
            if (ok[j]) atomicAdd(&a.ctl->dbg[1].v, 1ull);
    u32 newc = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        if (ok[j] && (int32_t)nd[j] < cd[j]) {
            v2_dmin(a.dist + t[j], (int32_t)nd[j]);
            if (PJ_V2_STATS) atomicAdd(&a.ctl->dbg[2].v, 1ull);
            if (LIGHT && (int32_t)nd[j] < a.hi) {
                if (PJ_V2_STATS) atomicAdd(&a.ctl->dbg[4].v, 1ull);
                if (v2_mark(fout, t[j])) {
                    if (PJ_V2_STATS) atomicAdd(&a.ctl->dbg[3].v, 1ull);
                    ++newc;
                    fe += a.lsplit[t[j]];
                }
            }
        }
    }
    return newc;
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
                                              V2Dense<Off>& sh) {
    const int tid = threadIdx.x, lane = lane_id();
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
        // long segments -> hub queue (wave-aggregated packed append, as v2_expand_k)
#pragma unroll
        for (int j = 0; j < V2_DV; ++j) {
            const bool hub = e[j] - b[j] > V2_DHT;
            const u64 hm = __ballot(hub);
            if (hm) {
                const u64 seg = hub ? e[j] - b[j] : 0;
                const u64 ie = wave_incl_scan(seg);
                const u64 tot = __shfl(ie, 63, 64);
                const int leader = __ffsll((long long)hm) - 1;
                u64 base = 0;
                if (lane == leader) base = atomicAdd(&a.ctl->hub[hs].v, ((u64)__popcll(hm) << V2_EB) | tot);
                base = __shfl(base, leader, 64);
                if (hub) {
                    const u64 slot = (base >> V2_EB) + (u64)__popcll(hm & lanemask_lt());
                    const u64 q = (u64)hs * a.hcap + slot;
                    a.hv[q] = (u32)(v0 + j);
                    a.hbeg[q] = b[j];
                    a.hoff[q] = (base & mask) + ie - seg;
                    e[j] = b[j];
                }
            }
        }
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
            newc += v2_relax_g<true, V2_DNJ>(a, ed, idx, dj, val, fout, fe);
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
    }
}

template <typename Off, bool LIGHT>
__device__ __forceinline__ void v2_expand_body(const V2Args& a, const Off* __restrict__ row, u64* __restrict__ fin,
                                               u64* __restrict__ fout, int cin, int hs, u64* red);

template <typename Off, bool LIGHT>
__global__ __launch_bounds__(DB) void v2_expand_k(V2Args a, const Off* __restrict__ row, u64* __restrict__ fin,
                                                  u64* __restrict__ fout, int cin, int hs, u64 pull_thresh,
                                                  u64 dense_min, u64* __restrict__ fclr) {
    constexpr int NWV = DB / WAVE;
    __shared__ u64 red[NWV];
    if (LIGHT) {
        v2_zero_slot(a, (cin + 2) & 3);
        v2_clear_words(fclr, a.nwords);
        if (v2_slot_sum(a.ctl->cnt[cin]) == 0) return;  // empty frontier (block-uniform)
        if (v2_slot_edges(a.ctl->cnt[cin]) > pull_thresh) return;  // v2_pull_round_k pulled this round
        if (v2_slot_sum(a.ctl->cnt[cin]) > dense_min) return;  // v2_pull_round_k ran it tile-dense
    }
    v2_expand_body<Off, LIGHT>(a, row, fin, fout, cin, hs, red);
}

template <typename Off, bool LIGHT>
__device__ __forceinline__ void v2_expand_body(const V2Args& a, const Off* __restrict__ row, u64* __restrict__ fin,
                                               u64* __restrict__ fout, int cin, int hs, u64* red) {
    constexpr int NWV = DB / WAVE;
    const int lane = lane_id();
    const u64 mask = (1ull << V2_EB) - 1ull;
    u32 newc = 0;
    u64 mh = 0, ml = 0, fe = 0;
    const i64 nsc = (a.nwords + V2_SC - 1) / V2_SC;
    for (i64 sc = (i64)blockIdx.x * NWV + wave_id(); sc < nsc; sc += (i64)gridDim.x * NWV) {
        const i64 wbase = sc * V2_SC;
        u64 mytodo = 0, mynew = 0;
        if (lane < V2_SC && wbase + lane < a.nwords) {
            mytodo = fin[wbase + lane];
            if (mytodo) {
                fin[wbase + lane] = 0;
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
                if (PJ_V2_STATS && LIGHT) atomicAdd(&a.ctl->dbg[0].v, 1ull);
                if (LIGHT) {  // light CSR (tail mode: the light prefix in cw)
                    b = a.ltail ? (u64)row[v] : a.lrow[v];
                    e = a.ltail ? b + a.lsplit[v] : a.lrow[v + 1];
                    if ((tn >> bit) & 1ull) {
                        mh += (u64)row[v + 1] - (u64)row[v] - (e - b);
                        ml += e - b;
                    }
                } else {      // heavy suffix of the row
                    b = (u64)row[v] + a.lsplit[v];
                    e = (u64)row[v + 1];
                }
            }
            // long segment -> hub queue (wave-aggregated packed append; all lanes here)
            const bool hub = e - b > V2_HT;
            const u64 hm = __ballot(hub);
            if (hm) {
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
                    e = b;  // the hub kernel relaxes this segment
                }
            }
            // lane-serial part
            u64 k = b;
            const u64 lim = (e - b > (u64)V2_LS) ? b + V2_LS : e;
            bool go = k < lim;
            while (__ballot(go)) {
                if (go) {
                    newc += v2_relax_n<LIGHT>(a, LIGHT ? v2_light_src(a) : v2_cw_src(a), k, lim, du, fout, fe);
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
                    if (gi < tot)
                        newc += v2_relax<LIGHT>(a, LIGHT ? v2_light_src(a) : v2_cw_src(a), kl + (gi - xl), dl, fout, fe);
                }
            }
        }
    }
    if (LIGHT) {
        v2_flush2(newc, fe, a.ctl->cnt[(cin + 1) & 3], red);
        v2_flush2(mh, ml, a.ctl->mh, red);
    }
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
                                            u64& fe, V2HubLds& L) {
    const u64 nq = packed >> V2_EB, total = packed & ((1ull << V2_EB) - 1ull);
    const u32* hv = a.hv + (u64)hs * a.hcap;
    const u64* hb = a.hbeg + (u64)hs * a.hcap;
    const u64* ho = a.hoff + (u64)hs * a.hcap;
    for (u64 e0 = (u64)blockIdx.x * V2_HTILE; e0 < total; e0 += (u64)gridDim.x * V2_HTILE) {
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
        newc += v2_relax_g<LIGHT, NJ>(a, LIGHT ? v2_light_src(a) : v2_cw_src(a), idx, du, val, fout, fe);
        __syncthreads();
    }
}

// The hub queue hs of one round in its own launch. Zeroes the next ring slot hz for
// later appends.
template <bool LIGHT>
__global__ __launch_bounds__(DB) void v2_hub_k(V2Args a, u64* __restrict__ fout, int cin, int hs, int hz) {
    __shared__ V2HubLds L;
    __shared__ u64 red[DB / WAVE];
    const u64 packed = a.ctl->hub[hs].v;
    if (blockIdx.x == 0 && threadIdx.x == 0) a.ctl->hub[hz].v = 0;
    if ((packed >> V2_EB) == 0) return;
    u32 newc = 0;
    u64 fe = 0;
    v2_hub_body<LIGHT>(a, fout, hs, packed, newc, fe, L);
    if (LIGHT) v2_flush2(newc, fe, a.ctl->cnt[(cin + 1) & 3], red);
}

// Next band [lo, hi): fout words = members, count into slot cout, min dist >= lo.
// A wave takes V2_SELW consecutive words per step with their distance loads issued
// together (one 256-byte load per step and wave left each wave one load in flight:
// 42.5 us for the 134 MB of s26 distances; 28 us with 4, profiles/r03/experiments_r3ab_select.txt).
#ifndef PJ_V2_SELW
#define PJ_V2_SELW 4
#endif
constexpr int V2_SELW = PJ_V2_SELW;
__global__ __launch_bounds__(DB) void v2_select_k(V2Args a, u64* __restrict__ fout, int cout) {
    __shared__ u64 red[DB / WAVE];
    const int lane = lane_id();
    u32 c = 0;
    u64 fe = 0;
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
            if (mem) fe += (a.fesplit ? a.fesplit : a.lsplit)[v];
            if (lane == 0) fout[wi] = m;
            c += lane == 0 ? (u32)__popcll(m) : 0u;
        }
    }
    v2_flush2(c, fe, a.ctl->cnt[cout], red);
    v2_flush_min(mn, a.ctl, red);
}

// Pull step of the heavy edges of band [lo, hi) fused with the selection of the
// next band [hi, nhi): see d_pull_heavy_k for the pull rule. The wave owns its
// PSC words: it writes the next band's member words of fout whole (and so clears
// them), counts them into slot cout and folds min{new dist >= hi} into minv.
template <typename Off>
__global__ __launch_bounds__(DB) void v2_pull_k(V2Args a, const Off* __restrict__ row, u64* __restrict__ fout,
                                                int32_t nhi, int cout, int32_t mlo, int32_t cap) {
    constexpr int NWV = DB / WAVE;
    __shared__ u32 s_new[NWV][2 * PSC];
    __shared__ u64 red[NWV];
    const int lane = lane_id();
    const int32_t lo = mlo, hi = a.hi;  // lo: the smallest member distance (early stop)
    u32* newb = s_new[wave_id()];
    u32 ccount = 0;
    u64 fe = 0;
    int32_t mn = INT_INF;
    const i64 ngroups = a.nwords;
    const i64 nsc = (ngroups + PSC - 1) / PSC;
    for (i64 sc = (i64)blockIdx.x * NWV + wave_id(); sc < nsc; sc += (i64)gridDim.x * NWV) {
        const i64 gbase = sc * PSC;
        u64 mytodo = 0;
#pragma unroll
        for (int k = 0; k < PSC; ++k) {
            const i64 v = (gbase + k) * 64 + lane;
            const int32_t d = v < a.n ? a.dist[v] : 0;
            const u64 m = __ballot(v < a.n && d >= hi);
            if (lane == k) mytodo = m;
            if (a.swrite) {
                const u64 sm = __ballot(v < a.n && d < hi);
                if (lane == k && gbase + k < a.nwords) a.swrite[gbase + k] = sm;
            }
        }
        if (lane < 2 * PSC) newb[lane] = 0;
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
            int32_t d0 = INT_INF, cur = INT_INF, bound = INT_INF;
            Off k = 0, e = 0;
            if (act) {
                d0 = a.dist[v];
                bound = min(d0, cap);  // cap (defer_heavy): only values that can land in [hi, nhi)
                cur = bound;
                k = row[v] + (Off)a.lsplit[v];
                e = row[v + 1];
            }  // (edges in a.cw)
            const Off lim = (e - k > (Off)PSERIAL) ? k + (Off)PSERIAL : e;
            bool go = act && k < lim, done = !act || k >= e;
#if PJ_V2_PSTATS
            const Off k0 = k;
#endif
            while (__ballot(go)) {
                if (go) {
                    // band members are exactly mb's bits: probe the (cache-resident)
                    // bitmap first, read dist only for members
                    if (pull_step_fin_cw<Off>(v2_cw_src(a), a.dist, a.mb, k, lim, lo, cur)) {
                        done = true;
                        go = false;
                    } else {
                        go = k < lim;
                        done = k >= e;
                    }
                }
            }
#if PJ_V2_PSTATS  // (heavy-pull scan lengths: candidates, stopped within 2 / 4 / 8 / the serial part)
            {
                const u64 sc = (u64)(k - k0);
                const u64 c0 = wave_sum((u64)act), c1 = wave_sum((u64)(act && done && sc <= 2)),
                          c2 = wave_sum((u64)(act && done && sc <= 4)), c3 = wave_sum((u64)(act && done && sc <= 8)),
                          c4 = wave_sum((u64)(act && done)), c5 = wave_sum(act ? (u64)(e - k0) : 0ull);
                if (lane == 0) {
                    atomicAdd(&a.ctl->dbg[2].v, c0);
                    atomicAdd(&a.ctl->dbg[3].v, c1);
                    atomicAdd(&a.ctl->dbg[4].v, c2);
                    atomicAdd(&a.ctl->dbg[5].v, c3);
                    atomicAdd(&a.ctl->dbg[6].v, c4);
                    atomicAdd(&a.ctl->dbg[7].v, c5);
                }
            }
#endif
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
                    int32_t cand = INT_INF;
                    if (!stop) {
                        const u32 u = (u32)x;
                        if ((a.mb[u >> 6] >> (u & 63)) & 1ull) {
                            const long long nd = (long long)a.dist[u] + w;
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
                if (cur == bound) cur = d0;  // nothing found below the bound
                if (cur < d0) a.dist[v] = cur;
                if (cur < mn) mn = cur;
                if (cur < nhi) {  // cur >= hi always here
                    const i64 wl = (v >> 6) - gbase;
                    atomicOr(&newb[2 * wl + ((v >> 5) & 1)], 1u << (v & 31));
                    fe += (a.fesplit ? a.fesplit : a.lsplit)[v];
                }
            }
        }
        if (lane < PSC && gbase + lane < a.nwords) {
            const u64 word = (u64)newb[2 * lane] | ((u64)newb[2 * lane + 1] << 32);
            fout[gbase + lane] = word;
            ccount += (u32)__popcll(word);
        }
    }
    v2_flush2(ccount, fe, a.ctl->cnt[cout], red);
    v2_flush_min(mn, a.ctl, red);
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
                                                   u32& newc, u64& fe, u64& mh, u64& ml, bool amin = false) {
    constexpr int NWV = DB / WAVE;
    const int lane = lane_id();
    const int32_t lo = a.lo, hi = a.hi;
    const i64 nsc = (a.nwords + PSC - 1) / PSC;
    for (i64 sc = (i64)blockIdx.x * NWV + wave_id(); sc < nsc; sc += (i64)gridDim.x * NWV) {
        const i64 gbase = sc * PSC;
        if (lane < PSC && gbase + lane < a.nwords) {
            const u64 f = fin[gbase + lane];
            if (f) {
                const u64 old = a.mb[gbase + lane];
                u64 nm = f & ~old;
                if (nm) a.mb[gbase + lane] = old | f;
                while (nm) {
                    const int b = __ffsll((long long)nm) - 1;
                    nm &= nm - 1;
                    const i64 v = (gbase + lane) * 64 + b;
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
            const u64 m = __ballot(v < a.n && d > lo);
            if (lane == k) mytodo = m;
        }
        // a vertex without light edges has no light in-edge (symmetric graph): not a candidate
        if (a.hl && mytodo) mytodo &= a.hl[gbase + lane];
        if (lane < 2 * PSC) newb[lane] = 0;
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
            u32 ls = 0;
            if (act) {
                d0 = a.dist[v];
                cur = d0;
                if (a.ltail) {  // the tail: the light prefix of the row in the whole CSR, no long-row list
                    k = row[v];
                    ls = a.lsplit[v];
                    e = k + (Off)ls;
                } else {
                    k = (Off)a.lrow[v];
                    ls = (u32)(a.lrow[v + 1] - a.lrow[v]);
                    e = ls > V2_PLMAX ? k : k + (Off)ls;  // long rows: v2_pull_long_body
                }
            }
            const Off lim = (e - k > (Off)PSERIAL) ? k + (Off)PSERIAL : e;
            bool go = act && k < lim, done = !act || k >= e;
            while (__ballot(go)) {
                if (go) {
                    if (pull_step_fin_cw<Off>(v2_light_src(a), a.dist, fin, k, lim, lo, cur)) {
                        done = true;
                        go = false;
                    } else {
                        go = k < lim;
                        done = k >= e;
                    }
                }
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
                    const bool stop = !valid || (long long)lo + w >= (long long)cl;
                    int32_t cand = INT_INF;
                    if (!stop) {
                        const u32 u = (u32)x;
                        if ((fin[u >> 6] >> (u & 63)) & 1ull) {
                            const long long nd = (long long)a.dist[u] + w;
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
            // amin: hub tiles of the previous round relax concurrently (fold_hub), so a
            // plain store could overwrite a lower distance they wrote
            if (act && cur < d0 && (!amin || cur < atomicMin(a.dist + v, cur))) {
                if (!amin) a.dist[v] = cur;
                if (cur < hi) {
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
// v2_pull_light_body: one lane scanning tens of thousands of edges would hold up
// its wave. Their pull runs here instead, over a static list of (vertex, chunk
// of V2_PCH light edges) built once per delta; a wave takes a chunk, skips it
// when even its lightest edge cannot help, and folds the result in with
// atomicMin (the vertex's chunks run in different waves).
__device__ __forceinline__ void v2_pull_long_body(const V2Args& a, const u64* __restrict__ fin, u64* __restrict__ fout,
                                                  const u32* __restrict__ lcv, const u32* __restrict__ lcc, u64 nlc,
                                                  u32& newc, u64& fe) {
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
        if ((long long)lo + (eat(v2_light_src(a), kb) >> 32) >= (long long)d0) continue;
        int32_t cur = d0;
        for (u64 kk = kb; kk < ke; kk += WAVE) {
            const u64 k0 = kk + lane;
            const bool valid = k0 < ke;
            const u64 x = valid ? eat(v2_light_src(a), k0) : 0ull;
            const u32 w = (u32)(x >> 32);
            const bool stop = !valid || (long long)lo + w >= (long long)cur;
            int32_t cand = INT_INF;
            if (!stop) {
                const u32 u = (u32)x;
                if ((fin[u >> 6] >> (u & 63)) & 1ull) {
                    const long long nd = (long long)a.dist[u] + w;
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
                const u64 bit = 1ull << (v & 63);
                if (!(atomicOr(fout + (v >> 6), bit) & bit)) {
                    ++newc;
                    fe += ls;
                }
            }
        }
    }
}

// Tile-dense form of v2_pull_light_body (dense_pull): the workgroup takes V2_DT
// consecutive vertices, 4 per thread with coalesced loads (distances, light-row
// bounds, the new members' row bounds), compacts the candidates' light rows (dist
// > lo, light edges, not a long row) into LDS with one block scan and scans all
// their edges edge-balanced, 4 independent edges per thread: an edge can help only
// when lo + w is below its vertex's best so far; a frontier in-neighbour's
// dist + w is folded into the vertex's LDS minimum. The block owns its vertices:
// improved distances are plain stores, the frontier words are OR-ed in (the long
// rows' chunks run concurrently).
template <typename Off>
struct V2DensePull {
    Off b[V2_DT];        // light-row begin (index into lcw)
    u32 off[V2_DT + 1];  // row start inside the tile's edge range
    int32_t best[V2_DT];
    uint16_t vi[V2_DT];  // vertex index inside the tile
    u32 newb[2 * (V2_DT / 64)];
    u64 fnew[V2_DT / 64];
    u64 red[DB / WAVE];
};

template <typename Off>
__device__ __forceinline__ void v2_dense_pull_body(const V2Args& a, const Off* __restrict__ row,
                                                   const u64* __restrict__ fin, u64* __restrict__ fout, u32& newc,
                                                   u64& fe, u64& mh, u64& ml, V2DensePull<Off>& sh) {
    const int tid = threadIdx.x;
    const int32_t lo = a.lo, hi = a.hi;
    const u64 mask = (1ull << V2_EB) - 1ull;
    const i64 ntiles = (a.n + V2_DT - 1) / V2_DT;
    for (i64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const i64 w0 = tile * (V2_DT / 64);
        if (tid < V2_DT / 64) {
            u64 nw = 0;
            if (w0 + tid < a.nwords) {
                const u64 f = fin[w0 + tid];
                if (f) {
                    const u64 old = a.mb[w0 + tid];  // the block owns these words of mb
                    nw = f & ~old;
                    if (nw) a.mb[w0 + tid] = old | f;
                }
            }
            sh.fnew[tid] = nw;
        }
        if (tid < 2 * (V2_DT / 64)) sh.newb[tid] = 0;
        __syncthreads();
        const int i0 = tid * V2_DV;
        const i64 v0 = tile * V2_DT + i0;
        const u32 nnew = (u32)(sh.fnew[i0 >> 6] >> (i0 & 63)) & V2_DVM;
        const u32 hlb = a.hl ? (u32)(a.hl[(v0 >> 6) < a.nwords ? (v0 >> 6) : 0] >> (v0 & 63)) & V2_DVM : V2_DVM;
        u64 b[V2_DV], e[V2_DV];
        int32_t d[V2_DV];
#pragma unroll
        for (int j = 0; j < V2_DV; ++j) {
            const i64 v = v0 + j;
            b[j] = e[j] = 0;
            d[j] = 0;
            if (v < a.n) {
                d[j] = a.dist[v];
                if ((nnew >> j) & 1u) {
                    const u64 ls = a.lsplit[v];
                    mh += (u64)row[v + 1] - (u64)row[v] - ls;
                    ml += ls;
                }
                if (d[j] > lo && ((hlb >> j) & 1u)) {
                    b[j] = a.lrow[v];
                    e[j] = a.lrow[v + 1];
                    if (e[j] - b[j] > V2_PLMAX) e[j] = b[j];  // long rows: v2_pull_long_body
                }
            }
        }
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
                sh.off[slot] = eo;
                sh.best[slot] = d[j];
                sh.vi[slot] = (uint16_t)(i0 + j);
                ++slot;
                eo += (u32)(e[j] - b[j]);
            }
        const u32 ns = (u32)(tot >> V2_EB), te = (u32)(tot & mask);
        if (tid == 0) sh.off[ns] = te;
        __syncthreads();
        for (u32 e0 = 0; e0 < te; e0 += DB * 4) {
            u32 sl[4], u[4], w[4];
            bool ok[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const u32 x = e0 + (u32)j * DB + (u32)tid;
                ok[j] = x < te;
                sl[j] = ok[j] ? v2_dense_find(sh.off, ns, x) : 0u;
                const u64 rec = ok[j] ? eat(v2_light_src(a), (u64)sh.b[sl[j]] + (x - sh.off[sl[j]])) : 0ull;
                u[j] = (u32)rec;
                w[j] = (u32)(rec >> 32);
            }
            u64 fw[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                ok[j] = ok[j] && (long long)lo + w[j] < (long long)sh.best[sl[j]];
                fw[j] = ok[j] ? fin[u[j] >> 6] : 0ull;
            }
            int32_t du[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                ok[j] = ok[j] && ((fw[j] >> (u[j] & 63)) & 1ull);
                du[j] = ok[j] ? a.dist[u[j]] : 0;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (ok[j]) {
                    const long long nd = (long long)du[j] + w[j];
                    if (nd < sh.best[sl[j]]) atomicMin(&sh.best[sl[j]], (int32_t)nd);
                }
        }
        __syncthreads();
        for (u32 q = tid; q < ns; q += DB) {
            const u32 i = sh.vi[q];
            const i64 v = tile * V2_DT + i;
            const int32_t bq = sh.best[q];
            if (bq < a.dist[v]) {  // (the block's own vertex: dist[v] is still d0)
                a.dist[v] = bq;
                if (bq < hi) {
                    atomicOr(&sh.newb[i >> 5], 1u << (i & 31));
                    ++newc;
                    fe += sh.off[q + 1] - sh.off[q];
                }
            }
        }
        __syncthreads();
        if (tid < V2_DT / 64 && w0 + tid < a.nwords) {
            const u64 word = (u64)sh.newb[2 * tid] | ((u64)sh.newb[2 * tid + 1] << 32);
            if (word) atomicOr(fout + w0 + tid, word);
        }
    }
}

template <typename Off>
union V2RoundLds {  // the round kernel's LDS: the folded hub tiles, then a dense push or a dense pull
    V2Dense<Off> push;
    V2DensePull<Off> pull;
    V2HubLds hub;
};

// Pull form of a light round, one launch: the chunks of the long light rows
// (v2_pull_long_body) and the short rows (v2_pull_light_body) over the whole
// grid. The two touch disjoint vertices; frontier words are OR-ed in.
template <typename Off>
__global__ __launch_bounds__(DB) void v2_pull_round_k(V2Args a, const Off* __restrict__ row, u64* __restrict__ fin,
                                                      u64* __restrict__ fout, int cin, u64 pull_thresh,
                                                      const u32* __restrict__ lcv, const u32* __restrict__ lcc, u64 nlc,
                                                      int hs, u64 dense_min, u64* __restrict__ fclr, int merged,
                                                      int fold, int hin) {
    constexpr int NWV = DB / WAVE;
    __shared__ u32 s_new[NWV][2 * PSC];
    __shared__ u64 red[NWV];
    __shared__ V2RoundLds<Off> lds;
    if (merged) {  // the whole round in this launch: no v2_expand_k behind it
        v2_zero_slot(a, (cin + 2) & 3);
        v2_clear_words(fclr, a.nwords);
    }
    // fold_hub: no hub launch behind the round. The hub tiles of the previous round
    // (queue hin, complete at this kernel boundary) are relaxed here first, into this
    // round's output frontier -- a label-correcting delay of one round, exact in any
    // order (R9). The round appends its own long segments to queue hs, which the next
    // round relaxes; block 0 zeroes the ring slot after hs for the round after that.
    bool hub_pending = false;
    if (fold) {
        if (blockIdx.x == 0 && threadIdx.x == 0) a.ctl->hub[(hs + 1) % 3].v = 0;
        const u64 packed = hin >= 0 ? a.ctl->hub[hin].v : 0ull;
        if (packed >> V2_EB) {
            hub_pending = true;
            u32 hn = 0;
            u64 hfe = 0;
            v2_hub_body<true>(a, fout, hin, packed, hn, hfe, lds.hub);
            v2_flush2(hn, hfe, a.ctl->cnt[(cin + 1) & 3], red);
        }
    }
    const u64 fcount = v2_slot_sum(a.ctl->cnt[cin]);
    if (a.rlog && merged && blockIdx.x == 0 && threadIdx.x == 0 && fcount) {  // (debug: round_log)
        const u64 fe0 = v2_slot_edges(a.ctl->cnt[cin]);
        const u64 i = atomicAdd(a.rlog, 1ull);
        if (i < 255) {
            a.rlog[1 + 3 * i] = fe0 > pull_thresh ? 2ull : (fcount > dense_min ? 1ull : 0ull);
            a.rlog[2 + 3 * i] = fcount;
            a.rlog[3 + 3 * i] = fe0 | ((u64)a.lo << 40);
        }
    }
    if (fcount == 0) return;
    if (v2_slot_edges(a.ctl->cnt[cin]) <= pull_thresh) {
        if (fcount <= dense_min) {  // a sparse push round
            if (merged) v2_expand_body<Off, true>(a, row, fin, fout, cin, hs, red);
            return;  // (else v2_expand_k)
        }
        u32 newc = 0;
        u64 mh = 0, ml = 0, fe = 0;
        v2_dense_body<Off>(a, row, fin, fout, hs, newc, fe, mh, ml, lds.push);
        v2_flush2(newc, fe, a.ctl->cnt[(cin + 1) & 3], red);
        v2_flush2(mh, ml, a.ctl->mh, red);
        return;
    }
    u32 newc = 0;
    u64 fe = 0, mh = 0, ml = 0;
    if (nlc && !a.ltail) v2_pull_long_body(a, fin, fout, lcv, lcc, nlc, newc, fe);
    if (a.dense_pull && !a.ltail) {
        v2_dense_pull_body<Off>(a, row, fin, fout, newc, fe, mh, ml, lds.pull);
    } else {
        v2_pull_light_body<Off>(a, row, fin, fout, s_new[wave_id()], newc, fe, mh, ml, hub_pending);
    }
    v2_flush2(newc, fe, a.ctl->cnt[(cin + 1) & 3], red);
    v2_flush2(mh, ml, a.ctl->mh, red);
}

// ---------------------------------------------------------------------------
// Binned light rounds (host-decided, symmetric graphs, outside the tail).
//
// A big push round is bound by its random accesses: per light edge a 4-byte
// probe of dist[t] (a 64-byte line from the Infinity Cache or HBM) and, when it
// improves, a device-scope atomicMin executed at the memory side (round 3: 24M
// and 32M light edges took 0.95 and 0.91 ms, 25-35 G edges/s; with the atomics
// replaced by plain stores, a timing-only build, still ~0.5 ms). A binned round
// has no random access and no global atomic per edge:
//   gen    : the frontier's light edges become pairs (t << 32 | dist[u] + w),
//            staged in LDS per coarse bucket (a vertex range holding ~1/64 of the
//            light-edge mass) and flushed in runs, one cursor atomic per run;
//            long segments go through the hub queue and v2_hub_k<BIN>
//   fine   : each chunk of a coarse bucket's pairs is counting-sorted in LDS by
//            fine bucket (2^14 vertices) and written out in runs
//   reduce : one workgroup per fine bucket: dist of its range into LDS, an LDS
//            atomicMin per pair, then improved distances and the next frontier's
//            words stored whole (the workgroup owns the range)
// Regions need no sizing pass: on a symmetric graph a vertex receives at most one
// pair per light in-edge = light out-edge, so the pairs of a vertex range fit the
// range's span of the light CSR, [lrow[a], lrow[b]), in both pair buffers.
// ---------------------------------------------------------------------------
constexpr int BIN_FLOG = 14;     // fine bucket: 2^14 vertices = 64 KB of LDS minima
constexpr int BIN_FINE = 1 << BIN_FLOG;
constexpr int BIN_NB1 = 128;     // most coarse buckets
constexpr int BIN_SB = 32;       // pairs staged per coarse bucket before a flush
constexpr int BIN_SPAN = 256;    // most fine buckets per coarse bucket
constexpr int BIN_CH = 4096;     // pairs per chunk of the fine pass
constexpr int BIN_MASS = 64;     // coarse buckets are cut at 1/BIN_MASS of the light-edge mass

struct BinArgs {
    u64* p1;             // pairs (t << 32 | nd) in coarse regions
    u64* p2;             // pairs in fine regions
    u64* c1;             // [BIN_NB1] coarse cursors (zeroed by the reduce)
    u64* c2;             // [nfine] fine cursors (zeroed by the reduce)
    const u64* r1;       // [nb1 + 1] coarse region starts
    const u64* r2;       // [nfine + 1] fine region starts = lrow[f << BIN_FLOG]
    const uint8_t* f2c;  // [nfine] coarse bucket of each fine bucket
    const u32* cb;       // [nb1 + 1] first fine bucket of each coarse bucket
    int nb1, nfine;
};

struct BinStage {
    u64 p[BIN_NB1][BIN_SB];
    u32 cnt[BIN_NB1];
    u64 base[BIN_NB1];
};

__device__ __forceinline__ void bin_stage_init(BinStage& st) {
    for (int c = threadIdx.x; c < BIN_NB1; c += blockDim.x) st.cnt[c] = 0;
}

// one pair into the block's staging (a full bucket goes straight to its region)
__device__ __forceinline__ void bin_put(const BinArgs& b, BinStage& st, u32 t, u32 nd) {
    const u32 c = b.f2c[t >> BIN_FLOG];
    const u64 pr = ((u64)t << 32) | nd;
    const u32 pos = atomicAdd(&st.cnt[c], 1u);
    if (pos < (u32)BIN_SB) st.p[c][pos] = pr;
    else b.p1[b.r1[c] + atomicAdd(&b.c1[c], 1ull)] = pr;
}

// collective: every staged run to its coarse region (one cursor atomic per run)
__device__ __forceinline__ void bin_flush(const BinArgs& b, BinStage& st) {
    __syncthreads();
    for (int c = threadIdx.x; c < b.nb1; c += blockDim.x) {
        const u32 k = min(st.cnt[c], (u32)BIN_SB);
        st.base[c] = k ? atomicAdd(&b.c1[c], (u64)k) : 0ull;
    }
    __syncthreads();
    const int nwv = (int)blockDim.x / WAVE, lane = lane_id();
    for (int c = wave_id(); c < b.nb1; c += nwv) {
        const u32 k = min(st.cnt[c], (u32)BIN_SB);
        if ((u32)lane < k) b.p1[b.r1[c] + st.base[c] + lane] = st.p[c][lane];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < b.nb1; c += blockDim.x) st.cnt[c] = 0;
    __syncthreads();
}

// gen: tile-dense screening of the frontier (as v2_dense_body), pairs for the light
// segments <= V2_DHT edges, longer ones to the hub queue; new members' degree sums
template <typename Off>
__global__ __launch_bounds__(DB) void v2_bin_gen_k(V2Args a, BinArgs b, const Off* __restrict__ row,
                                                   u64* __restrict__ fin, int cin, int hs, u64* __restrict__ fclr) {
    __shared__ V2Dense<Off> sh;
    __shared__ BinStage st;
    v2_zero_slot(a, (cin + 2) & 3);
    v2_clear_words(fclr, a.nwords);
    bin_stage_init(st);
    const int tid = threadIdx.x, lane = lane_id();
    const u64 mask = (1ull << V2_EB) - 1ull;
    const ESrc ed = v2_light_src(a);
    u64 mh = 0, ml = 0;
    const i64 ntiles = (a.n + V2_DT - 1) / V2_DT;
    for (i64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const i64 w0 = tile * (V2_DT / 64);
        if (tid < V2_DT / 64) {
            u64 f = 0, nw = 0;
            if (w0 + tid < a.nwords) {
                f = fin[w0 + tid];
                if (f) {
                    fin[w0 + tid] = 0;
                    const u64 old = a.mb[w0 + tid];
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
        u64 bb[V2_DV], e[V2_DV];
        int32_t du[V2_DV];
#pragma unroll
        for (int j = 0; j < V2_DV; ++j) {
            bb[j] = e[j] = 0;
            du[j] = 0;
            if ((nib >> j) & 1u) {
                const i64 v = v0 + j;
                du[j] = a.dist[v];
                bb[j] = a.lrow[v];
                e[j] = a.lrow[v + 1];
                if ((nnew >> j) & 1u) {
                    mh += (u64)row[v + 1] - (u64)row[v] - (e[j] - bb[j]);
                    ml += e[j] - bb[j];
                }
            }
        }
#pragma unroll
        for (int j = 0; j < V2_DV; ++j) {  // long segments -> hub queue (as v2_dense_body)
            const bool hub = e[j] - bb[j] > V2_DHT;
            const u64 hm = __ballot(hub);
            if (hm) {
                const u64 seg = hub ? e[j] - bb[j] : 0;
                const u64 ie = wave_incl_scan(seg);
                const u64 tot = __shfl(ie, 63, 64);
                const int leader = __ffsll((long long)hm) - 1;
                u64 base = 0;
                if (lane == leader) base = atomicAdd(&a.ctl->hub[hs].v, ((u64)__popcll(hm) << V2_EB) | tot);
                base = __shfl(base, leader, 64);
                if (hub) {
                    const u64 slot = (base >> V2_EB) + (u64)__popcll(hm & lanemask_lt());
                    const u64 q = (u64)hs * a.hcap + slot;
                    a.hv[q] = (u32)(v0 + j);
                    a.hbeg[q] = bb[j];
                    a.hoff[q] = (base & mask) + ie - seg;
                    e[j] = bb[j];
                }
            }
        }
        u64 cnt = 0, edges = 0;
#pragma unroll
        for (int j = 0; j < V2_DV; ++j)
            if (e[j] > bb[j]) {
                ++cnt;
                edges += e[j] - bb[j];
            }
        u64 tot;
        const u64 ex = block_excl_scan<DB / WAVE>((cnt << V2_EB) | edges, sh.red, tot);
        u32 slot = (u32)(ex >> V2_EB);
        u32 eo = (u32)(ex & mask);
#pragma unroll
        for (int j = 0; j < V2_DV; ++j)
            if (e[j] > bb[j]) {
                sh.b[slot] = (Off)bb[j];
                sh.du[slot] = du[j];
                sh.off[slot] = eo;
                ++slot;
                eo += (u32)(e[j] - bb[j]);
            }
        const u32 ns = (u32)(tot >> V2_EB), te = (u32)(tot & mask);
        __syncthreads();
        for (u32 e0 = 0; e0 < te; e0 += DB * V2_DNJ) {  // (te is block-uniform: the flush is collective)
#pragma unroll
            for (int j = 0; j < V2_DNJ; ++j) {
                const u32 x = e0 + (u32)j * DB + (u32)tid;
                if (x < te) {
                    const u32 sl = v2_dense_find(sh.off, ns, x);
                    const u64 r = eat(ed, (u64)sh.b[sl] + (x - sh.off[sl]));
                    const long long nd = (long long)sh.du[sl] + (long long)(r >> 32);
                    if (nd < INT_INF) bin_put(b, st, (u32)r, (u32)nd);
                }
            }
            bin_flush(b, st);
        }
        __syncthreads();
    }
    v2_flush2(mh, ml, a.ctl->mh, sh.red);
}

// hub segments of a binned round: the tiles of v2_hub_k, emitting pairs
__global__ __launch_bounds__(DB) void v2_hub_bin_k(V2Args a, BinArgs b, int hs, int hz) {
    __shared__ LbShared<V2_HTILE> sh;
    __shared__ int32_t s_du[V2_HTILE];
    __shared__ u64 s_b[V2_HTILE];
    __shared__ BinStage st;
    const u64 packed = a.ctl->hub[hs].v;
    if (blockIdx.x == 0 && threadIdx.x == 0) a.ctl->hub[hz].v = 0;
    const u64 nq = packed >> V2_EB, total = packed & ((1ull << V2_EB) - 1ull);
    if (nq == 0) return;
    bin_stage_init(st);
    const u32* hv = a.hv + (u64)hs * a.hcap;
    const u64* hb = a.hbeg + (u64)hs * a.hcap;
    const u64* ho = a.hoff + (u64)hs * a.hcap;
    const ESrc ed = v2_light_src(a);
    for (u64 e0 = (u64)blockIdx.x * V2_HTILE; e0 < total; e0 += (u64)gridDim.x * V2_HTILE) {
        u64 s0;
        u32 ns;
        lb_tile_load<V2_HTILE>(ho, nq, e0, sh, s0, ns);
        for (u32 i = threadIdx.x; i < ns; i += DB) {
            s_du[i] = a.dist[hv[s0 + i]];
            s_b[i] = hb[s0 + i];
        }
        __syncthreads();
        for (u32 j = 0; j < (u32)V2_HTILE; j += DB) {
            const u64 e = e0 + j + threadIdx.x;
            if (e < total) {
                const u32 sl = lb_find<V2_HTILE>(sh, ns, e);
                const u64 r = eat(ed, s_b[sl] + (e - sh.off[sl]));
                const long long nd = (long long)s_du[sl] + (long long)(r >> 32);
                if (nd < INT_INF) bin_put(b, st, (u32)r, (u32)nd);
            }
        }
        bin_flush(b, st);
    }
}

// fine: counting sort of each BIN_CH chunk of a coarse bucket's pairs by fine bucket
__global__ __launch_bounds__(DB) void v2_bin_fine_k(BinArgs b) {
    __shared__ u64 sp[BIN_CH];
    __shared__ u32 hist[BIN_SPAN], off[BIN_SPAN];
    __shared__ u64 gbase[BIN_SPAN];
    __shared__ u64 cpre[BIN_NB1 + 1];  // chunks before coarse bucket i
    __shared__ u32 red[DB / WAVE];
    const int tid = threadIdx.x;
    if (tid == 0) {
        u64 t = 0;
        for (int i = 0; i < b.nb1; ++i) {
            cpre[i] = t;
            t += (b.c1[i] + BIN_CH - 1) / BIN_CH;
        }
        cpre[b.nb1] = t;
    }
    __syncthreads();
    const u64 nchunks = cpre[b.nb1];
    constexpr int PT = BIN_CH / DB;
    for (u64 ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
        int i = 0;
        while (cpre[i + 1] <= ch) ++i;  // (<= 128 buckets, LDS)
        const u64 j0 = (ch - cpre[i]) * BIN_CH;
        const u64 cnt1 = b.c1[i];
        const u32 m = (u32)min((u64)BIN_CH, cnt1 - j0);
        const u32 fb0 = b.cb[i], nfb = b.cb[i + 1] - fb0;
        for (u32 k = tid; k < nfb; k += DB) hist[k] = 0;
        __syncthreads();
        u64 pr[PT];
        u32 lf[PT], rk[PT];
#pragma unroll
        for (int q = 0; q < PT; ++q) {
            const u32 x = (u32)q * DB + tid;
            pr[q] = x < m ? b.p1[b.r1[i] + j0 + x] : 0ull;
            lf[q] = x < m ? (u32)(pr[q] >> (32 + BIN_FLOG)) - fb0 : 0u;
        }
#pragma unroll
        for (int q = 0; q < PT; ++q) rk[q] = ((u32)q * DB + tid < m) ? atomicAdd(&hist[lf[q]], 1u) : 0u;
        __syncthreads();
        // exclusive offsets of the fine buckets inside the chunk, and their global bases
        u32 carry = 0;
        for (u32 k0 = 0; k0 < nfb; k0 += DB) {
            const u32 k = k0 + tid;
            const u32 h = k < nfb ? hist[k] : 0u;
            u32 tot;
            const u32 ex = block_excl_scan<DB / WAVE>(h, red, tot);
            if (k < nfb) {
                off[k] = carry + ex;
                gbase[k] = h ? atomicAdd(&b.c2[fb0 + k], (u64)h) : 0ull;
            }
            carry += tot;
            __syncthreads();
        }
#pragma unroll
        for (int q = 0; q < PT; ++q)
            if ((u32)q * DB + tid < m) sp[off[lf[q]] + rk[q]] = pr[q];
        __syncthreads();
        // runs out in LDS order: consecutive threads, consecutive addresses of one fine region
        for (u32 x = tid; x < m; x += DB) {
            const u64 p = sp[x];
            const u32 f = (u32)(p >> (32 + BIN_FLOG)), l = f - fb0;
            b.p2[b.r2[f] + gbase[l] + (x - off[l])] = p;
        }
        __syncthreads();
    }
}

// reduce: one workgroup per fine bucket (LDS minima), then the range's improved
// distances and next-frontier words; zeroes the cursors for the next binned round
__global__ __launch_bounds__(DB) void v2_bin_reduce_k(V2Args a, BinArgs b, u64* __restrict__ fout, int cin) {
    __shared__ int32_t best[BIN_FINE];
    __shared__ u64 words[BIN_FINE / 64];
    __shared__ u64 red[DB / WAVE];
    const int tid = threadIdx.x;
    if (blockIdx.x == 0)
        for (int c = tid; c < b.nb1; c += DB) b.c1[c] = 0;  // (the fine pass has read them)
    u64 newc = 0, fe = 0;
    for (int f = blockIdx.x; f < b.nfine; f += gridDim.x) {
        const u64 np = b.c2[f];
        if (np == 0) continue;  // block-uniform
        const i64 v0 = (i64)f << BIN_FLOG;
        const int nv = (int)min((i64)BIN_FINE, a.n - v0);
        for (int x = tid; x < nv; x += DB) best[x] = a.dist[v0 + x];
        __syncthreads();
        const u64* pp = b.p2 + b.r2[f];
        for (u64 k = tid; k < np; k += DB) {
            const u64 p = pp[k];
            const int32_t nd = (int32_t)(u32)p;
            const int x = (int)((p >> 32) - (u64)v0);
            if (nd < best[x]) atomicMin(&best[x], nd);
        }
        __syncthreads();
        // improved distances (plain stores: the workgroup owns the range) and the
        // range's next-frontier words, built in LDS and stored whole
        for (int x = tid; x < BIN_FINE / 64; x += DB) words[x] = 0;
        __syncthreads();
        for (int x = tid; x < nv; x += DB) {
            const int32_t bx = best[x];
            const i64 v = v0 + x;
            if (bx < a.dist[v]) {
                a.dist[v] = bx;
                if (bx < a.hi) {
                    atomicOr(&words[x >> 6], 1ull << (x & 63));
                    ++newc;
                    fe += a.lsplit[v];
                }
            }
        }
        __syncthreads();
        for (int x = tid; x < (nv + 63) / 64; x += DB) fout[(v0 >> 6) + x] = words[x];
        __syncthreads();
        if (tid == 0) b.c2[f] = 0;
    }
    v2_flush2(newc, fe, a.ctl->cnt[(cin + 1) & 3], red);
}

// fine region starts: r2[f] = lrow[min(f << BIN_FLOG, n)]
__global__ void v2_bin_r2_k(const u64* __restrict__ lrow, i64 n, int nfine, u64* __restrict__ r2) {
    for (int f = blockIdx.x * blockDim.x + threadIdx.x; f <= nfine; f += gridDim.x * blockDim.x)
        r2[f] = lrow[min((i64)f << BIN_FLOG, n)];
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

struct DeltaWork {
    DevBuf<u64> chg, sel, settled;  // 1 bit per vertex
    DevBuf<u32> qvl, qvh;
    DevBuf<u64> qbl, qbh, qol, qoh;
    DevBuf<u64> part, boff;
    DevBuf<DTot> tot;
    DevBuf<u32> flag;
    DevBuf<u32> lsplit;
    DevBuf<u32> lsplit2;   // light prefixes for the tail threshold (g.tail_delta)
    u32 lsplit2_delta = 0;
    DevBuf<u64> sb;        // settled-before-the-tail bitmap
    long long maxw = -1;   // largest edge weight (-1: not computed)
    DTot* host = nullptr;  // mapped pinned
    u32 lsplit_delta = 0;  // delta lsplit was computed for (0 = none)
    u64 heavy_total = 0;   // edges with w >= delta (for the pull decision)
    u64 light_total = 0;   // edges with w < delta
    // v2 band loop
    DevBuf<u64> f[3], mb;   // light-round frontier ring (v2_clear_words), band members
    DevBuf<V2Ctl> ctl;
    V2Ctl* hctl = nullptr;  // mapped pinned host copy, written by v2_publish_k
    V2Ctl* hctl_dev = nullptr;
    u64* hseq = nullptr;    // mapped pinned sequence word of v2_publish_k
    u64* hseq_dev = nullptr;
    u64 seq = 0;
    DevBuf<u32> hv;
    DevBuf<u64> hbeg, hoff;
    u64 hcap = 0;
    DevBuf<u32> lcv, lcc;  // long light rows: (vertex, chunk) work items
    u64 nlc = 0;
    DevBuf<u64> cw;        // interleaved relabeled edges
    ScanWs lscan;
    DevBuf<u64> lrow, lcw; // light CSR (per delta)
    DevBuf<u32> lcw32;     // the light CSR packed (col | w << lcb), when it fits
    u32 lcb = 0;
    int packed_for = -1;   // g.light_pack the light CSR was built for
    DevBuf<u64> hl;        // has-light-edges bitmap (per delta)
    // binned light rounds (per delta): pair buffers, cursors, bucket tables
    DevBuf<u64> bp1, bp2, bc1, bc2, br1, br2;
    DevBuf<uint8_t> bf2c;
    DevBuf<u32> bcb;
    int bnb1 = 0, bnfine = 0;
    u32 bin_for = 0;       // delta the tables were built for (0 = none)
    ~DeltaWork() {
        if (host) (void)hipHostFree(host);
        if (hctl) (void)hipHostFree(hctl);
        if (hseq) (void)hipHostFree(hseq);
    }
};

void delete_delta_work(DeltaWork* p) { delete p; }

namespace {

}  // namespace

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

// delta (explicit option, else 3.5 * mean weight / mean out-degree over all input
// ids: light edges are then ~5% of a row; swept on Kronecker s26 with weights
// 1..255 together with the tail switch, profiles/r01/tail_sweep.txt) and, once
// per delta, the light
// prefix length of every row and the number of heavy edges.
template <typename Off>
int32_t prepare_delta(Graph& g, DeltaWork& w) {
    Ctx& ctx = *g.ctx;
    hipStream_t s = ctx.stream;
    Relabeled& R = *g.rl;
    const i64 n = R.n_scan;
    const Off* row = static_cast<const Off*>(R.row_ptr(g.off64));
    const unsigned maxgrid = (unsigned)ctx.cu_count * 8u;
    int32_t delta = (int32_t)g.delta;
    if (delta <= 0) {
        const double mean_deg = g.n ? (double)g.nnz / (double)g.n : 1.0;
        const double d = 3.5 * g.mean_weight / std::max(1.0, mean_deg);
        delta = (int32_t)std::max(1.0, std::min(65536.0, std::round(d)));
    }
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
    return delta;
}

// Binned-round tables of the current light CSR: fine region starts (lrow at every
// 2^14-th vertex), coarse buckets cut greedily at 1/BIN_MASS of the light-edge mass
// or BIN_SPAN fine buckets, and the two pair buffers (the light CSR's size each).
// Returns false when the graph needs more than BIN_NB1 coarse buckets.
bool prepare_bins(DeltaWork& w, i64 n, hipStream_t s) {
    if (w.bin_for == w.lsplit_delta && w.bnb1 > 0) return true;
    const int nfine = (int)((n + BIN_FINE - 1) / BIN_FINE);
    w.br2.alloc((size_t)nfine + 1);
    v2_bin_r2_k<<<grid_for(nfine + 1, 256, 1024), 256, 0, s>>>(w.lrow.p, n, nfine, w.br2.p);
    PJ_LAUNCH_CHECK();
    std::vector<u64> r2((size_t)nfine + 1);
    PJ_HIP(hipMemcpyAsync(r2.data(), w.br2.p, sizeof(u64) * r2.size(), hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
    const u64 target = std::max<u64>(1, w.light_total / BIN_MASS);
    std::vector<u32> cb{0};
    for (int f = 0; f < nfine; ++f) {
        const u64 mass = r2[(size_t)f + 1] - r2[cb.back()];
        if (f + 1 < nfine && (mass >= target || (u32)(f + 1) - cb.back() >= (u32)BIN_SPAN)) cb.push_back((u32)f + 1);
    }
    cb.push_back((u32)nfine);
    const int nb1 = (int)cb.size() - 1;
    if (nb1 > BIN_NB1 || nfine == 0) return false;
    std::vector<u64> r1((size_t)nb1 + 1);
    std::vector<uint8_t> f2c((size_t)nfine);
    for (int i = 0; i <= nb1; ++i) r1[(size_t)i] = r2[cb[(size_t)i]];
    for (int i = 0; i < nb1; ++i)
        for (u32 f = cb[(size_t)i]; f < cb[(size_t)i + 1]; ++f) f2c[f] = (uint8_t)i;
    w.bcb.alloc(cb.size());
    w.br1.alloc(r1.size());
    w.bf2c.alloc(f2c.size());
    PJ_HIP(hipMemcpyAsync(w.bcb.p, cb.data(), sizeof(u32) * cb.size(), hipMemcpyHostToDevice, s));
    PJ_HIP(hipMemcpyAsync(w.br1.p, r1.data(), sizeof(u64) * r1.size(), hipMemcpyHostToDevice, s));
    PJ_HIP(hipMemcpyAsync(w.bf2c.p, f2c.data(), f2c.size(), hipMemcpyHostToDevice, s));
    w.bp1.ensure(std::max<u64>(w.light_total, 1));
    w.bp2.ensure(std::max<u64>(w.light_total, 1));
    w.bc1.ensure(BIN_NB1);
    w.bc2.alloc((size_t)nfine);
    PJ_HIP(hipMemsetAsync(w.bc1.p, 0, sizeof(u64) * BIN_NB1, s));
    PJ_HIP(hipMemsetAsync(w.bc2.p, 0, sizeof(u64) * (size_t)nfine, s));
    PJ_HIP(hipStreamSynchronize(s));
    w.bnb1 = nb1;
    w.bnfine = nfine;
    w.bin_for = w.lsplit_delta;
    return true;
}

template <typename Off>
void delta_run(Graph& g, DeltaWork& w, i64 source) {
    Ctx& ctx = *g.ctx;
    hipStream_t s = ctx.stream;
    Relabeled& R = *g.rl;
    const i64 n = R.n_scan;  // the solver works on the relabeled vertices with edges
    const i64 nwords = (n + 63) / 64;
    const Off* row = static_cast<const Off*>(R.row_ptr(g.off64));
    const unsigned maxgrid = (unsigned)ctx.cu_count * 8u;

    const int32_t delta = prepare_delta<Off>(g, w);
    ensure_w32(g);

    SelArgs a{};
    a.n = n;
    a.nwords = nwords;
    a.nwaves = (nwords + WPW - 1) / WPW;
    a.dist = R.dist.p;
    a.lsplit = w.lsplit.p;
    a.chg = w.chg.p;
    a.settled = w.settled.p;
    a.sel = w.sel.p;
    a.part = w.part.p;
    a.boff = w.boff.p;
    a.qvl = w.qvl.p;
    a.qvh = w.qvh.p;
    a.qbl = w.qbl.p;
    a.qbh = w.qbh.p;
    a.qol = w.qol.p;
    a.qoh = w.qoh.p;
    a.flag = w.flag.p;
    a.tot = w.tot.p;
    PJ_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&a.host), w.host, 0));
    const unsigned sgrid = (unsigned)((a.nwaves + SNW - 1) / SNW);

    auto select = [&](int mode, int32_t lo, int32_t hi) -> DTot {
        a.lo = lo;
        a.hi = hi;
        if (mode == SEL_DIST_L) sel_count_k<Off, SEL_DIST_L><<<sgrid, SB, 0, s>>>(a, row);
        else if (mode == SEL_DIST_H) sel_count_k<Off, SEL_DIST_H><<<sgrid, SB, 0, s>>>(a, row);
        else sel_count_k<Off, SEL_BITS><<<sgrid, SB, 0, s>>>(a, row);
        PJ_LAUNCH_CHECK();
        sel_scan_k<<<1, SCAN_T, 0, s>>>(a);
        PJ_LAUNCH_CHECK();
        if (PJ_SCAN_HOSTCOPY) PJ_HIP(hipMemcpyAsync(w.host, w.tot.p, sizeof(DTot), hipMemcpyDeviceToHost, s));
        PJ_HIP(hipStreamSynchronize(s));
        const volatile DTot* h = w.host;
        DTot t;
        t.nl = h->nl;
        t.ml = h->ml;
        t.nh = h->nh;
        t.mh = h->mh;
        t.members = h->members;
        t.minv = h->minv;
        t.overflow = h->overflow;
        return t;
    };
    pj_stats st{};
    // write the selected list, then relax it (light: with recursion; heavy: plain)
    auto relax = [&](int mode, const DTot& t, int32_t hi) {
        if (mode == SEL_DIST_L) sel_write_k<Off, SEL_DIST_L><<<sgrid, SB, 0, s>>>(a, row);
        else if (mode == SEL_DIST_H) sel_write_k<Off, SEL_DIST_H><<<sgrid, SB, 0, s>>>(a, row);
        else sel_write_k<Off, SEL_BITS><<<sgrid, SB, 0, s>>>(a, row);
        PJ_LAUNCH_CHECK();
        if (t.ml > 0) {
            const unsigned grid = grid_for((i64)((t.ml + D_TILE - 1) / D_TILE), 1, maxgrid);
            d_relax_k<Off, true><<<grid, DB, 0, s>>>(w.qvl.p, w.qbl.p, w.qol.p, w.tot.p, row, w.lsplit.p, R.col.p,
                                                     R.w.p, R.dist.p, hi, w.chg.p, w.flag.p, w.settled.p);
            PJ_LAUNCH_CHECK();
            st.relax_rounds++;
        }
        if (t.mh > 0) {
            const unsigned grid = grid_for((i64)((t.mh + D_TILE - 1) / D_TILE), 1, maxgrid);
            d_relax_k<Off, false><<<grid, DB, 0, s>>>(w.qvh.p, w.qbh.p, w.qoh.p, w.tot.p, row, w.lsplit.p,
                                                      R.col.p, R.w.p, R.dist.p, hi, w.chg.p, w.flag.p,
                                                      w.settled.p);
            PJ_LAUNCH_CHECK();
            st.relax_rounds++;
        }
    };

    const bool valid = source >= 0 && source < g.n;
    const i64 ls = valid ? relabeled_id(R, source, s) : -1;  // the source's new id (before the timed region)
    auto t_host0 = std::chrono::steady_clock::now();
    PJ_HIP(hipEventRecord(g.ev0, s));
    if (n > 0) {
        PJ_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(R.dist.p), INT_INF, (size_t)n, s));
        PJ_HIP(hipMemsetAsync(w.chg.p, 0, sizeof(u64) * (size_t)nwords, s));
        PJ_HIP(hipMemsetAsync(w.settled.p, 0, sizeof(u64) * (size_t)nwords, s));
        PJ_HIP(hipMemsetAsync(w.flag.p, 0, sizeof(u32), s));
    }
    if (valid && ls < n) {
        d_source_k<<<1, 1, 0, s>>>(ls, R.dist.p);
        PJ_LAUNCH_CHECK();
        long long lo = 0;
        u64 heavy_left = w.heavy_total;  // heavy edges of vertices not settled yet
        const bool can_pull = g.symmetric && g.pull_factor > 0.0;
        while (lo < INT_INF) {
            const int32_t hi = (int32_t)std::min<long long>(lo + delta, INT_INF);
            DTot t = select(SEL_DIST_L, (int32_t)lo, hi);
            if (t.members == 0) {
                if (t.minv >= (u64)INT_INF) break;  // nothing reached beyond the settled bands
                lo = (long long)t.minv / delta * delta;  // jump to the next occupied band
                continue;
            }
            st.levels++;
            // near phase: the members' light edges, cascades relaxed in-workgroup
            if (t.nl > 0) relax(SEL_DIST_L, t, hi);
            // heavy pass over the final members; deferred vertices (worklist
            // overflow, long light rows) first get BITS rounds of their own
            for (;;) {
                t = select(SEL_DIST_H, (int32_t)lo, hi);
                if (!t.overflow) break;
                DTot b = select(SEL_BITS, (int32_t)lo, hi);
                while (b.nl > 0) {
                    relax(SEL_BITS, b, hi);
                    b = select(SEL_BITS, (int32_t)lo, hi);
                }
            }
            // heavy edges: push the members' (t.mh) or let the unsettled vertices
            // pull (at most heavy_left edges, cut early by the weight order)
            heavy_left = heavy_left > t.mh ? heavy_left - t.mh : 0;
            if (t.nh > 0) {
                if (can_pull && (double)heavy_left < g.pull_factor * (double)t.mh) {
                    d_pull_heavy_k<Off><<<maxgrid, DB, 0, s>>>(row, w.lsplit.p, R.col.p, R.w.p, R.dist.p, n,
                                                               (int32_t)lo, hi);
                    PJ_LAUNCH_CHECK();
                    st.bu_levels++;
                } else {
                    relax(SEL_DIST_H, t, hi);
                    st.td_levels++;
                }
            }
            lo = hi;
        }
    }
    if (g.n > 0) {
        unlabel_k<<<grid_for(g.n, 256, maxgrid), 256, 0, s>>>(R.inv.p, R.dist.p, g.n, n, g.dist.p);
        PJ_LAUNCH_CHECK();
        if (valid && ls >= n) d_source_k<<<1, 1, 0, s>>>(source, g.dist.p);  // a source without edges
    }
    PJ_HIP(hipEventRecord(g.ev1, s));
    PJ_HIP(hipEventSynchronize(g.ev1));
    float ms = 0.f;
    PJ_HIP(hipEventElapsedTime(&ms, g.ev0, g.ev1));
    st.kernel_ms = ms;
    st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_host0).count();
    g.stats = st;
    g.have_result = true;
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
        if (threadIdx.x == 0 && src >= 0) ctl->cnt[0][0].v = 1;
    }
}

template <typename Off>
void delta2_run(Graph& g, DeltaWork& w, i64 source) {
    Ctx& ctx = *g.ctx;
    hipStream_t s = ctx.stream;
    Relabeled& R = *g.rl;
    const i64 n = R.n_scan;
    const i64 nwords = (n + 63) / 64;
    const Off* row = static_cast<const Off*>(R.row_ptr(g.off64));
    const unsigned maxgrid = (unsigned)ctx.cu_count * (unsigned)PJ_V2_GPC;  // workgroups per CU of the v2 kernels (grid-stride)
    const unsigned pullgrid = (unsigned)ctx.cu_count * (unsigned)PJ_V2_GPC_PULL;
    // light-round grids (grid-stride kernels): a launch that finds its round empty costs
    // in proportion to its workgroups, so these may be sized to the resident capacity
    const unsigned roundgrid = g.round_gpc > 0 ? (unsigned)ctx.cu_count * (unsigned)g.round_gpc : pullgrid;
    const unsigned hubgrid = g.hub_gpc > 0 ? (unsigned)ctx.cu_count * (unsigned)g.hub_gpc : maxgrid;
    const unsigned heavygrid = g.heavy_gpc > 0 ? (unsigned)ctx.cu_count * (unsigned)g.heavy_gpc : pullgrid;
    const int32_t delta = prepare_delta<Off>(g, w);
    // band width: at most the light threshold (an edge that can stay inside its
    // band must be light, so the band's light rounds see it)
    int32_t bw = g.band_width > 0 ? std::min<int32_t>(delta, (int32_t)g.band_width) : delta;
    if (!w.hctl) {
        const size_t nw = nwords ? (size_t)nwords : 1;
        w.f[0].alloc(nw);
        w.f[1].alloc(nw);
        w.f[2].alloc(nw);
        w.mb.alloc(nw);
        w.ctl.alloc(1);
        w.hcap = (u64)std::max<i64>(1, std::min<i64>(n, g.nnz / (i64)V2_HT + 1));
        w.hv.alloc(3 * w.hcap);
        w.hbeg.alloc(3 * w.hcap);
        w.hoff.alloc(3 * w.hcap);
        PJ_HIP(hipHostMalloc(reinterpret_cast<void**>(&w.hctl), sizeof(V2Ctl), hipHostMallocMapped));
        PJ_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&w.hctl_dev), w.hctl, 0));
        PJ_HIP(hipHostMalloc(reinterpret_cast<void**>(&w.hseq), 64, hipHostMallocMapped | hipHostMallocCoherent));
        PJ_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&w.hseq_dev), w.hseq, 0));
        *w.hseq = 0;
        w.seq = 0;
    }
    V2Args a{};
    a.n = n;
    a.nwords = nwords;
    a.dist = R.dist.p;
    a.lsplit = w.lsplit.p;
    a.cw = w.cw.p;
    a.lrow = w.lrow.p;
    a.lcw = w.lcw.p;
    a.lcw32 = w.lcb ? w.lcw32.p : nullptr;
    a.lcb = w.lcb;
    a.col = R.col.p;
    a.w8 = g.split_w ? R.w8.p : nullptr;
    a.hl = g.light_filter ? w.hl.p : nullptr;
    a.dense_pull = g.dense_pull;
    // light rounds whose frontier holds more than dense_frac x n vertices run tile-dense
    const u64 dense_min = g.dense_frac > 0.0 ? (u64)(g.dense_frac * (double)n) : ~0ull;
    a.mb = w.mb.p;
    a.ctl = w.ctl.p;
    a.hv = w.hv.p;
    a.hbeg = w.hbeg.p;
    a.hoff = w.hoff.p;
    a.hcap = w.hcap;
    DevBuf<u64> rlog;
    if (g.round_log) {
        rlog.alloc(1 + 3 * 255);
        PJ_HIP(hipMemsetAsync(rlog.p, 0, sizeof(u64), s));
        a.rlog = rlog.p;
    }
    // the host's view of the counters: one block copies them into mapped host memory
    // (a D2H hipMemcpyAsync of the same 3.3 KB ran as a ~30 us blit per sync)
    // The host spins on the sequence number (wakes within ~1 us of the copy instead of
    // the stream synchronization's latency); after 0.2 s of spinning it synchronizes the
    // stream, which surfaces a failed kernel instead of spinning forever.
    auto sync_ctl = [&]() {
        const u64 seq = ++w.seq;
        v2_publish_k<<<1, 256, 0, s>>>(w.ctl.p, reinterpret_cast<u64*>(w.hctl_dev), w.hseq_dev, seq);
        PJ_LAUNCH_CHECK();
        if (g.spin_sync) {
            const auto t0 = std::chrono::steady_clock::now();
            while (__atomic_load_n(w.hseq, __ATOMIC_ACQUIRE) != seq) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
                    PJ_HIP(hipStreamSynchronize(s));
                    break;
                }
            }
        } else {
            PJ_HIP(hipStreamSynchronize(s));
        }
    };
    auto slot = [&](int c) {
        u64 t = 0;
        for (int i = 0; i < V2_NSH; ++i) t += w.hctl->cnt[c][i].v;
        return t;
    };
    auto hminv = [&]() {
        u64 m = ~0ull;
        for (int i = 0; i < V2_NSH; ++i) m = std::min<u64>(m, w.hctl->minv[i].v);
        return m;
    };

    pj_stats st{};
    const bool valid = source >= 0 && source < g.n;
    const i64 ls = valid ? relabeled_id(R, source, s) : -1;  // the source's new id (before the timed region)
    auto t_host0 = std::chrono::steady_clock::now();
    PJ_HIP(hipEventRecord(g.ev0, s));
    if (n > 0) {
        v2_init_k<<<grid_for(n, 256, maxgrid), 256, 0, s>>>(R.dist.p, n, nwords, (valid && ls < n) ? ls : -1,
                                                            w.f[0].p, w.f[1].p, w.mb.p, w.ctl.p);
        PJ_LAUNCH_CHECK();
    }
    if (valid && ls < n) {
        int cs = 0, hr = 0, fi = 0;
        long long lo = 0;
        u64 heavy_left = w.heavy_total, light_left = w.light_total;
        const bool can_pull = g.symmetric && g.pull_factor > 0.0;
        bool can_pull_light = g.symmetric && g.light_pull > 0.0;
        double light_pull = g.light_pull;  // (tail_light_pull once in the tail)
        bool tail = false;
        u64 tail_unsettled = 0;
        const int32_t tdelta = (int32_t)std::min(65536.0, g.tail_delta < 0 ? 64.0 * delta : g.tail_delta);
        u64 last_fe = 1;  // light edges of the frontier at the last host sync (round 0: unknown)
        u64 last_cnt = 1; // its vertex count
        bool fe_known = false;  // last_fe / last_cnt describe the next round's frontier
        // binned light rounds: symmetric graphs with a light CSR, tables per delta
        BinArgs ba{};
        const bool bin_ok = g.bin_min > 0 && g.symmetric && !PJ_V2_STATS && w.light_total > 0 &&
                            prepare_bins(w, n, s);
        if (bin_ok) {
            ba.p1 = w.bp1.p;
            ba.p2 = w.bp2.p;
            ba.c1 = w.bc1.p;
            ba.c2 = w.bc2.p;
            ba.r1 = w.br1.p;
            ba.r2 = w.br2.p;
            ba.f2c = w.bf2c.p;
            ba.cb = w.bcb.p;
            ba.nb1 = w.bnb1;
            ba.nfine = w.bnfine;
        }
        // Deferred band check (merged rounds): after a heavy step the host does not wait
        // for its counters; it enqueues the next band's first rounds at once and learns at
        // their check whether that band had any vertex (its start slot survives the first
        // two rounds of the counter ring) and, if not, the next occupied band (minv of the
        // heavy step, copied by the same publish before it resets minv).
        const bool defer_ok = g.merged_round && g.defer_check && !PJ_V2_STATS && g.round_batch <= 2;
        // fold_hub: the hub tiles of light round r run inside round r + 1's launch (no hub
        // launch per round); not with binned rounds (their own hub kernel) or tile-dense
        // pulls (plain distance stores)
        const bool fold = g.fold_hub && g.merged_round && !bin_ok && !g.dense_pull;
        bool hub_pend = false;  // the last light round launched may have queued hub segments
        bool owed = false;      // defer_heavy: mb still holds the last band's members, whose heavier
        int32_t owed_lo = 0;    // edges (lo + w >= that band's nhi) are not relaxed yet; their lo
        u64 mh_owed = 0;        // and heavy-edge count
        bool deferred = false;
        bool finished = false;
        while (lo < INT_INF && !finished) {
            const int32_t hi = (int32_t)std::min<long long>(lo + bw, INT_INF);
            a.lo = (int32_t)lo;
            a.hi = hi;
            st.levels++;
            u64 mh = 0, ml = 0;  // members' heavy / light degree sums (reset by every publish)
            const int cs_start = cs;
            bool jumped = false;
            // light rounds until the band's frontier is empty
            // light rounds launched per host check: round_batch, doubling (starting
            // each band at the previous band's round count, or at 4 or 8, measured slower:
            // idle rounds cost more than the checks they save)
            int K = PJ_V2_STATS ? 1 : g.round_batch;
            for (;;) {
                const u64 pull_thresh = can_pull_light ? (u64)((double)light_left / light_pull) : ~0ull;
                // launch the pull kernels (which decide on the device, per round) only
                // when the last frontier seen could grow past the threshold in this batch
                const bool try_pull = can_pull_light && (double)last_fe * g.pull_grow > (double)pull_thresh;
                // binned round (host-decided, so the check before it must have seen the
                // frontier): its light edges are many, it is not a pull; a growing frontier
                // below that size gets single rounds, so the next big one is seen too
                const bool bin_can = bin_ok && fe_known && !a.ltail && g.merged_round;
                const bool pull_next = can_pull_light && last_fe > pull_thresh;
                const bool bin_now = bin_can && !pull_next && last_fe >= (u64)g.bin_min;
                const int k_now = (bin_can && !bin_now && last_fe >= (u64)g.bin_watch) ? 1 : K;
                if (bin_now) {
                    u64* fin = w.f[fi].p;
                    u64* fout = w.f[(fi + 1) % 3].p;
                    u64* fclr = w.f[(fi + 2) % 3].p;
                    v2_bin_gen_k<Off><<<roundgrid, DB, 0, s>>>(a, ba, row, fin, cs, hr, fclr);
                    PJ_LAUNCH_CHECK();
                    v2_hub_bin_k<<<hubgrid, DB, 0, s>>>(a, ba, hr, (hr + 1) % 3);
                    PJ_LAUNCH_CHECK();
                    v2_bin_fine_k<<<roundgrid, DB, 0, s>>>(ba);
                    PJ_LAUNCH_CHECK();
                    v2_bin_reduce_k<<<(unsigned)std::min<i64>(w.bnfine, (i64)ctx.cu_count * 4), DB, 0, s>>>(
                        a, ba, fout, cs);
                    PJ_LAUNCH_CHECK();
                    fi = (fi + 1) % 3;
                    cs = (cs + 1) & 3;
                    hr = (hr + 1) % 3;
                    st.relax_rounds++;
                }
                for (int q = 0; q < (bin_now ? 0 : k_now); ++q) {
                    u64* fin = w.f[fi].p;
                    u64* fout = w.f[(fi + 1) % 3].p;
                    u64* fclr = w.f[(fi + 2) % 3].p;
                    if (g.merged_round) {
                        // one launch decides pull / tile-dense push / sparse push on the device
                        v2_pull_round_k<Off><<<roundgrid, DB, 0, s>>>(a, row, fin, fout, cs,
                                                                     can_pull_light ? pull_thresh : ~0ull, w.lcv.p,
                                                                    w.lcc.p, w.nlc, hr, dense_min, fclr, 1,
                                                                    fold ? 1 : 0, hub_pend ? (hr + 2) % 3 : -1);
                        PJ_LAUNCH_CHECK();
                    } else {
                        // the round kernel also runs dense push rounds (v2_dense_body): whenever it
                        // is launched for pulls, else for the first round of a batch whose last
                        // seen frontier was dense
                        const bool try_dense =
                            dense_min != ~0ull && (try_pull || (q == 0 && last_cnt > dense_min));
                        const u64 dmin = try_dense ? dense_min : ~0ull;
                        if (try_pull || try_dense) {
                            v2_pull_round_k<Off><<<pullgrid, DB, 0, s>>>(a, row, fin, fout, cs,
                                                                        try_pull ? pull_thresh : ~0ull, w.lcv.p,
                                                                        w.lcc.p, w.nlc, hr, dmin, nullptr, 0, 0, -1);
                            PJ_LAUNCH_CHECK();
                        }
                        // (without the round kernel the expand must push every round)
                        v2_expand_k<Off, true><<<maxgrid, DB, 0, s>>>(a, row, fin, fout, cs, hr,
                                                                      try_pull ? pull_thresh : ~0ull, dmin, fclr);
                        PJ_LAUNCH_CHECK();
                    }
                    if (fold) {
                        hub_pend = true;  // (the next round relaxes this round's hub queue)
                    } else {
                        v2_hub_k<true><<<hubgrid, DB, 0, s>>>(a, fout, cs, hr, (hr + 1) % 3);
                        PJ_LAUNCH_CHECK();
                    }
                    fi = (fi + 1) % 3;
                    cs = (cs + 1) & 3;
                    hr = (hr + 1) % 3;
                    st.relax_rounds++;
                }
                sync_ctl();
                fe_known = true;
                // fold_hub: the band's light work is done only when the last round's frontier
                // AND its hub queue (relaxed by the next round) are empty
                const bool hubs_left = hub_pend && (w.hctl->hub[(hr + 2) % 3].v >> V2_EB) != 0;
                if (deferred) {
                    deferred = false;
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
                        v2_select_k<<<maxgrid, DB, 0, s>>>(a, w.f[fi].p, cs);
                        PJ_LAUNCH_CHECK();
                        fe_known = false;
                        jumped = true;
                        hub_pend = false;  // (idle rounds: no hubs queued)
                        break;
                    }
                }
                for (int i = 0; i < V2_NSH; ++i) {
                    mh += w.hctl->mh[i].v;
                    ml += w.hctl->mh[i].pad[0];
                }
                last_fe = 0;
                for (int i = 0; i < V2_NSH; ++i) last_fe += w.hctl->cnt[cs][i].pad[0];
                last_cnt = slot(cs);
                if (PJ_V2_STATS) {
                    fprintf(stderr, "band %d lo %lld rounds %d: frontier %llu edges %llu atomicmin %llu atomicor %llu marks %llu next %llu\n",
                            (int)st.levels, lo, K, w.hctl->dbg[0].v, w.hctl->dbg[1].v, w.hctl->dbg[2].v,
                            w.hctl->dbg[4].v, w.hctl->dbg[3].v, slot(cs));
                    PJ_HIP(hipMemsetAsync(w.ctl.p->dbg, 0, sizeof(w.ctl.p->dbg), s));
                }
                if (slot(cs) == 0 && !hubs_left) {
                    hub_pend = false;
                    break;
                }
                if (!bin_now && k_now == K) K = PJ_V2_STATS ? 1 : std::min(2 * K, 16);
            }
            if (finished) break;
            if (jumped) continue;  // (the select of the jumped-to band is enqueued)
            heavy_left = heavy_left > mh ? heavy_left - mh : 0;
            light_left = light_left > ml ? light_left - ml : 0;
            // Tail: past the dense first bands the remaining rows are short and the
            // bands sparse, so wide bands (few band steps) pay off. Once the edges of
            // the unsettled vertices drop below tail_frac x nnz, the bands after this
            // one use the light threshold tdelta (light prefixes from lsplit2, push
            // only: the packed light CSR belongs to delta) and width tdelta. Decided
            // here, before the heavy step, so that its fused selection already picks
            // the first tail band and writes the settled bitmap the tail's
            // relaxations filter their targets with. Exact at any band boundary:
            // everything below hi is settled and relaxed after this heavy step.
            const bool enter_tail = !tail && tdelta > delta && (int)st.levels >= g.tail_after &&
                                    (double)(heavy_left + light_left) < g.tail_frac * (double)g.nnz;
            const int32_t nbw = enter_tail ? tdelta : bw;
            const int32_t nhi_t = (int32_t)std::min<long long>((long long)hi + nbw, INT_INF);
            if (enter_tail) {
                if (w.lsplit2_delta != (u32)tdelta) {
                    w.lsplit2.ensure((size_t)n);
                    launch_light_split<Off>(R, row, n, (u32)tdelta, w.lsplit2.p, maxgrid, s);
                    w.lsplit2_delta = (u32)tdelta;
                }
                w.sb.ensure((size_t)nwords);
                a.swrite = w.sb.p;
                a.fesplit = w.lsplit2.p;
            }
            // defer_heavy: a heavy pull whose next band is not the tail relaxes only what can
            // land in the next band (lo + w < nhi: the lightest heavy edges) and keeps the
            // members in mb; the heavy step after the next band relaxes the rest for the
            // members of both bands in one pass over the heavy rows (R9: any relaxation
            // order is exact as long as an edge is relaxed before the band it lands in runs)
            const u64 mh_all = mh + mh_owed;
            const bool pull_now = can_pull && mh_all > 0 && (double)heavy_left < g.pull_factor * (double)mh_all;
            const bool medium = pull_now && g.defer_heavy && !owed && !enter_tail && nhi_t < INT_INF;
            if (pull_now) {
                v2_pull_k<Off><<<heavygrid, DB, 0, s>>>(a, row, w.f[fi].p, nhi_t, cs, owed ? owed_lo : a.lo,
                                                        medium ? nhi_t : INT_INF);
                PJ_LAUNCH_CHECK();
                if (medium) {
                    owed = true;
                    owed_lo = a.lo;
                    mh_owed = mh;
                } else {
                    PJ_HIP(hipMemsetAsync(w.mb.p, 0, sizeof(u64) * (size_t)nwords, s));
                    owed = false;
                    mh_owed = 0;
                }
                st.bu_levels++;
            } else {
                owed = false;  // the push relaxes every heavy edge of mb's members (both bands)
                mh_owed = 0;
                if (mh_all > 0) {
                    v2_expand_k<Off, false><<<maxgrid, DB, 0, s>>>(a, row, w.mb.p, nullptr, cs, hr, ~0ull, ~0ull, nullptr);
                    PJ_LAUNCH_CHECK();
                    v2_hub_k<false><<<maxgrid, DB, 0, s>>>(a, nullptr, cs, hr, (hr + 1) % 3);
                    PJ_LAUNCH_CHECK();
                    hr = (hr + 1) % 3;
                    st.td_levels++;
                } else {
                    PJ_HIP(hipMemsetAsync(w.mb.p, 0, sizeof(u64) * (size_t)nwords, s));
                }
                a.lo = hi;
                a.hi = nhi_t;
                v2_select_k<<<maxgrid, DB, 0, s>>>(a, w.f[fi].p, cs);
                PJ_LAUNCH_CHECK();
            }
            if (enter_tail) {
                tail = true;
                a.hl = nullptr;  // the tail's light prefixes come from lsplit2
                a.swrite = nullptr;
                a.fesplit = nullptr;
                a.sbits = w.sb.p;
                a.lsplit = w.lsplit2.p;
                a.ltail = 1;
                bw = tdelta;
                // light pulls in the tail (tail_pull): rows are scanned in weight order and
                // stop at the first w with lo + w >= the vertex's distance
                can_pull_light = g.symmetric && g.tail_pull;
                light_pull = g.tail_light_pull;
                tail_unsettled = heavy_left + light_left;
                if ((long long)tdelta > w.maxw) {
                    heavy_left = 0;  // every edge is light in the tail
                    light_left = tail_unsettled;
                } else {
                    PJ_HIP(hipMemsetAsync(&w.ctl.p->dbg[0], 0, sizeof(V2Line), s));
                    v2_heavy_left_k<Off><<<maxgrid, DB, 0, s>>>(row, a.lsplit, R.dist.p, n, hi, &w.ctl.p->dbg[0].v);
                    PJ_LAUNCH_CHECK();
                }
            }
            bool synced = false;
            if (medium) {  // (no deferred check: an empty next band needs the owed edges first)
                sync_ctl();
                synced = true;
                if (slot(cs) == 0) {  // the owed heavy edges decide where the solve goes on
                    v2_pull_k<Off><<<heavygrid, DB, 0, s>>>(a, row, w.f[fi].p, nhi_t, cs, owed_lo, INT_INF);
                    PJ_LAUNCH_CHECK();
                    PJ_HIP(hipMemsetAsync(w.mb.p, 0, sizeof(u64) * (size_t)nwords, s));
                    owed = false;
                    mh_owed = 0;
                    st.bu_levels++;
                    sync_ctl();
                }
            }
            if (!synced && defer_ok && !(enter_tail && (long long)tdelta <= w.maxw)) {
                deferred = true;  // checked at the next band's first publish
                fe_known = false;
                lo = hi;
                continue;
            }
            if (!synced) sync_ctl();
            if (enter_tail && (long long)tdelta <= w.maxw) {
                heavy_left = w.hctl->dbg[0].v;
                light_left = tail_unsettled > heavy_left ? tail_unsettled - heavy_left : 0;
            }
            last_fe = 0;
            for (int i = 0; i < V2_NSH; ++i) last_fe += w.hctl->cnt[cs][i].pad[0];
            last_cnt = slot(cs);
            if (slot(cs) == 0) {
                const u64 mv = hminv();
                if (mv >= (u64)INT_INF) break;  // nothing reached beyond the settled bands
                lo = (long long)mv / bw * bw;  // jump to the next occupied band
                a.lo = (int32_t)lo;
                a.hi = (int32_t)std::min<long long>(lo + bw, INT_INF);
                v2_select_k<<<maxgrid, DB, 0, s>>>(a, w.f[fi].p, cs);
                PJ_LAUNCH_CHECK();
                fe_known = false;
                continue;
            }
            lo = hi;
        }
    }
    if (g.n > 0) {
        unlabel_k<<<grid_for(g.n, 256, maxgrid), 256, 0, s>>>(R.inv.p, R.dist.p, g.n, n, g.dist.p);
        PJ_LAUNCH_CHECK();
        if (valid && ls >= n) d_source_k<<<1, 1, 0, s>>>(source, g.dist.p);  // a source without edges
    }
    PJ_HIP(hipEventRecord(g.ev1, s));
    PJ_HIP(hipEventSynchronize(g.ev1));
    float ms = 0.f;
    PJ_HIP(hipEventElapsedTime(&ms, g.ev0, g.ev1));
    st.kernel_ms = ms;
    st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_host0).count();
    g.stats = st;
    g.have_result = true;
    if (PJ_V2_PSTATS) {
        V2Ctl h;
        PJ_HIP(hipMemcpy(&h, w.ctl.p, sizeof(V2Ctl), hipMemcpyDeviceToHost));
        fprintf(stderr, "heavy pulls: candidates %llu stopped within 2 %llu, 4 %llu, 8 %llu, serial %llu; "
                "heavy edges of the candidates %llu\n", (unsigned long long)h.dbg[2].v, (unsigned long long)h.dbg[3].v,
                (unsigned long long)h.dbg[4].v, (unsigned long long)h.dbg[5].v, (unsigned long long)h.dbg[6].v,
                (unsigned long long)h.dbg[7].v);
    }
    if (g.round_log) {  // debug: one stderr line per non-empty light round
        std::vector<u64> h(1 + 3 * 255);
        PJ_HIP(hipMemcpy(h.data(), rlog.p, sizeof(u64) * h.size(), hipMemcpyDeviceToHost));
        static const char* kind[3] = {"push", "dense", "pull"};
        for (u64 i = 0; i < std::min<u64>(h[0], 255); ++i)
            fprintf(stderr, "round %llu lo %llu %s frontier %llu light_edges %llu\n", (unsigned long long)i,
                    (unsigned long long)(h[3 + 3 * i] >> 40), kind[h[1 + 3 * i] % 3], (unsigned long long)h[2 + 3 * i],
                    (unsigned long long)(h[3 + 3 * i] & ((1ull << 40) - 1)));
    }
}

}  // namespace

void delta_solve(Graph& g, i64 source) {
    const size_t n = (size_t)g.n;
    const size_t nwords = (n + 63) / 64;
    g.dist.ensure(n ? n : 1);
    if (!g.ev0) PJ_HIP(hipEventCreate(&g.ev0));
    if (!g.ev1) PJ_HIP(hipEventCreate(&g.ev1));
    if (!g.rl) {
        build_relabeled(g);
        g.delta_work.reset();
    }
    if (!g.delta_work) {
        g.delta_work.reset(new DeltaWork());
        DeltaWork& w = *g.delta_work;
        const size_t m = n ? n : 1;
        const size_t nwaves = (nwords + WPW - 1) / WPW + 1;
        w.chg.alloc(nwords ? nwords : 1);
        w.settled.alloc(nwords ? nwords : 1);
        w.sel.alloc(nwords ? nwords : 1);
        w.qvl.alloc(m);
        w.qvh.alloc(m);
        w.qbl.alloc(m);
        w.qbh.alloc(m);
        w.qol.alloc(m + 1);
        w.qoh.alloc(m + 1);
        w.part.alloc(6 * nwaves);
        w.boff.alloc(4 * nwaves);
        w.tot.alloc(1);
        w.flag.alloc(1);
        w.lsplit.alloc(m);
        PJ_HIP(hipHostMalloc(reinterpret_cast<void**>(&w.host), sizeof(DTot), hipHostMallocMapped));
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
    if (g.delta_impl == 1) {
        if (g.off64) delta_run<u64>(g, *g.delta_work, source);
        else delta_run<u32>(g, *g.delta_work, source);
    } else {
        if (g.off64) delta2_run<u64>(g, *g.delta_work, source);
        else delta2_run<u32>(g, *g.delta_work, source);
    }
}

}  // namespace pj
