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
constexpr int SCAN_T = 1024;        // threads of the one-block scan

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
// relax overflow flag. The partials are walked in chunks of SCAN_T consecutive
// entries (coalesced loads; the four scans of a chunk share two barriers).
__global__ __launch_bounds__(SCAN_T) void sel_scan_k(SelArgs a) {
    __shared__ u64 lds[4][SCAN_T / WAVE];
    const i64 nw = a.nwaves;
    const int lane = lane_id(), wid = wave_id();
    u64 run[4] = {0, 0, 0, 0}, m = 0, mi = INT_INF;
    for (i64 c0 = 0; c0 < nw; c0 += SCAN_T) {
        const i64 i = c0 + threadIdx.x;
        const bool ok = i < nw;
        u64 x[4], inc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = ok ? a.part[j * nw + i] : 0;
        if (ok) {
            m += a.part[4 * nw + i];
            const u64 y = a.part[5 * nw + i];
            mi = y < mi ? y : mi;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            inc[j] = wave_incl_scan(x[j]);
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
            if (ok) a.boff[j * nw + i] = run[j] + wp[j] + inc[j] - x[j];
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
        a.host->nl = t.nl;
        a.host->ml = t.ml;
        a.host->nh = t.nh;
        a.host->mh = t.mh;
        a.host->members = t.members;
        a.host->minv = t.minv;
        a.host->overflow = t.overflow;
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

// One edge: relax u -> col[idx]; true if the target was lowered into the band.
__device__ __forceinline__ bool relax_edge(u64 idx, int32_t du, const u32* __restrict__ col,
                                           const u32* __restrict__ wt, int32_t* __restrict__ dist, int32_t hi,
                                           const u64* __restrict__ settled, u32& v) {
    v = col[idx];
    const long long nd = (long long)du + (long long)wt[idx];
    // a target settled in an earlier band cannot improve: skip its dist probe (the
    // settled bitmap is 1/32 of dist and mostly L2-resident; dist lines are not)
    if (PJ_D_SETTLED && ((settled[v >> 6] >> (v & 63)) & 1ull)) return false;
    if (nd < INT_INF && (int32_t)nd < dist[v]) {
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

// distances back to input ids: out[v] = dist'[inv[v]] (INT_INF past n_scan)
__global__ void unlabel_k(const u32* __restrict__ inv, const int32_t* __restrict__ dl, i64 n, i64 n_scan,
                          int32_t* __restrict__ out) {
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x) {
        const u32 x = inv[v];
        out[v] = (i64)x < n_scan ? dl[x] : INT_INF;
    }
}

// lsplit[v] = number of edges of v with weight < delta (rows are weight-sorted)
template <typename Off>
__global__ void light_split_k(const Off* __restrict__ row, const u32* __restrict__ w, i64 n, u32 delta,
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

__global__ __launch_bounds__(DB) void wsum_k(const u32* __restrict__ w, i64 n, u64* __restrict__ out) {
    u64 acc = 0;
    for (i64 i = (i64)blockIdx.x * DB + threadIdx.x; i < n; i += (i64)gridDim.x * DB) acc += w[i];
    acc = wave_sum(acc);
    if (lane_id() == 0 && acc) atomicAdd(out, acc);
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
    DTot* host = nullptr;  // mapped pinned
    u32 lsplit_delta = 0;  // delta lsplit was computed for (0 = none)
    ~DeltaWork() {
        if (host) (void)hipHostFree(host);
    }
};

void delete_delta_work(DeltaWork* p) { delete p; }

namespace {

template <typename Off>
void delta_run(Graph& g, DeltaWork& w, i64 source) {
    Ctx& ctx = *g.ctx;
    hipStream_t s = ctx.stream;
    Relabeled& R = *g.rl;
    const i64 n = R.n_scan;  // the solver works on the relabeled vertices with edges
    const i64 nwords = (n + 63) / 64;
    const Off* row = static_cast<const Off*>(R.row_ptr(g.off64));
    const unsigned maxgrid = (unsigned)ctx.cu_count * 8u;

    // delta: explicit option, else 6 * mean weight / mean out-degree (over all
    // input ids) — light edges are then ~10% of a row. Swept on Kronecker s22 and
    // s26 with weights 1..255 (profiles/r01/delta_sweep.txt): flat from 24 to 48.
    int32_t delta = (int32_t)g.delta;
    if (delta <= 0) {
        const double mean_deg = g.n ? (double)g.nnz / (double)g.n : 1.0;
        const double d = 6.0 * g.mean_weight / std::max(1.0, mean_deg);
        delta = (int32_t)std::max(1.0, std::min(65536.0, std::round(d)));
    }
    if (w.lsplit_delta != (u32)delta && n > 0) {
        light_split_k<Off><<<grid_for(n, 256, maxgrid), 256, 0, s>>>(row, R.w.p, n, (u32)delta, w.lsplit.p);
        PJ_LAUNCH_CHECK();
        w.lsplit_delta = (u32)delta;
    }

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

    auto t_host0 = std::chrono::steady_clock::now();
    PJ_HIP(hipEventRecord(g.ev0, s));
    const bool valid = source >= 0 && source < g.n;
    const i64 ls = valid ? (i64)R.inv_h[(size_t)source] : -1;  // the source's new id
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
            if (t.nh > 0) relax(SEL_DIST_H, t, hi);
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
        u64 sum = 0;
        if (g.nnz > 0) {
            DevBuf<u64> acc;
            acc.alloc(1);
            PJ_HIP(hipMemsetAsync(acc.p, 0, sizeof(u64), g.ctx->stream));
            wsum_k<<<grid_for(g.nnz, DB, (unsigned)g.ctx->cu_count * 8u), DB, 0, g.ctx->stream>>>(g.w.p, g.nnz, acc.p);
            PJ_LAUNCH_CHECK();
            PJ_HIP(hipMemcpyAsync(&sum, acc.p, sizeof(u64), hipMemcpyDeviceToHost, g.ctx->stream));
            PJ_HIP(hipStreamSynchronize(g.ctx->stream));
        }
        g.mean_weight = g.nnz > 0 ? (double)sum / (double)g.nnz : 1.0;
    }
    if (g.off64) delta_run<u64>(g, *g.delta_work, source);
    else delta_run<u32>(g, *g.delta_work, source);
}

}  // namespace pj
