// bfs.hip — unit-weight SSSP: direction-optimizing level-synchronous BFS.
//
// Replaces the reference's relaxation core (extract_local_pq :226-278 driven by
// the BSP round loop :507-594). With w == 1 (:147) the reference computes hop
// distances capped at INT_INF; the result does not depend on
// pop order, so each BFS level settles exactly the vertices the heap would
// settle at that distance, and no level assigns a distance >= INT_INF.
//
// Device state (HBM):
//   dist[n]      int32, PJ_INT_INF = unreached              (the reference's sp[] :443)
//   vis[2]       visited bitmaps, 1 bit / vertex, seeded with the isolated-vertex
//                mask (such vertices are never reached and never act as parents)
//   normal queue frontier vertices with 1 <= out-degree <= HUBT, vertex ids only,
//                in NQS segments of capacity n, one append counter per segment
//                (counters on separate 64-B lines: NQS x the single-word atomic rate)
//   hub queue    (v, row begin, edge offset) of frontier vertices with out-degree >
//                HUBT; slot and edge offset come from ONE packed 64-bit atomic, so
//                the offsets are monotonic in the slot index without a scan
//   C[3], S[2]   per-level counters and control state (ring buffers, see below)
//
// One kernel launch per level and no host round trip inside a batch of levels:
//   * every block re-derives the direction decision (Beamer's alpha/beta rule) from
//     the previous level's counters C[(L+2)%3] and state S[(L+1)%2]; block 0
//     publishes S[L%2] and zeroes C[(L+1)%3]; the level accumulates into C[L%3].
//   * push (top-down) levels: a block takes 256 normal entries, reads their rows and
//     walks their edges in 256-edge steps (owner found by binary search in LDS);
//     hub edges go in 1024-edge tiles (slot found by binary search in LDS), so a
//     300K-edge hub is spread over ~300 workgroups. Claims: atomicOr on vis.
//   * pull (bottom-up) levels: a wave takes WPI 64-vertex words; an unvisited vertex
//     looks for any in-neighbour that is already visited (for an unvisited vertex
//     that is exactly "in the frontier"). Lanes probe their first edges with
//     independent loads, then the whole wave scans the rest of long rows. The wave
//     owns its words and writes vis_next[w] = vis[w] | found without atomics.
//   * new frontier entries are staged in LDS and published with one atomic per
//     block step (per segment), not one per wave.
#include <chrono>

#include "lb.h"

namespace pj {

namespace {

#ifndef PJ_RPI
#define PJ_RPI 1  // 4 until round 6: with hub-first rows and the dense first in-neighbours one round of 64
                  // candidates at a time is faster (K22 mean kernel time 0.1906 -> 0.1827 ms, web-Google
                  // 0.2277 -> 0.2216; 2: 0.1847 / 0.2222, 8: 0.245 / 0.255; profiles/r06/bfs_rpi_r6av.txt)
#endif
#ifndef PJ_PB2
#define PJ_PB2 8
#endif
#ifndef PJ_BFS_STAMPS
#define PJ_BFS_STAMPS 0  // diagnostic build: block 0 stamps s_memrealtime per launch / small level (stderr)
#endif
#ifndef PJ_SMALL_WG_ATOMIC
#define PJ_SMALL_WG_ATOMIC 1  // small_levels claims: workgroup-scope atomics (one block is running)
#endif
constexpr int TB = 256;
constexpr int NW = TB / WAVE;
constexpr u32 HUBT = 256;     // out-degree above which a frontier vertex goes to the hub queue
constexpr int HUB_TILE = 1024;
constexpr int WPI = 4;        // pull levels: visited words per wave and iteration
constexpr int QCAP = TB * WPI;  // staging: most normal entries one block step can produce
constexpr int HCAP = 256;     // staging for hubs (overflow goes straight to global)
constexpr int BU_SERIAL = 16; // edges a lane probes alone before the wave helps
constexpr int PB1 = 2;        // pull probes, stage A (every candidate)
constexpr int PB2 = PJ_PB2;   // pull probes, stage B (candidates still open)
constexpr int NSH = 16;       // shards of the summed counters
constexpr int NQS = 8;        // normal-queue segments
constexpr int SC = 16;        // pull levels: visited words a wave screens at once
constexpr int RPI = PJ_RPI;   // pull levels: rounds of 64 candidates in flight per wave
constexpr u32 SMALL_N = TB;   // one-workgroup levels: frontier vertices (one per thread)
constexpr u32 SEPT = 8;       // one-workgroup levels: frontier edges per thread
constexpr u32 SMALL_M = SEPT * TB;
struct alignas(64) Line {
    u64 v;
    u64 pad[7];
};

struct LevelCnt {
    Line n_norm[NQS];  // normal-queue entries appended, per segment
    Line hub_packed;   // (hub count << eb) | hub edges
    u64 m_next[NSH];   // out-degree sum of the new frontier (edges of the next push level)
    u64 found[NSH];    // newly visited vertices
    u64 in_next[NSH];  // in-degree sum of newly visited vertices
    u64 fnz[NSH];      // newly visited vertices with out-degree > 0 (the next frontier)
    u64 scan[NSH];     // pull levels: in-edges probed (a push level's edges are its frontier's, d.mq)
};

struct LevelState {
    int32_t mode;  // 0 push, 1 pull
    int32_t done;
    int32_t vsel;  // visited buffer holding "dist <= level" at the start of the next level
    int32_t level; // last level computed
    double m_u;    // Beamer: in-edges of unvisited vertices
    u64 prev_found;
    double n_u;    // unvisited vertices with an edge (the pull level's candidates: pull_vertex rule)
    u64 nr, mr;    // reached vertices and their out-edges, summed over the levels whose counters were read
    u64 pad[2];
};

struct BfsArgs {
    i64 n, nwords;
    int eb;  // edge bits of the packed hub counter
    double alpha, beta;
    double pv;  // pull_vertex: push -> pull also when the frontier's out-edges exceed pv x the unvisited
                // vertices (0 = Beamer's rule alone)
    int force;  // 0 auto, 1 push only, 2 pull whenever possible
    int small;  // one-workgroup levels for small push frontiers
    int32_t max_levels;  // debug: stop after this many levels
    int32_t* dist;
    u64* vis[2];
    u64* fnew;   // pull levels: bitmap of the vertices they found (next frontier)
    u32* qv[2];  // [parity], NQS segments of n entries
    u32* hv[2];
    u64* hbeg[2];
    u64* hoff[2];
    LevelCnt* C;    // [3]
    LevelState* S;  // [2]
    u64* nmode;     // [2] push / pull levels run (device)
    int64_t* host;  // mapped host words: [0] levels run (-1 while running), [1] push, [2] pull, [3] launches,
                    // [4] edges scanned (push: every frontier out-edge; pull: every in-edge probed),
                    // [5] reached vertices, [6] their out-edges (n_r, m_r: the levels' counters summed)
    u64* wtot;      // device: edges scanned by the levels so far (block 0 of each launch adds the last one's)
    u64* llog;      // level_log option: per launch (L, mode | kind << 8, frontier, its out-edges, found, scanned
                    // by the previous launch), or null
    u64* stamps;    // PJ_BFS_STAMPS builds: [launch * 64 + slot] 100 MHz timestamps of block 0
};

// (PJ_BFS_STAMPS) thread 0 of block 0 records the real-time counter in slot k of launch li
__device__ __forceinline__ void bfs_stamp(const BfsArgs& a, int32_t li, int k) {
#if PJ_BFS_STAMPS
    if (threadIdx.x == 0 && blockIdx.x == 0 && li < 64 && k < 64)
        a.stamps[(u64)li * 64 + (u64)k] = __builtin_amdgcn_s_memrealtime();
#else
    (void)a;
    (void)li;
    (void)k;
#endif
}

template <typename Off>
struct Graph_d {
    const Off* row;
    const u32* col;
    const Off* crow;
    const u32* ccol;
    const u64* hf2;  // (option pull_first) per vertex its in-row's first two entries, ccol[crow[v]] in the
                     // low half and ccol[crow[v] + 1] in the high half (~0u past the row's end); else null
};

struct Decision {
    int32_t L;  // the level this launch computes
    int32_t mode, vsel, prev_mode;
    double m_u, n_u;
    u64 nr, mr;  // LevelState::nr / mr with the previous launch's counters added
    u64 found;
    u64 nseg[NQS];
    u64 nh, he, mq;
};

// Decision of launch li, identical in every block: 2 = run level d.L, 1 = the BFS
// ends at this level, 0 = it ended before. The counter / state rings are indexed
// by launch, not by level, since one launch may run several levels (small_levels):
// launch li reads C[(li + 2) % 3] and S[(li + 1) % 2], accumulates into C[li % 3],
// publishes S[li % 2] and zeroes C[(li + 1) % 3] -- none of which it reads.
__device__ __forceinline__ int decide(const BfsArgs& a, int32_t li, Decision& d) {
    const LevelState& ps = a.S[(li + 1) & 1];
    const LevelCnt& pc = a.C[(li + 2) % 3];
    const int32_t L = ps.level + 1;
    d.L = L;
    d.mode = ps.mode;
    d.prev_mode = ps.mode;
    d.vsel = ps.vsel;
    d.m_u = ps.m_u;
    d.n_u = ps.n_u;
    d.found = ps.prev_found;
    d.nh = d.he = d.mq = 0;
    d.nr = ps.nr;
    d.mr = ps.mr;
    if (ps.done) return 0;
    u64 nn = 0;
#pragma unroll
    for (int k = 0; k < NQS; ++k) {
        d.nseg[k] = pc.n_norm[k].v;
        nn += d.nseg[k];
    }
    const u64 hp = pc.hub_packed.v;
    d.nh = hp >> a.eb;
    d.he = hp & ((1ull << a.eb) - 1ull);
    u64 mq = 0, fd = 0, in = 0, fz = 0;
#pragma unroll
    for (int k = 0; k < NSH; ++k) {
        mq += pc.m_next[k];
        fd += pc.found[k];
        in += pc.in_next[k];
        fz += pc.fnz[k];
    }
    d.mq = mq;
    d.found = fd;
    d.nr += fd;
    d.mr += mq;
    d.m_u = ps.m_u - (double)in;
    d.n_u = ps.n_u - (double)fd;
    if (fz == 0 || L + 1 >= INT_INF || L >= a.max_levels) return 1;
    if (a.force == 1) d.mode = 0;
    else if (a.force == 2) d.mode = 1;
    else if (d.mode == 0) {
        // Beamer's rule (the pull's cost as every unvisited in-edge), or with hub-first in-rows,
        // where most unvisited vertices stop at their first probe, the unvisited vertices
        if ((double)mq > d.m_u / a.alpha || (a.pv > 0.0 && (double)mq > a.pv * d.n_u)) d.mode = 1;
    } else if ((double)fd < (double)a.n / a.beta && fd < ps.prev_found) {
        d.mode = 0;
    }
    // a queued frontier small enough for one workgroup stays push: a pull level costs a
    // pass over the whole visited bitmap, small_levels a few dependent loads (web-graph
    // tails, where the unvisited in-edges are few but the unvisited vertices are not)
    if (a.small && a.force == 0 && d.mode == 1 && d.prev_mode == 0 && nn + d.nh <= SMALL_N && mq <= SMALL_M)
        d.mode = 0;
    return 2;
}

struct BlockQ {
    u32 n, nh;
    u64 base, hbase;
    u32 v[QCAP];
    u32 hv[HCAP];
    u32 hdeg[HCAP];
    u64 hbeg[HCAP];
    u64 scan[NW];
};

struct Acc {
    u64 m = 0, f = 0, in = 0, fz = 0;
    u64 scan = 0;  // (pull levels, lane 0 of each wave: the wave's in-edge probes)
};

__device__ __forceinline__ void hub_direct(const BfsArgs& a, LevelCnt* cacc, int32_t L, bool ish, u32 v, u32 deg,
                                           u64 beg) {
    // staging full: publish this wave's hubs with one packed atomic
    const u64 hm = __ballot(ish);
    if (!hm) return;
    const int np = (L + 1) & 1;
    const u64 d = ish ? (u64)deg : 0ull;
    const u64 incl = wave_incl_scan(d);
    const u64 tot = __shfl(incl, 63, 64);
    const int leader = __ffsll((long long)hm) - 1;
    u64 old = 0;
    if (lane_id() == leader) old = atomicAdd(&cacc->hub_packed.v, ((u64)__popcll(hm) << a.eb) + tot);
    old = __shfl(old, leader, 64);
    if (ish) {
        const u64 hs = (old >> a.eb) + (u64)__popcll(hm & lanemask_lt());
        a.hv[np][hs] = v;
        a.hbeg[np][hs] = beg;
        a.hoff[np][hs] = (old & ((1ull << a.eb) - 1ull)) + incl - d;
    }
}

// Stage one candidate per lane (whole wave calls). KNOWN: row bounds supplied.
template <typename Off, bool SYM, bool KNOWN = false>
__device__ __forceinline__ void stage(BlockQ& q, const BfsArgs& a, LevelCnt* cacc, const Graph_d<Off>& g, int32_t L,
                                      bool pred, u32 v, u64 in_deg, Acc& acc, Off kb = 0, Off ke = 0) {
    u32 deg = 0;
    u64 beg = 0;
    if (pred) {
        Off b = kb, e = ke;
        if (!KNOWN) {
            b = g.row[v];
            e = g.row[v + 1];
        }
        deg = (u32)(e - b);
        beg = (u64)b;
        acc.m += deg;
        acc.f += 1;
        acc.fz += deg > 0;
        acc.in += SYM ? (u64)deg : in_deg;
    }
    const bool isn = pred && deg > 0 && deg <= HUBT;
    const u64 m = __ballot(isn);
    if (m) {
        const int leader = __ffsll((long long)m) - 1;
        u32 pos = 0;
        if (lane_id() == leader) pos = atomicAdd(&q.n, (u32)__popcll(m));
        pos = __shfl(pos, leader, 64) + (u32)__popcll(m & lanemask_lt());
        if (isn) q.v[pos] = v;
    }
    const bool ish = pred && deg > HUBT;
    const u64 hm = __ballot(ish);
    if (hm) {
        const int leader = __ffsll((long long)hm) - 1;
        u32 pos = 0;
        if (lane_id() == leader) pos = atomicAdd(&q.nh, (u32)__popcll(hm));
        pos = __shfl(pos, leader, 64) + (u32)__popcll(hm & lanemask_lt());
        // q.nh only grows, so every staging slot below HCAP is taken exactly once; hubs past
        // the end go straight to the global queue and flush() reads min(q.nh, HCAP). (Handing
        // a whole overflowing wave back with a subtraction let a later wave's slots land above
        // the restored count: lost hubs, seen as rare push-only mismatches on Kronecker.)
        const bool fits = pos < (u32)HCAP;
        if (ish && fits) {
            q.hv[pos] = v;
            q.hdeg[pos] = deg;
            q.hbeg[pos] = beg;
        }
        const bool over = ish && !fits;
        if (__ballot(over)) hub_direct(a, cacc, L, over, v, deg, beg);
    }
}

// Block-uniform: publish everything staged (one atomic per queue).
__device__ __forceinline__ void flush(BlockQ& q, const BfsArgs& a, LevelCnt* c, int32_t L) {
    __syncthreads();
    const u32 n = q.n, nh = min(q.nh, (u32)HCAP);
    if (!(n | nh)) return;
    const int np = (L + 1) & 1;
    const u32 t = threadIdx.x;
    const int seg = blockIdx.x % NQS;
    // hub edge offsets: block scan of the staged hub degrees (one per thread, HCAP == TB)
    const u64 hd = t < nh ? (u64)q.hdeg[t] : 0ull;
    u64 tot;
    const u64 ex = block_excl_scan<NW>(hd, q.scan, tot);
    if (t == 0) {
        if (n) q.base = atomicAdd(&c->n_norm[seg].v, (u64)n);
        if (nh) q.hbase = atomicAdd(&c->hub_packed.v, ((u64)nh << a.eb) + tot);
    }
    __syncthreads();
    u32* qout = a.qv[np] + (u64)seg * (u64)a.n + q.base;
    for (u32 i = t; i < n; i += TB) qout[i] = q.v[i];
    if (t < nh) {
        const u64 hs = (q.hbase >> a.eb) + t;
        a.hv[np][hs] = q.hv[t];
        a.hbeg[np][hs] = q.hbeg[t];
        a.hoff[np][hs] = (q.hbase & ((1ull << a.eb) - 1ull)) + ex;
    }
    __syncthreads();
    if (t == 0) q.n = q.nh = 0;
    __syncthreads();
}

__device__ __forceinline__ void flush_acc(LevelCnt* c, const Acc& acc, u64* red) {
    const u64 m = block_sum<NW>(acc.m, red);
    const u64 f = block_sum<NW>(acc.f, red);
    const u64 in = block_sum<NW>(acc.in, red);
    const u64 fz = block_sum<NW>(acc.fz, red);
    const u64 sc = block_sum<NW>(acc.scan, red);
    if (threadIdx.x == 0) {
        const int sh = blockIdx.x % NSH;
        if (m) atomicAdd(&c->m_next[sh], m);
        if (f) atomicAdd(&c->found[sh], f);
        if (in) atomicAdd(&c->in_next[sh], in);
        if (fz) atomicAdd(&c->fnz[sh], fz);
        if (sc) atomicAdd(&c->scan[sh], sc);
    }
}

// claim v for level L+1 through the visited bitmap (push levels)
// prefilter (levels with at least n/4 edges): read the word first and skip the atomic
// for visited targets, most of a big level's (K22 push-only 6.97 -> 2.52 ms); smaller
// levels are latency-bound and take the atomic directly, one dependent round trip less
// (web-Google-shaped 0.233 -> 0.217 ms, K22 0.194 -> 0.184 ms per solve)
__device__ __forceinline__ bool claim(u64* vis, u32 v, bool prefilter) {
    u64* wp = vis + (v >> 6);
    const u64 bit = 1ull << (v & 63);
    if (prefilter && (*wp & bit)) return false;
    return !(atomicOr(wp, bit) & bit);
}

struct LevelShared {
    LbShared<HUB_TILE> sh;
    BlockQ q;
    u32 s_excl[TB];
    u64 s_beg[TB];
    u32 s_wex[TB];
    u64 s_fw[TB];
    u32 s_new[NW][2 * SC];
};

struct SmallShared {
    u32 cv[SMALL_N];  // frontier of the current level: vertex, out-degree (>= 1), row begin
    u32 cdeg[SMALL_N];
    u64 cbeg[SMALL_N];
    u32 cex[SMALL_N];  // exclusive scan of cdeg
    u32 nv[SMALL_M];   // vertices the level claims with out-degree >= 1 (at most one per edge)
    u32 ndeg[SMALL_M];
    u64 nbeg[SMALL_M];
    u32 nn;
    u32 scan[NW];
};

// One-workgroup levels. While the frontier is small (<= SMALL_N vertices and
// <= SMALL_M edges) and the decision is push, block 0 of the launch runs the levels
// itself with the frontier in LDS: per level one edge-to-owner search in LDS, one
// column load, one claim atomic (the row loads of the claimed vertices are issued
// beside it) and the block barriers -- instead of a kernel boundary plus the
// dependent global round trips of a grid level (decision counters, queue read,
// staging and publication atomics). Small frontiers are where a web graph's BFS
// spends its first and last levels. The loop leaves the queues, counters and state
// exactly as the grid kernel would after its last level, or ends the BFS.
template <typename Off, bool SYM>
__device__ void small_levels(const BfsArgs& a, const Graph_d<Off>& g, const Decision& d, int32_t li, SmallShared& ss,
                             u64* red) {
    const u32 t = threadIdx.x;
    u64 nn = 0;
#pragma unroll
    for (int k = 0; k < NQS; ++k) nn += d.nseg[k];
    u32 F = (u32)(nn + d.nh);
    if (t < F) {  // the frontier of level d.L, from the normal segments and the hub queue
        const int cp = d.L & 1;
        u32 v;
        if (t < nn) {
            u64 r = 0, pre = 0;
            int k = 0;
#pragma unroll
            for (int j = 0; j < NQS; ++j) {  // unrolled: no dynamic index into d.nseg
                if (t >= pre && t < pre + d.nseg[j]) {
                    k = j;
                    r = t - pre;
                }
                pre += d.nseg[j];
            }
            v = a.qv[cp][(u64)k * (u64)a.n + r];
        } else {
            v = a.hv[cp][t - nn];
        }
        const Off b = g.row[v], e = g.row[v + 1];
        ss.cv[t] = v;
        ss.cdeg[t] = (u32)(e - b);
        ss.cbeg[t] = (u64)b;
    }
    u64* vis = a.vis[d.vsel];
    int32_t L = d.L;
    double m_u = d.m_u, n_u = d.n_u;
    u64 fprev = d.found, nlev = 0;
    u64 nr = d.nr, mr = d.mr;  // (plus the levels this launch consumes itself)
    for (;;) {
        __syncthreads();
        bfs_stamp(a, li, 2 + 3 * (int)nlev);
        u32 E;
        const u32 ex = block_excl_scan<NW>(t < F ? ss.cdeg[t] : 0u, ss.scan, E);
        ss.cex[t] = ex;
        if (t == 0) *a.wtot += E;  // (the level walks every frontier out-edge)
        if (t == 0) ss.nn = 0;
        __syncthreads();
        u32 vv[SEPT];
        bool ok[SEPT];
#pragma unroll
        for (u32 k = 0; k < SEPT; ++k) {
            const u32 e = k * TB + t;
            ok[k] = e < E;
            vv[k] = 0;
            if (ok[k]) {
                u32 lo = 0;  // owner: last entry with cex <= e (degrees >= 1: cex ascends strictly)
#pragma unroll
                for (u32 step = SMALL_N / 2; step > 0; step >>= 1)
                    if (lo + step < F && ss.cex[lo + step] <= e) lo += step;
                vv[k] = g.col[ss.cbeg[lo] + (e - ss.cex[lo])];
            }
        }
        bool c[SEPT];
        Off rb[SEPT], re[SEPT];
        u64 ind[SEPT];
#pragma unroll
        for (u32 k = 0; k < SEPT; ++k) {
            c[k] = false;
            if (ok[k]) {
                const u64 bit = 1ull << (vv[k] & 63);
#if PJ_SMALL_WG_ATOMIC
                // block 0 is the launch's only writer of vis: workgroup scope suffices, and the
                // kernel's end publishes the words to the next launch
                const u64 old = __hip_atomic_fetch_or(vis + (vv[k] >> 6), bit, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
#else
                const u64 old = atomicOr(vis + (vv[k] >> 6), bit);
#endif
                c[k] = !(old & bit);
            }
        }
#pragma unroll
        for (u32 k = 0; k < SEPT; ++k) {  // issued beside the claims, needed only by the winners
            rb[k] = re[k] = 0;
            ind[k] = 0;
            if (ok[k]) {
                rb[k] = g.row[vv[k]];
                re[k] = g.row[vv[k] + 1];
                if (!SYM) ind[k] = (u64)(g.crow[vv[k] + 1] - g.crow[vv[k]]);
            }
        }
        const int32_t nl = L + 1;
        Acc acc;
#pragma unroll
        for (u32 k = 0; k < SEPT; ++k) {
            const bool cl = ok[k] && c[k];
            const u32 dg = cl ? (u32)(re[k] - rb[k]) : 0u;
            if (cl) {
                a.dist[vv[k]] = nl;
                acc.f += 1;
                acc.m += dg;
                acc.fz += dg > 0;
                acc.in += SYM ? (u64)dg : ind[k];
            }
            const bool app = cl && dg > 0;
            const u64 m = __ballot(app);
            if (m) {
                const int leader = __ffsll((long long)m) - 1;
                u32 pos = 0;
                if (lane_id() == leader) pos = atomicAdd(&ss.nn, (u32)__popcll(m));
                pos = __shfl(pos, leader, 64) + (u32)__popcll(m & lanemask_lt());
                if (app) {
                    ss.nv[pos] = vv[k];
                    ss.ndeg[pos] = dg;
                    ss.nbeg[pos] = (u64)rb[k];
                }
            }
        }
        const u64 mq = block_sum<NW>(acc.m, red);
        bfs_stamp(a, li, 3 + 3 * (int)nlev);
        const u64 f = block_sum<NW>(acc.f, red);
        const u64 in = block_sum<NW>(acc.in, red);
        const u32 NF = ss.nn;  // = the level's found vertices with out-degree > 0
        bfs_stamp(a, li, 4 + 3 * (int)nlev);
        ++nlev;
        // decide() for level L + 1, from what level L would publish
        const int32_t L2 = L + 1;
        const double m_u2 = m_u - (double)in;
        const bool end = NF == 0 || L2 + 1 >= INT_INF || L2 >= a.max_levels;
        // (decide() keeps a frontier this small in push mode unless the caller forces pull)
        if (!end && a.force != 2 && NF <= SMALL_N && mq <= SMALL_M) {
            if (t < NF) {
                ss.cv[t] = ss.nv[t];
                ss.cdeg[t] = ss.ndeg[t];
                ss.cbeg[t] = ss.nbeg[t];
            }
            F = NF;
            fprev = f;
            nr += f;
            mr += mq;
            m_u = m_u2;
            n_u -= (double)f;
            L = L2;
            continue;
        }
        if (end) {  // what the grid kernel publishes when decide() ends the BFS at L2
            if (t == 0) {
                a.nmode[0] += nlev;
                LevelState& s = a.S[li & 1];
                s.mode = 0;
                s.done = 1;
                s.vsel = d.vsel;
                s.level = L2;
                s.m_u = m_u2;
                s.n_u = n_u - (double)f;
                s.prev_found = f;
                s.nr = nr + f;
                s.mr = mr + mq;
                a.host[1] = (int64_t)a.nmode[0];
                a.host[2] = (int64_t)a.nmode[1];
                a.host[3] = (int64_t)li + 1;
                a.host[4] = (int64_t)*a.wtot;
                a.host[5] = (int64_t)(nr + f);
                a.host[6] = (int64_t)(mr + mq);
                __atomic_store_n(&a.host[0], (int64_t)L2, __ATOMIC_RELEASE);
            }
            return;
        }
        // hand level L2 to the grid: its frontier into normal segment 0 and the hub queue
        // (thread t takes entries [t * SEPT, t * SEPT + SEPT), so slots keep one order),
        // level L's counters into C[li % 3], level L's state into S[li % 2]
        u32 cn = 0, ch = 0;
        u64 che = 0;
#pragma unroll
        for (u32 k = 0; k < SEPT; ++k) {
            const u32 j = t * SEPT + k;
            if (j < NF) {
                const u32 dg = ss.ndeg[j];
                if (dg <= HUBT) ++cn;
                else {
                    ++ch;
                    che += dg;
                }
            }
        }
        u32 tn, th;
        u64 the;
        u32 pn = block_excl_scan<NW>(cn, ss.scan, tn);
        u32 ph = block_excl_scan<NW>(ch, ss.scan, th);
        u64 pe = block_excl_scan<NW>(che, red, the);
        const int np = L2 & 1;
#pragma unroll
        for (u32 k = 0; k < SEPT; ++k) {
            const u32 j = t * SEPT + k;
            if (j < NF) {
                const u32 v = ss.nv[j], dg = ss.ndeg[j];
                if (dg <= HUBT) {
                    a.qv[np][pn++] = v;
                } else {
                    a.hv[np][ph] = v;
                    a.hbeg[np][ph] = ss.nbeg[j];
                    a.hoff[np][ph] = pe;
                    ++ph;
                    pe += dg;
                }
            }
        }
        if (t == 0) {
            a.nmode[0] += nlev;
            LevelCnt* c = a.C + li % 3;  // zeroed by launch li - 1
            c->n_norm[0].v = tn;
            c->hub_packed.v = ((u64)th << a.eb) | the;
            c->m_next[0] = mq;
            c->found[0] = f;
            c->in_next[0] = in;
            c->fnz[0] = NF;
            LevelState& s = a.S[li & 1];
            s.mode = 0;
            s.done = 0;
            s.vsel = d.vsel;
            s.level = L;
            s.m_u = m_u;
            s.n_u = n_u;
            s.prev_found = fprev;
            s.nr = nr;  // (level L's own counts go to C: the next launch's decide adds them)
            s.mr = mr;
        }
        return;
    }
}


template <typename Off, bool SYM>
__global__ __launch_bounds__(TB) void bfs_level_k(BfsArgs a, Graph_d<Off> g, int32_t li) {
    __shared__ union {
        LevelShared lv;
        SmallShared sm;
    } U;
    __shared__ u64 red[NW];
    Decision d;
    bfs_stamp(a, li, 0);
    const int dec = decide(a, li, d);
    bfs_stamp(a, li, 1);
    const bool go = dec == 2;
    const u32 t = threadIdx.x;
    const int32_t L = d.L;
    u64 nfr = d.nh;
#pragma unroll
    for (int k = 0; k < NQS; ++k) nfr += d.nseg[k];
    // every block reaches the same verdict: the inputs are not written by this launch
    const bool queued = d.prev_mode == 0;  // the frontier is in the queues (else in fnew)
    const bool small = go && a.small && d.mode == 0 && queued && nfr <= SMALL_N && d.mq <= SMALL_M;
    if (blockIdx.x == 0) {
        u64* zp = reinterpret_cast<u64*>(a.C + (li + 1) % 3);
        for (u32 i = t; i < sizeof(LevelCnt) / 8; i += TB) zp[i] = 0;
        if (t == 0 && dec > 0) {
            // edges scanned: the previous launch's pull probes, and this launch's push edges
            // (small levels add their own)
            const LevelCnt& pc = a.C[(li + 2) % 3];
            u64 ps = 0;
#pragma unroll
            for (int k = 0; k < NSH; ++k) ps += pc.scan[k];
            *a.wtot += ps + ((go && d.mode == 0 && !small) ? d.mq : 0ull);
        }
        if (t == 0 && a.llog && li < 64) {  // (every launch, the idle ones behind the end too)
            const LevelCnt& pc = a.C[(li + 2) % 3];
            u64 ps = 0;
#pragma unroll
            for (int k = 0; k < NSH; ++k) ps += pc.scan[k];
            u64* e = a.llog + 6 * (u64)li;
            e[0] = (u64)(int64_t)L;
            e[1] = (u64)d.mode | ((u64)(small ? 2 : dec == 2 ? (queued ? 0 : 1) : dec == 1 ? 3 : 4) << 8);
            e[2] = queued ? nfr : d.found;
            e[3] = d.mq;
            e[4] = d.found;
            e[5] = dec > 0 ? ps : 0;
        }
        if (t == 0 && !small) {
            LevelState& s = a.S[li & 1];
            s.mode = d.mode;
            s.done = go ? 0 : 1;
            s.vsel = (go && d.mode == 1) ? 1 - d.vsel : d.vsel;
            s.level = L;
            s.m_u = d.m_u;
            s.n_u = d.n_u;
            s.prev_found = d.found;
            s.nr = d.nr;
            s.mr = d.mr;
            if (go) a.nmode[d.mode] += 1;
            if (dec == 1) {
                a.host[1] = (int64_t)a.nmode[0];
                a.host[2] = (int64_t)a.nmode[1];
                a.host[3] = (int64_t)li + 1;
                a.host[4] = (int64_t)*a.wtot;
                a.host[5] = (int64_t)d.nr;
                a.host[6] = (int64_t)d.mr;
                __atomic_store_n(&a.host[0], (int64_t)L, __ATOMIC_RELEASE);
            }
        }
    }
    if (small) {
        if (blockIdx.x == 0) small_levels<Off, SYM>(a, g, d, li, U.sm, red);
        return;
    }
    if (!go) return;
    LbShared<HUB_TILE>& sh = U.lv.sh;
    BlockQ& q = U.lv.q;
    u32* s_excl = U.lv.s_excl;
    u64* s_beg = U.lv.s_beg;
    u32* s_wex = U.lv.s_wex;
    u64* s_fw = U.lv.s_fw;
    LevelCnt* cacc = a.C + li % 3;
    if (t == 0) q.n = q.nh = 0;
    const int32_t nl = L + 1;
    const int cp = L & 1;
    Acc acc;
    const int lane = lane_id();

    if (d.mode == 0) {
        u64* vis = a.vis[d.vsel];
        const bool prefilter = d.mq >= (u64)a.n / 4;  // block-uniform
        // ---- hub queue: 1024-edge tiles over monotonic edge offsets
        const u64 ntiles = (d.he + HUB_TILE - 1) / HUB_TILE;
        for (u64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
            const u64 e0 = tile * HUB_TILE;
            const u64 e1 = min(e0 + (u64)HUB_TILE, d.he);
            u64 s0;
            u32 ns;
            lb_tile_load<HUB_TILE>(a.hoff[cp], d.nh, e0, sh, s0, ns);
            bool c[HUB_TILE / TB];
            u32 vv[HUB_TILE / TB];
#pragma unroll
            for (int k = 0; k < HUB_TILE / TB; ++k) {
                const u64 e = e0 + (u64)k * TB + t;
                c[k] = false;
                vv[k] = 0;
                if (e < e1) {
                    const u32 j = lb_find<HUB_TILE>(sh, ns, e);
                    vv[k] = g.col[a.hbeg[cp][s0 + j] + (e - sh.off[j])];
                }
            }
#pragma unroll
            for (int k = 0; k < HUB_TILE / TB; ++k) {
                if (e0 + (u64)k * TB + t < e1) {
                    c[k] = claim(vis, vv[k], prefilter);
                    if (c[k]) a.dist[vv[k]] = nl;
                }
            }
#pragma unroll
            for (int k = 0; k < HUB_TILE / TB; ++k)
                stage<Off, SYM>(q, a, cacc, g, L, c[k], vv[k],
                                c[k] && !SYM ? (u64)(g.crow[vv[k] + 1] - g.crow[vv[k]]) : 0ull, acc);
            flush(q, a, cacc, L);
        }
        // Walk the edges of up to 256 frontier vertices (one per thread: deg, beg) in
        // 256-edge steps; owner of an edge = binary search over the block's degree scan.
        auto expand_group = [&](u32 deg, u64 beg) {
            s_beg[t] = beg;
            u32 tot;
            s_excl[t] = block_excl_scan<NW>(deg, reinterpret_cast<u32*>(red), tot);
            __syncthreads();
            for (u32 base = 0; base < tot; base += TB) {
                const u32 e = base + t;
                bool c = false;
                u32 v = 0;
                if (e < tot) {
                    u32 lo = 0;  // largest j with s_excl[j] <= e
#pragma unroll
                    for (u32 step = TB / 2; step > 0; step >>= 1)
                        if (s_excl[lo + step] <= e) lo += step;
                    v = g.col[s_beg[lo] + (e - s_excl[lo])];
                    c = claim(vis, v, prefilter);
                    if (c) a.dist[v] = nl;
                }
                stage<Off, SYM>(q, a, cacc, g, L, c, v, c && !SYM ? (u64)(g.crow[v + 1] - g.crow[v]) : 0ull, acc);
                __syncthreads();
                // block-uniform: tot is uniform and q.n is read after the barrier
                if (base + TB >= tot || q.n > (u32)(QCAP - TB)) flush(q, a, cacc, L);
            }
        };
        if (queued) {
            // ---- normal queue: a block takes G entries. A block walks its group's edges
            // in dependent 256-edge steps, so a small frontier in 256-entry groups would run
            // on a handful of blocks; G shrinks while the groups still fit in one pass of the grid.
            u64 nn = 0;
#pragma unroll
            for (int k = 0; k < NQS; ++k) nn += d.nseg[k];
            u32 G = TB;
            while (G > 1 && (nn + G / 2 - 1) / (G / 2) <= (u64)gridDim.x) G >>= 1;
            u64 gcount = 0, gpre[NQS];
#pragma unroll
            for (int k = 0; k < NQS; ++k) {
                gpre[k] = gcount;
                gcount += (d.nseg[k] + G - 1) / G;
            }
            for (u64 grp = blockIdx.x; grp < gcount; grp += gridDim.x) {
                int seg = 0;
                u64 sbase = 0, scount = d.nseg[0];
#pragma unroll
                for (int k = 1; k < NQS; ++k)
                    if (grp >= gpre[k]) {
                        seg = k;
                        sbase = gpre[k];
                        scount = d.nseg[k];
                    }
                const u64 i = (grp - sbase) * G + t;
                u32 deg = 0;
                u64 beg = 0;
                if (t < G && i < scount) {
                    const u32 u = a.qv[cp][(u64)seg * (u64)a.n + i];
                    const Off b = g.row[u], e = g.row[u + 1];
                    deg = (u32)(e - b);
                    beg = (u64)b;
                }
                expand_group(deg, beg);
            }
        } else {
            // ---- frontier found by the previous (pull) level, as a bitmap: a block takes
            // 256 words, ranks their bits, and expands 256 frontier vertices at a time.
            u32 WB = TB;  // words per block step, halved while the steps do not cover the grid
            while (WB > 16 && (a.nwords + WB - 1) / WB < (i64)gridDim.x) WB >>= 1;
            for (i64 wc = blockIdx.x; wc * WB < a.nwords; wc += gridDim.x) {
                const i64 w = wc * WB + t;
                const u64 fw = (t < WB && w < a.nwords) ? a.fnew[w] : 0ull;
                u32 F;
                const u32 wex = block_excl_scan<NW>((u32)__popcll(fw), reinterpret_cast<u32*>(red), F);
                s_wex[t] = wex;
                s_fw[t] = fw;
                __syncthreads();
                for (u32 fb = 0; fb < F; fb += TB) {
                    const u32 f = fb + t;
                    u32 deg = 0;
                    u64 beg = 0;
                    if (f < F) {
                        u32 lo = 0;  // word holding the f-th frontier vertex of this block
#pragma unroll
                        for (u32 step = TB / 2; step > 0; step >>= 1)
                            if (s_wex[lo + step] <= f) lo += step;
                        const u32 u = (u32)((wc * WB + lo) * 64 + select_bit(s_fw[lo], f - s_wex[lo]));
                        const Off b = g.row[u], e = g.row[u + 1];
                        deg = (u32)(e - b);
                        beg = (u64)b;
                    }
                    expand_group(deg, beg);
                }
                __syncthreads();
            }
        }
    } else {
        // ---- pull level: a wave screens SC visited words, compacts their unvisited
        // (non-isolated) vertices into lanes, and works through them RPI rounds of 64
        // at a time. Output is bitmaps only (vis_next, fnew): no queue, no block barrier.
        const u64* vis = a.vis[d.vsel];
        u64* vout = a.vis[1 - d.vsel];
        u32* newb = U.lv.s_new[wave_id()];  // found bits of the scw words, as 32-bit halves
        // words per wave task: SC, halved while the tasks do not cover the grid's waves
        // (a small graph would otherwise leave most of the chip idle)
        u32 scw = SC;
        while (scw > 1 && (a.nwords + scw - 1) / scw < (i64)gridDim.x * NW) scw >>= 1;
        const i64 nsc = (a.nwords + scw - 1) / scw;
        u32 lsc = 0;  // in-edge probes of this lane's candidates (the wave's ones, for the wave-wide scans)
        for (i64 sc = (i64)blockIdx.x * NW + wave_id(); sc < nsc; sc += (i64)gridDim.x * NW) {
            const i64 wbase = sc * scw;
            const bool mine = lane < (int)scw && wbase + lane < a.nwords;
            u64 myvis = ~0ull, mytodo = 0;
            if (mine) {
                const i64 wd = wbase + lane;
                myvis = vis[wd];
                const u64 valid = (wd == a.nwords - 1 && (a.n & 63)) ? ((1ull << (a.n & 63)) - 1ull) : ~0ull;
                mytodo = ~myvis & valid;
            }
            if (lane < 2 * SC) newb[lane] = 0;
            const u32 cnt = (u32)__popcll(mytodo);
            const u32 incl = wave_incl_scan(cnt);
            const u32 myex = incl - cnt;
            const u32 T = __shfl(incl, 63, 64);
            for (u32 r0 = 0; r0 < T; r0 += RPI * WAVE) {
                bool fnd[RPI], act[RPI];
                Off b[RPI], e[RPI], k[RPI];
                u32 v[RPI];
#pragma unroll
                for (int j = 0; j < RPI; ++j) {
                    const u32 c = r0 + (u32)j * WAVE + lane;
                    act[j] = c < T;
                    // word of candidate c: largest lane jw < SC with ex[jw] <= c
                    u32 jw = 0;
                    for (u32 step = scw / 2; step > 0; step >>= 1) {
                        const u32 x = __shfl(myex, jw + step, 64);
                        if (x <= c) jw += step;
                    }
                    const u32 ex = __shfl(myex, jw, 64);
                    const u64 tw = __shfl(mytodo, jw, 64);
                    v[j] = act[j] ? (u32)((wbase + jw) * 64 + select_bit(tw, c - ex)) : 0u;
                    fnd[j] = false;
                    b[j] = e[j] = k[j] = 0;
                }
#pragma unroll
                for (int j = 0; j < RPI; ++j)
                    if (act[j]) {
                        b[j] = g.crow[v[j]];
                        e[j] = g.crow[v[j] + 1];
                    }
                // probes, stage A: the first PB1 in-edges of every candidate (independent
                // loads); most vertices of a dense pull level find a parent here. With the
                // dense copy hf2 the candidates' ids come 8 bytes per vertex from consecutive
                // addresses, instead of one in-row start (a line of its own) per candidate.
                u32 u[RPI][PB1];
                static_assert(PB1 == 2, "hf2 holds two in-neighbours");
                if (g.hf2) {
#pragma unroll
                    for (int j = 0; j < RPI; ++j) {
                        const u64 h = act[j] ? g.hf2[v[j]] : ~0ull;
                        u[j][0] = (u32)h;
                        u[j][1] = (u32)(h >> 32);
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < RPI; ++j)
#pragma unroll
                        for (int p = 0; p < PB1; ++p) u[j][p] = (b[j] + p < e[j]) ? g.ccol[b[j] + p] : 0u;
                }
                bool open_any = false;
#pragma unroll
                for (int j = 0; j < RPI; ++j) {
#pragma unroll
                    for (int p = 0; p < PB1; ++p)
                        fnd[j] |= (b[j] + p < e[j]) && ((vis[u[j][p] >> 6] >> (u[j][p] & 63)) & 1ull);
                    k[j] = b[j] + PB1;
                    open_any |= !fnd[j] && k[j] < e[j];
                }
                // stage B: the next PB2 in-edges at once, only for candidates still open
                if (PB2 > 0 && __ballot(open_any)) {
                    u32 x[RPI][PB2 > 0 ? PB2 : 1];
#pragma unroll
                    for (int j = 0; j < RPI; ++j)
#pragma unroll
                        for (int p = 0; p < PB2; ++p)
                            x[j][p] = (!fnd[j] && k[j] + p < e[j]) ? g.ccol[k[j] + p] : 0u;
#pragma unroll
                    for (int j = 0; j < RPI; ++j) {
                        if (!fnd[j]) {
#pragma unroll
                            for (int p = 0; p < PB2; ++p)
                                fnd[j] |= (k[j] + p < e[j]) && ((vis[x[j][p] >> 6] >> (x[j][p] & 63)) & 1ull);
                            k[j] += PB2;
                        }
                    }
                }
                // serial probes up to BU_SERIAL edges: a wave-uniform loop with predicated
                // bodies (all RPI rounds advance together; no divergent loop exits)
                Off lim[RPI];
                bool go[RPI];
#pragma unroll
                for (int j = 0; j < RPI; ++j) {
                    lim[j] = (e[j] - b[j] > (Off)BU_SERIAL) ? b[j] + (Off)BU_SERIAL : e[j];
                    go[j] = !fnd[j] && k[j] < lim[j];
                }
                for (;;) {
                    bool any = false;
#pragma unroll
                    for (int j = 0; j < RPI; ++j) any |= go[j];
                    if (!__ballot(any)) break;
                    u32 y[RPI];
#pragma unroll
                    for (int j = 0; j < RPI; ++j) y[j] = go[j] ? g.ccol[k[j]] : 0u;
#pragma unroll
                    for (int j = 0; j < RPI; ++j) {
                        if (go[j]) {
                            fnd[j] = (vis[y[j] >> 6] >> (y[j] & 63)) & 1ull;
                            ++k[j];
                            go[j] = !fnd[j] && k[j] < lim[j];
                        }
                    }
                }
                // (probes so far: stage A took min(PB1, row), stage B min(PB2, rest) of the open
                // candidates, the serial loop one per step, so k - b up to the row's end)
#pragma unroll
                for (int j = 0; j < RPI; ++j) lsc += act[j] ? (u32)(min(k[j], e[j]) - b[j]) : 0u;
                // wave-cooperative scan of the long rows that are still open
#pragma unroll
                for (int j = 0; j < RPI; ++j) {
                    u64 open = __ballot(!fnd[j] && k[j] < e[j]);
                    while (open) {
                        const int l = __ffsll((long long)open) - 1;
                        open &= open - 1;
                        const Off kb = __shfl(k[j], l, 64), ke = __shfl(e[j], l, 64);
                        bool hit = false;
                        Off kk = kb;
                        for (; kk < ke; kk += 2 * WAVE) {
                            const Off k0 = kk + lane, k1 = kk + WAVE + lane;
                            const u32 u0 = k0 < ke ? g.ccol[k0] : 0u;
                            const u32 u1 = k1 < ke ? g.ccol[k1] : 0u;
                            const u64 x0 = vis[u0 >> 6], x1 = vis[u1 >> 6];
                            const bool h = (k0 < ke && ((x0 >> (u0 & 63)) & 1ull)) ||
                                           (k1 < ke && ((x1 >> (u1 & 63)) & 1ull));
                            if (__ballot(h)) {
                                hit = true;
                                break;
                            }
                        }
                        if (lane == l) {
                            fnd[j] = hit;
                            lsc += (u32)(min(kk + (Off)(2 * WAVE), ke) - kb);  // (the steps up to the hit)
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < RPI; ++j) {
                    if (fnd[j]) {
                        a.dist[v[j]] = nl;
                        atomicOr(&newb[2 * ((v[j] >> 6) - wbase) + ((v[j] >> 5) & 1)], 1u << (v[j] & 31));
                        Off rb = b[j], re = e[j];
                        if (!SYM) {
                            rb = g.row[v[j]];
                            re = g.row[v[j] + 1];
                        }
                        const u32 deg = (u32)(re - rb);
                        acc.m += deg;
                        acc.f += 1;
                        acc.fz += deg > 0;
                        acc.in += (u64)(e[j] - b[j]);
                    }
                }
            }
            if (mine) {
                const u64 mynew = (u64)newb[2 * lane] | ((u64)newb[2 * lane + 1] << 32);
                vout[wbase + lane] = myvis | mynew;
                a.fnew[wbase + lane] = mynew;
            }
        }
        acc.scan += lsc;
    }
    flush(q, a, cacc, L);
    flush_acc(cacc, acc, red);
    bfs_stamp(a, li, 63);
}

// dist := INF, vis := isolated-vertex mask, then the source; level -1's counters
// C[2] / state S[1] describe the one-vertex frontier.
template <typename Off>
__global__ __launch_bounds__(TB) void bfs_init_k(BfsArgs a, Graph_d<Off> g, const u64* __restrict__ zmask, i64 s,
                                                 double nnz, double n_live) {
    const i64 n4 = a.n / 4;
    const i64 tid = (i64)blockIdx.x * TB + threadIdx.x, nth = (i64)gridDim.x * TB;
    int4* d4 = reinterpret_cast<int4*>(a.dist);
    for (i64 i = tid; i < n4; i += nth) {
        int4 x = make_int4(INT_INF, INT_INF, INT_INF, INT_INF);
        if (i == (s >> 2)) {
            const int r = (int)(s & 3);
            if (r == 0) x.x = 0;
            else if (r == 1) x.y = 0;
            else if (r == 2) x.z = 0;
            else x.w = 0;
        }
        d4[i] = x;
    }
    for (i64 i = n4 * 4 + tid; i < a.n; i += nth) a.dist[i] = (i == s) ? 0 : INT_INF;
    for (i64 w = tid; w < a.nwords; w += nth) a.vis[0][w] = zmask[w] | (w == (s >> 6) ? 1ull << (s & 63) : 0ull);
    if (blockIdx.x == 0) {
        u64* z0 = reinterpret_cast<u64*>(a.C);
        for (u32 i = threadIdx.x; i < 3 * sizeof(LevelCnt) / 8; i += TB) z0[i] = 0;
    }
    __syncthreads();
    if (tid == 0) {
        const Off b = g.row[s], e = g.row[s + 1];
        const u32 deg = (u32)(e - b);
        LevelCnt& c = a.C[2];
        if (deg > 0 && deg <= HUBT) {
            a.qv[0][0] = (u32)s;  // segment 0
            c.n_norm[0].v = 1;
        } else if (deg > HUBT) {
            a.hv[0][0] = (u32)s;
            a.hbeg[0][0] = (u64)b;
            a.hoff[0][0] = 0;
            c.hub_packed.v = (1ull << a.eb) | (u64)deg;
        }
        c.m_next[0] = deg;
        c.found[0] = 1;
        c.fnz[0] = deg > 0;
        c.in_next[0] = (u64)(g.crow[s + 1] - g.crow[s]);
        LevelState& st = a.S[1];
        st = LevelState{};
        st.level = -1;
        st.m_u = nnz;
        st.n_u = n_live;
        a.nmode[0] = a.nmode[1] = 0;
        *a.wtot = 0;
        a.host[0] = -1;
        a.host[3] = 0;
        a.host[4] = 0;
    }
}

// Isolated vertices (no in- and no out-edges). They can never be reached, and,
// having no out-edges, never serve as the "visited in-neighbour" of a pull test,
// so they may start out marked visited. (A vertex with in-degree 0 but
// out-edges may not: it would pose as a parent without ever being reached.)
template <typename Off>
__global__ void zmask_k(const Off* __restrict__ row, const Off* __restrict__ crow, i64 n, i64 nwords,
                        u64* __restrict__ z, u64* __restrict__ nz) {
    u64 c = 0;
    for (i64 w = (i64)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += (i64)gridDim.x * blockDim.x) {
        u64 m = 0;
        for (int j = 0; j < 64; ++j) {
            const i64 v = w * 64 + j;
            if (v < n && crow[v + 1] == crow[v] && row[v + 1] == row[v]) m |= 1ull << j;
        }
        z[w] = m;
        c += (u64)__popcll(m);
    }
    c = wave_sum(c);
    if (lane_id() == 0 && c) atomicAdd(nz, c);  // (isolated vertices)
}

template <typename Off>
__global__ void reach_k(const int32_t* __restrict__ dist, i64 n, const Off* __restrict__ row,
                        u64* __restrict__ out) {
    __shared__ u64 red[NW];
    u64 c = 0, m = 0;
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) {
        if (dist[i] < INT_INF) {
            c += 1;
            m += (u64)(row[i + 1] - row[i]);
        }
    }
    c = block_sum<NW>(c, red);
    m = block_sum<NW>(m, red);
    if (threadIdx.x == 0) {
        if (c) atomicAdd(out, c);
        if (m) atomicAdd(out + 1, m);
    }
}

// Hub-first in-rows for the pull levels (option hub_first): key of in-edge k of row r =
// (r << kb) | (2^kb - 1 - bucket(in-degree of its source u)), bucket = floor(8 log2(deg + 1))
// capped at 2^kb - 1, so one stable radix sort of (key, u) lays every in-row out with its
// highest-degree in-neighbours first (ties in file order). A pull probes a row in order and
// stops at its first visited in-neighbour; the hubs are visited in the first levels.
template <typename Off>
__global__ void hub_first_keys_k(const Off* __restrict__ crow, const u32* __restrict__ ccol, i64 n, i64 nnz, int kb,
                                 u32* __restrict__ key, u32* __restrict__ val) {
    const u32 top = (1u << kb) - 1u;
    for (i64 k = (i64)blockIdx.x * blockDim.x + threadIdx.x; k < nnz; k += (i64)gridDim.x * blockDim.x) {
        i64 lo = 0, hi = n;  // the row holding entry k: largest r with crow[r] <= k
        while (hi - lo > 1) {
            const i64 mid = (lo + hi) >> 1;
            if ((i64)crow[mid] <= k) lo = mid;
            else hi = mid;
        }
        const u32 u = ccol[k];
        const u64 deg = (u64)(crow[u + 1] - crow[u]);
        const u32 b = min(top, (u32)(8.0f * log2f((float)deg + 1.0f)));
        key[k] = ((u32)lo << kb) | (top - b);
        val[k] = u;
    }
}

// hf2[v] = the first two entries of in-row v (~0u for the missing ones)
template <typename Off>
__global__ void first_in_k(const Off* __restrict__ crow, const u32* __restrict__ ccol, i64 n, u64* __restrict__ hf2) {
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x) {
        const Off b = crow[v], e = crow[v + 1];
        const u32 x0 = b < e ? ccol[b] : ~0u, x1 = b + 1 < e ? ccol[b + 1] : ~0u;
        hf2[v] = (u64)x0 | ((u64)x1 << 32);
    }
}

int edge_bits(i64 nnz) {
    int b = 1;
    while (b < 63 && ((u64)1 << b) <= (u64)nnz) ++b;
    return b;
}

}  // namespace

struct BfsWorkHolder {
    DevBuf<u32> qv[2];  // NQS segments of n entries
    DevBuf<u32> hv[2];
    DevBuf<u64> hbeg[2], hoff[2];
    DevBuf<u64> vis2;   // second visited buffer
    DevBuf<u64> zmask;  // isolated vertices
    DevBuf<u64> fnew;   // frontier bitmap written by pull levels
    DevBuf<uint8_t> ctl;  // C[3] + S[2] + nmode[2]
    int64_t* host = nullptr;  // mapped pinned host words (see BfsArgs::host)
    int64_t* host_dev = nullptr;  // their device address
    int32_t last_launches = 0;  // level launches the previous solve used: sizes the first batch
    i64 n_live = 0;             // vertices with an edge (not in zmask)
    DevBuf<u64> hf2;            // (pull_first) the first two entries of every in-row of hf2_src
    const u32* hf2_src = nullptr;
    ~BfsWorkHolder() {
        if (host) (void)hipHostFree(host);
    }
};

void delete_bfs_work(BfsWorkHolder* p) { delete p; }

namespace {

// Host wait for a level batch: spin on the mapped done word (the BFS ended) or on
// the batch's end event, instead of a blocking synchronisation whose wake-up
// costs several microseconds per solve (a web-Google solve is ~0.22 ms). After
// 0.2 s it falls back to a blocking wait, which also surfaces a failed kernel.
static void spin_wait(hipStream_t s, hipEvent_t ev, const int64_t* done) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 0;; ++it) {
        if (done && *(volatile const int64_t*)done >= 0) return;
        if ((it & 15) == 15) {
            const hipError_t e = hipEventQuery(ev);
            if (e == hipSuccess) return;
            if (e != hipErrorNotReady) PJ_HIP(e);
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
                PJ_HIP(hipStreamSynchronize(s));
                return;
            }
        }
    }
}

template <typename Off>
void bfs_run(Graph& g, BfsWorkHolder& w, i64 source) {
    Ctx& ctx = *g.ctx;
    hipStream_t s = ctx.stream;
    const i64 n = g.n;
    const i64 nwords = (n + 63) / 64;

    BfsArgs a{};
    a.n = n;
    a.nwords = nwords;
    a.eb = edge_bits(g.nnz);
    a.alpha = g.alpha;
    a.beta = g.beta;
    a.force = g.force_mode;
    a.small = g.bfs_small;
    a.max_levels = g.max_levels > 0 ? g.max_levels : INT_INF;
    a.dist = g.dist.p;
    a.vis[0] = g.visited.p;
    a.vis[1] = w.vis2.p;
    a.fnew = w.fnew.p;
    for (int i = 0; i < 2; ++i) {
        a.qv[i] = w.qv[i].p;
        a.hv[i] = w.hv[i].p;
        a.hbeg[i] = w.hbeg[i].p;
        a.hoff[i] = w.hoff[i].p;
    }
    a.C = reinterpret_cast<LevelCnt*>(w.ctl.p);
    a.S = reinterpret_cast<LevelState*>(w.ctl.p + 3 * sizeof(LevelCnt));
    a.nmode = reinterpret_cast<u64*>(w.ctl.p + 3 * sizeof(LevelCnt) + 2 * sizeof(LevelState));
    a.wtot = a.nmode + 2;
    DevBuf<u64> llog;
    if (g.level_log) {
        llog.alloc(6 * 64);
        PJ_HIP(hipMemsetAsync(llog.p, 0xFF, 6 * 64 * sizeof(u64), s));
        a.llog = llog.p;
    }
    a.host = w.host_dev;
    Graph_d<Off> gd{static_cast<const Off*>(g.row_ptr()), g.col.p, static_cast<const Off*>(g.crow_ptr()),
                    pull_ccol(g), nullptr};
    // the vertex-count rule's cost model (a pull probes ~2 in-edges per unvisited vertex) holds for
    // hub-first in-rows only: without them (option off, or nnz >= 2^32) Beamer's rule alone. On
    // Kronecker s28 (no hub-first copy) one bench root's second level pulled 1.19G in-edges in
    // 20.6 ms under it, against a 9 ms push (profiles/r06/k28_single_r6y.txt)
    a.pv = (g.hub_first && g.ccol_hf.p && gd.ccol == g.ccol_hf.p) ? g.pull_vertex : 0.0;
    if (g.pull_first && n > 0) {  // (built once per in-row order: hub_first may switch it)
        if (w.hf2_src != gd.ccol) {
            w.hf2.ensure((size_t)n);
            first_in_k<Off><<<grid_for(n, 256, (unsigned)ctx.cu_count * 8u), 256, 0, s>>>(gd.crow, gd.ccol, n, w.hf2.p);
            PJ_LAUNCH_CHECK();
            w.hf2_src = gd.ccol;
        }
        gd.hf2 = w.hf2.p;
    }
#if PJ_BFS_STAMPS
    static DevBuf<u64> stamps;
    stamps.ensure(64 * 64);
    PJ_HIP(hipMemsetAsync(stamps.p, 0, 64 * 64 * sizeof(u64), s));
    a.stamps = stamps.p;
#endif

    // workgroups per CU: 4, or 2 on small graphs (< 2^25 entries), whose levels are short and
    // latency-bound, so a smaller grid drains faster (web-Google-shaped: 0.297 -> 0.281 ms per
    // solve; Kronecker s22 is fastest at 4: tools/probe_wg_opts.py grid_per_cu=...)
    const int gpc = g.grid_per_cu > 0 ? g.grid_per_cu : (g.nnz < ((i64)1 << 25) ? 2 : 4);
    const unsigned grid = (unsigned)ctx.cu_count * (unsigned)gpc;
    auto t_host0 = std::chrono::steady_clock::now();
    PJ_HIP(hipEventRecord(g.ev0, s));
    pj_stats st{};
    const bool valid = source >= 0 && source < n;
    if (!valid) {
        if (n > 0) PJ_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(g.dist.p), INT_INF, (size_t)n, s));
    } else {
        // the done word still holds the previous solve's level count until bfs_init_k runs;
        // clear it here, or the first spin_wait sees it and ends the solve after one batch
        *(volatile int64_t*)w.host = -1;
        bfs_init_k<Off><<<grid_for(std::max(n / 4, nwords), TB, (unsigned)ctx.cu_count * 4u), TB, 0, s>>>(
            a, gd, w.zmask.p, source, (double)g.nnz, (double)w.n_live);
        PJ_LAUNCH_CHECK();
        int32_t li = 0;  // launch index (a launch runs one level, or several small ones)
        // first batch: the previous solve's launches, so a repeated solve on the same graph
        // usually needs one host check and no idle launch behind the last level
        // (bfs_spare extra launches cover a solve one level longer than the previous one
        // without a host round trip; measured slower, off by default)
        int batch = g.level_batch > 0 ? g.level_batch : std::max(2, w.last_launches + g.bfs_spare);
        // a solve that outlasts the first batch usually needs one or two more levels:
        // continue with 2, 4, 8, ... (doubling the first batch put up to a whole batch
        // of idle ~7 us launches inside the timed region: K22, 14 behind an 8-level solve)
        int next = 2;
        for (;;) {
            for (int i = 0; i < batch && li < INT_INF; ++i, ++li) {
                if (g.symmetric) bfs_level_k<Off, true><<<grid, TB, 0, s>>>(a, gd, li);
                else bfs_level_k<Off, false><<<grid, TB, 0, s>>>(a, gd, li);
                PJ_LAUNCH_CHECK();
            }
            // end event right behind this batch's last level (re-recorded per batch), so the
            // device time does not include the host's done-word round trip
            PJ_HIP(hipEventRecord(g.ev1, s));
            spin_wait(s, g.ev1, w.host);
            if (*(volatile int64_t*)w.host >= 0 || li >= INT_INF) break;
            batch = g.level_batch > 0 ? batch : next;
            next = next < 1024 ? next * 2 : next;
        }
        st.levels = *(volatile int64_t*)w.host;
        w.last_launches = (int32_t)((volatile int64_t*)w.host)[3];
    }
    if (!valid) PJ_HIP(hipEventRecord(g.ev1, s));
    spin_wait(s, g.ev1, nullptr);
    float ms = 0.f;
    PJ_HIP(hipEventElapsedTime(&ms, g.ev0, g.ev1));
    st.kernel_ms = ms;
    st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_host0).count();
    if (valid) {
        st.td_levels = ((volatile int64_t*)w.host)[1];
        st.bu_levels = ((volatile int64_t*)w.host)[2];
        // edges scanned: every record read is a u32 column id and every one probes a visited bit
        // (an 8-byte bitmap word; the N-bit bitmap stays in the L2s)
        st.scanned_edges = st.probes = ((volatile int64_t*)w.host)[4];
        st.work_bytes = 4 * st.scanned_edges + 8 * st.probes;
        // n_r and m_r from the levels' counters (what pj_reach_stats computes with a pass of its own)
        st.reached = ((volatile int64_t*)w.host)[5];
        st.reached_edges = ((volatile int64_t*)w.host)[6];
    }
    g.stats = st;
    g.have_result = true;
    if (g.level_log && valid) {  // debug: one stderr line per level launch
        std::vector<u64> h(6 * 64);
        PJ_HIP(hipMemcpy(h.data(), llog.p, h.size() * sizeof(u64), hipMemcpyDeviceToHost));
        static const char* kind[5] = {"queued", "bitmap", "small", "end", "idle"};
        for (int l = 0; l < 64 && h[6 * (size_t)l] != ~0ull; ++l) {
            const u64* e = &h[6 * (size_t)l];
            std::fprintf(stderr, "level_launch %d level %lld mode %s frontier_from %s frontier %llu frontier_edges %llu "
                         "prev_found %llu prev_scanned %llu\n", l, (long long)(int64_t)e[0], (e[1] & 255) ? "pull" : "push",
                         kind[std::min<u64>((e[1] >> 8) & 7, 4)], (unsigned long long)e[2], (unsigned long long)e[3],
                         (unsigned long long)e[4], (unsigned long long)e[5]);
        }
    }
#if PJ_BFS_STAMPS
    {  // per launch: decide, then per small level (start, edges done, counters done), block 0's end
        std::vector<u64> h(64 * 64);
        PJ_HIP(hipMemcpy(h.data(), stamps.p, h.size() * sizeof(u64), hipMemcpyDeviceToHost));
        const u64 t0 = h[0];
        for (int l = 0; l < 64 && h[(size_t)l * 64]; ++l) {
            std::fprintf(stderr, "stamps launch %d:", l);
            for (int k = 0; k < 64; ++k)
                if (h[(size_t)l * 64 + k])
                    std::fprintf(stderr, " %d@%.2f", k, (double)(h[(size_t)l * 64 + k] - t0) / 100.0);
            std::fprintf(stderr, "\n");
        }
    }
#endif
}

// the hub-first in-rows (once per graph, at the first solve that asks for them); graphs whose
// row ids leave fewer than 3 key bits keep their file-order rows
template <typename Off>
void build_hub_first(Graph& g) {
    int rb = 1;
    while (rb < 40 && ((i64)1 << rb) < g.n + 1) ++rb;
    const int kb = std::min(8, 32 - rb);
    if (g.ccol_hf.p || g.nnz == 0 || kb < 3 || g.nnz >= ((i64)1 << 32)) return;
    hipStream_t s = g.ctx->stream;
    DevBuf<u32> key((size_t)g.nnz), kalt((size_t)g.nnz), vals((size_t)g.nnz), valt((size_t)g.nnz);
    hub_first_keys_k<Off><<<grid_for(g.nnz, 256, (unsigned)g.ctx->cu_count * 16u), 256, 0, s>>>(
        static_cast<const Off*>(g.crow_ptr()), g.ccol_ptr(), g.n, g.nnz, kb, key.p, vals.p);
    PJ_LAUNCH_CHECK();
    SortWs ws;
    u32 *kr = nullptr, *vr = nullptr;
    radix_sort_pairs<u32>(key.p, kalt.p, vals.p, valt.p, g.nnz, rb + kb, ws, s, &kr, &vr);
    if (vr == vals.p) g.ccol_hf = std::move(vals);
    else g.ccol_hf = std::move(valt);
    PJ_HIP(hipStreamSynchronize(s));
}

void bfs_workspace(Graph& g) {
    const size_t n = (size_t)g.n;
    const size_t nwords = (n + 63) / 64;
    g.dist.ensure(n ? n : 1);
    g.visited.ensure(nwords ? nwords : 1);
    if (g.bfs_work) return;
    g.bfs_work.reset(new BfsWorkHolder());
    BfsWorkHolder& w = *g.bfs_work;
    for (int i = 0; i < 2; ++i) {
        w.qv[i].alloc(n ? (size_t)NQS * n : 1);
        w.hv[i].alloc(n ? n : 1);
        w.hbeg[i].alloc(n ? n : 1);
        w.hoff[i].alloc(n ? n : 1);
    }
    w.vis2.alloc(nwords ? nwords : 1);
    w.zmask.alloc(nwords ? nwords : 1);
    w.fnew.alloc(nwords ? nwords : 1);
    w.ctl.alloc(3 * sizeof(LevelCnt) + 2 * sizeof(LevelState) + 3 * sizeof(u64));  // (+ nmode[2], wtot)
    PJ_HIP(hipHostMalloc(reinterpret_cast<void**>(&w.host), 8 * sizeof(int64_t), hipHostMallocMapped));
    PJ_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&w.host_dev), w.host, 0));
    if (nwords) {
        hipStream_t s = g.ctx->stream;
        DevBuf<u64> nz(1);
        PJ_HIP(hipMemsetAsync(nz.p, 0, sizeof(u64), s));
        if (g.off64)
            zmask_k<u64><<<grid_for((i64)nwords, 256), 256, 0, s>>>(static_cast<const u64*>(g.row_ptr()),
                                                                    static_cast<const u64*>(g.crow_ptr()), g.n,
                                                                    (i64)nwords, w.zmask.p, nz.p);
        else
            zmask_k<u32><<<grid_for((i64)nwords, 256), 256, 0, s>>>(static_cast<const u32*>(g.row_ptr()),
                                                                    static_cast<const u32*>(g.crow_ptr()), g.n,
                                                                    (i64)nwords, w.zmask.p, nz.p);
        PJ_LAUNCH_CHECK();
        u64 iso = 0;
        PJ_HIP(hipMemcpyAsync(&iso, nz.p, sizeof(u64), hipMemcpyDeviceToHost, s));
        PJ_HIP(hipStreamSynchronize(s));
        w.n_live = g.n - (i64)iso;
    }
    if (!g.ev0) PJ_HIP(hipEventCreate(&g.ev0));
    if (!g.ev1) PJ_HIP(hipEventCreate(&g.ev1));
}

}  // namespace

const u32* pull_ccol(Graph& g) {
    if (!g.hub_first) return g.ccol_ptr();
    if (g.off64) build_hub_first<u64>(g);
    else build_hub_first<u32>(g);
    return g.ccol_hf.p ? g.ccol_hf.p : g.ccol_ptr();
}

void bfs_solve(Graph& g, i64 source) {
    bfs_workspace(g);
    if (g.off64) bfs_run<u64>(g, *g.bfs_work, source);
    else bfs_run<u32>(g, *g.bfs_work, source);
}

void reach_stats(Graph& g, i64* n_r, i64* m_r) {
    hipStream_t s = g.ctx->stream;
    DevBuf<u64> out(2);
    PJ_HIP(hipMemsetAsync(out.p, 0, 2 * sizeof(u64), s));
    const unsigned grid = grid_for(g.n, 256, (unsigned)g.ctx->cu_count * 8u);
    if (g.n > 0) {
        if (g.off64) reach_k<u64><<<grid, 256, 0, s>>>(g.dist.p, g.n, g.row64.p, out.p);
        else reach_k<u32><<<grid, 256, 0, s>>>(g.dist.p, g.n, g.row32.p, out.p);
        PJ_LAUNCH_CHECK();
    }
    u64 h[2];
    PJ_HIP(hipMemcpyAsync(h, out.p, sizeof(h), hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
    *n_r = (i64)h[0];
    *m_r = (i64)h[1];
}

}  // namespace pj

namespace pj {
// debug: copy both visited buffers and fnew to the host
void debug_bitmaps(Graph& g, u64* vis0, u64* vis1, u64* fnew) {
    const size_t nw = (size_t)((g.n + 63) / 64);
    if (!g.bfs_work || !nw) return;
    PJ_HIP(hipMemcpy(vis0, g.visited.p, 8 * nw, hipMemcpyDeviceToHost));
    PJ_HIP(hipMemcpy(vis1, g.bfs_work->vis2.p, 8 * nw, hipMemcpyDeviceToHost));
    PJ_HIP(hipMemcpy(fnew, g.bfs_work->fnew.p, 8 * nw, hipMemcpyDeviceToHost));
}
}  // namespace pj
