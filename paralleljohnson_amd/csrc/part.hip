// part.hip — 1D vertex-partitioned BFS, one process per GPU (SURVEY.md §8e.2,
// BASELINE.json configs[3]: Kronecker s28 across 2/4/8 MI355X).
//
// This is the GPU form of the reference's distributed layout: nn2rank /
// get_start_nn (ParallelJohnson.cpp:169-200) give each rank a contiguous
// vertex block and the scatter at :344-410 hands it the out-rows of that
// block. Here blocks are multiples of 64 vertices (owner(v) = v / block) so
// that no 64-bit visited word is shared by two ranks; partitioning is
// result-neutral.
//
// Per rank (HBM):
//   row/col     out-rows of the owned block, global column ids (u32), offsets
//               u32 or u64 (nnz_local >= 2^32)
//   crow/ccol   in-rows of the owned block (pull levels); alias row/col when the
//               graph is symmetric (Kronecker, both directions written)
//   dist[nl]    int32, PJ_INT_INF = unreached
//   vis         caller-owned (torch) replicated visited bitmap of ALL vertices,
//               world slices of bw = block/64 words; exact for the owned slice,
//               exact everywhere after the per-level all-gather of slices
//   fr / frn    own-slice bitmaps: current and next frontier
//   sent        replicated-size bitmap (world x bw words) of the remote targets this
//               rank claimed in the current push level; the pack turns it into the
//               owner-major id list and clears it. With it, the exchange buffers are
//               sized to the traffic (the ids actually sent / received, grown to the
//               largest level), not to the partition: per-rank state is the owned
//               rows + O(N/P) vertex state + three N-bit bitmaps (vis, iso, sent)
//               + the traffic (round 3: world x 8 x block u32 send regions and world x
//               block u32 send / recv buffers, ~40 N bytes per rank at every world)
//
// A level (driven by paralleljohnson_amd/partition.py):
//   push : queue := fr (vertices with out-degree >= 1), edge-balanced expansion;
//          a target is claimed with atomicOr on vis; owned targets are settled
//          at once, others are marked in `sent` and counted per owner, then packed
//          owner-major for the exchange; pj_part_apply settles the received
//          ids (claim on the owner's exact slice). This is the analogue of the
//          reference's per-owner send buffers and MPI_Alltoall(v) at :522-554.
//   pull : every unvisited owned vertex probes its in-neighbours in the exact
//          global vis snapshot (for an unvisited vertex "an in-neighbour is
//          visited" is exactly "an in-neighbour is in the frontier").
//   end  : fr := frn, own vis slice |= fr, counts (n_f, frontier with edges,
//          m_f); the driver sums them over ranks (the analogue of the
//          MPI_Allreduce termination test at :589-590) and all-gathers the vis
//          slices before pull levels.
#include <chrono>
#include <memory>
#include <cmath>
#include <thread>

#include "kron.h"
#include "lb.h"
#include "engine.h"

namespace pj {

namespace {

constexpr int TB = 256;
constexpr int NW = TB / WAVE;
constexpr int EPT = 4;              // push: edges per lane per tile
constexpr int PTILE = TB * EPT;     // push: edges per tile
constexpr int SH = 8;               // send-counter shards per owner (own 64-B lines)
constexpr int MAXW = 64;            // largest world size
constexpr int SC = 16;              // pull: visited words a wave screens at once
constexpr int PB1 = 4;              // pull: independent first probes per candidate
constexpr int BU_SERIAL = 32;       // pull: edges a lane probes alone before the wave helps
constexpr int IPT = 8;              // filter: items per thread per block

template <typename Off>
struct PartD {
    const Off* row;
    const u32* col;
    const Off* crow;
    const u32* ccol;
};

__device__ __forceinline__ bool claim(u64* vis, u32 v) {
    u64* wp = vis + (v >> 6);
    const u64 bit = 1ull << (v & 63);
    if (*wp & bit) return false;
    return !(atomicOr(wp, bit) & bit);
}

// ---------------------------------------------------------------- build ----
// Stable filter of an edge source into the local COO of one rank: entries whose
// key (src for out-rows, dst for in-rows) lies in [lo, hi) are written as
// (key - lo, other) in source order. Two passes over the same enumeration: a
// per-block count, an exclusive scan, and the write.
struct CooSrc {
    const u32* src;
    const u32* dst;
    i64 n;
    static constexpr int K = 1;
    __device__ __forceinline__ i64 items() const { return n; }
    __device__ __forceinline__ void get(u64 i, u32* s, u32* d) const {
        s[0] = src[i];
        d[0] = dst[i];
    }
};

struct KronSrc {
    int scale;
    u64 seed;
    u64 M;  // tuples
    PermKeys pk;
    static constexpr int K = 2;
    __device__ __forceinline__ i64 items() const { return (i64)M; }
    __device__ __forceinline__ void get(u64 i, u32* s, u32* d) const {
        u32 pu, pv;
        kron_tuple(scale, seed, pk, i, pu, pv);
        s[0] = pu;
        d[0] = pv;
        s[1] = pv;
        d[1] = pu;
    }
};

template <class S>
#ifndef PJ_PART_GPC
#define PJ_PART_GPC 32  // push/pull workgroups per CU (swept 4..48 on s28 at world 1: 8 -> 32 is 14.66 -> 13.80 ms, profiles/r01/part_grid_sweep.txt)
#endif
__global__ __launch_bounds__(TB) void filter_count_k(S src, bool by_dst, u64 lo, u64 hi, u32* __restrict__ bcnt) {
    __shared__ u32 red[NW];
    const i64 base = (i64)blockIdx.x * TB * IPT;
    const i64 ni = src.items();
    u32 c = 0;
    for (int k = 0; k < IPT; ++k) {
        const i64 i = base + (i64)k * TB + threadIdx.x;
        if (i < ni) {
            u32 s[S::K], d[S::K];
            src.get((u64)i, s, d);
#pragma unroll
            for (int j = 0; j < S::K; ++j) {
                const u64 key = by_dst ? d[j] : s[j];
                c += (key >= lo && key < hi);
            }
        }
    }
    const u32 tot = block_sum<NW>(c, red);
    if (threadIdx.x == 0) bcnt[blockIdx.x] = tot;
}

template <class S>
__global__ __launch_bounds__(TB) void filter_write_k(S src, bool by_dst, u64 lo, u64 hi, const u64* __restrict__ boff,
                                                     u32* __restrict__ okey, u32* __restrict__ oval) {
    __shared__ u32 red[NW];
    const i64 base = (i64)blockIdx.x * TB * IPT;
    const i64 ni = src.items();
    u64 pos = boff[blockIdx.x];
    for (int k = 0; k < IPT; ++k) {
        const i64 i = base + (i64)k * TB + threadIdx.x;
        u32 s[S::K], d[S::K];
        u32 c = 0;
        bool keep[S::K];
#pragma unroll
        for (int j = 0; j < S::K; ++j) keep[j] = false;
        if (i < ni) {
            src.get((u64)i, s, d);
#pragma unroll
            for (int j = 0; j < S::K; ++j) {
                const u64 key = by_dst ? d[j] : s[j];
                keep[j] = key >= lo && key < hi;
                c += keep[j];
            }
        }
        u32 tot;
        u64 p = pos + block_excl_scan<NW>(c, red, tot);
#pragma unroll
        for (int j = 0; j < S::K; ++j)
            if (keep[j]) {
                okey[p] = (by_dst ? d[j] : s[j]) - (u32)lo;
                oval[p] = by_dst ? s[j] : d[j];
                ++p;
            }
        pos += tot;
    }
}

// Own-slice isolated mask: no in- and no out-edges (never reached, never a
// parent), plus the padding bits past the last owned vertex. Such bits start
// out visited so that pull levels never test them.
template <typename Off>
__global__ void part_zmask_k(PartD<Off> g, i64 nl, i64 bw, u64* __restrict__ z) {
    for (i64 w = (i64)blockIdx.x * blockDim.x + threadIdx.x; w < bw; w += (i64)gridDim.x * blockDim.x) {
        u64 m = 0;
        for (int b = 0; b < 64; ++b) {
            const i64 v = w * 64 + b;
            bool iso = true;
            if (v < nl) iso = g.row[v] == g.row[v + 1] && g.crow[v] == g.crow[v + 1];
            m |= (u64)iso << b;
        }
        z[w] = m;
    }
}

// --------------------------------------------------------------- solve ----
struct PartArgs {
    i64 n, lo, nl, block, bw;
    int rank, world;
    int32_t* dist;
    u64* vis;   // world * bw words (global)
    u64* fr;    // bw
    u64* frn;   // bw
    u32* q;     // frontier queue (local ids)
    u32* qdeg;
    u64* qoff;
    u64* sent;  // world * bw: remote targets claimed by this push level
    u64* ctr;   // world * SH counters, 8 words apart (this level's remote claims per owner)
    u64* cur;   // world cursors, 8 words apart (pack)
    u64* stat;  // [0] n_f, [1] m_f, [2] frontier with out-edges, [3] queue fill, [4] bad ids, [8..8+world) packed counts
};

// dist := INF, vis := iso (global), fr = frn = 0; then the source: its vis bit
// on every rank, and on its owner dist 0 and the frn bit (end_level makes it
// the frontier of level 0).
__global__ void part_begin_k(PartArgs a, const u64* __restrict__ iso, i64 s) {
    const i64 gs = (i64)gridDim.x * blockDim.x;
    const i64 t0 = (i64)blockIdx.x * blockDim.x + threadIdx.x;
    for (i64 i = t0; i < a.nl; i += gs) a.dist[i] = INT_INF;
    for (i64 i = t0; i < (i64)a.world * a.bw; i += gs) a.vis[i] = iso[i];
    for (i64 i = t0; i < a.bw; i += gs) {
        a.fr[i] = 0;
        a.frn[i] = 0;
    }
    if (t0 < 16) a.stat[t0] = 0;
}

__global__ void part_source_k(PartArgs a, i64 s) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && s >= 0 && s < a.n) {
        a.vis[s >> 6] |= 1ull << (s & 63);
        const i64 l = s - a.lo;
        if (l >= 0 && l < a.nl) {
            a.dist[l] = 0;
            a.frn[l >> 6] |= 1ull << (l & 63);
        }
    }
}

// fr := frn, frn := 0, own vis |= fr; stat[0..2] += (n_f, m_f, frontier vertices with out-edges)
template <typename Off>
__global__ __launch_bounds__(TB) void part_end_k(PartArgs a, PartD<Off> g) {
    __shared__ u64 red[NW];
    u64 nf = 0, mf = 0, nz = 0;
    for (i64 w = (i64)blockIdx.x * TB + threadIdx.x; w < a.bw; w += (i64)gridDim.x * TB) {
        const u64 f = a.frn[w];
        a.frn[w] = 0;
        a.fr[w] = f;
        if (f) {
            a.vis[(i64)a.rank * a.bw + w] |= f;
            nf += (u64)__popcll(f);
            u64 m = f;
            while (m) {
                const int b = __ffsll((long long)m) - 1;
                m &= m - 1;
                const i64 v = w * 64 + b;
                const u64 d = (u64)(g.row[v + 1] - g.row[v]);
                mf += d;
                nz += d > 0;
            }
        }
    }
    nf = block_sum<NW>(nf, red);
    mf = block_sum<NW>(mf, red);
    nz = block_sum<NW>(nz, red);
    if (threadIdx.x == 0) {
        if (nf) atomicAdd(&a.stat[0], nf);
        if (mf) atomicAdd(&a.stat[1], mf);
        if (nz) atomicAdd(&a.stat[2], nz);
    }
}

// Push queue: frontier vertices with out-degree >= 1 (local ids) and their degrees.
template <typename Off>
__global__ __launch_bounds__(TB) void part_queue_k(PartArgs a, PartD<Off> g) {
    __shared__ u32 red[NW];
    __shared__ u64 base_s;
    for (i64 w0 = (i64)blockIdx.x * TB; w0 < a.bw; w0 += (i64)gridDim.x * TB) {
        const i64 w = w0 + threadIdx.x;
        u64 f = w < a.bw ? a.fr[w] : 0;
        // drop vertices without out-edges (the edge-balanced mapping needs >= 1 edge per slot)
        u64 keep = 0;
        for (u64 m = f; m;) {
            const int b = __ffsll((long long)m) - 1;
            m &= m - 1;
            const i64 v = w * 64 + b;
            if (g.row[v + 1] != g.row[v]) keep |= 1ull << b;
        }
        u32 tot;
        const u32 ex = block_excl_scan<NW>((u32)__popcll(keep), red, tot);
        if (threadIdx.x == 0) base_s = tot ? atomicAdd(&a.stat[3], (u64)tot) : 0;
        __syncthreads();
        u64 p = base_s + ex;
        while (keep) {
            const int b = __ffsll((long long)keep) - 1;
            keep &= keep - 1;
            const i64 v = w * 64 + b;
            a.q[p] = (u32)v;
            a.qdeg[p] = (u32)(g.row[v + 1] - g.row[v]);
            ++p;
        }
        __syncthreads();
    }
}

template <typename Off>
__global__ __launch_bounds__(TB) void part_push_k(PartArgs a, PartD<Off> g, u64 nq, u64 mq, int32_t nlev) {
    __shared__ LbShared<PTILE> sh;
    __shared__ u32 lcnt[MAXW];
    const int shard = blockIdx.x % SH;
    const u32 blk = (u32)a.block;
    for (u64 e0 = (u64)blockIdx.x * PTILE; e0 < mq; e0 += (u64)gridDim.x * PTILE) {
        u64 s0;
        u32 ns;
        lb_tile_load<PTILE>(a.qoff, nq, e0, sh, s0, ns);
        if (threadIdx.x < (u32)a.world) lcnt[threadIdx.x] = 0;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const u64 e = e0 + (u64)j * TB + threadIdx.x;
            if (e < mq) {
                const u32 slot = lb_find<PTILE>(sh, ns, e);
                const u32 u = a.q[s0 + slot];
                const u32 t = g.col[(u64)g.row[u] + (e - sh.off[slot])];
                if (claim(a.vis, t)) {
                    const u32 o = t / blk;
                    if ((int)o == a.rank) {
                        const u32 l = t - (u32)a.lo;
                        a.dist[l] = nlev;
                        atomicOr(&a.frn[l >> 6], 1ull << (l & 63));
                    } else {  // (the claim is this rank's only one of t: the bit is new)
                        atomicOr(&a.sent[t >> 6], 1ull << (t & 63));
                        atomicAdd(&lcnt[o], 1u);
                    }
                }
            }
        }
        __syncthreads();
        if (threadIdx.x < (u32)a.world) {
            const u32 c = lcnt[threadIdx.x];
            if (c) atomicAdd(&a.ctr[((u64)threadIdx.x * SH + shard) * 8], (u64)c);
        }
        __syncthreads();
    }
}

// Per-owner counts of the level's remote claims: stat[8 + o] = sum of o's shards;
// the shards and the pack cursors are cleared for the next level (one block).
__global__ void part_counts_k(PartArgs a) {
    for (int o = threadIdx.x; o < a.world; o += blockDim.x) {
        u64 c = 0;
        for (int sh = 0; sh < SH; ++sh) {
            c += a.ctr[((u64)o * SH + sh) * 8];
            a.ctr[((u64)o * SH + sh) * 8] = 0;
        }
        a.stat[8 + o] = c;
        a.cur[(u64)o * 8] = 0;
    }
}

// Pack: the `sent` bits of every remote slice become the owner-major id list
// packed = [owner 0 | owner 1 | ...] (owner offsets from stat[8 ..]); a wave takes 64
// words of one owner's slice, places its ids with one cursor atomic and clears the
// words. (Order inside an owner's segment is free: the owner settles ids in any order.)
// Only the words [wlo, wlo + span) of each owner's slice (a piece of the level, engine.h).
__global__ __launch_bounds__(TB) void part_pack_k(PartArgs a, u32* __restrict__ packed, i64 wlo, i64 span) {
    const int lane = lane_id();
    const i64 cpo = (span + 63) / 64;  // chunks per owner slice
    const i64 nch = cpo * a.world;
    for (i64 c = (i64)blockIdx.x * NW + wave_id(); c < nch; c += (i64)gridDim.x * NW) {
        const int o = (int)(c / cpo);
        if (o == a.rank) continue;  // (wave-uniform)
        const i64 wr = (c - (i64)o * cpo) * 64 + lane, wi = wlo + wr;
        u64 bits = 0;
        if (wr < span && wi < a.bw) {
            bits = a.sent[(i64)o * a.bw + wi];
            if (bits) a.sent[(i64)o * a.bw + wi] = 0;
        }
        const u32 cnt = (u32)__popcll(bits);
        const u32 incl = wave_incl_scan(cnt);
        const u32 tot = __shfl(incl, 63, 64);
        if (!tot) continue;
        u64 base = 0;
        if (lane == 63) base = atomicAdd(&a.cur[(u64)o * 8], (u64)tot);
        base = __shfl(base, 63, 64);
        u64 off = 0;  // owner o's segment start
        for (int q = 0; q < o; ++q) off += a.stat[8 + q];
        u64 p = off + base + incl - cnt;
        const u64 w0 = ((u64)((i64)o * a.bw + wi)) << 6;
        while (bits) {
            const int b = __ffsll((long long)bits) - 1;
            bits &= bits - 1;
            packed[p++] = (u32)(w0 + (u64)b);
        }
    }
}

// Per-owner claim counts of the words [wlo, wlo + span) of every remote slice (a piece):
// cnt[o] (zeroed by the caller), one atomic per (wave, owner).
__global__ __launch_bounds__(TB) void part_piece_counts_k(PartArgs a, i64 wlo, i64 span, u64* __restrict__ cnt) {
    const int lane = lane_id();
    const i64 tot = (i64)a.world * span;
    for (i64 b0 = ((i64)blockIdx.x * NW + wave_id()) * 64; b0 < tot; b0 += (i64)gridDim.x * NW * 64) {
        const i64 i = b0 + lane;
        int o = -1;
        u32 c = 0;
        if (i < tot) {
            o = (int)(i / span);
            const i64 wi = wlo + (i - (i64)o * span);
            if (o != a.rank && wi < a.bw) c = (u32)__popcll(a.sent[(i64)o * a.bw + wi]);
        }
        u64 pending = __ballot(c != 0);
        while (pending) {
            const int l = __ffsll((long long)pending) - 1;
            const int oo = __shfl(o, l, 64);
            const bool mine = c != 0 && o == oo;
            pending &= ~__ballot(mine);
            const u32 t = wave_sum(mine ? c : 0u);
            if (lane == l) atomicAdd(&cnt[oo], (u64)t);
        }
    }
}

// Settle received ids (all owned by this rank).
__global__ void part_apply_k(PartArgs a, const u32* __restrict__ recv, i64 nr, int32_t nlev) {
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < nr; i += (i64)gridDim.x * blockDim.x) {
        const u32 t = recv[i];
        const i64 l = (i64)t - a.lo;
        if (l < 0 || l >= a.nl) {
            atomicAdd(&a.stat[4], 1ull);  // not ours: exchange corrupted (reported as PJ_ERR_COMM)
            continue;
        }
        if (claim(a.vis, t)) {
            a.dist[l] = nlev;
            atomicOr(&a.frn[l >> 6], 1ull << (l & 63));
        }
    }
}

__device__ __forceinline__ bool vbit(const u64* vis, u32 u) { return (vis[u >> 6] >> (u & 63)) & 1ull; }

// Pull level over the owned slice. A wave screens SC own words, compacts their
// unvisited vertices into lanes, probes PB1 in-edges per candidate with
// independent loads, then probes serially (wave-uniform loop, predicated
// bodies) up to BU_SERIAL edges, then scans the remaining long rows with the
// whole wave. The wave owns its words: frn is written without atomics.
template <typename Off>
__global__ __launch_bounds__(TB) void part_pull_k(PartArgs a, PartD<Off> g, int32_t nlev) {
    __shared__ u32 s_new[NW][2 * SC];
    const int lane = lane_id();
    const u64* vis = a.vis;
    const i64 obase = (i64)a.rank * a.bw;
    u32* newb = s_new[wave_id()];
    const i64 nsc = (a.bw + SC - 1) / SC;
    for (i64 sc = (i64)blockIdx.x * NW + wave_id(); sc < nsc; sc += (i64)gridDim.x * NW) {
        const i64 wbase = sc * SC;
        const bool mine = lane < SC && wbase + lane < a.bw;
        u64 mytodo = 0;
        if (mine) mytodo = ~vis[obase + wbase + lane];
        if (lane < 2 * SC) newb[lane] = 0;
        const u32 cnt = (u32)__popcll(mytodo);
        const u32 incl = wave_incl_scan(cnt);
        const u32 myex = incl - cnt;
        const u32 T = __shfl(incl, 63, 64);
        for (u32 r0 = 0; r0 < T; r0 += WAVE) {
            const u32 c = r0 + lane;
            const bool act = c < T;
            u32 jw = 0;  // word of candidate c: largest lane jw < SC with ex[jw] <= c
#pragma unroll
            for (u32 step = SC / 2; step > 0; step >>= 1) {
                const u32 x = __shfl(myex, jw + step, 64);
                if (x <= c) jw += step;
            }
            const u32 ex = __shfl(myex, jw, 64);
            const u64 tw = __shfl(mytodo, jw, 64);
            const u32 v = act ? (u32)((wbase + jw) * 64 + select_bit(tw, c - ex)) : 0u;  // local id
            Off b = 0, e = 0;
            if (act) {
                b = g.crow[v];
                e = g.crow[v + 1];
            }
            bool fnd = false;
            u32 u[PB1];
#pragma unroll
            for (int p = 0; p < PB1; ++p) u[p] = (b + p < e) ? g.ccol[b + p] : 0u;
#pragma unroll
            for (int p = 0; p < PB1; ++p) fnd |= (b + p < e) && vbit(vis, u[p]);
            Off k = b + PB1;
            const Off lim = (e - b > (Off)BU_SERIAL) ? b + (Off)BU_SERIAL : e;
            bool go = !fnd && k < lim;
            while (__ballot(go)) {
                const u32 y = go ? g.ccol[k] : 0u;
                if (go) {
                    fnd = vbit(vis, y);
                    ++k;
                    go = !fnd && k < lim;
                }
            }
            u64 open = __ballot(!fnd && k < e);
            while (open) {
                const int l = __ffsll((long long)open) - 1;
                open &= open - 1;
                const Off kb = __shfl(k, l, 64), ke = __shfl(e, l, 64);
                bool hit = false;
                for (Off kk = kb; kk < ke; kk += WAVE) {
                    const Off k0 = kk + lane;
                    const u32 u0 = k0 < ke ? g.ccol[k0] : 0u;
                    const bool h = k0 < ke && vbit(vis, u0);
                    if (__ballot(h)) {
                        hit = true;
                        break;
                    }
                }
                if (lane == l) fnd = hit;
            }
            if (fnd) {
                a.dist[v] = nlev;
                atomicOr(&newb[2 * ((v >> 6) - wbase) + ((v >> 5) & 1)], 1u << (v & 31));
            }
        }
        if (mine) a.frn[wbase + lane] = (u64)newb[2 * lane] | ((u64)newb[2 * lane + 1] << 32);
    }
}

template <typename Off>
__global__ __launch_bounds__(TB) void part_reach_k(PartArgs a, PartD<Off> g) {
    __shared__ u64 red[NW];
    u64 nr = 0, mr = 0;
    for (i64 v = (i64)blockIdx.x * TB + threadIdx.x; v < a.nl; v += (i64)gridDim.x * TB)
        if (a.dist[v] < INT_INF) {
            ++nr;
            mr += (u64)(g.row[v + 1] - g.row[v]);
        }
    nr = block_sum<NW>(nr, red);
    mr = block_sum<NW>(mr, red);
    if (threadIdx.x == 0) {
        if (nr) atomicAdd(&a.stat[5], nr);
        if (mr) atomicAdd(&a.stat[6], mr);
    }
}

}  // namespace

// ------------------------------------------------------------------ host ---
struct Part {
    Ctx* ctx = nullptr;
    int rank = 0, world = 1;
    i64 n = 0, block = 64, lo = 0, hi = 0, nl = 0, bw = 1;
    i64 nnz_local = 0, nnz_in_local = 0;
    bool symmetric = false, off64 = false;
    DevBuf<u32> row32, crow32, col, ccol;
    DevBuf<u64> row64, crow64;
    DevBuf<int32_t> dist;
    DevBuf<u64> zmask, fr, frn, qoff, ctr, cur, stat, sent;
    DevBuf<u32> q, qdeg;
    PinnedBuf<u64> hstat;
    ScanWs scan;
    u64 nq = 0, mq = 0;  // push queue of the current frontier (host copy from end_level)
    i64 exch_bytes = 0;  // the engine view's send + recv buffers (sized to the largest level)
    i64 pw_lo = 0, pw_span = 0;  // the piece the next part_pack packs (span 0: the whole level)
    int32_t level = 0;
    std::unique_ptr<BfsSteps> steps;  // engine view with its own exchange buffers (lazy)
    int single_gpu = 1;               // world 1: solve with bfs.hip's single-GPU BFS (part_solve_single)
    std::unique_ptr<Graph> g1;        // (its Graph: borrows this partition's rows for each solve)
    const Comm* iso_comm = nullptr;   // transport the replicated isolated mask was gathered over
    bool iso_ok = false;
    BfsParams prm;
    // build phases (host wall seconds, each ending at a stream sync): [0] enumerate + count
    // (filter_count_k: every tuple generated, the owned ones counted), [1] enumerate + write
    // (filter_write_k), [2] radix sort of the local COO, [3] CSR bounds, [4] device
    // allocations, [5] per-solve state, [6] total, [7] device frees; [8] the slowest single
    // allocation and [9] its GB
    double bt[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
};

void delete_part(Part* p) { delete p; }

namespace {
// host wall clock since the last call, added to acc (the build phases of Part::bt)
struct PhaseClock {
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(double& acc) {
        const auto u = std::chrono::steady_clock::now();
        acc += std::chrono::duration<double>(u - t).count();
        t = u;
    }
};
// one timed device allocation (bt[4]; the slowest one in bt[8], its GB in bt[9]) and
// one timed free (bt[7]); the caller laps whatever ran before into its own phase
template <typename T>
void timed_alloc(double* bt, PhaseClock& pc, DevBuf<T>& b, size_t count) {
    const auto t0 = std::chrono::steady_clock::now();
    b.alloc(count);
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (dt > bt[8]) {
        bt[8] = dt;
        bt[9] = (double)(count * sizeof(T)) / 1e9;
    }
    pc.lap(bt[4]);
}
template <typename T>
void timed_free(double* bt, PhaseClock& pc, DevBuf<T>& b) {
    b.release();
    pc.lap(bt[7]);
}
}  // namespace

namespace {

template <typename Off>
PartD<Off> part_d(const Part& p) {
    PartD<Off> d;
    if (sizeof(Off) == 8) {
        d.row = (const Off*)p.row64.p;
        d.crow = (const Off*)(p.symmetric ? p.row64.p : p.crow64.p);
    } else {
        d.row = (const Off*)p.row32.p;
        d.crow = (const Off*)(p.symmetric ? p.row32.p : p.crow32.p);
    }
    d.col = p.col.p;
    d.ccol = p.symmetric ? p.col.p : p.ccol.p;
    return d;
}

PartArgs part_args(Part& p, u64* vis) {
    PartArgs a;
    a.n = p.n;
    a.lo = p.lo;
    a.nl = p.nl;
    a.block = p.block;
    a.bw = p.bw;
    a.rank = p.rank;
    a.world = p.world;
    a.dist = p.dist.p;
    a.vis = vis;
    a.fr = p.fr.p;
    a.frn = p.frn.p;
    a.q = p.q.p;
    a.qdeg = p.qdeg.p;
    a.qoff = p.qoff.p;
    a.sent = p.sent.p;
    a.ctr = p.ctr.p;
    a.cur = p.cur.p;
    a.stat = p.stat.p;
    return a;
}

// (on fctx's stream: the rank's own, or the context that parsed a file for every rank)
template <class S>
i64 filter_into(Part& p, Ctx& fctx, const S& src, i64 items, bool by_dst, i64 lo, i64 hi, DevBuf<u32>& key,
                DevBuf<u32>& val, PhaseClock& pc) {
    hipStream_t s = fctx.stream;
    const i64 per = (i64)TB * IPT;
    const i64 nb = (items + per - 1) / per;
    if (nb == 0) {
        key.alloc(0);
        val.alloc(0);
        return 0;
    }
    DevBuf<u32> bcnt;
    DevBuf<u64> boff;
    ScanWs ws;
    pc.lap(p.bt[0]);
    timed_alloc(p.bt, pc, bcnt, (size_t)nb);
    timed_alloc(p.bt, pc, boff, (size_t)nb + 1);
    filter_count_k<S><<<(unsigned)nb, TB, 0, s>>>(src, by_dst, (u64)lo, (u64)hi, bcnt.p);
    PJ_LAUNCH_CHECK();
    exclusive_scan_u32(bcnt.p, boff.p, nb, ws, s);
    u64 total = 0;
    PJ_HIP(hipMemcpyAsync(&total, boff.p + nb, sizeof(u64), hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
    pc.lap(p.bt[0]);
    timed_alloc(p.bt, pc, key, (size_t)total);
    timed_alloc(p.bt, pc, val, (size_t)total);
    if (total) {
        filter_write_k<S><<<(unsigned)nb, TB, 0, s>>>(src, by_dst, (u64)lo, (u64)hi, boff.p, key.p, val.p);
        PJ_LAUNCH_CHECK();
    }
    PJ_HIP(hipStreamSynchronize(s));
    pc.lap(p.bt[1]);
    timed_free(p.bt, pc, bcnt);
    timed_free(p.bt, pc, boff);
    return (i64)total;
}

// sort the local COO by key and turn it into rows [nl+1] (Off) + vals
void rows_from_local(Part& p, DevBuf<u32>& key, DevBuf<u32>& val, i64 m, DevBuf<u32>& r32, DevBuf<u64>& r64,
                     DevBuf<u32>& out, PhaseClock& pc) {
    hipStream_t s = p.ctx->stream;
    int bits = 0;
    while (bits < 32 && ((u64)1 << bits) < (u64)p.nl) ++bits;
    SortWs ws;
    DevBuf<u32> kalt, valt;
    timed_alloc(p.bt, pc, kalt, (size_t)m);
    timed_alloc(p.bt, pc, valt, (size_t)m);
    u32 *kr, *vr;
    radix_sort_pairs<u32>(key.p, kalt.p, val.p, valt.p, m, bits, ws, s, &kr, &vr);
    PJ_HIP(hipStreamSynchronize(s));
    pc.lap(p.bt[2]);
    if (p.off64) {
        timed_alloc(p.bt, pc, r64, (size_t)p.nl + 1);
        csr_bounds<u64>(kr, m, p.nl, r64.p, s);
    } else {
        timed_alloc(p.bt, pc, r32, (size_t)p.nl + 1);
        csr_bounds<u32>(kr, m, p.nl, r32.p, s);
    }
    PJ_HIP(hipStreamSynchronize(s));
    pc.lap(p.bt[3]);
    out = std::move(vr == val.p ? val : valt);
    timed_free(p.bt, pc, key);
    timed_free(p.bt, pc, val);
    timed_free(p.bt, pc, kalt);
    timed_free(p.bt, pc, valt);
    ws = SortWs();
    pc.lap(p.bt[7]);
}

// The rank's rows from its local COO (key = owned id - lo, in file order): out-rows from
// (key, val), and for a graph not known symmetric the in-rows from (ikey, ival).
void build_part_local(Part& p, DevBuf<u32>& key, DevBuf<u32>& val, i64 m, DevBuf<u32>& ikey, DevBuf<u32>& ival,
                      i64 mi, bool symmetric, PhaseClock& pc, std::chrono::steady_clock::time_point t0);

template <class S>
void build_part(Part& p, const S& src, i64 items, bool symmetric) {
    const auto t0 = std::chrono::steady_clock::now();
    PhaseClock pc;
    DevBuf<u32> key, val;
    const i64 m = filter_into(p, *p.ctx, src, items, false, p.lo, p.hi, key, val, pc);
    i64 mi = m;
    DevBuf<u32> ikey, ival;
    if (!symmetric) mi = filter_into(p, *p.ctx, src, items, true, p.lo, p.hi, ikey, ival, pc);
    build_part_local(p, key, val, m, ikey, ival, mi, symmetric, pc, t0);
}

void build_part_local(Part& p, DevBuf<u32>& key, DevBuf<u32>& val, i64 m, DevBuf<u32>& ikey, DevBuf<u32>& ival,
                      i64 mi, bool symmetric, PhaseClock& pc, std::chrono::steady_clock::time_point t0) {
    hipStream_t s = p.ctx->stream;
    p.symmetric = symmetric;
    p.nnz_local = m;
    p.nnz_in_local = mi;
    p.off64 = (u64)std::max(m, mi) > 0xFFFFFFFFull;
    rows_from_local(p, key, val, m, p.row32, p.row64, p.col, pc);
    if (!symmetric) rows_from_local(p, ikey, ival, mi, p.crow32, p.crow64, p.ccol, pc);
    // per-solve state
    p.dist.alloc((size_t)std::max<i64>(p.nl, 1));
    p.zmask.alloc((size_t)p.bw);
    p.fr.alloc((size_t)p.bw);
    p.frn.alloc((size_t)p.bw);
    p.q.alloc((size_t)std::max<i64>(p.nl, 1));
    p.qdeg.alloc((size_t)std::max<i64>(p.nl, 1));
    p.qoff.alloc((size_t)std::max<i64>(p.nl, 1) + 1);
    if (p.world > 1) {
        p.sent.alloc((size_t)p.world * (size_t)p.bw);
        PJ_HIP(hipMemsetAsync(p.sent.p, 0, p.sent.bytes(), s));
    }
    p.ctr.alloc((size_t)p.world * SH * 8);
    p.cur.alloc((size_t)p.world * 8);
    PJ_HIP(hipMemsetAsync(p.cur.p, 0, p.cur.bytes(), s));
    p.stat.alloc(64);
    p.hstat.alloc(64);
    p.scan.ensure(std::max<i64>(p.nl, 1));
    PJ_HIP(hipMemsetAsync(p.ctr.p, 0, p.ctr.bytes(), s));
    if (p.off64) part_zmask_k<u64><<<grid_for(p.bw, 256, 4096), 256, 0, s>>>(part_d<u64>(p), p.nl, p.bw, p.zmask.p);
    else part_zmask_k<u32><<<grid_for(p.bw, 256, 4096), 256, 0, s>>>(part_d<u32>(p), p.nl, p.bw, p.zmask.p);
    PJ_LAUNCH_CHECK();
    PJ_HIP(hipStreamSynchronize(s));
    pc.lap(p.bt[5]);
    p.bt[6] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

void part_geometry(Part& p, i64 n, int rank, int world) {
    if (world < 1 || world > MAXW || rank < 0 || rank >= world) throw Error(PJ_ERR_ARG, "rank/world out of range");
    p.n = n;
    p.rank = rank;
    p.world = world;
    const i64 per = (n + world - 1) / world;
    p.block = std::max<i64>(64, (per + 63) / 64 * 64);
    if ((u64)p.block * (u64)world > 0xFFFFFFFFull + 1ull) throw Error(PJ_ERR_RANGE, "too many vertices for u32 ids");
    p.bw = p.block / 64;
    p.lo = std::min<i64>((i64)rank * p.block, n);
    p.hi = std::min<i64>(p.lo + p.block, n);
    p.nl = p.hi - p.lo;
}

template <typename Off>
void end_level_impl(Part& p, u64* vis) {
    hipStream_t s = p.ctx->stream;
    PartArgs a = part_args(p, vis);
    part_end_k<Off><<<grid_for(p.bw, TB, 2048), TB, 0, s>>>(a, part_d<Off>(p));
    PJ_LAUNCH_CHECK();
}

}  // namespace

Part* part_from_kronecker(Ctx& ctx, int scale, int edgefactor, uint64_t seed, int rank, int world) {
    auto p = std::make_unique<Part>();
    p->ctx = &ctx;
    part_geometry(*p, (i64)1 << scale, rank, world);
    KronSrc ks;
    ks.scale = scale;
    ks.seed = seed;
    ks.M = (u64)edgefactor << scale;
    ks.pk = make_perm_keys(scale, seed);
    build_part(*p, ks, (i64)ks.M, true);
    return p.release();
}

// Parse once, scatter (the reference's rank 0 reads the file and scatters row blocks,
// :313-338, :344-410): the device COO on ctxs[0] is filtered into every rank's piece there
// (entries whose source, and for the in-rows whose target, the rank owns; file order kept),
// each piece is copied to its rank's GPU (peer copy, or a device copy on a shared GPU), and
// every rank builds its rows from its piece alone, the ranks in parallel (one host thread
// each). The COO is consumed.
std::vector<Part*> parts_from_coo_group(const std::vector<Ctx*>& ctxs, DevBuf<u32>& src, DevBuf<u32>& dst, i64 nnz,
                                        i64 n, bool symmetric) {
    const int world = (int)ctxs.size();
    Ctx& c0 = *ctxs[0];
    std::vector<std::unique_ptr<Part>> parts((size_t)world);
    struct Piece {
        DevBuf<u32> key, val, ikey, ival;
        i64 m = 0, mi = 0;
    };
    std::vector<Piece> pc_((size_t)world);
    std::vector<std::chrono::steady_clock::time_point> t0((size_t)world);
    CooSrc cs;
    cs.src = src.p;
    cs.dst = dst.p;
    cs.n = nnz;
    for (int r = 0; r < world; ++r) {
        parts[(size_t)r].reset(new Part());
        Part& p = *parts[(size_t)r];
        p.ctx = ctxs[(size_t)r];
        part_geometry(p, n, r, world);
        t0[(size_t)r] = std::chrono::steady_clock::now();
        PhaseClock pc;
        Piece& q = pc_[(size_t)r];
        DevBuf<u32> k0, v0, ik0, iv0;
        PJ_HIP(hipSetDevice(c0.device));
        q.m = filter_into(p, c0, cs, nnz, false, p.lo, p.hi, k0, v0, pc);
        q.mi = q.m;
        if (!symmetric) q.mi = filter_into(p, c0, cs, nnz, true, p.lo, p.hi, ik0, iv0, pc);
        if (p.ctx == &c0) {
            q.key = std::move(k0);
            q.val = std::move(v0);
            q.ikey = std::move(ik0);
            q.ival = std::move(iv0);
            continue;
        }
        PJ_HIP(hipSetDevice(p.ctx->device));
        auto ship = [&](DevBuf<u32>& from, DevBuf<u32>& to, i64 cnt) {
            to.alloc((size_t)cnt);
            if (cnt)
                PJ_HIP(hipMemcpyPeerAsync(to.p, p.ctx->device, from.p, c0.device, sizeof(u32) * (size_t)cnt,
                                          c0.stream));
        };
        ship(k0, q.key, q.m);
        ship(v0, q.val, q.m);
        if (!symmetric) {
            ship(ik0, q.ikey, q.mi);
            ship(iv0, q.ival, q.mi);
        }
        PJ_HIP(hipSetDevice(c0.device));
        PJ_HIP(hipStreamSynchronize(c0.stream));
        pc.lap(p.bt[1]);
    }
    src.release();
    dst.release();
    std::vector<std::exception_ptr> errs((size_t)world);
    std::vector<std::thread> th;
    for (int r = 0; r < world; ++r)
        th.emplace_back([&, r] {
            try {
                Part& p = *parts[(size_t)r];
                PJ_HIP(hipSetDevice(p.ctx->device));
                Piece& q = pc_[(size_t)r];
                PhaseClock pc;
                build_part_local(p, q.key, q.val, q.m, q.ikey, q.ival, q.mi, symmetric, pc, t0[(size_t)r]);
            } catch (...) {
                errs[(size_t)r] = std::current_exception();
            }
        });
    for (auto& t : th) t.join();
    for (auto& e : errs)
        if (e) std::rethrow_exception(e);
    std::vector<Part*> out;
    for (auto& p : parts) out.push_back(p.release());
    return out;
}

Part* part_from_coo(Ctx& ctx, DevBuf<u32>& src, DevBuf<u32>& dst, i64 nnz, i64 n, int rank, int world,
                    bool symmetric) {
    auto p = std::make_unique<Part>();
    p->ctx = &ctx;
    part_geometry(*p, n, rank, world);
    CooSrc cs;
    cs.src = src.p;
    cs.dst = dst.p;
    cs.n = nnz;
    build_part(*p, cs, nnz, symmetric);
    return p.release();
}

void part_info(const Part& p, i64* out) {
    out[0] = p.n;
    out[1] = p.lo;
    out[2] = p.hi;
    out[3] = p.block;
    out[4] = p.bw;
    out[5] = p.nnz_local;
    out[6] = p.symmetric;
    out[7] = p.off64;
    out[8] = p.rank;
    out[9] = p.world;
    out[10] = p.nnz_in_local;
    // device bytes of this rank: owned rows; O(N/P) vertex state; the N-bit bitmaps
    // (sent, and the engine view's replicated vis / iso); the exchange buffers
    out[11] = (i64)(p.row32.bytes() + p.row64.bytes() + p.col.bytes() + p.crow32.bytes() + p.crow64.bytes() +
                    p.ccol.bytes());
    out[12] = (i64)(p.dist.bytes() + p.zmask.bytes() + p.fr.bytes() + p.frn.bytes() + p.q.bytes() + p.qdeg.bytes() +
                    p.qoff.bytes() + p.ctr.bytes() + p.cur.bytes() + p.stat.bytes());
    out[13] = (i64)p.sent.bytes() + (p.steps ? 2 * (i64)p.world * p.bw * 8 + p.bw * 8 : 0);
    out[14] = p.exch_bytes;
    for (int k = 0; k < 10; ++k)  // build phases: microseconds ([9]: the slowest allocation's MB)
        out[15 + k] = (i64)std::llround(p.bt[k] * (k == 9 ? 1e3 : 1e6));
}

void part_zmask(Part& p, u64* out_dev) {
    PJ_HIP(hipMemcpyAsync(out_dev, p.zmask.p, sizeof(u64) * (size_t)p.bw, hipMemcpyDeviceToDevice, p.ctx->stream));
}

static void read_stats(Part& p, i64* out3) {
    hipStream_t s = p.ctx->stream;
    PJ_HIP(hipMemcpyAsync(p.hstat.p, p.stat.p, sizeof(u64) * 8, hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
    if (p.hstat.p[4]) throw Error(PJ_ERR_COMM, "received ids owned by another rank (corrupted exchange)");
    p.nq = p.hstat.p[2];
    p.mq = p.hstat.p[1];
    out3[0] = (i64)p.hstat.p[0];
    out3[1] = (i64)p.hstat.p[1];
    out3[2] = (i64)p.hstat.p[2];
    PJ_HIP(hipMemsetAsync(p.stat.p, 0, sizeof(u64) * 8, s));
}

void part_end_level(Part& p, u64* vis, i64* out3) {
    if (p.off64) end_level_impl<u64>(p, vis);
    else end_level_impl<u32>(p, vis);
    read_stats(p, out3);
}

// device-row form of part_end_level: the kernel leaves stat[0..4]; the transport
// gathers the rows; finish takes this rank's row (already on the host)
static void part_end_level_async(Part& p, u64* vis) {
    if (p.off64) end_level_impl<u64>(p, vis);
    else end_level_impl<u32>(p, vis);
}
static void part_end_level_finish(Part& p, const i64* own5) {
    if (own5[4]) throw Error(PJ_ERR_COMM, "received ids owned by another rank (corrupted exchange)");
    p.nq = (u64)own5[2];
    p.mq = (u64)own5[1];
    PJ_HIP(hipMemsetAsync(p.stat.p, 0, sizeof(u64) * 8, p.ctx->stream));
}

void part_begin(Part& p, i64 source, const u64* iso, u64* vis, i64* out3) {
    hipStream_t s = p.ctx->stream;
    PartArgs a = part_args(p, vis);
    const i64 work = std::max<i64>(p.nl, (i64)p.world * p.bw);
    part_begin_k<<<grid_for(work, 256, 8192), 256, 0, s>>>(a, iso, source);
    PJ_LAUNCH_CHECK();
    part_source_k<<<1, 64, 0, s>>>(a, source);
    PJ_LAUNCH_CHECK();
    p.level = 0;
    part_end_level(p, vis, out3);
}

// The level's remote claims (marked in `sent` by the push) as the owner-major id list;
// packed holds at least the sum of the level's counts.
void part_pack(Part& p, u64* vis, u32* packed) {
    if (p.world < 2) return;
    PartArgs a = part_args(p, vis);
    const i64 span = p.pw_span > 0 ? p.pw_span : p.bw;
    const i64 nch = (span + 63) / 64 * p.world;
    part_pack_k<<<grid_for(nch, NW, (unsigned)p.ctx->cu_count * 8), TB, 0, p.ctx->stream>>>(a, packed, p.pw_lo,
                                                                                             span);
    PJ_LAUNCH_CHECK();
    p.pw_lo = 0;  // (the next pack is a whole level unless a piece is counted first)
    p.pw_span = 0;
}

// Piece k of npieces of the level's claims (words [k bw / npieces, (k + 1) bw / npieces) of
// every remote slice): per-owner counts into counts[] and stat[8 ..], pack cursors cleared;
// the next part_pack packs this piece.
void part_piece_counts(Part& p, int k, int npieces, i64* counts) {
    hipStream_t s = p.ctx->stream;
    const i64 wlo = p.bw * k / npieces, whi = p.bw * (k + 1) / npieces;
    PJ_HIP(hipMemsetAsync(p.stat.p + 8, 0, sizeof(u64) * (size_t)p.world, s));
    PJ_HIP(hipMemsetAsync(p.cur.p, 0, p.cur.bytes(), s));
    if (whi > wlo && p.world > 1) {
        PartArgs a = part_args(p, nullptr);
        const i64 tot = (i64)p.world * (whi - wlo);
        part_piece_counts_k<<<grid_for((tot + 63) / 64, NW, (unsigned)p.ctx->cu_count * 8), TB, 0, s>>>(
            a, wlo, whi - wlo, p.stat.p + 8);
        PJ_LAUNCH_CHECK();
    }
    PJ_HIP(hipMemcpyAsync(p.hstat.p + 8, p.stat.p + 8, sizeof(u64) * (size_t)p.world, hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
    for (int o = 0; o < p.world; ++o) counts[o] = (i64)p.hstat.p[8 + o];
    p.pw_lo = wlo;
    p.pw_span = whi - wlo;
}

namespace {
template <typename Off>
void push_impl(Part& p, int level, u64* vis, u32* packed, i64* counts) {
    hipStream_t s = p.ctx->stream;
    PartArgs a = part_args(p, vis);
    if (p.nq) {
        PJ_HIP(hipMemsetAsync(p.stat.p + 3, 0, sizeof(u64), s));
        part_queue_k<Off><<<grid_for(p.bw, TB, 2048), TB, 0, s>>>(a, part_d<Off>(p));
        PJ_LAUNCH_CHECK();
        exclusive_scan_u32(p.qdeg.p, p.qoff.p, (i64)p.nq, p.scan, s);
        const u64 tiles = (p.mq + PTILE - 1) / PTILE;
        const unsigned grid = (unsigned)std::min<u64>(tiles, (u64)p.ctx->cu_count * PJ_PART_GPC);
        part_push_k<Off><<<grid, TB, 0, s>>>(a, part_d<Off>(p), p.nq, p.mq, level + 1);
        PJ_LAUNCH_CHECK();
    }
    part_counts_k<<<1, 64, 0, s>>>(a);
    PJ_LAUNCH_CHECK();
    if (packed) part_pack(p, vis, packed);
    if (!counts) return;  // device rows: the transport reads stat[8 ..] itself
    PJ_HIP(hipMemcpyAsync(p.hstat.p + 8, p.stat.p + 8, sizeof(u64) * (size_t)p.world, hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
    for (int o = 0; o < p.world; ++o) counts[o] = (i64)p.hstat.p[8 + o];
}
}  // namespace

void part_push(Part& p, int level, u64* vis, u32* packed, i64* counts) {
    if (p.off64) push_impl<u64>(p, level, vis, packed, counts);
    else push_impl<u32>(p, level, vis, packed, counts);
}

void part_apply(Part& p, int level, u64* vis, const u32* recv, i64 nr) {
    if (nr <= 0) return;
    PartArgs a = part_args(p, vis);
    part_apply_k<<<grid_for(nr, 256, 8192), 256, 0, p.ctx->stream>>>(a, recv, nr, level + 1);
    PJ_LAUNCH_CHECK();
}

void part_pull(Part& p, int level, u64* vis) {
    hipStream_t s = p.ctx->stream;
    PartArgs a = part_args(p, vis);
    const i64 nsc = (p.bw + SC - 1) / SC;
    const unsigned grid = grid_for(nsc, NW, (unsigned)p.ctx->cu_count * PJ_PART_GPC);
    if (p.off64) part_pull_k<u64><<<grid, TB, 0, s>>>(a, part_d<u64>(p), level + 1);
    else part_pull_k<u32><<<grid, TB, 0, s>>>(a, part_d<u32>(p), level + 1);
    PJ_LAUNCH_CHECK();
}

void part_reach(Part& p, i64* out2) {
    hipStream_t s = p.ctx->stream;
    PartArgs a = part_args(p, nullptr);
    PJ_HIP(hipMemsetAsync(p.stat.p + 5, 0, 2 * sizeof(u64), s));
    if (p.off64) part_reach_k<u64><<<grid_for(p.nl, TB, 4096), TB, 0, s>>>(a, part_d<u64>(p));
    else part_reach_k<u32><<<grid_for(p.nl, TB, 4096), TB, 0, s>>>(a, part_d<u32>(p));
    PJ_LAUNCH_CHECK();
    PJ_HIP(hipMemcpyAsync(p.hstat.p + 5, p.stat.p + 5, 2 * sizeof(u64), hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
    out2[0] = (i64)p.hstat.p[5];
    out2[1] = (i64)p.hstat.p[6];
}

void part_copy_dist(Part& p, int32_t* host) {
    hipStream_t s = p.ctx->stream;
    if (p.nl) PJ_HIP(hipMemcpyAsync(host, p.dist.p, sizeof(int32_t) * (size_t)p.nl, hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
}

const int32_t* part_dist_device(const Part& p) { return p.dist.p; }

// ------------------------------------------------------------ engine view ---
namespace {

// The exchange buffers are sized to the traffic: the level's counts are known (on the
// host) before the exchange, so exchange_buffers grows send / recv to the largest level
// seen so far and packs the claimed ids into send.
struct PartGpuSteps final : BfsSteps {
    Part& p;
    DevBuf<u64> vis_b, iso_b, zown_b;
    DevBuf<u32> send_b, recv_b;
    explicit PartGpuSteps(Part& part) : p(part) {
        n = p.n;
        nnz_local = p.nnz_local;
        bw = p.bw;
        block = p.block;
        rank = p.rank;
        world = p.world;
        vis_b.alloc((size_t)world * (size_t)bw);
        iso_b.alloc((size_t)world * (size_t)bw);
        zown_b.alloc((size_t)bw);
        send_b.alloc(1);
        recv_b.alloc(1);
        vis = vis_b.p;
        iso = iso_b.p;
        zown = zown_b.p;
        send = send_b.p;
        recv = recv_b.p;
    }
    hipStream_t stream() override { return p.ctx->stream; }
    void zmask() override { part_zmask(p, zown_b.p); }
    void begin(i64 source, i64* st3) override { part_begin(p, source, iso_b.p, vis_b.p, st3); }
    void push(int level, i64* counts) override { part_push(p, level, vis_b.p, nullptr, counts); }
    // growth: x1.25 of the need, but never past the cap unless the need itself is; a piece
    // (pw_span > 0) takes the cap whole, so every later piece and level fits
    size_t grow_to(i64 need) {
        const i64 cap = exchange_cap();
        i64 t = need + need / 4;
        if (cap > 0) t = std::max(need, p.pw_span > 0 ? cap : std::min(t, cap));
        return (size_t)t;
    }
    void exchange_buffers(i64 nsend, i64 nrecv) override {
        if ((size_t)nsend > send_b.n) {
            send_b.ensure(grow_to(nsend));
            send = send_b.p;
        }
        if ((size_t)nrecv > recv_b.n) {
            recv_b.ensure(grow_to(nrecv));
            recv = recv_b.p;
        }
        p.exch_bytes = (i64)(send_b.bytes() + recv_b.bytes());
        part_pack(p, vis_b.p, send_b.p);
    }
    void apply(int level, i64 nr) override { part_apply(p, level, vis_b.p, recv_b.p, nr); }
    i64 exchange_cap() override { return p.prm.xcap < 0 ? std::max<i64>(p.block / 16, 4096) : p.prm.xcap; }
    void piece_counts(int k, int npieces, i64* counts) override { part_piece_counts(p, k, npieces, counts); }
    void pull(int level) override { part_pull(p, level, vis_b.p); }
    void end_level(i64* st3) override { part_end_level(p, vis_b.p, st3); }
    const i64* counts_dev() override { return reinterpret_cast<const i64*>(p.stat.p + 8); }
    const i64* stats_dev() override { return reinterpret_cast<const i64*>(p.stat.p); }
    void end_level_async() override { part_end_level_async(p, vis_b.p); }
    void end_level_finish(const i64* own5) override { part_end_level_finish(p, own5); }
};

}  // namespace

// World 1: the one rank owns every vertex and its rows are the whole CSR (and CSC), so the
// solve is bfs.hip's -- the single-GPU path's level kernels (hub-first in-rows, the dense first
// in-neighbours, one-workgroup small levels, launch batches), not this file's level loop -- on
// a Graph that borrows the partition's row arrays and distance array for the solve (swapped in
// and out, no copy). Its workspace and derived rows stay with it for the next solve. The
// distances land in p.dist, so the gather, the reach pass and the step API see them as the
// level loop's. Option "single_gpu" 0 keeps the level loop (what every rank runs at world > 1).
void part_solve_single(Part& p, i64 source, pj_part_stats* st) {
    const auto t0 = std::chrono::steady_clock::now();
    if (!p.g1) {
        auto g = std::make_unique<Graph>();
        g->ctx = p.ctx;
        g->n = p.n;
        g->nnz = p.nnz_local;
        g->symmetric = p.symmetric;
        g->off64 = p.off64;
        p.g1 = std::move(g);
    }
    Graph& g = *p.g1;
    g.alpha = p.prm.alpha;
    g.beta = p.prm.beta;
    g.force_mode = p.prm.force;
    struct Lend {  // the partition's arrays in the Graph for the solve, back on every exit
        Part& p;
        Graph& g;
        void swap_all() {
            std::swap(p.row32, g.row32);
            std::swap(p.row64, g.row64);
            std::swap(p.col, g.col);
            std::swap(p.crow32, g.crow32);
            std::swap(p.crow64, g.crow64);
            std::swap(p.ccol, g.ccol);
            std::swap(p.dist, g.dist);
        }
        Lend(Part& pp, Graph& gg) : p(pp), g(gg) { swap_all(); }
        ~Lend() { swap_all(); }
    } lend(p, g);
    bfs_solve(g, source);
    if (st) {
        *st = pj_part_stats{};
        st->solve_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        st->levels = g.stats.levels;
        st->td_levels = g.stats.td_levels;
        st->bu_levels = g.stats.bu_levels;
        st->reached = g.stats.reached;
        st->reached_edges = g.stats.reached_edges;
    }
}
bool part_single(const Part& p) { return p.world == 1 && p.single_gpu; }
int& part_single_gpu(Part& p) { return p.single_gpu; }

BfsSteps& part_steps(Part& p) {
    if (!p.steps) p.steps.reset(new PartGpuSteps(p));
    return *p.steps;
}

BfsParams& part_params(Part& p) { return p.prm; }

const Ctx& part_ctx(const Part& p) { return *p.ctx; }

bool& part_iso_ready(Part& p, const Comm* comm) {
    if (p.iso_comm != comm) {
        p.iso_comm = comm;
        p.iso_ok = false;
    }
    return p.iso_ok;
}

void part_gather_dist(Part& p, Comm& comm, int32_t* out) {
    hipStream_t s = p.ctx->stream;
    // every rank contributes a block of int32 (padded with INT_INF past its last vertex)
    DevBuf<int32_t> own((size_t)p.block), all((size_t)p.world * (size_t)p.block);
    PJ_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(own.p), INT_INF, (size_t)p.block, s));
    if (p.nl) PJ_HIP(hipMemcpyAsync(own.p, p.dist.p, sizeof(int32_t) * (size_t)p.nl, hipMemcpyDeviceToDevice, s));
    comm.allgather(own.p, all.p, sizeof(int32_t) * (size_t)p.block, s);
    if (out && p.n) PJ_HIP(hipMemcpyAsync(out, all.p, sizeof(int32_t) * (size_t)p.n, hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
}

}  // namespace pj
