// tree.hip — shortest-path tree of a single-source solve and its Graph500-style
// validation (the reference has no counterpart: it writes
// distances only, output_vector :32-46).
//
// parent[v] = the smallest u with an edge u -> v of weight w > 0 and dist[u] + w
// == dist[v] (< PJ_INT_INF), parent[source] = source, -1 for unreached vertices.
// A reached v with no such edge is entered only through zero-weight tight edges
// from vertices of the same distance: those are parented level by level from
// the vertices parented so far (hop depth h inside the zero-weight tight
// subgraph, h = 0 for the source and every vertex with a positive tight
// in-edge): parent[v] = the smallest u with a zero-weight edge u -> v,
// dist[u] == dist[v] and h(u) == h(v) - 1. Every parent step lowers (dist, h),
// so the tree is acyclic with zero weights too; it is a function of the
// distances alone, identical for every solver path (BFS levels, delta bands,
// either direction) and for a CPU restatement.
//
// Validation (the Graph500 BFS / SSSP checks, restated for the capped int32
// distances of the reference), against the graph's CSR and the
// solve's distances:
//   root   parent[source] == source and dist[source] == 0
//   reach  parent[v] != -1 exactly when dist[v] < PJ_INT_INF
//   tree   every parent edge u -> v exists with dist[u] + w == dist[v]
//   edge   no edge u -> v with dist[u] < INF relaxes: dist[v] <= min(dist[u] + w, INF)
//   cycle  every reached vertex's parent chain ends at the source (pointer
//          jumping, ceil(log2 n) + 1 rounds)
#include "devutil.h"

namespace pj {

namespace {

constexpr int LONG_ROW = 32;  // rows longer than this are walked by the whole wave

struct TreeCnt {
    u64 reached, bad_root, bad_reach, bad_tree, bad_edge, bad_cycle;
};

// Every CSR edge u -> v of a reached row, visited once: short rows by their lane,
// long rows by the whole wave (lanes over consecutive entries). f(u, du, v, w).
// (hop != null: only the rows u with hop[u] == lvl, the frontier of a zero-weight level)
template <typename Off, bool W, typename F>
__device__ __forceinline__ void for_reached_edges(const Off* __restrict__ row, const u32* __restrict__ col,
                                                  const u32* __restrict__ wt, const int32_t* __restrict__ dist,
                                                  i64 n, F f, const u32* __restrict__ hop = nullptr, u32 lvl = 0) {
    const int lane = lane_id();
    const i64 stride = (i64)gridDim.x * blockDim.x;
    for (i64 base = (i64)blockIdx.x * blockDim.x + (threadIdx.x & ~63); base < n; base += stride) {
        const i64 u = base + lane;
        const bool ok = u < n && (!hop || hop[u] == lvl) && dist[u] < INT_INF;
        const int32_t du = ok ? dist[u] : 0;
        const Off b = ok ? row[u] : 0, e = ok ? row[u + 1] : 0;
        const bool lng = ok && e - b > (Off)LONG_ROW;
        if (ok && !lng)
            for (Off k = b; k < e; ++k) f(u, du, col[k], W ? wt[k] : 1u);
        u64 m = __ballot(lng);
        while (m) {
            const int l = __ffsll((long long)m) - 1;
            m &= m - 1;
            const Off kb = __shfl(b, l, 64), ke = __shfl(e, l, 64);
            const i64 ul = __shfl(u, l, 64);
            const int32_t dl = __shfl(du, l, 64);
            for (Off k = kb + (Off)lane; k < ke; k += WAVE) f(ul, dl, col[k], W ? wt[k] : 1u);
        }
    }
}

constexpr u32 NO_HOP = 0xffffffffu;

// positive tight edges; zflag counts the zero-weight tight edges (the second phase runs only then)
template <typename Off, bool W>
__global__ __launch_bounds__(256) void parent_k(const Off* __restrict__ row, const u32* __restrict__ col,
                                                const u32* __restrict__ wt, const int32_t* __restrict__ dist, i64 n,
                                                u32* __restrict__ par, u32* __restrict__ zflag) {
    u32 zero = 0;
    for_reached_edges<Off, W>(row, col, wt, dist, n, [&](i64 u, int32_t du, u32 v, u32 w) {
        const int32_t dv = dist[v];
        if (dv < INT_INF && (i64)du + (i64)w == (i64)dv) {
            if (w == 0) zero = 1;
            else if (par[v] > (u32)u) atomicMin(&par[v], (u32)u);
        }
    });
    if (zero) atomicOr(zflag, 1u);
}

__global__ void hop_init_k(const u32* __restrict__ par, i64 n, i64 source, u32* __restrict__ hop) {
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x)
        hop[v] = (v == source || par[v] != 0xffffffffu) ? 0u : NO_HOP;
}

// one level of the zero-weight phase: the rows u with hop[u] == lvl (only those rows'
// edges are read) parent their zero-weight tight targets that have no hop yet (every
// writer stores lvl + 1). Levels are enqueued in batches: flags is a ring of 3, level lvl
// sets flags[lvl % 3] when it parents anything, exits at once when level lvl - 1
// (flags[(lvl + 2) % 3]) parented nothing, and clears flags[(lvl + 1) % 3] for level lvl + 1.
template <typename Off>
__global__ __launch_bounds__(256) void parent_zero_k(const Off* __restrict__ row, const u32* __restrict__ col,
                                                     const u32* __restrict__ wt, const int32_t* __restrict__ dist,
                                                     i64 n, u32 lvl, u32* __restrict__ hop, u32* __restrict__ par,
                                                     u32* __restrict__ flags) {
    if (blockIdx.x == 0 && threadIdx.x == 0) flags[(lvl + 1) % 3] = 0;
    if (flags[(lvl + 2) % 3] == 0) return;  // (block-uniform)
    u32 any = 0;
    for_reached_edges<Off, true>(row, col, wt, dist, n, [&](i64 u, int32_t du, u32 v, u32 w) {
        if (w != 0 || dist[v] != du) return;
        const u32 hv = hop[v];
        if (hv != NO_HOP && hv != lvl + 1) return;
        hop[v] = lvl + 1;
        if (par[v] > (u32)u) atomicMin(&par[v], (u32)u);
        any = 1;
    }, hop, lvl);
    if (any) atomicOr(&flags[lvl % 3], 1u);
}

__global__ void parent_out_k(const u32* __restrict__ par, i64 n, i64 source, int64_t* __restrict__ out) {
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x)
        out[v] = v == source ? source : (par[v] == 0xffffffffu ? -1 : (int64_t)par[v]);
}

template <typename Off, bool W>
__global__ __launch_bounds__(256) void tree_edges_k(const Off* __restrict__ row, const u32* __restrict__ col,
                                                    const u32* __restrict__ wt, const int32_t* __restrict__ dist,
                                                    i64 n, const int64_t* __restrict__ par, u32* __restrict__ ok,
                                                    TreeCnt* __restrict__ c) {
    u64 bad = 0;
    for_reached_edges<Off, W>(row, col, wt, dist, n, [&](i64 u, int32_t du, u32 v, u32 w) {
        const int32_t dv = dist[v];
        const i64 via = (i64)du + (i64)w;
        bad += (i64)dv > (via < INT_INF ? via : (i64)INT_INF);
        if (dv < INT_INF && via == (i64)dv && par[v] == u) atomicOr(&ok[v >> 5], 1u << (v & 31));
    });
    bad = wave_sum(bad);  // (one atomic per wave: a per-thread add on one word serializes)
    if (lane_id() == 0 && bad) atomicAdd(&c->bad_edge, bad);
}

__global__ void tree_vertices_k(const int32_t* __restrict__ dist, i64 n, i64 source, const int64_t* __restrict__ par,
                                const u32* __restrict__ ok, int64_t* __restrict__ anc, TreeCnt* __restrict__ c) {
    u64 reached = 0, root = 0, reach = 0, tree = 0;
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x) {
        const int64_t p = par[v];
        const int32_t d = dist[v];
        int64_t a = -1;
        if (v == source) {
            root += p != source || d != 0;
            reached += 1;
            a = source;
        } else if (d >= INT_INF) {
            reach += p != -1;
        } else {
            reached += 1;
            if (p < 0 || p >= n || p == v) reach += 1;
            else {
                tree += !((ok[v >> 5] >> (v & 31)) & 1u);
                a = p;
            }
        }
        anc[v] = a;
    }
    reached = wave_sum(reached);
    root = wave_sum(root);
    reach = wave_sum(reach);
    tree = wave_sum(tree);
    if (lane_id() == 0) {
        if (reached) atomicAdd(&c->reached, reached);
        if (root) atomicAdd(&c->bad_root, root);
        if (reach) atomicAdd(&c->bad_reach, reach);
        if (tree) atomicAdd(&c->bad_tree, tree);
    }
}

// one pointer-jumping round: anc[v] = anc[anc[v]] (in place: any ancestor stays an ancestor)
__global__ void jump_k(int64_t* __restrict__ anc, i64 n) {
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x) {
        const int64_t a = anc[v];
        if (a >= 0) anc[v] = anc[a];
    }
}

__global__ void cycle_k(const int32_t* __restrict__ dist, const int64_t* __restrict__ anc, i64 n, i64 source,
                        TreeCnt* __restrict__ c) {
    u64 bad = 0;
    for (i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (i64)gridDim.x * blockDim.x)
        bad += dist[v] < INT_INF && v != source && anc[v] != source;
    bad = wave_sum(bad);
    if (lane_id() == 0 && bad) atomicAdd(&c->bad_cycle, bad);
}

unsigned grid_of(const Graph& g, i64 work) { return grid_for(work, 256, (unsigned)g.ctx->cu_count * 8u); }

template <typename Off, bool W>
void parent_run(Graph& g, i64 source, u32* par) {
    const Off* row = static_cast<const Off*>(g.row_ptr());
    hipStream_t s = g.ctx->stream;
    DevBuf<u32> flag(1);
    PinnedBuf<u32> hflag;
    hflag.alloc(1);
    PJ_HIP(hipMemsetAsync(flag.p, 0, sizeof(u32), s));
    parent_k<Off, W><<<grid_of(g, g.n), 256, 0, s>>>(row, g.col.p, g.w.p, g.dist.p, g.n, par, flag.p);
    PJ_LAUNCH_CHECK();
    if constexpr (W) {
        PJ_HIP(hipMemcpyAsync(hflag.p, flag.p, sizeof(u32), hipMemcpyDeviceToHost, s));
        PJ_HIP(hipStreamSynchronize(s));
        if (!hflag.p[0]) return;
        DevBuf<u32> hop((size_t)g.n), flags(3);
        hop_init_k<<<grid_of(g, g.n), 256, 0, s>>>(par, g.n, source, hop.p);
        PJ_LAUNCH_CHECK();
        const u32 f0[3] = {0, 0, 1};  // "level -1" parented something
        PJ_HIP(hipMemcpyAsync(flags.p, f0, sizeof(f0), hipMemcpyHostToDevice, s));
        // levels in batches of 8 between host checks (a level whose predecessor parented
        // nothing exits at once); ends when a level parents nothing
        for (u32 lvl = 0;;) {
            for (int b = 0; b < 8; ++b, ++lvl) {
                parent_zero_k<Off><<<grid_of(g, g.n), 256, 0, s>>>(row, g.col.p, g.w.p, g.dist.p, g.n, lvl, hop.p,
                                                                   par, flags.p);
                PJ_LAUNCH_CHECK();
            }
            PJ_HIP(hipMemcpyAsync(hflag.p, flags.p + (lvl - 1) % 3, sizeof(u32), hipMemcpyDeviceToHost, s));
            PJ_HIP(hipStreamSynchronize(s));
            if (!hflag.p[0]) break;
        }
    }
}

template <typename Off, bool W>
void edges_run(Graph& g, const int64_t* par, u32* ok, TreeCnt* c) {
    const Off* row = static_cast<const Off*>(g.row_ptr());
    tree_edges_k<Off, W><<<grid_of(g, g.n), 256, 0, g.ctx->stream>>>(row, g.col.p, g.w.p, g.dist.p, g.n, par, ok, c);
    PJ_LAUNCH_CHECK();
}

}  // namespace

void parent_tree(Graph& g, i64 source, int64_t* host_out) {
    const i64 n = g.n;
    if (n == 0) return;
    hipStream_t s = g.ctx->stream;
    DevBuf<u32> par((size_t)n);
    DevBuf<int64_t> out((size_t)n);
    PJ_HIP(hipMemsetAsync(par.p, 0xff, 4 * (size_t)n, s));
    const bool w = g.weighted;
    if (g.off64) w ? parent_run<u64, true>(g, source, par.p) : parent_run<u64, false>(g, source, par.p);
    else w ? parent_run<u32, true>(g, source, par.p) : parent_run<u32, false>(g, source, par.p);
    parent_out_k<<<grid_of(g, n), 256, 0, s>>>(par.p, n, source, out.p);
    PJ_LAUNCH_CHECK();
    PJ_HIP(hipMemcpyAsync(host_out, out.p, 8 * (size_t)n, hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
}

void validate_tree(Graph& g, i64 source, const int64_t* host_parent, pj_tree_report* rep) {
    const i64 n = g.n;
    *rep = pj_tree_report{};
    if (n == 0) return;
    hipStream_t s = g.ctx->stream;
    DevBuf<int64_t> par((size_t)n), anc((size_t)n);
    DevBuf<u32> ok((size_t)((n + 31) / 32));
    DevBuf<TreeCnt> cnt(1);
    PJ_HIP(hipMemcpyAsync(par.p, host_parent, 8 * (size_t)n, hipMemcpyHostToDevice, s));
    PJ_HIP(hipMemsetAsync(ok.p, 0, 4 * (size_t)((n + 31) / 32), s));
    PJ_HIP(hipMemsetAsync(cnt.p, 0, sizeof(TreeCnt), s));
    const bool w = g.weighted;
    if (g.off64) w ? edges_run<u64, true>(g, par.p, ok.p, cnt.p) : edges_run<u64, false>(g, par.p, ok.p, cnt.p);
    else w ? edges_run<u32, true>(g, par.p, ok.p, cnt.p) : edges_run<u32, false>(g, par.p, ok.p, cnt.p);
    const unsigned gr = grid_of(g, n);
    tree_vertices_k<<<gr, 256, 0, s>>>(g.dist.p, n, source, par.p, ok.p, anc.p, cnt.p);
    PJ_LAUNCH_CHECK();
    int rounds = 1;
    while (((i64)1 << (rounds - 1)) < n) ++rounds;  // ceil(log2 n) + 1
    for (int r = 0; r < rounds; ++r) {
        jump_k<<<gr, 256, 0, s>>>(anc.p, n);
        PJ_LAUNCH_CHECK();
    }
    cycle_k<<<gr, 256, 0, s>>>(g.dist.p, anc.p, n, source, cnt.p);
    PJ_LAUNCH_CHECK();
    TreeCnt h{};
    PJ_HIP(hipMemcpyAsync(&h, cnt.p, sizeof(h), hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
    rep->reached = (int64_t)h.reached;
    rep->bad_root = (int64_t)h.bad_root;
    rep->bad_reach = (int64_t)h.bad_reach;
    rep->bad_tree_edge = (int64_t)h.bad_tree;
    rep->bad_edge = (int64_t)h.bad_edge;
    rep->bad_cycle = (int64_t)h.bad_cycle;
}

}  // namespace pj
