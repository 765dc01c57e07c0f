// bfs.hip — unit-weight SSSP: direction-optimizing level-synchronous BFS.
//
// Replaces the reference's relaxation core (extract_local_pq :226-278 driven by
// the BSP round loop :507-594). With w == 1 (:147) the reference computes hop
// distances capped at INT_INF; the result does not depend on
// pop order, so each BFS level settles exactly the vertices the heap would
// settle at that distance.
//
// Device state (HBM):
//   dist[n]      int32, PJ_INT_INF = unreached            (the reference's sp[] :443)
//   visited      1 bit / vertex (u64 words)               (replaces the in-heap marker sp==INT_INF)
//   fcur/fnext   frontier bitmaps for pull levels
//   queue        (v, out-degree, row begin) per frontier vertex with out-degree > 0,
//                plus an exclusive scan of the degrees for edge-balanced push levels
// Push (top-down) level: every frontier edge is one work item; a 1024-edge
//   tile finds its frontier slots by binary search in LDS, so a 300K-edge hub
//   is split over ~300 workgroups. Claims use atomicOr on the visited word.
// Pull (bottom-up) level: one wave per 64-vertex visited word; lanes scan the
//   in-edges (CSC) of unvisited vertices and stop at the first parent in fcur.
//   The wave owns its visited/fnext words, so no atomics are needed.
// Switching follows Beamer's heuristic (alpha, beta).
#include <chrono>

#include "lb.h"

namespace pj {

namespace {

struct BfsCnt {
    u64 n_next;   // queue entries appended (new vertices with out-degree > 0)
    u64 m_next;   // sum of their out-degrees (edges of the next push level)
    u64 found;    // newly visited vertices
    u64 in_next;  // sum of in-degrees of newly visited vertices (Beamer's m_u bookkeeping)
};

constexpr int TB = 256;
constexpr int TD_IPT = 4;
constexpr int TD_TILE = TB * TD_IPT;

template <typename Off>
__global__ void bfs_source_k(i64 s, const Off* __restrict__ row, const Off* __restrict__ crow,
                             int32_t* __restrict__ dist, u64* __restrict__ visited, u32* __restrict__ qv,
                             u32* __restrict__ qdeg, u64* __restrict__ qbeg, BfsCnt* __restrict__ c) {
    dist[s] = 0;
    visited[s >> 6] |= 1ull << (s & 63);
    const Off b = row[s], e = row[s + 1];
    const u32 deg = (u32)(e - b);
    if (deg) {
        qv[0] = (u32)s;
        qdeg[0] = deg;
        qbeg[0] = (u64)b;
        c->n_next = 1;
        c->m_next = deg;
    }
    c->found = 1;
    c->in_next = (u64)(crow[s + 1] - crow[s]);
}

template <typename T>
__device__ __forceinline__ void block_add3(T a, T b, T c, T* lds, u64* da, u64* db, u64* dc) {
    a = block_sum<TB / WAVE>(a, lds);
    b = block_sum<TB / WAVE>(b, lds);
    c = block_sum<TB / WAVE>(c, lds);
    if (threadIdx.x == 0) {
        if (a) atomicAdd(da, (u64)a);
        if (b) atomicAdd(db, (u64)b);
        if (c) atomicAdd(dc, (u64)c);
    }
}

// Push level over `total` frontier edges.
template <typename Off, bool SYM>
__global__ __launch_bounds__(TB) void td_expand_k(const u64* __restrict__ qbeg, const u64* __restrict__ qoff,
                                                  u64 nq, u64 total, const u32* __restrict__ col,
                                                  const Off* __restrict__ row, const Off* __restrict__ crow,
                                                  u64* __restrict__ visited, int32_t* __restrict__ dist,
                                                  int32_t nl, u32* __restrict__ qv_n, u32* __restrict__ qdeg_n,
                                                  u64* __restrict__ qbeg_n, BfsCnt* __restrict__ cnt) {
    __shared__ LbShared<TD_TILE> sh;
    __shared__ u64 red[TB / WAVE];
    const int t = threadIdx.x;
    const u64 ntiles = (total + TD_TILE - 1) / TD_TILE;
    u64 my_m = 0, my_found = 0, my_in = 0;
    for (u64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const u64 e0 = tile * TD_TILE;
        const u64 e1 = min(e0 + (u64)TD_TILE, total);
        u64 s0;
        u32 ns;
        lb_tile_load<TD_TILE>(qoff, nq, e0, sh, s0, ns);
#pragma unroll
        for (int k = 0; k < TD_IPT; ++k) {
            const u64 e = e0 + (u64)k * TB + t;
            const bool valid = e < e1;
            u32 v = 0;
            bool claim = false;
            if (valid) {
                const u32 j = lb_find<TD_TILE>(sh, ns, e);
                v = col[qbeg[s0 + j] + (e - sh.off[j])];
                u64* wp = visited + (v >> 6);
                const u64 bit = 1ull << (v & 63);
                if (!(*wp & bit)) claim = !(atomicOr(wp, bit) & bit);
            }
            u32 deg = 0;
            u64 beg = 0;
            if (claim) {
                dist[v] = nl;
                const Off b = row[v], en = row[v + 1];
                deg = (u32)(en - b);
                beg = (u64)b;
                my_m += deg;
                my_found += 1;
                my_in += SYM ? (u64)deg : (u64)(crow[v + 1] - crow[v]);
            }
            const bool app = claim && deg > 0;
            const u64 slot = wave_append(app, &cnt->n_next);
            if (app) {
                qv_n[slot] = v;
                qdeg_n[slot] = deg;
                qbeg_n[slot] = beg;
            }
        }
        __syncthreads();
    }
    block_add3<u64>(my_m, my_found, my_in, red, &cnt->m_next, &cnt->found, &cnt->in_next);
}

// Pull level: one wave per 64-vertex word of the visited bitmap.
template <typename Off>
__global__ __launch_bounds__(TB) void bu_step_k(i64 n, i64 nwords, u64* __restrict__ visited,
                                                const u64* __restrict__ fcur, u64* __restrict__ fnext,
                                                const Off* __restrict__ crow, const u32* __restrict__ ccol,
                                                const Off* __restrict__ row, int32_t* __restrict__ dist,
                                                int32_t nl, u32* __restrict__ qv_n, u32* __restrict__ qdeg_n,
                                                u64* __restrict__ qbeg_n, BfsCnt* __restrict__ cnt) {
    __shared__ u64 red[TB / WAVE];
    const int lane = lane_id();
    const i64 gw0 = (i64)blockIdx.x * (TB / WAVE) + wave_id();
    const i64 gstride = (i64)gridDim.x * (TB / WAVE);
    u64 my_m = 0, my_found = 0, my_in = 0;
    for (i64 wd = gw0; wd < nwords; wd += gstride) {
        const u64 vis = visited[wd];
        const u64 valid = (wd == nwords - 1 && (n & 63)) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
        const u64 todo = ~vis & valid;
        if (todo == 0) {
            if (lane == 0) fnext[wd] = 0;
            continue;
        }
        const i64 v = wd * 64 + lane;
        bool found = false;
        Off b = 0, e = 0;
        if ((todo >> lane) & 1ull) {
            b = crow[v];
            e = crow[v + 1];
            for (Off k = b; k < e; ++k) {
                const u32 u = ccol[k];
                if ((fcur[u >> 6] >> (u & 63)) & 1ull) {
                    found = true;
                    break;
                }
            }
        }
        const u64 m = __ballot(found);
        if (lane == 0) {
            visited[wd] = vis | m;
            fnext[wd] = m;
        }
        u32 deg = 0;
        u64 beg = 0;
        if (found) {
            dist[v] = nl;
            const Off rb = row[v], re = row[v + 1];
            deg = (u32)(re - rb);
            beg = (u64)rb;
            my_m += deg;
            my_found += 1;
            my_in += (u64)(e - b);
        }
        const bool app = found && deg > 0;
        const u64 slot = wave_append(app, &cnt->n_next);
        if (app) {
            qv_n[slot] = (u32)v;
            qdeg_n[slot] = deg;
            qbeg_n[slot] = beg;
        }
    }
    block_add3<u64>(my_m, my_found, my_in, red, &cnt->m_next, &cnt->found, &cnt->in_next);
}

__global__ void q_to_bits_k(const u32* __restrict__ qv, u64 nq, u64* __restrict__ bits) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < nq; i += (u64)gridDim.x * blockDim.x) {
        const u32 v = qv[i];
        atomicOr(bits + (v >> 6), 1ull << (v & 63));
    }
}

template <typename Off>
__global__ void reach_k(const int32_t* __restrict__ dist, i64 n, const Off* __restrict__ row,
                        u64* __restrict__ out) {
    __shared__ u64 red[TB / WAVE];
    u64 c = 0, m = 0;
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) {
        if (dist[i] < INT_INF) {
            c += 1;
            m += (u64)(row[i + 1] - row[i]);
        }
    }
    c = block_sum<TB / WAVE>(c, red);
    m = block_sum<TB / WAVE>(m, red);
    if (threadIdx.x == 0) {
        if (c) atomicAdd(out, c);
        if (m) atomicAdd(out + 1, m);
    }
}

template <typename Off>
void bfs_run(Graph& g, i64 source) {
    Ctx& ctx = *g.ctx;
    hipStream_t s = ctx.stream;
    const i64 n = g.n;
    const i64 nwords = (n + 63) / 64;
    const Off* row = static_cast<const Off*>(g.row_ptr());
    const Off* crow = static_cast<const Off*>(g.crow_ptr());
    const u32* ccol = g.ccol_ptr();
    const bool sym = g.symmetric;
    BfsCnt* dcnt = reinterpret_cast<BfsCnt*>(g.counters.p);
    BfsCnt* hcnt = reinterpret_cast<BfsCnt*>(g.hcounters.p);
    const unsigned maxgrid = (unsigned)ctx.cu_count * 8u;

    auto t_host0 = std::chrono::steady_clock::now();
    PJ_HIP(hipEventRecord(g.ev0, s));
    if (n > 0) {
        PJ_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(g.dist.p), INT_INF, (size_t)n, s));
        PJ_HIP(hipMemsetAsync(g.visited.p, 0, sizeof(u64) * (size_t)nwords, s));
    }
    pj_stats st{};
    if (source >= 0 && source < n) {
        PJ_HIP(hipMemsetAsync(dcnt, 0, sizeof(BfsCnt), s));
        bfs_source_k<Off><<<1, 1, 0, s>>>(source, row, crow, g.dist.p, g.visited.p, g.qv[0].p, g.qdeg[0].p,
                                          g.qbeg[0].p, dcnt);
        PJ_LAUNCH_CHECK();
        PJ_HIP(hipMemcpyAsync(hcnt, dcnt, sizeof(BfsCnt), hipMemcpyDeviceToHost, s));
        PJ_HIP(hipStreamSynchronize(s));
        u64 nq = hcnt->n_next, mq = hcnt->m_next, nfound = hcnt->found;
        double m_u = (double)g.nnz - (double)hcnt->in_next;
        int cur = 0;
        bool bottom_up = false;
        u64 prev_found = 0;
        int32_t level = 0;
        while (nq > 0 && level + 1 < INT_INF) {
            const int32_t nl = level + 1;
            const int nx = 1 - cur;
            if (!bottom_up) {
                const bool go = g.force_mode == 2 ? true
                                : g.force_mode == 1 ? false
                                                    : (double)mq > m_u / g.alpha;
                if (go) {
                    PJ_HIP(hipMemsetAsync(g.fcur.p, 0, sizeof(u64) * (size_t)nwords, s));
                    q_to_bits_k<<<grid_for((i64)nq, 256, maxgrid), 256, 0, s>>>(g.qv[cur].p, nq, g.fcur.p);
                    PJ_LAUNCH_CHECK();
                    bottom_up = true;
                }
            } else if (g.force_mode != 2 && (double)nfound < (double)n / g.beta && nfound < prev_found) {
                bottom_up = false;
            }
            PJ_HIP(hipMemsetAsync(dcnt, 0, sizeof(BfsCnt), s));
            if (!bottom_up) {
                exclusive_scan_u32(g.qdeg[cur].p, g.qoff.p, (i64)nq, g.scan, s);
                const unsigned grid = grid_for((i64)((mq + TD_TILE - 1) / TD_TILE), 1, maxgrid);
                if (sym)
                    td_expand_k<Off, true><<<grid, TB, 0, s>>>(g.qbeg[cur].p, g.qoff.p, nq, mq, g.col.p, row, crow,
                                                               g.visited.p, g.dist.p, nl, g.qv[nx].p,
                                                               g.qdeg[nx].p, g.qbeg[nx].p, dcnt);
                else
                    td_expand_k<Off, false><<<grid, TB, 0, s>>>(g.qbeg[cur].p, g.qoff.p, nq, mq, g.col.p, row,
                                                                crow, g.visited.p, g.dist.p, nl, g.qv[nx].p,
                                                                g.qdeg[nx].p, g.qbeg[nx].p, dcnt);
                PJ_LAUNCH_CHECK();
                st.td_levels++;
            } else {
                const unsigned grid = grid_for((nwords + 3) / 4, 1, (unsigned)ctx.cu_count * 16u);
                bu_step_k<Off><<<grid, TB, 0, s>>>(n, nwords, g.visited.p, g.fcur.p, g.fnext.p, crow, ccol, row,
                                                   g.dist.p, nl, g.qv[nx].p, g.qdeg[nx].p, g.qbeg[nx].p, dcnt);
                PJ_LAUNCH_CHECK();
                std::swap(g.fcur, g.fnext);
                st.bu_levels++;
            }
            PJ_HIP(hipMemcpyAsync(hcnt, dcnt, sizeof(BfsCnt), hipMemcpyDeviceToHost, s));
            PJ_HIP(hipStreamSynchronize(s));
            prev_found = nfound;
            nq = hcnt->n_next;
            mq = hcnt->m_next;
            nfound = hcnt->found;
            m_u -= (double)hcnt->in_next;
            cur = nx;
            level = nl;
        }
        st.levels = level;
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

void bfs_workspace(Graph& g) {
    const size_t n = (size_t)g.n;
    const size_t nwords = (n + 63) / 64;
    g.dist.ensure(n ? n : 1);
    g.visited.ensure(nwords ? nwords : 1);
    g.fcur.ensure(nwords ? nwords : 1);
    g.fnext.ensure(nwords ? nwords : 1);
    for (int i = 0; i < 2; ++i) {
        g.qv[i].ensure(n ? n : 1);
        g.qdeg[i].ensure(n ? n : 1);
        g.qbeg[i].ensure(n ? n : 1);
    }
    g.qoff.ensure(n + 1);
    g.scan.ensure((i64)n);
    g.counters.ensure(16);
    if (!g.hcounters.p) g.hcounters.alloc(16);
    if (!g.ev0) PJ_HIP(hipEventCreate(&g.ev0));
    if (!g.ev1) PJ_HIP(hipEventCreate(&g.ev1));
}

}  // namespace

void bfs_solve(Graph& g, i64 source) {
    bfs_workspace(g);
    if (g.off64) bfs_run<u64>(g, source);
    else bfs_run<u32>(g, source);
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
