// delta.hip — weighted SSSP: delta-stepping with light/heavy edges.
//
// Generalises the reference's label-correcting relaxation (extract_local_pq
// :226-278, apply loop :557-573) to integer weights >= 0, keeping its output
// contract: candidates >= INT_INF are discarded and the
// result is the true distance when it is < INT_INF. The reference settles one
// vertex per heap pop; here a whole distance band [thr - delta, thr) is
// settled at once (Meyer & Sanders' delta-stepping):
//   rows are sorted by weight (graph.hip), so the light edges (w < delta) of v
//   are the prefix row[v] .. row[v] + lsplit[v];
//   near rounds : the vertices improved below thr relax their LIGHT edges,
//                 edge-balanced (lb.h tiles), dist lowered with atomicMin;
//                 improvements below thr re-enter the near queue, the rest go
//                 to the far pile (per-epoch stamp: each vertex at most once)
//   heavy pass  : when the band is stable, every vertex settled in it relaxes
//                 its HEAVY edges once (their targets land at >= thr)
//   split       : thr jumps to the first band holding a far vertex; far entries
//                 below the new thr become the near queue
// Each round / pass is one kernel; the host reads a few counters between them
// (the analogue of the reference's termination allreduce :579-593).
#include <chrono>
#include <cmath>

#include "lb.h"

namespace pj {

namespace {

struct DCnt {
    u64 n_near;   // near-queue entries appended
    u64 m_near;   // their light-edge sum
    u64 n_far;    // far-pile entries appended
    u64 min_far;  // smallest distance in the far pile (split pre-pass)
    u64 n_r;      // settled-in-band entries with heavy edges appended
    u64 m_r;      // their heavy-edge sum
    u64 pad[2];
};

constexpr int DB = 256;
constexpr int D_IPT = 4;
constexpr int D_TILE = DB * D_IPT;

struct DQueues {
    // near queue (next), band list, far pile (current epoch)
    u32 *qv, *qdeg;
    u64* qbeg;
    u32 *rv, *rdeg;
    u64* rbeg;
    u32* far;
    int32_t *st_near, *st_band, *st_far;
    int32_t round, band, epoch;
};

// v's distance just dropped below thr (or v came out of the far pile): queue its
// light edges for the next near round and, once per band, its heavy edges.
template <typename Off>
__device__ __forceinline__ void near_append(u32 v, const Off* __restrict__ row, const u32* __restrict__ lsplit,
                                            bool pred, const DQueues& q, DCnt* c, u64& m_acc, u64& h_acc) {
    u32 lc = 0, hc = 0;
    u64 beg = 0;
    bool first_in_band = false;
    if (pred) {
        const Off b = row[v], e = row[v + 1];
        lc = lsplit[v];
        hc = (u32)(e - b) - lc;
        beg = (u64)b;
        first_in_band = atomicExch(q.st_band + v, q.band) != q.band;
    }
    const bool app = pred && lc > 0;
    const u64 slot = wave_append(app, &c->n_near);
    if (app) {
        q.qv[slot] = v;
        q.qdeg[slot] = lc;
        q.qbeg[slot] = beg;
        m_acc += lc;
    }
    const bool rap = first_in_band && hc > 0;
    const u64 rslot = wave_append(rap, &c->n_r);
    if (rap) {
        q.rv[rslot] = v;
        q.rdeg[rslot] = hc;
        q.rbeg[rslot] = beg + lc;
        h_acc += hc;
    }
}

template <typename Off>
__global__ void d_source_k(i64 s, const Off* __restrict__ row, const u32* __restrict__ lsplit,
                           int32_t* __restrict__ dist, DQueues q, DCnt* __restrict__ c) {
    dist[s] = 0;
    const Off b = row[s], e = row[s + 1];
    const u32 lc = lsplit[s], hc = (u32)(e - b) - lc;
    q.st_band[s] = q.band;
    if (lc) {
        q.qv[0] = (u32)s;
        q.qdeg[0] = lc;
        q.qbeg[0] = (u64)b;
        c->n_near = 1;
        c->m_near = lc;
    }
    if (hc) {
        q.rv[0] = (u32)s;
        q.rdeg[0] = hc;
        q.rbeg[0] = (u64)b + lc;
        c->n_r = 1;
        c->m_r = hc;
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

// Relax the edges [qbeg[i], qbeg[i] + qdeg[i]) of queue entries (light edges in
// near rounds, heavy edges in the band's heavy pass), edge-balanced.
template <typename Off>
__global__ __launch_bounds__(DB) void d_relax_k(const u32* __restrict__ iv, const u64* __restrict__ ibeg,
                                                const u64* __restrict__ ioff, u64 nq, u64 total,
                                                const u32* __restrict__ col, const u32* __restrict__ wt,
                                                const Off* __restrict__ row, const u32* __restrict__ lsplit,
                                                int32_t* __restrict__ dist, int32_t thr, DQueues q,
                                                DCnt* __restrict__ cnt) {
    __shared__ LbShared<D_TILE> sh;
    __shared__ int32_t s_du[D_TILE];
    __shared__ u64 red[DB / WAVE];
    const u64 ntiles = (total + D_TILE - 1) / D_TILE;
    u64 m_acc = 0, h_acc = 0;
    for (u64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const u64 e0 = tile * D_TILE;
        const u64 e1 = min(e0 + (u64)D_TILE, total);
        u64 s0;
        u32 ns;
        lb_tile_load<D_TILE>(ioff, nq, e0, sh, s0, ns);
        for (u32 i = threadIdx.x; i < ns; i += DB) s_du[i] = dist[iv[s0 + i]];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < D_IPT; ++k) {
            const u64 e = e0 + (u64)k * DB + threadIdx.x;
            bool to_near = false, to_far = false;
            u32 v = 0;
            if (e < e1) {
                const u32 j = lb_find<D_TILE>(sh, ns, e);
                const u64 idx = ibeg[s0 + j] + (e - sh.off[j]);
                v = col[idx];
                const long long nd = (long long)s_du[j] + (long long)wt[idx];
                if (nd < INT_INF && (int32_t)nd < dist[v]) {
                    const int32_t old = atomicMin(dist + v, (int32_t)nd);
                    if ((int32_t)nd < old) {
                        if ((int32_t)nd < thr) to_near = atomicExch(q.st_near + v, q.round) != q.round;
                        else to_far = atomicExch(q.st_far + v, q.epoch) != q.epoch;
                    }
                }
            }
            near_append<Off>(v, row, lsplit, to_near, q, cnt, m_acc, h_acc);
            const u64 fslot = wave_append(to_far, &cnt->n_far);
            if (to_far) q.far[fslot] = v;
        }
        __syncthreads();
    }
    m_acc = block_sum<DB / WAVE>(m_acc, red);
    h_acc = block_sum<DB / WAVE>(h_acc, red);
    if (threadIdx.x == 0) {
        if (m_acc) atomicAdd(&cnt->m_near, m_acc);
        if (h_acc) atomicAdd(&cnt->m_r, h_acc);
    }
}

__global__ __launch_bounds__(DB) void d_far_min_k(const u32* __restrict__ far, u64 nf,
                                                  const int32_t* __restrict__ dist, int32_t thr,
                                                  DCnt* __restrict__ cnt) {
    long long mn = INT_INF;
    for (u64 i = (u64)blockIdx.x * DB + threadIdx.x; i < nf; i += (u64)gridDim.x * DB) {
        const int32_t d = dist[far[i]];
        if (d >= thr && d < mn) mn = d;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        long long y = __shfl_xor(mn, off, 64);
        mn = y < mn ? y : mn;
    }
    if (lane_id() == 0 && mn < INT_INF) atomicMin(&cnt->min_far, (u64)mn);
}

template <typename Off>
__global__ __launch_bounds__(DB) void d_split_k(const u32* __restrict__ far, u64 nf, const Off* __restrict__ row,
                                                const u32* __restrict__ lsplit, const int32_t* __restrict__ dist,
                                                int32_t old_thr, int32_t thr, DQueues q,
                                                DCnt* __restrict__ cnt) {
    __shared__ u64 red[DB / WAVE];
    u64 m_acc = 0, h_acc = 0;
    const u64 nloop = (nf + DB - 1) / DB;
    for (u64 it = blockIdx.x; it < nloop; it += gridDim.x) {
        const u64 i = it * DB + threadIdx.x;
        bool to_near = false, to_far = false;
        u32 v = 0;
        if (i < nf) {
            v = far[i];
            const int32_t d = dist[v];
            if (d >= old_thr) {  // entries below old_thr were settled in an earlier band
                if (d < thr) to_near = atomicExch(q.st_near + v, q.round) != q.round;
                else to_far = atomicExch(q.st_far + v, q.epoch) != q.epoch;
            }
        }
        near_append<Off>(v, row, lsplit, to_near, q, cnt, m_acc, h_acc);
        const u64 fslot = wave_append(to_far, &cnt->n_far);
        if (to_far) q.far[fslot] = v;
    }
    m_acc = block_sum<DB / WAVE>(m_acc, red);
    h_acc = block_sum<DB / WAVE>(h_acc, red);
    if (threadIdx.x == 0) {
        if (m_acc) atomicAdd(&cnt->m_near, m_acc);
        if (h_acc) atomicAdd(&cnt->m_r, h_acc);
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
    DevBuf<int32_t> st_near, st_band, st_far;
    DevBuf<u32> far[2];
    DevBuf<u32> rv, rdeg;
    DevBuf<u64> rbeg;
    DevBuf<u32> lsplit;
    u32 lsplit_delta = 0;  // delta lsplit was computed for (0 = none)
};

void delete_delta_work(DeltaWork* p) { delete p; }

namespace {

template <typename Off>
void delta_run(Graph& g, DeltaWork& w, i64 source) {
    Ctx& ctx = *g.ctx;
    hipStream_t s = ctx.stream;
    const i64 n = g.n;
    const Off* row = static_cast<const Off*>(g.row_ptr());
    DCnt* dcnt = reinterpret_cast<DCnt*>(g.counters.p);
    DCnt* hcnt = reinterpret_cast<DCnt*>(g.hcounters.p);
    const unsigned maxgrid = (unsigned)ctx.cu_count * 8u;

    // delta: explicit option, else (mean weight / mean out-degree) * 4 — light
    // edges are then a small fraction of each row (tuned on Kronecker)
    int32_t delta = (int32_t)g.delta;
    if (delta <= 0) {
        const double mean_deg = n ? (double)g.nnz / (double)n : 1.0;
        const double d = 4.0 * g.mean_weight / std::max(1.0, mean_deg);
        delta = (int32_t)std::max(1.0, std::min(65536.0, std::round(d)));
    }
    if (w.lsplit_delta != (u32)delta && n > 0) {
        light_split_k<Off><<<grid_for(n, 256, maxgrid), 256, 0, s>>>(row, g.w.p, n, (u32)delta, w.lsplit.p);
        PJ_LAUNCH_CHECK();
        w.lsplit_delta = (u32)delta;
    }

    DQueues q{};
    q.st_near = w.st_near.p;
    q.st_band = w.st_band.p;
    q.st_far = w.st_far.p;
    q.rv = w.rv.p;
    q.rdeg = w.rdeg.p;
    q.rbeg = w.rbeg.p;

    auto t_host0 = std::chrono::steady_clock::now();
    PJ_HIP(hipEventRecord(g.ev0, s));
    pj_stats st{};
    if (n > 0) {
        PJ_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(g.dist.p), INT_INF, (size_t)n, s));
        PJ_HIP(hipMemsetAsync(w.st_near.p, 0xFF, sizeof(int32_t) * (size_t)n, s));
        PJ_HIP(hipMemsetAsync(w.st_band.p, 0xFF, sizeof(int32_t) * (size_t)n, s));
        PJ_HIP(hipMemsetAsync(w.st_far.p, 0xFF, sizeof(int32_t) * (size_t)n, s));
    }
    if (source >= 0 && source < n) {
        int cur = 0, fcur = 0;
        q.round = 0;
        q.band = 0;
        q.epoch = 0;
        q.qv = g.qv[0].p;
        q.qdeg = g.qdeg[0].p;
        q.qbeg = g.qbeg[0].p;
        PJ_HIP(hipMemsetAsync(dcnt, 0, sizeof(DCnt), s));
        d_source_k<Off><<<1, 1, 0, s>>>(source, row, w.lsplit.p, g.dist.p, q, dcnt);
        PJ_LAUNCH_CHECK();
        PJ_HIP(hipMemcpyAsync(hcnt, dcnt, sizeof(DCnt), hipMemcpyDeviceToHost, s));
        PJ_HIP(hipStreamSynchronize(s));
        u64 nq = hcnt->n_near, mq = hcnt->m_near, nf = 0, nr = hcnt->n_r, mr = hcnt->m_r;
        int32_t round = 0, epoch = 0, band = 0;
        int32_t thr = delta;
        for (;;) {
            // ---- near rounds: light edges of the vertices improved below thr
            while (nq > 0) {
                ++round;
                const int nx = 1 - cur;
                PJ_HIP(hipMemsetAsync(dcnt, 0, sizeof(DCnt), s));
                exclusive_scan_u32(g.qdeg[cur].p, g.qoff.p, (i64)nq, g.scan, s);
                q.round = round;
                q.band = band;
                q.epoch = epoch;
                q.qv = g.qv[nx].p;
                q.qdeg = g.qdeg[nx].p;
                q.qbeg = g.qbeg[nx].p;
                q.rv = w.rv.p + nr;
                q.rdeg = w.rdeg.p + nr;
                q.rbeg = w.rbeg.p + nr;
                q.far = w.far[fcur].p + nf;
                const unsigned grid = grid_for((i64)((mq + D_TILE - 1) / D_TILE), 1, maxgrid);
                d_relax_k<Off><<<grid, DB, 0, s>>>(g.qv[cur].p, g.qbeg[cur].p, g.qoff.p, nq, mq, g.col.p, g.w.p,
                                                   row, w.lsplit.p, g.dist.p, thr, q, dcnt);
                PJ_LAUNCH_CHECK();
                PJ_HIP(hipMemcpyAsync(hcnt, dcnt, sizeof(DCnt), hipMemcpyDeviceToHost, s));
                PJ_HIP(hipStreamSynchronize(s));
                nq = hcnt->n_near;
                mq = hcnt->m_near;
                nf += hcnt->n_far;
                nr += hcnt->n_r;
                mr += hcnt->m_r;
                cur = nx;
                st.relax_rounds++;
            }
            // ---- heavy pass: the band's settled vertices relax their heavy edges once
            if (nr > 0) {
                ++round;
                PJ_HIP(hipMemsetAsync(dcnt, 0, sizeof(DCnt), s));
                exclusive_scan_u32(w.rdeg.p, g.qoff.p, (i64)nr, g.scan, s);
                q.round = round;
                q.band = band;
                q.epoch = epoch;
                q.qv = g.qv[1 - cur].p;  // unused: heavy targets land at >= thr
                q.qdeg = g.qdeg[1 - cur].p;
                q.qbeg = g.qbeg[1 - cur].p;
                q.rv = w.rv.p;  // unused for the same reason
                q.rdeg = w.rdeg.p;
                q.rbeg = w.rbeg.p;
                q.far = w.far[fcur].p + nf;
                const unsigned grid = grid_for((i64)((mr + D_TILE - 1) / D_TILE), 1, maxgrid);
                d_relax_k<Off><<<grid, DB, 0, s>>>(w.rv.p, w.rbeg.p, g.qoff.p, nr, mr, g.col.p, g.w.p, row,
                                                   w.lsplit.p, g.dist.p, thr, q, dcnt);
                PJ_LAUNCH_CHECK();
                PJ_HIP(hipMemcpyAsync(hcnt, dcnt, sizeof(DCnt), hipMemcpyDeviceToHost, s));
                PJ_HIP(hipStreamSynchronize(s));
                nf += hcnt->n_far;
                nr = 0;
                mr = 0;
                st.relax_rounds++;
            }
            st.levels++;
            if (nf == 0) break;
            // ---- next non-empty band
            DCnt init{};
            init.min_far = (u64)INT_INF;
            PJ_HIP(hipMemcpyAsync(dcnt, &init, sizeof(DCnt), hipMemcpyHostToDevice, s));
            d_far_min_k<<<grid_for((i64)nf, DB, maxgrid), DB, 0, s>>>(w.far[fcur].p, nf, g.dist.p, thr, dcnt);
            PJ_LAUNCH_CHECK();
            PJ_HIP(hipMemcpyAsync(hcnt, dcnt, sizeof(DCnt), hipMemcpyDeviceToHost, s));
            PJ_HIP(hipStreamSynchronize(s));
            const u64 mn = hcnt->min_far;
            if (mn >= (u64)INT_INF) break;  // every far entry was settled below thr
            const int32_t old_thr = thr;
            const long long nthr = ((long long)mn / delta + 1) * (long long)delta;
            thr = (int32_t)std::min<long long>(nthr, INT_INF);
            ++round;
            ++epoch;
            ++band;
            q.round = round;
            q.band = band;
            q.epoch = epoch;
            q.qv = g.qv[cur].p;
            q.qdeg = g.qdeg[cur].p;
            q.qbeg = g.qbeg[cur].p;
            q.rv = w.rv.p;
            q.rdeg = w.rdeg.p;
            q.rbeg = w.rbeg.p;
            q.far = w.far[1 - fcur].p;
            PJ_HIP(hipMemsetAsync(dcnt, 0, sizeof(DCnt), s));
            d_split_k<Off><<<grid_for((i64)nf, DB, maxgrid), DB, 0, s>>>(w.far[fcur].p, nf, row, w.lsplit.p, g.dist.p,
                                                                         old_thr, thr, q, dcnt);
            PJ_LAUNCH_CHECK();
            PJ_HIP(hipMemcpyAsync(hcnt, dcnt, sizeof(DCnt), hipMemcpyDeviceToHost, s));
            PJ_HIP(hipStreamSynchronize(s));
            nq = hcnt->n_near;
            mq = hcnt->m_near;
            nf = hcnt->n_far;
            nr = hcnt->n_r;
            mr = hcnt->m_r;
            fcur = 1 - fcur;
        }
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
    g.dist.ensure(n ? n : 1);
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
    if (!g.delta_work) {
        g.delta_work.reset(new DeltaWork());
        DeltaWork& w = *g.delta_work;
        const size_t m = n ? n : 1;
        w.st_near.alloc(m);
        w.st_band.alloc(m);
        w.st_far.alloc(m);
        w.far[0].alloc(m);  // each epoch appends every vertex at most once
        w.far[1].alloc(m);
        w.rv.alloc(m);  // each band appends every vertex at most once
        w.rdeg.alloc(m);
        w.rbeg.alloc(m);
        w.lsplit.alloc(m);
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
