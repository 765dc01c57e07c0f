// delta.hip — weighted SSSP: near-far delta-stepping on the GPU.
//
// Generalises the reference's label-correcting relaxation (extract_local_pq
// :226-278, apply loop :557-573) to integer weights >= 0, keeping its output
// contract: candidates >= INT_INF are discarded and the
// result is the true distance when it is < INT_INF. The reference settles one
// vertex per heap pop; here a whole distance band [thr - delta, thr) is
// relaxed at once:
//   near queue : vertices whose distance dropped below thr this round; relaxed
//                edge-balanced (lb.h tiles), dist[v] lowered with atomicMin
//   far pile   : improved vertices with distance >= thr, kept with a per-epoch
//                stamp so each vertex appears at most once
//   split      : when the near queue drains, thr jumps to the first band that
//                holds a far vertex; far entries below the new thr move to near
// Each relax round and each split is one kernel; the host reads three counters
// between them (the analogue of the reference's termination allreduce
// :579-593).
#include <chrono>
#include <cmath>

#include "lb.h"

namespace pj {

namespace {

struct DCnt {
    u64 n_near;  // near-queue entries appended
    u64 m_near;  // their out-degree sum
    u64 n_far;   // far-pile entries appended
    u64 min_far; // smallest distance in the far pile (split pre-pass)
};

constexpr int DB = 256;
constexpr int D_IPT = 4;
constexpr int D_TILE = DB * D_IPT;

template <typename Off>
__device__ __forceinline__ void near_append(u32 v, const Off* __restrict__ row, u32* __restrict__ qv,
                                            u32* __restrict__ qdeg, u64* __restrict__ qbeg, bool pred, DCnt* c,
                                            u64& m_acc) {
    u32 deg = 0;
    u64 beg = 0;
    if (pred) {
        const Off b = row[v], e = row[v + 1];
        deg = (u32)(e - b);
        beg = (u64)b;
    }
    const bool app = pred && deg > 0;
    const u64 slot = wave_append(app, &c->n_near);
    if (app) {
        qv[slot] = v;
        qdeg[slot] = deg;
        qbeg[slot] = beg;
        m_acc += deg;
    }
}

template <typename Off>
__global__ void d_source_k(i64 s, const Off* __restrict__ row, int32_t* __restrict__ dist, u32* __restrict__ qv,
                           u32* __restrict__ qdeg, u64* __restrict__ qbeg, DCnt* __restrict__ c) {
    dist[s] = 0;
    const Off b = row[s], e = row[s + 1];
    if (e > b) {
        qv[0] = (u32)s;
        qdeg[0] = (u32)(e - b);
        qbeg[0] = (u64)b;
        c->n_near = 1;
        c->m_near = (u64)(e - b);
    }
}

template <typename Off>
__global__ __launch_bounds__(DB) void d_relax_k(const u32* __restrict__ qv, const u64* __restrict__ qbeg,
                                                const u64* __restrict__ qoff, u64 nq, u64 total,
                                                const u32* __restrict__ col, const u32* __restrict__ wt,
                                                const Off* __restrict__ row, int32_t* __restrict__ dist,
                                                int32_t thr, int32_t round, int32_t epoch,
                                                int32_t* __restrict__ st_near, int32_t* __restrict__ st_far,
                                                u32* __restrict__ qv_n, u32* __restrict__ qdeg_n,
                                                u64* __restrict__ qbeg_n, u32* __restrict__ far_out,
                                                DCnt* __restrict__ cnt) {
    __shared__ LbShared<D_TILE> sh;
    __shared__ int32_t s_du[D_TILE];
    __shared__ u64 red[DB / WAVE];
    const u64 ntiles = (total + D_TILE - 1) / D_TILE;
    u64 m_acc = 0;
    for (u64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const u64 e0 = tile * D_TILE;
        const u64 e1 = min(e0 + (u64)D_TILE, total);
        u64 s0;
        u32 ns;
        lb_tile_load<D_TILE>(qoff, nq, e0, sh, s0, ns);
        for (u32 i = threadIdx.x; i < ns; i += DB) s_du[i] = dist[qv[s0 + i]];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < D_IPT; ++k) {
            const u64 e = e0 + (u64)k * DB + threadIdx.x;
            bool to_near = false, to_far = false;
            u32 v = 0;
            if (e < e1) {
                const u32 j = lb_find<D_TILE>(sh, ns, e);
                const u64 idx = qbeg[s0 + j] + (e - sh.off[j]);
                v = col[idx];
                const long long nd = (long long)s_du[j] + (long long)wt[idx];
                if (nd < INT_INF && (int32_t)nd < dist[v]) {
                    const int32_t old = atomicMin(dist + v, (int32_t)nd);
                    if ((int32_t)nd < old) {
                        if ((int32_t)nd < thr) to_near = atomicExch(st_near + v, round) != round;
                        else to_far = atomicExch(st_far + v, epoch) != epoch;
                    }
                }
            }
            near_append<Off>(v, row, qv_n, qdeg_n, qbeg_n, to_near, cnt, m_acc);
            const u64 fslot = wave_append(to_far, &cnt->n_far);
            if (to_far) far_out[fslot] = v;
        }
        __syncthreads();
    }
    m_acc = block_sum<DB / WAVE>(m_acc, red);
    if (threadIdx.x == 0 && m_acc) atomicAdd(&cnt->m_near, m_acc);
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
                                                const int32_t* __restrict__ dist, int32_t old_thr, int32_t thr,
                                                int32_t round, int32_t epoch, int32_t* __restrict__ st_near,
                                                int32_t* __restrict__ st_far, u32* __restrict__ qv_n,
                                                u32* __restrict__ qdeg_n, u64* __restrict__ qbeg_n,
                                                u32* __restrict__ far_out, DCnt* __restrict__ cnt) {
    __shared__ u64 red[DB / WAVE];
    u64 m_acc = 0;
    const u64 nloop = (nf + DB - 1) / DB;
    for (u64 it = blockIdx.x; it < nloop; it += gridDim.x) {
        const u64 i = it * DB + threadIdx.x;
        bool to_near = false, to_far = false;
        u32 v = 0;
        if (i < nf) {
            v = far[i];
            const int32_t d = dist[v];
            if (d >= old_thr) {  // entries below old_thr were settled through the near queue
                if (d < thr) to_near = atomicExch(st_near + v, round) != round;
                else to_far = atomicExch(st_far + v, epoch) != epoch;
            }
        }
        near_append<Off>(v, row, qv_n, qdeg_n, qbeg_n, to_near, cnt, m_acc);
        const u64 fslot = wave_append(to_far, &cnt->n_far);
        if (to_far) far_out[fslot] = v;
    }
    m_acc = block_sum<DB / WAVE>(m_acc, red);
    if (threadIdx.x == 0 && m_acc) atomicAdd(&cnt->m_near, m_acc);
}

template <typename Off>
void delta_run(Graph& g, i64 source, DevBuf<int32_t>& st_near, DevBuf<int32_t>& st_far, DevBuf<u32> far[2]) {
    Ctx& ctx = *g.ctx;
    hipStream_t s = ctx.stream;
    const i64 n = g.n;
    const Off* row = static_cast<const Off*>(g.row_ptr());
    DCnt* dcnt = reinterpret_cast<DCnt*>(g.counters.p);
    DCnt* hcnt = reinterpret_cast<DCnt*>(g.hcounters.p);
    const unsigned maxgrid = (unsigned)ctx.cu_count * 8u;

    // delta: explicit option, else mean weight / mean out-degree scaled so a
    // band holds a few relax rounds (tuned on Kronecker).
    int32_t delta = (int32_t)g.delta;
    if (delta <= 0) {
        const double mean_deg = n ? (double)g.nnz / (double)n : 1.0;
        const double d = 8.0 * 128.0 / std::max(1.0, mean_deg);
        delta = (int32_t)std::max(1.0, std::min(4096.0, std::round(d)));
    }

    auto t_host0 = std::chrono::steady_clock::now();
    PJ_HIP(hipEventRecord(g.ev0, s));
    pj_stats st{};
    if (n > 0) {
        PJ_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(g.dist.p), INT_INF, (size_t)n, s));
        PJ_HIP(hipMemsetAsync(st_near.p, 0xFF, sizeof(int32_t) * (size_t)n, s));
        PJ_HIP(hipMemsetAsync(st_far.p, 0xFF, sizeof(int32_t) * (size_t)n, s));
    }
    if (source >= 0 && source < n) {
        PJ_HIP(hipMemsetAsync(dcnt, 0, sizeof(DCnt), s));
        d_source_k<Off><<<1, 1, 0, s>>>(source, row, g.dist.p, g.qv[0].p, g.qdeg[0].p, g.qbeg[0].p, dcnt);
        PJ_LAUNCH_CHECK();
        PJ_HIP(hipMemcpyAsync(hcnt, dcnt, sizeof(DCnt), hipMemcpyDeviceToHost, s));
        PJ_HIP(hipStreamSynchronize(s));
        u64 nq = hcnt->n_near, mq = hcnt->m_near, nf = 0;
        int cur = 0, fcur = 0;
        int32_t round = 0, epoch = 0;
        int32_t thr = delta;
        for (;;) {
            while (nq > 0) {
                ++round;
                const int nx = 1 - cur;
                PJ_HIP(hipMemsetAsync(dcnt, 0, sizeof(DCnt), s));
                exclusive_scan_u32(g.qdeg[cur].p, g.qoff.p, (i64)nq, g.scan, s);
                // relaxations append to the far pile after its current nf entries
                const unsigned grid = grid_for((i64)((mq + D_TILE - 1) / D_TILE), 1, maxgrid);
                d_relax_k<Off><<<grid, DB, 0, s>>>(g.qv[cur].p, g.qbeg[cur].p, g.qoff.p, nq, mq, g.col.p, g.w.p,
                                                   row, g.dist.p, thr, round, epoch, st_near.p, st_far.p,
                                                   g.qv[nx].p, g.qdeg[nx].p, g.qbeg[nx].p, far[fcur].p + nf, dcnt);
                PJ_LAUNCH_CHECK();
                PJ_HIP(hipMemcpyAsync(hcnt, dcnt, sizeof(DCnt), hipMemcpyDeviceToHost, s));
                PJ_HIP(hipStreamSynchronize(s));
                nq = hcnt->n_near;
                mq = hcnt->m_near;
                nf += hcnt->n_far;
                cur = nx;
                st.relax_rounds++;
            }
            st.levels++;
            if (nf == 0) break;
            // next non-empty band
            DCnt init{};
            init.min_far = (u64)INT_INF;
            PJ_HIP(hipMemcpyAsync(dcnt, &init, sizeof(DCnt), hipMemcpyHostToDevice, s));
            d_far_min_k<<<grid_for((i64)nf, DB, maxgrid), DB, 0, s>>>(far[fcur].p, nf, g.dist.p, thr, dcnt);
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
            PJ_HIP(hipMemsetAsync(dcnt, 0, sizeof(DCnt), s));
            d_split_k<Off><<<grid_for((i64)nf, DB, maxgrid), DB, 0, s>>>(
                far[fcur].p, nf, row, g.dist.p, old_thr, thr, round, epoch, st_near.p, st_far.p, g.qv[cur].p,
                g.qdeg[cur].p, g.qbeg[cur].p, far[1 - fcur].p, dcnt);
            PJ_LAUNCH_CHECK();
            PJ_HIP(hipMemcpyAsync(hcnt, dcnt, sizeof(DCnt), hipMemcpyDeviceToHost, s));
            PJ_HIP(hipStreamSynchronize(s));
            nq = hcnt->n_near;
            mq = hcnt->m_near;
            nf = hcnt->n_far;
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
    // stamps + far piles (each epoch appends every vertex at most once: <= n entries)
    DevBuf<int32_t> st_near(n ? n : 1), st_far(n ? n : 1);
    DevBuf<u32> far[2];
    far[0].alloc(n ? n : 1);
    far[1].alloc(n ? n : 1);
    if (g.off64) delta_run<u64>(g, source, st_near, st_far, far);
    else delta_run<u32>(g, source, st_near, st_far, far);
}

}  // namespace pj
