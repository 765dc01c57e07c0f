// msbfs.hip — batched multi-source unit-weight SSSP (Johnson-style rows of
// the all-pairs matrix), 64 sources per pass.
//
// The reference answers one source per run (`atoi(argv[2])`, :448); a batch of
// 64 runs shares every CSR read here. Per vertex v the pass keeps three 64-bit
// words, one bit per source of the batch:
//   V[v]  sources that have reached v          (the 64 reference sp[] arrays, as bits)
//   F[v]  sources that reached v at the last level (their frontier)
//   Fn[v] the same for the level being computed
// A level is a pull over in-edges: Fn[v] = (OR over in-neighbours u of F[u]) & ~V[v],
// with the scan stopping as soon as every source still missing at v is covered.
// Distances follow the R9 contract per source: the level number, capped at INT_INF.
//
// Work mapping: one wave per 64 consecutive vertices; each lane walks its first
// MS_SERIAL in-edges in a wave-uniform loop (predicated body), then the whole wave
// scans the rest of long rows (web-graph in-hubs) 64 edges at a time.
#include <chrono>

#include "devutil.h"

namespace pj {

namespace {

constexpr int MB = 256;
constexpr int MS_SERIAL = 16;

struct MsCtl {
    u64 active[3];  // ring: level L reads [(L+2)%3] (level L-1), writes [L%3], block 0 zeroes [(L+1)%3]
    u64 done;       // set once by block 0 of the first level that finds nothing to do
};

__device__ __forceinline__ u64 wave_or(u64 x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x |= __shfl_xor(x, off, 64);
    return x;
}

__global__ __launch_bounds__(MB) void ms_init_k(u64* __restrict__ V, u64* __restrict__ F, i64 n,
                                                int32_t* __restrict__ dist, i64 nb_dist) {
    const i64 tid = (i64)blockIdx.x * MB + threadIdx.x, nth = (i64)gridDim.x * MB;
    for (i64 i = tid; i < n; i += nth) {
        V[i] = 0;
        F[i] = 0;
    }
    int4* d4 = reinterpret_cast<int4*>(dist);
    const i64 n4 = nb_dist / 4;
    for (i64 i = tid; i < n4; i += nth) d4[i] = make_int4(INT_INF, INT_INF, INT_INF, INT_INF);
    for (i64 i = n4 * 4 + tid; i < nb_dist; i += nth) dist[i] = INT_INF;
}

__global__ void ms_sources_k(const int64_t* __restrict__ src, int ns, i64 n, u64* __restrict__ V, u64* __restrict__ F,
                             int32_t* __restrict__ dist, MsCtl* ctl, int64_t* host_done) {
    // one thread: sources may repeat
    u64 any = 0;
    for (int i = 0; i < ns; ++i) {
        const int64_t s = src[i];
        if (s < 0 || s >= n) continue;
        V[s] |= 1ull << i;
        F[s] |= 1ull << i;
        dist[(i64)i * n + s] = 0;
        any = 1;
    }
    ctl->active[2] = any;  // "level -1" found the sources
    ctl->active[0] = 0;
    ctl->active[1] = 0;
    ctl->done = 0;
    *host_done = -1;
}

template <typename Off>
__global__ __launch_bounds__(MB) void ms_level_k(i64 n, const Off* __restrict__ crow, const u32* __restrict__ ccol,
                                                 u64* __restrict__ V, const u64* __restrict__ F,
                                                 u64* __restrict__ Fn, int32_t* __restrict__ dist, int32_t L,
                                                 u64 smask, MsCtl* ctl, int64_t* host_done) {
    // level L computes distance L+1 from the frontier of level L-1
    if (ctl->active[(L + 2) % 3] == 0 || L + 1 >= INT_INF) {
        if (blockIdx.x == 0 && threadIdx.x == 0 && !ctl->done) {
            ctl->done = 1;
            *host_done = L;
        }
        return;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) ctl->active[(L + 1) % 3] = 0;
    const int lane = lane_id();
    u64 found_any = 0;
    const i64 nwaves = (i64)gridDim.x * (MB / WAVE);
    for (i64 base = ((i64)blockIdx.x * (MB / WAVE) + wave_id()) * 64; base < n; base += nwaves * 64) {
        const i64 v = base + lane;
        const bool inr = v < n;
        const u64 vv = inr ? V[v] : ~0ull;
        const u64 need = ~vv & smask;  // sources of this batch that have not reached v
        if (__ballot(need != 0) == 0) {
            if (inr) Fn[v] = 0;
            continue;
        }
        Off b = 0, e = 0;
        if (need) {
            b = crow[v];
            e = crow[v + 1];
        }
        u64 acc = 0;
        Off k = b;
        const Off lim = (e - b > (Off)MS_SERIAL) ? b + (Off)MS_SERIAL : e;
        bool go = need && k < lim;
        while (__ballot(go)) {
            if (go) {
                acc |= F[ccol[k]];
                ++k;
                go = (need & ~acc) && k < lim;
            }
        }
        u64 open = __ballot((need & ~acc) != 0 && k < e);
        while (open) {
            const int l = __ffsll((long long)open) - 1;
            open &= open - 1;
            const Off kb = __shfl(k, l, 64), ke = __shfl(e, l, 64);
            const u64 want = __shfl(need, l, 64);
            u64 got = __shfl(acc, l, 64);
            for (Off kk = kb; kk < ke && (want & ~got); kk += WAVE) {
                const Off kx = kk + lane;
                const u64 x = kx < ke ? F[ccol[kx]] : 0ull;
                got |= wave_or(x);
            }
            if (lane == l) acc = got;
        }
        const u64 newb = acc & need;
        if (inr) {
            Fn[v] = newb;
            if (newb) V[v] = vv | newb;
        }
        found_any |= newb;
        // distances of the newly reached (source, v) pairs: a wave-uniform loop
        u64 rest = newb;
        while (__ballot(rest != 0)) {
            if (rest) {
                const int sbit = __ffsll((long long)rest) - 1;
                rest &= rest - 1;
                dist[(i64)sbit * n + v] = L + 1;
            }
        }
    }
    if (__ballot(found_any != 0) && lane == 0) ctl->active[L % 3] = 1;
}

}  // namespace

struct MsWork {
    DevBuf<u64> V, F, Fn;
    DevBuf<int32_t> dist;
    DevBuf<int64_t> src;
    DevBuf<MsCtl> ctl;
    int64_t* host = nullptr;
    ~MsWork() {
        if (host) (void)hipHostFree(host);
    }
};

void delete_ms_work(MsWork* p) { delete p; }

template <typename Off>
static void ms_pass(Graph& g, MsWork& w, const int64_t* sources, int ns, int32_t* dist_out, double* kernel_ms,
                    i64* levels) {
    hipStream_t s = g.ctx->stream;
    const i64 n = g.n;
    const Off* crow = static_cast<const Off*>(g.crow_ptr());
    const u32* ccol = g.ccol_ptr();
    PJ_HIP(hipMemcpyAsync(w.src.p, sources, sizeof(int64_t) * (size_t)ns, hipMemcpyHostToDevice, s));
    int64_t* host_dev = nullptr;
    PJ_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&host_dev), w.host, 0));
    u64 smask = 0;  // bits of the valid sources of this batch
    for (int i = 0; i < ns; ++i)
        if (sources[i] >= 0 && sources[i] < n) smask |= 1ull << i;
    const unsigned grid = (unsigned)g.ctx->cu_count * 4u;
    PJ_HIP(hipEventRecord(g.ev0, s));
    ms_init_k<<<grid_for(std::max<i64>(n, (i64)ns * n / 4), MB, (unsigned)g.ctx->cu_count * 8u), MB, 0, s>>>(
        w.V.p, w.F.p, n, w.dist.p, (i64)ns * n);
    PJ_LAUNCH_CHECK();
    ms_sources_k<<<1, 1, 0, s>>>(w.src.p, ns, n, w.V.p, w.F.p, w.dist.p, w.ctl.p, host_dev);
    PJ_LAUNCH_CHECK();
    int32_t L = 0;
    int batch = 16;
    u64* F = w.F.p;
    u64* Fn = w.Fn.p;
    for (;;) {
        for (int i = 0; i < batch && L < INT_INF; ++i, ++L) {
            ms_level_k<Off><<<grid, MB, 0, s>>>(n, crow, ccol, w.V.p, F, Fn, w.dist.p, L, smask, w.ctl.p, host_dev);
            PJ_LAUNCH_CHECK();
            std::swap(F, Fn);
        }
        PJ_HIP(hipStreamSynchronize(s));
        if (*(volatile int64_t*)w.host >= 0 || L >= INT_INF || smask == 0) break;
        batch = batch < 1024 ? batch * 2 : batch;
    }
    PJ_HIP(hipEventRecord(g.ev1, s));
    PJ_HIP(hipEventSynchronize(g.ev1));
    float ms = 0.f;
    PJ_HIP(hipEventElapsedTime(&ms, g.ev0, g.ev1));
    *kernel_ms += ms;
    const i64 lv = (i64)*(volatile int64_t*)w.host;
    *levels = std::max<i64>(*levels, lv);
    if (dist_out && n) PJ_HIP(hipMemcpy(dist_out, w.dist.p, sizeof(int32_t) * (size_t)ns * (size_t)n, hipMemcpyDeviceToHost));
}

void msbfs_solve(Graph& g, const int64_t* sources, int n_src, int32_t* dist_out) {
    const size_t n = (size_t)g.n;
    if (!g.ms_work) {
        g.ms_work.reset(new MsWork());
        MsWork& w = *g.ms_work;
        w.V.alloc(n ? n : 1);
        w.F.alloc(n ? n : 1);
        w.Fn.alloc(n ? n : 1);
        w.dist.alloc(n ? 64 * n : 1);
        w.src.alloc(64);
        w.ctl.alloc(1);
        PJ_HIP(hipHostMalloc(reinterpret_cast<void**>(&w.host), sizeof(int64_t), hipHostMallocMapped));
    }
    if (!g.ev0) PJ_HIP(hipEventCreate(&g.ev0));
    if (!g.ev1) PJ_HIP(hipEventCreate(&g.ev1));
    auto t0 = std::chrono::steady_clock::now();
    pj_stats st{};
    double kms = 0;
    i64 levels = 0;
    for (int off = 0; off < n_src; off += 64) {
        const int ns = std::min(64, n_src - off);
        int32_t* out = dist_out ? dist_out + (size_t)off * n : nullptr;
        if (g.off64) ms_pass<u64>(g, *g.ms_work, sources + off, ns, out, &kms, &levels);
        else ms_pass<u32>(g, *g.ms_work, sources + off, ns, out, &kms, &levels);
    }
    st.kernel_ms = kms;
    st.levels = levels;
    st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    g.stats = st;
    // the per-source result of the last pass's final source is not kept in g.dist
}

}  // namespace pj
