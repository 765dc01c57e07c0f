// graph.hip — CSR/CSC construction from device COO, and the benchmark generators.
//
// CSR build = stable radix sort by src + lower-bound row offsets: the GPU form
// of coord2csr (ParallelJohnson.cpp:117-159), keeping duplicate edges,
// self-loops and file order inside each row. The CSC (in-edges, used only by
// the pull/bottom-up BFS step) is a second sort of the CSR by column.
// Weighted graphs (no reference counterpart: the reference hard-codes w = 1,
// :147) keep each row sorted by weight instead, for delta-stepping.
#include "devutil.h"
#include "kron.h"

namespace pj {

namespace {

__global__ void pack_k(const u32* __restrict__ lo, const u32* __restrict__ hi, u64* __restrict__ out, i64 n) {
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x)
        out[i] = (u64)lo[i] | ((u64)hi[i] << 32);
}

// (src | dst << 32) records in weight order, the sorted weights -> key src, record (dst | w << 32)
__global__ void split_k(const u64* __restrict__ rec, const u32* __restrict__ wsorted, u32* __restrict__ key,
                        u64* __restrict__ out, i64 n) {
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) {
        const u64 r = rec[i];
        key[i] = (u32)r;
        out[i] = (r >> 32) | ((u64)wsorted[i] << 32);
    }
}

__global__ void unpack_k(const u64* __restrict__ rec, u32* __restrict__ lo, u32* __restrict__ hi, i64 n) {
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) {
        const u64 r = rec[i];
        lo[i] = (u32)r;
        hi[i] = (u32)(r >> 32);
    }
}

__global__ void max_k(const u32* __restrict__ in, i64 n, u32* __restrict__ out) {
    u32 m = 0;
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) m = max(m, in[i]);
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0 && m) atomicMax(out, m);
}

// number of significant bits of max(w[0..n))
int max_bits_device(const u32* w, i64 n, hipStream_t s) {
    if (n == 0) return 0;
    DevBuf<u32> m(1);
    PJ_HIP(hipMemsetAsync(m.p, 0, sizeof(u32), s));
    max_k<<<grid_for(n, 256, 4096), 256, 0, s>>>(w, n, m.p);
    PJ_LAUNCH_CHECK();
    u32 h = 0;
    PJ_HIP(hipMemcpyAsync(&h, m.p, sizeof(u32), hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
    int b = 0;
    while (b < 32 && (h >> b)) ++b;
    return b;
}

int key_bits(i64 n) {
    int b = 0;
    while (b < 32 && ((u64)1 << b) < (u64)n) ++b;
    return b;
}

template <typename Off>
void bounds_into(Graph& g, const u32* keys, bool csc) {
    hipStream_t s = g.ctx->stream;
    if (sizeof(Off) == 8) {
        DevBuf<u64>& r = csc ? g.crow64 : g.row64;
        r.alloc((size_t)g.n + 1);
        csr_bounds<u64>(keys, g.nnz, g.n, r.p, s);
    } else {
        DevBuf<u32>& r = csc ? g.crow32 : g.row32;
        r.alloc((size_t)g.n + 1);
        csr_bounds<u32>(keys, g.nnz, g.n, r.p, s);
    }
}

void bounds(Graph& g, const u32* keys, bool csc) {
    if (g.off64) bounds_into<u64>(g, keys, csc);
    else bounds_into<u32>(g, keys, csc);
}

}  // namespace

namespace {

// flags |= 1: row[0] != 0, a decreasing offset or row[n] != nnz; 2: a column id >= n
template <typename Off>
__global__ void csr_check_k(const Off* __restrict__ row, const u32* __restrict__ col, i64 n, i64 nnz,
                            u32* __restrict__ flags) {
    u32 f = 0;
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (i64)gridDim.x * blockDim.x) {
        const u64 r = (u64)row[i];
        if ((i == 0 && r != 0) || (i == n && r != (u64)nnz) || (i > 0 && (u64)row[i - 1] > r) || r > (u64)nnz) f |= 1u;
    }
    for (i64 k = (i64)blockIdx.x * blockDim.x + threadIdx.x; k < nnz; k += (i64)gridDim.x * blockDim.x)
        if ((i64)col[k] >= n) f |= 2u;
    if (f) atomicOr(flags, f);
}

}  // namespace

void check_csr_device(const void* row, bool off64, const u32* col, i64 n, i64 nnz, hipStream_t s) {
    DevBuf<u32> flag(1);
    PJ_HIP(hipMemsetAsync(flag.p, 0, sizeof(u32), s));
    const unsigned grid = grid_for(std::max(n + 1, nnz), 256, 8192);
    if (off64) csr_check_k<u64><<<grid, 256, 0, s>>>(static_cast<const u64*>(row), col, n, nnz, flag.p);
    else csr_check_k<u32><<<grid, 256, 0, s>>>(static_cast<const u32*>(row), col, n, nnz, flag.p);
    PJ_LAUNCH_CHECK();
    u32 h = 0;
    PJ_HIP(hipMemcpyAsync(&h, flag.p, sizeof(u32), hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
    if (h & 1u) throw Error(PJ_ERR_PARSE, "CSR file: row offsets are not a valid CSR (corrupted payload)");
    if (h & 2u) throw Error(PJ_ERR_PARSE, "CSR file: a column id is out of range (corrupted payload)");
}

Graph::~Graph() {
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
}

void build_graph_from_coo(Graph& g, DevBuf<u32>& src, DevBuf<u32>& dst, DevBuf<u32>* w, i64 nnz, i64 n,
                          bool symmetric) {
    hipStream_t s = g.ctx->stream;
    g.n = n;
    g.nnz = nnz;
    g.weighted = (w != nullptr);
    g.symmetric = symmetric;
    g.off64 = (u64)nnz > 0xFFFFFFFFull;
    const int bits = key_bits(n);
    SortWs ws;
    if (!g.weighted) {
        DevBuf<u32> kalt((size_t)nnz), valt((size_t)nnz);
        u32 *kr, *vr;
        radix_sort_pairs<u32>(src.p, kalt.p, dst.p, valt.p, nnz, bits, ws, s, &kr, &vr);
        DevBuf<u32>& K = (kr == src.p) ? src : kalt;
        DevBuf<u32>& Kspare = (kr == src.p) ? kalt : src;
        DevBuf<u32>& Vb = (vr == dst.p) ? dst : valt;
        DevBuf<u32>& Vspare = (vr == dst.p) ? valt : dst;
        bounds(g, K.p, false);
        g.col = std::move(Vb);
        if (!symmetric) {
            // CSC: sort the (col, src) pairs of the CSR by col.
            DevBuf<u32> k2((size_t)nnz);
            if (nnz) PJ_HIP(hipMemcpyAsync(k2.p, g.col.p, sizeof(u32) * (size_t)nnz, hipMemcpyDeviceToDevice, s));
            u32 *kr2, *vr2;
            radix_sort_pairs<u32>(k2.p, Kspare.p, K.p, Vspare.p, nnz, bits, ws, s, &kr2, &vr2);
            bounds(g, kr2, true);
            PJ_HIP(hipStreamSynchronize(s));  // k2 is freed at scope exit
            if (vr2 == K.p) g.ccol = std::move(K);
            else g.ccol = std::move(Vspare);
        }
        PJ_HIP(hipStreamSynchronize(s));
    } else {
        // Weighted: rows sorted by weight (ties in file order), so that for any
        // delta the light edges of a vertex are a prefix of its row. Two stable
        // LSD sorts of whole records (no random gathers): by weight, carrying
        // (src, dst), then by src, carrying (dst, w).
        const int wbits = max_bits_device(w->p, nnz, s);
        DevBuf<u64> rec((size_t)nnz), ralt((size_t)nnz);
        DevBuf<u32> kalt((size_t)nnz);
        u32* kr = w->p;
        u64* rr = rec.p;
        if (nnz) {
            pack_k<<<grid_for(nnz, 256, 8192), 256, 0, s>>>(src.p, dst.p, rec.p, nnz);
            PJ_LAUNCH_CHECK();
            radix_sort_pairs<u64>(w->p, kalt.p, rec.p, ralt.p, nnz, wbits, ws, s, &kr, &rr);
        }
        // keys := src, records := (dst, w) in weight order
        u32* skey = (kr == w->p) ? kalt.p : w->p;  // the free key buffer
        u64* rfree = (rr == rec.p) ? ralt.p : rec.p;
        if (nnz) {
            split_k<<<grid_for(nnz, 256, 8192), 256, 0, s>>>(rr, kr, skey, rfree, nnz);
            PJ_LAUNCH_CHECK();
        }
        PJ_HIP(hipStreamSynchronize(s));
        src.release();
        dst.release();
        u32* kfree = (skey == kalt.p) ? w->p : kalt.p;
        u64* rfree2 = (rfree == rec.p) ? ralt.p : rec.p;
        u32* kr2 = skey;
        u64* rr2 = rfree;
        radix_sort_pairs<u64>(skey, kfree, rfree, rfree2, nnz, bits, ws, s, &kr2, &rr2);
        bounds(g, kr2, false);
        g.col.alloc((size_t)nnz);
        g.w.alloc((size_t)nnz);
        if (nnz) {
            unpack_k<<<grid_for(nnz, 256, 8192), 256, 0, s>>>(rr2, g.col.p, g.w.p, nnz);
            PJ_LAUNCH_CHECK();
        }
        PJ_HIP(hipStreamSynchronize(s));
    }
}

// ------------------------------------------------------------------------
// Kronecker generator (benchmark input; no reference counterpart). Spec in
// DESIGN.md §Inputs; restated independently in oracle/pj_oracle.c for tests.
// ------------------------------------------------------------------------
namespace {

__global__ __launch_bounds__(256) void kronecker_k(int scale, u64 M, u64 seed, int weighted, PermKeys pk,
                                                   u32* __restrict__ src, u32* __restrict__ dst,
                                                   u32* __restrict__ w) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < M; i += (u64)gridDim.x * blockDim.x) {
        u32 pu, pv;
        kron_tuple(scale, seed, pk, i, pu, pv);
        src[2 * i] = pu;
        dst[2 * i] = pv;
        src[2 * i + 1] = pv;
        dst[2 * i + 1] = pu;
        if (w) {
            const u32 wt = kron_weight(seed, i, weighted != 0);
            w[2 * i] = wt;
            w[2 * i + 1] = wt;
        }
    }
}

}  // namespace

void generate_kronecker_device(Ctx& ctx, int scale, int edgefactor, uint64_t seed, bool weighted,
                               DevBuf<u32>& src, DevBuf<u32>& dst, DevBuf<u32>* w) {
    const u64 M = (u64)edgefactor << scale;
    src.alloc((size_t)(2 * M));
    dst.alloc((size_t)(2 * M));
    if (w) w->alloc((size_t)(2 * M));
    const PermKeys pk = make_perm_keys(scale, seed);
    if (M) {
        kronecker_k<<<grid_for((i64)M, 256, 256u * 64u), 256, 0, ctx.stream>>>(
            scale, M, seed, weighted ? 1 : 0, pk, src.p, dst.p, w ? w->p : nullptr);
        PJ_LAUNCH_CHECK();
    }
}

// ------------------------------------------------------------------------
// web-Google-shaped generator (the SNAP file is not in the
// image; configs[0] runs on a seeded synthetic of the same shape). Edge i:
//   source rank  = floor(np * u1^g_out)            power-law out-degree
//   target rank  = floor(np * u2^g_in)             power-law in-degree, or with
//                  probability 3/10 a "same-site" link: source rank + 1..64
// ranks are mapped to ids by an affine bijection mod n_ids over the first np
// ranks (np ~ 95.6% of the id range, as in web-Google), and edge 0 is pinned
// to the largest id so that N = max id + 1 = n_ids.
// ------------------------------------------------------------------------
namespace {

__device__ __forceinline__ double u01(u64 h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }

__global__ __launch_bounds__(256) void webgraph_k(u64 n_ids, u64 np, u64 m, u64 seed, u64 mul, u64 add, double g_out,
                                                  double g_in, u32* __restrict__ src, u32* __restrict__ dst) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (u64)gridDim.x * blockDim.x) {
        const u64 h1 = splitmix64(seed ^ (i * 4 + 0));
        const u64 h2 = splitmix64(seed ^ (i * 4 + 1));
        const u64 h3 = splitmix64(seed ^ (i * 4 + 2));
        u64 rs = (u64)((double)np * pow(u01(h1), g_out));
        if (rs >= np) rs = np - 1;
        u64 rd;
        if ((h3 % 10) < 3) {
            rd = (rs + 1 + (h3 >> 8) % 64) % np;
        } else {
            rd = (u64)((double)np * pow(u01(h2), g_in));
            if (rd >= np) rd = np - 1;
        }
        u64 a = (rs * mul + add) % n_ids, b = (rd * mul + add) % n_ids;
        if (i == 0) b = n_ids - 1;
        src[i] = (u32)a;
        dst[i] = (u32)b;
    }
}

u64 gcd_u64(u64 a, u64 b) {
    while (b) {
        u64 t = a % b;
        a = b;
        b = t;
    }
    return a;
}

}  // namespace

void generate_webgraph_device(Ctx& ctx, i64 n_ids, i64 n_edges, uint64_t seed, DevBuf<u32>& src,
                              DevBuf<u32>& dst) {
    src.alloc((size_t)n_edges);
    dst.alloc((size_t)n_edges);
    const u64 np = (u64)((double)n_ids * 0.9556);
    u64 mul = (splitmix64_h(seed ^ 0x6A09E667F3BCC908ull) % (u64)n_ids) | 1ull;
    while (gcd_u64(mul, (u64)n_ids) != 1) mul += 2;
    const u64 add = splitmix64_h(seed ^ 0xBB67AE8584CAA73Bull) % (u64)n_ids;
    if (n_edges) {
        webgraph_k<<<grid_for(n_edges, 256, 256u * 64u), 256, 0, ctx.stream>>>(
            (u64)n_ids, np ? np : 1, (u64)n_edges, seed, mul, add, 1.47, 2.0, src.p, dst.p);
        PJ_LAUNCH_CHECK();
    }
}

}  // namespace pj
