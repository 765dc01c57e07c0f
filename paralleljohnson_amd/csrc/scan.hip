// scan.hip — device-wide exclusive scan (reduce-then-scan, 2048 items per
// 256-thread block). Used for frontier edge offsets (top-down load balance),
// radix-sort digit offsets and ingestion line offsets.
#include "devutil.h"

namespace pj {

namespace {

constexpr int SB = 256;         // threads per block
constexpr int SIPT = 8;         // items per thread
constexpr int STILE = SB * SIPT;

template <typename T>
__global__ __launch_bounds__(SB) void scan_reduce_k(const T* __restrict__ in, i64 n,
                                                    u64* __restrict__ part) {
    __shared__ u64 lds[SB / WAVE];
    const i64 base = (i64)blockIdx.x * STILE;
    u64 s = 0;
#pragma unroll
    for (int k = 0; k < SIPT; ++k) {
        i64 i = base + (i64)k * SB + threadIdx.x;
        if (i < n) s += (u64)in[i];
    }
    s = block_sum<SB / WAVE>(s, lds);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// Each thread owns SIPT consecutive items (blocked layout) so the running
// prefix is sequential in registers.
template <typename T>
__global__ __launch_bounds__(SB) void scan_down_k(const T* __restrict__ in, u64* __restrict__ out,
                                                  i64 n, const u64* __restrict__ part_excl) {
    __shared__ u64 lds[SB / WAVE];
    const i64 base = (i64)blockIdx.x * STILE + (i64)threadIdx.x * SIPT;
    u64 v[SIPT];
    u64 s = 0;
#pragma unroll
    for (int k = 0; k < SIPT; ++k) {
        i64 i = base + k;
        v[k] = i < n ? (u64)in[i] : 0ull;
        s += v[k];
    }
    u64 tot;
    u64 pre = block_excl_scan<SB / WAVE>(s, lds, tot);
    const u64 boff = part_excl ? part_excl[blockIdx.x] : 0ull;
    pre += boff;
#pragma unroll
    for (int k = 0; k < SIPT; ++k) {
        i64 i = base + k;
        if (i < n) out[i] = pre;
        pre += v[k];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = boff + tot;
}

i64 scan_ws_need(i64 n) {
    i64 nb = (n + STILE - 1) / STILE;
    if (nb <= 1) return 0;
    return nb + (nb + 1) + scan_ws_need(nb);
}

template <typename T>
void scan_impl(const T* in, u64* out, i64 n, u64* ws, hipStream_t s) {
    i64 nb = (n + STILE - 1) / STILE;
    if (nb <= 1) {
        scan_down_k<T><<<1, SB, 0, s>>>(in, out, n, nullptr);
        PJ_LAUNCH_CHECK();
        return;
    }
    u64* part = ws;
    u64* part_scan = ws + nb;
    scan_reduce_k<T><<<(unsigned)nb, SB, 0, s>>>(in, n, part);
    PJ_LAUNCH_CHECK();
    scan_impl<u64>(part, part_scan, nb, ws + nb + (nb + 1), s);
    scan_down_k<T><<<(unsigned)nb, SB, 0, s>>>(in, out, n, part_scan);
    PJ_LAUNCH_CHECK();
}

}  // namespace

void ScanWs::ensure(i64 n) {
    i64 need = scan_ws_need(n);
    part.ensure((size_t)(need > 0 ? need : 1));
}

void exclusive_scan_u32(const u32* in, u64* out, i64 n, ScanWs& ws, hipStream_t s) {
    ws.ensure(n);
    scan_impl<u32>(in, out, n, ws.part.p, s);
}

void exclusive_scan_u64(const u64* in, u64* out, i64 n, ScanWs& ws, hipStream_t s) {
    ws.ensure(n);
    scan_impl<u64>(in, out, n, ws.part.p, s);
}

}  // namespace pj
