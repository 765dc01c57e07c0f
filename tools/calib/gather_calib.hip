// gather_calib.hip -- calibration of rocprofv3's FETCH_SIZE for the access shapes of the
// weighted solve (MI355X_MICROARCH.md, HBM section: "calibrate on a known
// byte count in your own access pattern"). Measurement tooling, not part of libpj.
//
// Three kernels over one table far larger than the 256 MB Infinity Cache (default 4 GiB):
//   cal_stream_k   every 16-byte piece read once, coalesced (the guide's calibrated case)
//   cal_lines_k    random 128-byte lines, each read whole by 32 consecutive lanes (known bytes:
//                  lines x 128, nothing wasted)
//   cal_dwords_k   random 4-byte words, one per lane (the solve's probe shape: a dist read)
// and the same random-dword kernel over a 64 MiB table (Infinity-Cache resident), which shows
// whether cache hits are counted. Each kernel runs REPS times; the program prints one JSON line
// per kernel with the requested bytes (and gathers) per launch and the mean launch time
// (HIP events), so a FETCH_SIZE / WRITE_SIZE pass of the same command gives bytes per request.
// Usage: pj_gather_calib [table_MiB=4096 (a power of two)] [reps=5]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                       \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

typedef unsigned long long u64;

__device__ __forceinline__ u64 mix(u64 x) {  // splitmix64 finaliser
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

__global__ void cal_fill_k(unsigned* t, u64 n) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x)
        t[i] = (unsigned)mix(i);
}

// every uint4 of the table once (grid-stride, coalesced); sink keeps the loads alive
__global__ void cal_stream_k(const uint4* __restrict__ t, u64 n4, unsigned* sink) {
    unsigned acc = 0;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (u64)gridDim.x * blockDim.x) {
        const uint4 v = t[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// G random 128-byte lines per half-wave (32 lanes x 4 bytes), the G loads issued together
constexpr int G = 4;
__global__ void cal_lines_k(const unsigned* __restrict__ t, u64 nlines, u64 steps, u64 seed, unsigned* sink) {
    const u64 hw = ((u64)blockIdx.x * blockDim.x + threadIdx.x) >> 5;
    const unsigned l = threadIdx.x & 31;
    unsigned acc = 0;
    for (u64 s = 0; s < steps; ++s) {
        unsigned v[G];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const u64 line = mix(seed ^ (hw * steps + s) * G + j) & (nlines - 1);
            v[j] = t[line * 32 + l];
        }
#pragma unroll
        for (int j = 0; j < G; ++j) acc ^= v[j];
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// G random dwords per lane, the G loads issued together (TAG only names the dispatches apart)
template <int TAG>
__global__ void cal_dwords_k(const unsigned* __restrict__ t, u64 n, u64 steps, u64 seed, unsigned* sink) {
    const u64 gid = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned acc = 0;
    for (u64 s = 0; s < steps; ++s) {
        unsigned v[G];
#pragma unroll
        for (int j = 0; j < G; ++j) v[j] = t[mix(seed ^ (gid * steps + s) * G + j) & (n - 1)];
#pragma unroll
        for (int j = 0; j < G; ++j) acc ^= v[j];
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
    const u64 mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 4096;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    if (mib < 64 || (mib & (mib - 1))) {
        std::fprintf(stderr, "table_MiB must be a power of two >= 64\n");
        return 2;
    }
    const u64 n = mib << 18;  // dwords
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned *t = nullptr, *sink = nullptr;
    CK(hipMalloc(&t, n * 4));
    CK(hipMalloc(&sink, 64));
    cal_fill_k<<<cus * 8, 256>>>(t, n);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned grid = (unsigned)cus * 16u, block = 256;  // 16 waves per CU
    const u64 threads = (u64)grid * block;
    auto timed = [&](const char* name, u64 bytes, u64 gathers, u64 table_bytes, auto launch) {
        launch(0);  // warm-up
        CK(hipDeviceSynchronize());
        float tot = 0.f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            launch(r + 1);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            tot += ms;
        }
        const double ms = tot / reps;
        std::printf("{\"kernel\": \"%s\", \"table_bytes\": %llu, \"launches\": %d, \"bytes_requested_per_launch\": %llu, "
                    "\"gathers_per_launch\": %llu, \"ms_per_launch\": %.4f, \"GBps_requested\": %.1f, "
                    "\"Ggathers_per_s\": %.3f}\n",
                    name, table_bytes, reps + 1, bytes, gathers, ms, bytes / ms / 1e6, gathers / ms / 1e6);
        std::fflush(stdout);
    };
    // streaming: every byte of the table once
    timed("cal_stream_k", n * 4, 0, n * 4, [&](int) { cal_stream_k<<<grid, block>>>(reinterpret_cast<const uint4*>(t), n / 4, sink); });
    // random lines: 4 x 128 B per half-wave step, 2^30 bytes per launch
    const u64 line_steps = ((u64)1 << 30) / (threads / 32 * G * 128);
    timed("cal_lines_k", threads / 32 * line_steps * G * 128, threads / 32 * line_steps * G, n * 4,
          [&](int r) { cal_lines_k<<<grid, block>>>(t, n / 32, line_steps, 1000 + r, sink); });
    // random dwords: 2^27 gathers per launch
    const u64 dw_steps = ((u64)1 << 27) / (threads * G);
    timed("cal_dwords_k", threads * dw_steps * G * 4, threads * dw_steps * G, n * 4,
          [&](int r) { cal_dwords_k<0><<<grid, block>>>(t, n, dw_steps, 2000 + r, sink); });
    // random dwords over 64 MiB (Infinity-Cache resident)
    const u64 small = (u64)64 << 18;
    timed("cal_dwords_small_k", threads * dw_steps * G * 4, threads * dw_steps * G, small * 4,
          [&](int r) { cal_dwords_k<1><<<grid, block>>>(t, small, dw_steps, 3000 + r, sink); });
    CK(hipFree(t));
    CK(hipFree(sink));
    return 0;
}
