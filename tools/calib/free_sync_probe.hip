// free_sync_probe.hip — does hipFree / hipHostFree wait for kernels still running on a
// non-blocking stream? (libpj frees DevBufs with hipFree and relies on its implicit
// device synchronization.) A one-wave kernel spins ~200 ms on the clock on a
// hipStreamNonBlocking stream, touching nothing but its own flag word; the host then
// frees an unrelated device buffer (and a pinned host buffer) and times the call.
// A free that returns well before the kernel ends does not order against that stream.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                 \
            return 1;                                                           \
        }                                                                       \
    } while (0)

__global__ void spin_k(long long cycles, int* flag) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < cycles) {
    }
    if (threadIdx.x == 0) *flag = 1;
}

static double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main() {
    int rate_khz = 0;
    CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
    const long long cycles = (long long)rate_khz * 200;  // ~200 ms
    hipStream_t nb = nullptr, bl = nullptr;
    CK(hipStreamCreateWithFlags(&nb, hipStreamNonBlocking));
    CK(hipStreamCreate(&bl));
    int* flag = nullptr;
    CK(hipMalloc(&flag, 64));
    struct Case {
        const char* what;
        hipStream_t s;
        int kind;  // 0 hipFree of a small buffer, 1 hipFree of a 2 GiB buffer, 2 hipHostFree
    } cases[] = {{"hipFree small, non-blocking stream", nb, 0}, {"hipFree 2GiB, non-blocking stream", nb, 1},
                 {"hipHostFree, non-blocking stream", nb, 2},    {"hipFree small, blocking stream", bl, 0},
                 {"hipHostFree, blocking stream", bl, 2}};
    for (const Case& c : cases) {
        void* p = nullptr;
        if (c.kind == 0) CK(hipMalloc(&p, 4096));
        if (c.kind == 1) CK(hipMalloc(&p, (size_t)2 << 30));
        if (c.kind == 2) CK(hipHostMalloc(&p, 4096, hipHostMallocMapped));
        CK(hipMemsetAsync(flag, 0, 4, c.s));
        CK(hipStreamSynchronize(c.s));
        const auto t0 = std::chrono::steady_clock::now();
        spin_k<<<1, 64, 0, c.s>>>(cycles, flag);
        CK(hipGetLastError());
        const double launch_ms = ms_since(t0);
        const auto t1 = std::chrono::steady_clock::now();
        if (c.kind == 2) CK(hipHostFree(p));
        else CK(hipFree(p));
        const double free_ms = ms_since(t1);
        const hipError_t q = hipStreamQuery(c.s);
        CK(hipStreamSynchronize(c.s));
        const double total_ms = ms_since(t0);
        std::printf("{\"case\": \"%s\", \"launch_ms\": %.3f, \"free_ms\": %.3f, \"kernel_running_after_free\": %s, "
                    "\"total_ms\": %.1f}\n",
                    c.what, launch_ms, free_ms, q == hipErrorNotReady ? "true" : "false", total_ms);
    }
    CK(hipFree(flag));
    return 0;
}
