// kron_tts.cpp — time to solution of the generated-graph configs (BASELINE.json
// configs[1]/[2]) as one wall clock, the way SURVEY.md §8d defines it for the
// CLI: process start -> sol_file closed. The reference cannot read a 2^31-line
// text file (:66/:117), so the graph comes from the on-device Kronecker
// generator instead of pj_load_snap; everything else is the CLI's path:
// pj_create -> build (generate + radix sort + CSR) -> solve (the first solve
// includes the solver's preparation) -> D2H -> pj_write_sol.
//
//   pj_kron_tts scale edgefactor seed weighted source sol_file
// source "sample:<seed>": the first root pj_sample_roots(seed) picks on the built graph
// (the bench's first root), chosen inside the timed process.
// stdout: one line "phases_s <create> <build> <solve> <d2h> <write> <launch> <teardown>
// root <source> exit_ns <t>" (the parent times the whole process itself; launch = the
// parent's PJ_TTS_LAUNCH_NS (CLOCK_MONOTONIC) -> main, teardown = graph + context
// destruction (PJ_TTS_TEARDOWN=1, else ~0), exit_ns = CLOCK_MONOTONIC just before main returns, so the parent can
// report the process exit too).
//
// The n-entry host distance buffer is allocated without zero-filling, its pages are
// faulted in by host threads and then pinned (pj_host_pin) while the GPU builds the
// graph, so the D2H is one DMA copy (a zero-filled std::vector cost ~0.05 s of page
// faults on the critical path at s26: 268 MB; the staged copy into pageable memory
// 0.056 s, r4a). After the sol_file is closed and the phases are printed the process
// ends with _exit: the HIP runtime's teardown at exit cost 0.12 s and the graph and
// context destruction 0.03 s (r4a) that no result depends on; PJ_TTS_TEARDOWN=1
// destroys the graph and the context and returns from main instead.
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/pj.h"

static long long now_ns() {
    return (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}
static double now_s() { return (double)now_ns() * 1e-9; }

static int fail(const char* what) {
    std::fprintf(stderr, "pj_kron_tts: %s: %s\n", what, pj_last_error());
    return 1;
}

// n int32 of anonymous memory, its pages faulted in by `nt` threads (one byte per page).
struct HostRows {
    int32_t* p = nullptr;
    size_t bytes = 0;
    std::vector<std::thread> th;
    void start(size_t n, int nt) {
        bytes = std::max<size_t>(n, 1) * sizeof(int32_t);
        void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (m == MAP_FAILED) return;
        p = static_cast<int32_t*>(m);
        const size_t page = 4096, chunk = (bytes + nt - 1) / nt;
        for (int t = 0; t < nt; ++t)
            th.emplace_back([this, t, chunk, page] {
                char* b = reinterpret_cast<char*>(p);
                const size_t lo = (size_t)t * chunk, hi = std::min(bytes, lo + chunk);
                for (size_t o = lo; o < hi; o += page) b[o] = 0;
            });
    }
    void join() {
        for (auto& x : th) x.join();
        th.clear();
    }
    // after pj_create: one thread waits for the faulting threads, then pins the rows
    std::thread pinner;
    bool pinned = false;
    void pin() {
        if (!p) return;
        pinner = std::thread([this] {
            join();
            pinned = pj_host_pin(p, bytes) == PJ_OK;
        });
    }
    void finish() {
        if (pinner.joinable()) pinner.join();
        join();
    }
    ~HostRows() { finish(); }  // (the mapping goes with the process)
};

int main(int argc, char** argv) {
    const long long t0n = now_ns();
    if (argc != 7) {
        std::fprintf(stderr, "usage: pj_kron_tts scale edgefactor seed weighted source sol_file\n");
        return 2;
    }
    const char* launch = std::getenv("PJ_TTS_LAUNCH_NS");
    const double launch_s = launch ? (double)(t0n - std::atoll(launch)) * 1e-9 : -1.0;
    const int scale = std::atoi(argv[1]);
    HostRows rows;
    if (scale >= 0 && scale < 40) rows.start((size_t)1 << scale, 4);  // overlaps pj_create and the build
    const double t0 = (double)t0n * 1e-9;
    pj_ctx* ctx = nullptr;
    if (pj_create(0, &ctx) != PJ_OK) return fail("pj_create");
    rows.pin();
    const double t1 = now_s();
    pj_graph* g = nullptr;
    if (pj_generate_kronecker(ctx, scale, std::atoi(argv[2]), std::strtoull(argv[3], nullptr, 10), std::atoi(argv[4]),
                              &g) != PJ_OK)
        return fail("pj_generate_kronecker");
    const double t2 = now_s();
    int64_t n = 0;
    pj_graph_info(g, &n, nullptr, nullptr, nullptr);
    int64_t source = 0;
    if (std::strncmp(argv[5], "sample:", 7) == 0) {
        int found = 0;
        if (pj_sample_roots(g, std::strtoull(argv[5] + 7, nullptr, 10), 1, &source, &found) != PJ_OK || found != 1)
            return fail("pj_sample_roots");
    } else {
        source = std::atoll(argv[5]);
    }
    if (pj_sssp(g, source, nullptr) != PJ_OK) return fail("pj_sssp");
    const double t3 = now_s();
    rows.finish();
    std::vector<int32_t> fallback;
    int32_t* dist = rows.p;
    if (!dist || (size_t)n * sizeof(int32_t) > rows.bytes) {
        fallback.resize((size_t)std::max<int64_t>(n, 1));
        dist = fallback.data();
    }
    if (pj_copy_dist(g, dist) != PJ_OK) return fail("pj_copy_dist");
    const double t4 = now_s();
    if (pj_write_sol(dist, n, argv[6], 1) != PJ_OK) return fail("pj_write_sol");
    const double t5 = now_s();
    const bool teardown = std::getenv("PJ_TTS_TEARDOWN") && std::atoi(std::getenv("PJ_TTS_TEARDOWN"));
    if (teardown) {
        if (rows.pinned) pj_host_unpin(rows.p);
        pj_graph_destroy(g);
        pj_destroy(ctx);
    }
    const long long t6n = now_ns();
    std::printf("phases_s %.4f %.4f %.4f %.4f %.4f %.4f %.4f root %lld exit_ns %lld\n", t1 - t0, t2 - t1, t3 - t2,
                t4 - t3, t5 - t4, launch_s, (double)t6n * 1e-9 - t5, (long long)source, t6n);
    std::fflush(stdout);
    if (!teardown) _exit(0);
    return 0;
}
