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
// stdout: one line "phases_s <create> <build> <solve+d2h> <write> root <source>" (the
// parent times the whole process itself).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/pj.h"

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int fail(const char* what) {
    std::fprintf(stderr, "pj_kron_tts: %s: %s\n", what, pj_last_error());
    return 1;
}

int main(int argc, char** argv) {
    if (argc != 7) {
        std::fprintf(stderr, "usage: pj_kron_tts scale edgefactor seed weighted source sol_file\n");
        return 2;
    }
    const double t0 = now_s();
    pj_ctx* ctx = nullptr;
    if (pj_create(0, &ctx) != PJ_OK) return fail("pj_create");
    const double t1 = now_s();
    pj_graph* g = nullptr;
    if (pj_generate_kronecker(ctx, std::atoi(argv[1]), std::atoi(argv[2]), std::strtoull(argv[3], nullptr, 10),
                              std::atoi(argv[4]), &g) != PJ_OK)
        return fail("pj_generate_kronecker");
    const double t2 = now_s();
    int64_t n = 0;
    pj_graph_info(g, &n, nullptr, nullptr, nullptr);
    std::vector<int32_t> dist((size_t)n);
    int64_t source = 0;
    if (std::strncmp(argv[5], "sample:", 7) == 0) {
        int found = 0;
        if (pj_sample_roots(g, std::strtoull(argv[5] + 7, nullptr, 10), 1, &source, &found) != PJ_OK || found != 1)
            return fail("pj_sample_roots");
    } else {
        source = std::atoll(argv[5]);
    }
    if (pj_sssp(g, source, dist.data()) != PJ_OK) return fail("pj_sssp");
    const double t3 = now_s();
    if (pj_write_sol(dist.data(), n, argv[6], 1) != PJ_OK) return fail("pj_write_sol");
    const double t4 = now_s();
    std::printf("phases_s %.4f %.4f %.4f %.4f root %lld\n", t1 - t0, t2 - t1, t3 - t2, t4 - t3, (long long)source);
    pj_graph_destroy(g);
    pj_destroy(ctx);
    return 0;
}
