// cli.cpp — `parallel_johnson webfile source_node sol_file`, the drop-in for
// the reference's process boundary (README:9; parallel_johnson() :286-676,
// main :678-684). Same arguments, same stderr progress lines, same stdout
// `Time:` line and the same sol_file bytes; the work runs on the GPU through
// libpj (include/pj.h).
//
// Differences that are not parity targets: lines the
// reference reads as undefined behaviour are rejected with a message and exit
// status 255 (the reference's error status, :35/:82/:302).
//
// Environment: PJ_DEVICE (HIP ordinal, default 0 or LOCAL_RANK), PJ_WEIGHTED=1
// (third column = weight, delta-stepping), PJ_CSR_CACHE (binary CSR cache: "1"
// for <webfile>.pjcsr, or a path; loaded instead of parsing when its stamp --
// the text's size and mtime -- and weight mode match, else written after the
// parse). Under an MPI-style launcher only rank 0 works; the other ranks exit 0.
//
// Multi-source (Johnson-style rows; no reference counterpart, the reference
// takes one source per run, :448): PJ_SOURCES = a list of sources separated by
// commas or blanks, or "@file" with one source per line (each read with atoi,
// like argv[2]). argv[2] is then ignored and argv[3] is a pattern: "{s}" is
// replaced by the source, "{i}" by its index (no token: argv[3].<source>). Each
// file is byte-identical to a single-source run. With PJ_GPUS = P > 1 the
// sources are sharded over P GPUs (source r, r+P, ... on GPU r), each holding a
// copy of the graph.
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pj.h"

namespace {

int env_int(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return v && *v ? std::atoi(v) : dflt;
}

int launcher_rank() {
    for (const char* k : {"OMPI_COMM_WORLD_RANK", "PMI_RANK", "PMIX_RANK", "RANK"}) {
        const char* v = std::getenv(k);
        if (v && *v) return std::atoi(v);
    }
    return 0;
}

// The graph of `path`: from the binary CSR cache when PJ_CSR_CACHE names a fresh one,
// else parsed (pj_load_snap) and, with PJ_CSR_CACHE set, cached for the next run.
int load_graph(pj_ctx* ctx, const char* path, int weighted, pj_graph** g) {
    const char* cache = std::getenv("PJ_CSR_CACHE");
    struct stat sb {};
    if (!cache || !*cache || stat(path, &sb) != 0) return pj_load_snap(ctx, path, weighted, g);
    const std::string cpath = std::string(cache) == "1" ? std::string(path) + ".pjcsr" : std::string(cache);
    const int64_t size = (int64_t)sb.st_size;
    const int64_t mtime = (int64_t)sb.st_mtim.tv_sec * 1000000000ll + (int64_t)sb.st_mtim.tv_nsec;
    if (pj_load_csr_file(ctx, cpath.c_str(), size, mtime, g) == PJ_OK) {
        int w = 0;
        pj_graph_info(*g, nullptr, nullptr, &w, nullptr);
        if (w == (weighted != 0)) return PJ_OK;
        pj_graph_destroy(*g);
        *g = nullptr;
    }
    const int rc = pj_load_snap(ctx, path, weighted, g);
    if (rc == PJ_OK && pj_graph_save(*g, cpath.c_str(), size, mtime) != PJ_OK)
        std::cerr << "warning: could not write the CSR cache " << cpath << ": " << pj_last_error() << std::endl;
    return rc;
}

// print_msg :49-53
void print_msg(const std::string& msg, int rank) {
    if (rank == 0) std::cerr << msg << std::endl;
}

[[noreturn]] void fail(const char* what, int rc) {
    std::cerr << what << " failed (" << rc << "): " << pj_last_error() << std::endl;
    std::exit(-1);
}

int device_count() {
    static int n = -1;
    if (n < 0) {
        n = 0;
        pj_device_count(&n);
    }
    return n;
}

// PJ_SOURCES: "a,b c" or "@file" (one per line); every token read with atoi (:448)
std::vector<int64_t> parse_sources(const char* spec) {
    std::string text;
    if (spec[0] == '@') {
        std::ifstream f(spec + 1);
        if (!f) {
            std::cerr << "cannot read the source list " << (spec + 1) << std::endl;
            std::exit(-1);
        }
        std::stringstream ss;
        ss << f.rdbuf();
        text = ss.str();
    } else {
        text = spec;
    }
    std::vector<int64_t> out;
    std::string tok;
    auto flush = [&] {
        if (!tok.empty()) out.push_back(std::atoi(tok.c_str()));
        tok.clear();
    };
    for (char c : text) {
        if (c == ',' || c == '\n' || c == '\r' || c == ' ' || c == '\t') flush();
        else tok += c;
    }
    flush();
    return out;
}

// Per-source sol_file path: every "{s}" in the pattern becomes the source (decimal,
// as atoi read it), every "{i}" its index in the list; no token: pattern + "." + source.
std::string sol_path(const std::string& pat, int64_t src, size_t idx) {
    std::string out;
    bool tok = false;
    for (size_t i = 0; i < pat.size(); ++i) {
        if (pat.compare(i, 3, "{s}") == 0 || pat.compare(i, 3, "{i}") == 0) {
            out += std::to_string(pat[i + 1] == 's' ? src : (int64_t)idx);
            i += 2;
            tok = true;
        } else {
            out += pat[i];
        }
    }
    if (!tok) out += "." + std::to_string(src);
    return out;
}

// Source-sharded multi-source run: GPU r solves sources r, r+P, ... and writes their files.
int run_multi_source(const char* webfile, const std::vector<int64_t>& sources, const char* pattern, int gpus,
                     int weighted) {
    std::cerr << "compute shortest paths from " << sources.size() << " source nodes on " << gpus << " GPU(s)"
              << std::endl;
    std::cerr << "parallel Johnson's algorithm starts......" << std::endl;
    std::vector<double> kms((size_t)gpus, 0.0);
    std::vector<int> rcs((size_t)gpus, PJ_OK);
    std::vector<std::string> errs((size_t)gpus);
    std::vector<std::thread> th;
    int64_t n_all = 0;
    for (int r = 0; r < gpus; ++r)
        th.emplace_back([&, r] {
            pj_ctx* ctx = nullptr;
            pj_graph* g = nullptr;
            int rc = pj_create(r % std::max(1, device_count()), &ctx);
            if (rc == PJ_OK) rc = load_graph(ctx, webfile, weighted, &g);
            std::vector<int64_t> mine;
            std::vector<std::string> paths;
            for (size_t i = (size_t)r; i < sources.size(); i += (size_t)gpus) {
                mine.push_back(sources[i]);
                paths.push_back(sol_path(pattern, sources[i], i));
            }
            std::vector<const char*> pp;
            for (auto& q : paths) pp.push_back(q.c_str());
            if (rc == PJ_OK && r == 0) pj_graph_info(g, &n_all, nullptr, nullptr, nullptr);
            if (rc == PJ_OK && !mine.empty()) {
                rc = pj_sssp_batch_write(g, mine.data(), (int)mine.size(), pp.data(), 0);
                pj_stats st{};
                if (rc == PJ_OK && pj_last_stats(g, &st) == PJ_OK) kms[(size_t)r] = st.kernel_ms;
            }
            if (rc != PJ_OK) errs[(size_t)r] = pj_last_error();
            rcs[(size_t)r] = rc;
            pj_graph_destroy(g);
            pj_destroy(ctx);
        });
    for (auto& t : th) t.join();
    for (int r = 0; r < gpus; ++r)
        if (rcs[(size_t)r] != PJ_OK) {
            std::cerr << "GPU " << r << " failed (" << rcs[(size_t)r] << "): " << errs[(size_t)r] << std::endl;
            std::exit(-1);
        }
    std::cerr << "N = " << n_all << std::endl;
    std::cerr << "parallel Johnson's algorithm completes." << std::endl;
    const double t = *std::max_element(kms.begin(), kms.end()) / 1000.0;
    std::cout << "Time: " << t << " seconds when using " << gpus << " processes." << std::endl;
    std::cerr << "the shortest path distance vectors have been saved in files " << pattern << std::endl;
    return 0;
}

}  // namespace

int main(int argc, char* argv[]) {
    const int rank = launcher_rank();
    if (argc != 4) {  // :294-303
        if (rank == 0) {
            std::cerr << "to run this program must supply the following command "
                         "line arguments (in order)"
                      << std::endl;
            std::cerr << "argv[1]---web graph file." << std::endl;
            std::cerr << "argv[2]---source node number." << std::endl;
            std::cerr << "argv[3]---file to save the solution." << std::endl;
        }
        std::exit(-1);
    }
    if (rank != 0) return 0;

    const char* srcs = std::getenv("PJ_SOURCES");
    if (srcs && *srcs) {
        print_msg("process 0 reads in the web graph data......", rank);
        const int gpus = std::max(1, env_int("PJ_GPUS", 1));
        return run_multi_source(argv[1], parse_sources(srcs), argv[3], gpus, env_int("PJ_WEIGHTED", 0));
    }

    print_msg("process 0 reads in the web graph data......", rank);
    pj_ctx* ctx = nullptr;
    int rc = pj_create(env_int("PJ_DEVICE", env_int("LOCAL_RANK", 0)), &ctx);
    if (rc != PJ_OK) fail("pj_create", rc);
    pj_graph* g = nullptr;
    rc = load_graph(ctx, argv[1], env_int("PJ_WEIGHTED", 0), &g);
    if (rc != PJ_OK) fail("pj_load_snap", rc);
    int64_t n = 0;
    pj_graph_info(g, &n, nullptr, nullptr, nullptr);
    std::cerr << "N = " << n << std::endl;  // :320
    print_msg("read in the webgraph is done.", rank);
    print_msg("distribute sparse matrix is done.", rank);

    const int source_node = std::atoi(argv[2]);  // :448
    std::cerr << "compute shortest paths from source node: " << source_node << std::endl;
    std::cerr << "parallel Johnson's algorithm starts......" << std::endl;

    std::vector<int32_t> dist((size_t)n);
    rc = pj_sssp(g, source_node, dist.data());
    if (rc != PJ_OK) fail("pj_sssp", rc);
    pj_stats st{};
    pj_last_stats(g, &st);
    const double t_elapsed = st.kernel_ms / 1000.0;  // device time of the solve (:597-605 analogue)
    std::cerr << "parallel Johnson's algorithm completes." << std::endl;
    std::cout << "Time: " << t_elapsed << " seconds when using " << 1 << " processes." << std::endl;

    rc = pj_write_sol(dist.data(), n, argv[3], 0);  // :615-618
    if (rc != PJ_OK) fail("pj_write_sol", rc);
    std::cerr << "the shortest path distance vector has been saved in file " << argv[3] << std::endl;

    pj_graph_destroy(g);
    pj_destroy(ctx);
    return 0;
}
