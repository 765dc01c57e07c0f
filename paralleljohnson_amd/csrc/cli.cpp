// cli.cpp — `[mpirun -np P] parallel_johnson webfile source_node sol_file`, the
// drop-in for the reference's process boundary (README:9; parallel_johnson()
// :286-676, main :678-684). Same arguments, same stderr progress lines, same
// stdout `Time:` line and the same sol_file bytes; the work runs on the GPU
// through libpj (include/pj.h).
//
// Differences that are not parity targets: lines the
// reference reads as undefined behaviour are rejected with a message and exit
// status 255 (the reference's error status, :35/:82/:302).
//
// Processes: P = PJ_GPUS, else the launcher's world size (OMPI_COMM_WORLD_SIZE,
// PMI_SIZE, PMIX_SIZE), else 1. Under a launcher only rank 0 works (the other
// ranks exit 0): it runs the P ranks of the 1D vertex partition itself through
// the n-GPU handle pj_multi (one host thread and one pj_ctx per rank, rank r on
// GPU r mod (visible GPUs)), over
// RCCL when every rank has its own GPU and over device copies otherwise
// (PJ_TRANSPORT=rccl|host overrides). P = 1 runs the single-GPU solver. The
// `Time:` line reports P, as the reference does (:603-604).
//
// Environment: PJ_DEVICE (HIP ordinal for P = 1, default 0 or LOCAL_RANK),
// PJ_WEIGHTED=1 (third column = weight, delta-stepping), PJ_CSR_CACHE (binary
// CSR cache: "1" for <webfile>.pjcsr, or a path; loaded instead of parsing when
// its stamp -- the text's size and mtime -- and weight mode match, else written
// after the parse; P = 1 only), PJ_PHASES=1 (phase times on stderr).
//
// Multi-source (Johnson-style rows; no reference counterpart, the reference
// takes one source per run, :448): PJ_SOURCES = a list of sources separated by
// commas or blanks, or "@file" with one source per line (each read with atoi,
// like argv[2]). argv[2] is then ignored and argv[3] is a pattern: "{s}" is
// replaced by the source, "{i}" by its index (no token: argv[3].<source>). Each
// file is byte-identical to a single-source run. With P > 1 the sources are
// sharded over P GPUs (source i on GPU i mod P), each holding a copy of the
// graph.
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
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

int launcher_value(std::initializer_list<const char*> keys, int dflt) {
    for (const char* k : keys) {
        const char* v = std::getenv(k);
        if (v && *v) return std::atoi(v);
    }
    return dflt;
}

int launcher_rank() { return launcher_value({"OMPI_COMM_WORLD_RANK", "PMI_RANK", "PMIX_RANK"}, 0); }

int process_count() {
    const int p = env_int("PJ_GPUS", 0);
    if (p > 0) return p;
    return std::max(1, launcher_value({"OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "PMIX_SIZE"}, 1));
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Phases {
    bool on = env_int("PJ_PHASES", 0) != 0;
    double t = now_s();
    void mark(const char* name) {
        const double u = now_s();
        if (on) std::cerr << "phase " << name << ": " << (u - t) << " s" << std::endl;
        t = u;
    }
};

// PJ_CSR_CACHE: "1" -> <webfile>.pjcsr, else the path given; unset -> no cache
std::string cache_path(const char* webfile) {
    const char* c = std::getenv("PJ_CSR_CACHE");
    if (!c || !*c) return "";
    return std::string(c) == "1" ? std::string(webfile) + ".pjcsr" : std::string(c);
}

// print_msg :49-53 (rank 0 only; only rank 0 gets this far)
void print_msg(const std::string& msg) { std::cerr << msg << std::endl; }

[[noreturn]] void fail(const std::string& what, int rc, const std::string& msg) {
    std::cerr << what << " failed (" << rc << "): " << msg << std::endl;
    std::exit(-1);
}
[[noreturn]] void fail(const char* what, int rc) { fail(what, rc, pj_last_error()); }

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

int transport_from_env() {
    const char* t = std::getenv("PJ_TRANSPORT");
    if (!t || !*t || !std::strcmp(t, "auto")) return PJ_TRANSPORT_AUTO;
    if (!std::strcmp(t, "rccl")) return PJ_TRANSPORT_RCCL;
    if (!std::strcmp(t, "host")) return PJ_TRANSPORT_HOST;
    std::cerr << "PJ_TRANSPORT must be auto, rccl or host" << std::endl;
    std::exit(-1);
}

// P ranks in this process through the n-GPU handle of the C-ABI (pj_multi)
pj_multi* make_multi(int P) {
    pj_multi* m = nullptr;
    const int rc = pj_multi_create(P, transport_from_env(), &m);
    if (rc != PJ_OK) fail("pj_multi_create", rc);
    return m;
}

// Source-sharded multi-source run: GPU r solves sources r, r+P, ... and writes their files.
int run_multi_source(const char* webfile, const std::vector<int64_t>& sources, const char* pattern, int P,
                     int weighted) {
    Phases ph;
    pj_multi* m = make_multi(P);
    const std::string cache = cache_path(webfile);
    pj_multi_set_csr_cache(m, cache.c_str());
    int rc = pj_multi_load_snap(m, webfile, weighted, PJ_LAYOUT_REPLICATED);
    if (rc != PJ_OK) fail("pj_load_snap", rc);
    pj_multi_info_t mi{};
    pj_multi_info(m, &mi);
    std::cerr << "N = " << mi.n << std::endl;
    print_msg("read in the webgraph is done.");
    ph.mark("load");
    std::cerr << "compute shortest paths from " << sources.size() << " source nodes" << std::endl;
    print_msg("parallel Johnson's algorithm starts......");
    std::vector<std::string> paths;
    std::vector<const char*> pp;
    for (size_t i = 0; i < sources.size(); ++i) paths.push_back(sol_path(pattern, sources[i], i));
    for (auto& q : paths) pp.push_back(q.c_str());
    double kms = 0;
    rc = pj_multi_sssp_batch_write(m, sources.data(), (int)sources.size(), pp.data(), 0, &kms);
    if (rc != PJ_OK) fail("pj_sssp_batch_write", rc);
    ph.mark("solve+write");
    print_msg("parallel Johnson's algorithm completes.");
    std::cout << "Time: " << kms / 1000.0 << " seconds when using " << P << " processes." << std::endl;
    std::cerr << "the shortest path distance vectors have been saved in files " << pattern << std::endl;
    pj_multi_destroy(m);
    return 0;
}

// The 1D vertex partition over P ranks in this process (the reference's np = P run).
int run_partitioned(const char* webfile, int source, const char* out, int P, int weighted) {
    Phases ph;
    pj_multi* m = make_multi(P);
    // rank 0's GPU parses the file once, every rank gets its block's entries (:313-338, :344-410)
    int rc = pj_multi_load_snap(m, webfile, weighted, PJ_LAYOUT_PARTITIONED);
    if (rc != PJ_OK) fail("load", rc);
    pj_multi_info_t mi{};
    pj_multi_info(m, &mi);
    const int64_t n = mi.n;
    std::cerr << "N = " << n << std::endl;  // :320
    print_msg("read in the webgraph is done.");
    print_msg("distribute sparse matrix is done.");
    ph.mark("load");
    std::cerr << "compute shortest paths from source node: " << source << std::endl;
    print_msg("parallel Johnson's algorithm starts......");
    std::vector<int32_t> dist((size_t)n);
    pj_part_stats st{};
    rc = pj_multi_sssp(m, source, dist.data(), &st);  // solve + MPI_Gatherv :612-614
    if (rc != PJ_OK) fail(weighted ? "pj_wpart_delta_group" : "pj_part_bfs_group", rc);
    ph.mark("solve+gather");
    print_msg("parallel Johnson's algorithm completes.");
    std::cout << "Time: " << st.solve_ms / 1000.0 << " seconds when using " << P << " processes." << std::endl;
    rc = pj_write_sol(dist.data(), n, out, 0);  // :615-618
    if (rc != PJ_OK) fail("pj_write_sol", rc);
    ph.mark("write");
    std::cerr << "the shortest path distance vector has been saved in file " << out << std::endl;
    pj_multi_destroy(m);
    return 0;
}

// PJ_PARENTS=<path>: the shortest-path tree of the solve, validated by the Graph500
// checks on the device (a failed check is an error, rc 255), written as one parent
// id per line. No reference counterpart.
void write_tree(pj_graph* g, int source, int64_t n, const char* path) {
    std::vector<int64_t> parent((size_t)n);
    int rc = pj_parent_tree(g, parent.data());
    if (rc != PJ_OK) fail("pj_parent_tree", rc);
    pj_tree_report r{};
    rc = pj_validate_tree(g, source, parent.data(), &r);
    if (rc != PJ_OK) fail("pj_validate_tree", rc);
    const int64_t bad = r.bad_root + r.bad_reach + r.bad_tree_edge + r.bad_edge + r.bad_cycle;
    std::cerr << "parent tree: " << r.reached << " vertices reached, validation "
              << (bad ? "FAILED" : "passed") << " (root " << r.bad_root << ", reach " << r.bad_reach << ", tree edges "
              << r.bad_tree_edge << ", edges " << r.bad_edge << ", cycles " << r.bad_cycle << ")" << std::endl;
    if (bad) std::exit(-1);
    rc = pj_write_parents(parent.data(), n, path);
    if (rc != PJ_OK) fail("pj_write_parents", rc);
    std::cerr << "the parent tree has been saved in file " << path << std::endl;
}

int run_single(const char* webfile, int source, const char* out, int weighted) {
    Phases ph;
    pj_ctx* ctx = nullptr;
    int rc = pj_create(env_int("PJ_DEVICE", env_int("LOCAL_RANK", 0)), &ctx);
    if (rc != PJ_OK) fail("pj_create", rc);
    ph.mark("init");
    pj_graph* g = nullptr;
    const std::string cache = cache_path(webfile);
    rc = pj_load_snap_cached(ctx, webfile, weighted, cache.empty() ? nullptr : cache.c_str(), 1, &g);
    if (rc != PJ_OK) fail("pj_load_snap", rc);
    int64_t n = 0;
    pj_graph_info(g, &n, nullptr, nullptr, nullptr);
    std::cerr << "N = " << n << std::endl;  // :320
    print_msg("read in the webgraph is done.");
    print_msg("distribute sparse matrix is done.");
    ph.mark("load");
    pj_load_stats ls{};
    if (ph.on && pj_graph_load_stats(g, &ls) == PJ_OK)
        std::cerr << "phase load: file->HBM " << ls.read_ms / 1000.0 << " s (read and H2D overlapped), parse "
                  << ls.parse_ms / 1000.0 << " s, csr " << ls.csr_ms / 1000.0 << " s (" << ls.text_bytes
                  << " bytes of text)" << std::endl;
    std::cerr << "compute shortest paths from source node: " << source << std::endl;
    print_msg("parallel Johnson's algorithm starts......");
    // the distance buffer: not zero-filled; a host thread faults its pages in while the
    // GPU solves, so the D2H copy lands in resident memory
    std::unique_ptr<int32_t[]> dist(new int32_t[(size_t)std::max<int64_t>(n, 1)]);
    std::thread warm([&] {
        char* b = reinterpret_cast<char*>(dist.get());
        for (size_t o = 0; o < (size_t)n * sizeof(int32_t); o += 4096) b[o] = 0;
    });
    rc = pj_sssp(g, source, nullptr);
    warm.join();
    if (rc != PJ_OK) fail("pj_sssp", rc);
    pj_stats st{};
    pj_last_stats(g, &st);
    const double t_elapsed = st.kernel_ms / 1000.0;  // device time of the solve (:597-605 analogue)
    ph.mark("solve");
    rc = pj_copy_dist(g, dist.get());  // :612-614's gather
    if (rc != PJ_OK) fail("pj_copy_dist", rc);
    ph.mark("d2h");
    print_msg("parallel Johnson's algorithm completes.");
    std::cout << "Time: " << t_elapsed << " seconds when using " << 1 << " processes." << std::endl;
    rc = pj_write_sol(dist.get(), n, out, 0);  // :615-618
    if (rc != PJ_OK) fail("pj_write_sol", rc);
    ph.mark("write");
    std::cerr << "the shortest path distance vector has been saved in file " << out << std::endl;
    if (const char* pp = std::getenv("PJ_PARENTS"); pp && *pp) write_tree(g, source, n, pp);
    if (!env_int("PJ_TEARDOWN", 0)) {
        // the sol_file is closed: end without the graph / context destruction and the
        // HIP runtime's exit-time teardown (~0.15 s at s26, r4a), which no output needs
        std::cout.flush();
        std::cerr.flush();
        std::fflush(nullptr);
        _exit(0);
    }
    pj_graph_destroy(g);
    pj_destroy(ctx);
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
    const int P = process_count();
    const int weighted = env_int("PJ_WEIGHTED", 0);

    print_msg("process 0 reads in the web graph data......");
    const char* srcs = std::getenv("PJ_SOURCES");
    const char* parents = std::getenv("PJ_PARENTS");
    if (parents && *parents && (P > 1 || (srcs && *srcs))) {
        std::cerr << "PJ_PARENTS: the parent tree needs a single-source run on one GPU (P = 1, no PJ_SOURCES)"
                  << std::endl;
        std::exit(-1);
    }
    if (srcs && *srcs) return run_multi_source(argv[1], parse_sources(srcs), argv[3], P, weighted);
    const int source_node = std::atoi(argv[2]);  // :448
    if (P > 1) return run_partitioned(argv[1], source_node, argv[3], P, weighted);
    return run_single(argv[1], source_node, argv[3], weighted);
}
