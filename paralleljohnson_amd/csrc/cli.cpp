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
// ranks exit 0): it runs the P ranks of the 1D vertex partition itself, one
// host thread and one pj_ctx each, rank r on GPU r mod (visible GPUs), over
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
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
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

int device_count() {
    int n = 0;
    pj_device_count(&n);
    return n;
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

// print_msg :49-53 (rank 0 only; only rank 0 gets this far)
void print_msg(const std::string& msg) { std::cerr << msg << std::endl; }

[[noreturn]] void fail(const std::string& what, int rc, const std::string& msg) {
    std::cerr << what << " failed (" << rc << "): " << msg << std::endl;
    std::exit(-1);
}
[[noreturn]] void fail(const char* what, int rc) { fail(what, rc, pj_last_error()); }

// fn(r) on one thread per rank; exits on the first failure (the root cause, not a peer's)
template <typename F>
void per_rank(int P, const char* what, F&& fn) {
    std::vector<int> rcs((size_t)P, PJ_OK);
    std::vector<std::string> msgs((size_t)P);
    std::vector<std::thread> th;
    for (int r = 0; r < P; ++r)
        th.emplace_back([&, r] {
            rcs[(size_t)r] = fn(r);
            if (rcs[(size_t)r] != PJ_OK) msgs[(size_t)r] = pj_last_error();
        });
    for (auto& t : th) t.join();
    for (int r = 0; r < P; ++r)
        if (rcs[(size_t)r] != PJ_OK && rcs[(size_t)r] != PJ_ERR_COMM)
            fail(std::string(what) + " (rank " + std::to_string(r) + ")", rcs[(size_t)r], msgs[(size_t)r]);
    for (int r = 0; r < P; ++r)
        if (rcs[(size_t)r] != PJ_OK)
            fail(std::string(what) + " (rank " + std::to_string(r) + ")", rcs[(size_t)r], msgs[(size_t)r]);
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

std::vector<pj_ctx*> make_ctxs(int P) {
    const int ndev = std::max(1, device_count());
    std::vector<pj_ctx*> ctxs((size_t)P, nullptr);
    for (int r = 0; r < P; ++r) {
        const int rc = pj_create(r % ndev, &ctxs[(size_t)r]);
        if (rc != PJ_OK) fail("pj_create", rc);
    }
    return ctxs;
}

// Source-sharded multi-source run: GPU r solves sources r, r+P, ... and writes their files.
int run_multi_source(const char* webfile, const std::vector<int64_t>& sources, const char* pattern, int P,
                     int weighted) {
    Phases ph;
    std::vector<pj_ctx*> ctxs = make_ctxs(P);
    std::vector<pj_graph*> gs((size_t)P, nullptr);
    per_rank(P, "pj_load_snap", [&](int r) { return load_graph(ctxs[(size_t)r], webfile, weighted, &gs[(size_t)r]); });
    int64_t n = 0;
    pj_graph_info(gs[0], &n, nullptr, nullptr, nullptr);
    std::cerr << "N = " << n << std::endl;
    print_msg("read in the webgraph is done.");
    ph.mark("load");
    std::cerr << "compute shortest paths from " << sources.size() << " source nodes" << std::endl;
    print_msg("parallel Johnson's algorithm starts......");
    std::vector<double> kms((size_t)P, 0.0);
    per_rank(P, "pj_sssp_batch_write", [&](int r) {
        std::vector<int64_t> mine;
        std::vector<std::string> paths;
        for (size_t i = (size_t)r; i < sources.size(); i += (size_t)P) {
            mine.push_back(sources[i]);
            paths.push_back(sol_path(pattern, sources[i], i));
        }
        if (mine.empty()) return (int)PJ_OK;
        std::vector<const char*> pp;
        for (auto& q : paths) pp.push_back(q.c_str());
        int rc = pj_sssp_batch_write(gs[(size_t)r], mine.data(), (int)mine.size(), pp.data(), 0);
        pj_stats st{};
        if (rc == PJ_OK && pj_last_stats(gs[(size_t)r], &st) == PJ_OK) kms[(size_t)r] = st.kernel_ms;
        return rc;
    });
    ph.mark("solve+write");
    print_msg("parallel Johnson's algorithm completes.");
    const double t = *std::max_element(kms.begin(), kms.end()) / 1000.0;
    std::cout << "Time: " << t << " seconds when using " << P << " processes." << std::endl;
    std::cerr << "the shortest path distance vectors have been saved in files " << pattern << std::endl;
    for (int r = 0; r < P; ++r) {
        pj_graph_destroy(gs[(size_t)r]);
        pj_destroy(ctxs[(size_t)r]);
    }
    return 0;
}

int transport_from_env() {
    const char* t = std::getenv("PJ_TRANSPORT");
    if (!t || !*t || !std::strcmp(t, "auto")) return PJ_TRANSPORT_AUTO;
    if (!std::strcmp(t, "rccl")) return PJ_TRANSPORT_RCCL;
    if (!std::strcmp(t, "host")) return PJ_TRANSPORT_HOST;
    std::cerr << "PJ_TRANSPORT must be auto, rccl or host" << std::endl;
    std::exit(-1);
}

// The 1D vertex partition over P ranks in this process (the reference's np = P run).
int run_partitioned(const char* webfile, int source, const char* out, int P, int weighted) {
    Phases ph;
    std::vector<pj_ctx*> ctxs = make_ctxs(P);
    std::vector<pj_comm*> comms((size_t)P, nullptr);
    int rc = pj_comm_create_group(ctxs.data(), P, transport_from_env(), comms.data());
    if (rc != PJ_OK) fail("pj_comm_create_group", rc);
    std::vector<pj_part*> parts((size_t)P, nullptr);
    std::vector<pj_wpart*> wparts((size_t)P, nullptr);
    // every rank builds its own rows on its GPU: no scatter (:344-410)
    per_rank(P, "load", [&](int r) {
        return weighted ? pj_wpart_load_snap(ctxs[(size_t)r], webfile, r, P, &wparts[(size_t)r])
                        : pj_part_load_snap(ctxs[(size_t)r], webfile, r, P, &parts[(size_t)r]);
    });
    int64_t n = 0;
    if (weighted) {
        int64_t info[8];
        pj_wpart_info(wparts[0], info);
        n = info[0];
    } else {
        pj_part_info pi{};
        pj_part_info_get(parts[0], &pi);
        n = pi.n;
    }
    std::cerr << "N = " << n << std::endl;  // :320
    print_msg("read in the webgraph is done.");
    print_msg("distribute sparse matrix is done.");
    ph.mark("load");
    std::cerr << "compute shortest paths from source node: " << source << std::endl;
    print_msg("parallel Johnson's algorithm starts......");
    std::vector<pj_part_stats> st((size_t)P);
    rc = weighted ? pj_wpart_delta_group(P, wparts.data(), comms.data(), source, 0, st.data())
                  : pj_part_bfs_group(P, parts.data(), comms.data(), source, st.data());
    if (rc != PJ_OK) fail(weighted ? "pj_wpart_delta_group" : "pj_part_bfs_group", rc);
    double t = 0;
    for (auto& s : st) t = std::max(t, s.solve_ms / 1000.0);  // max over ranks (:597-605)
    ph.mark("solve");
    std::vector<int32_t> dist((size_t)n);
    per_rank(P, "gather", [&](int r) {  // MPI_Gatherv :612-614
        int32_t* o = r == 0 ? dist.data() : nullptr;
        return weighted ? pj_wpart_gather_dist(wparts[(size_t)r], comms[(size_t)r], o)
                        : pj_part_gather_dist(parts[(size_t)r], comms[(size_t)r], o);
    });
    print_msg("parallel Johnson's algorithm completes.");
    std::cout << "Time: " << t << " seconds when using " << P << " processes." << std::endl;
    rc = pj_write_sol(dist.data(), n, out, 0);  // :615-618
    if (rc != PJ_OK) fail("pj_write_sol", rc);
    ph.mark("gather+write");
    std::cerr << "the shortest path distance vector has been saved in file " << out << std::endl;
    for (int r = 0; r < P; ++r) {
        pj_part_destroy(parts[(size_t)r]);
        pj_wpart_destroy(wparts[(size_t)r]);
        pj_comm_destroy(comms[(size_t)r]);
        pj_destroy(ctxs[(size_t)r]);
    }
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
    rc = load_graph(ctx, webfile, weighted, &g);
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
    std::vector<int32_t> dist((size_t)n);
    rc = pj_sssp(g, source, nullptr);
    if (rc != PJ_OK) fail("pj_sssp", rc);
    pj_stats st{};
    pj_last_stats(g, &st);
    const double t_elapsed = st.kernel_ms / 1000.0;  // device time of the solve (:597-605 analogue)
    ph.mark("solve");
    rc = pj_copy_dist(g, dist.data());  // :612-614's gather
    if (rc != PJ_OK) fail("pj_copy_dist", rc);
    ph.mark("d2h");
    print_msg("parallel Johnson's algorithm completes.");
    std::cout << "Time: " << t_elapsed << " seconds when using " << 1 << " processes." << std::endl;
    rc = pj_write_sol(dist.data(), n, out, 0);  // :615-618
    if (rc != PJ_OK) fail("pj_write_sol", rc);
    ph.mark("write");
    std::cerr << "the shortest path distance vector has been saved in file " << out << std::endl;
    if (const char* pp = std::getenv("PJ_PARENTS"); pp && *pp) write_tree(g, source, n, pp);
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
