// internal.h — shared declarations of libpj (host + device). Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <stdexcept>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/pj.h"

namespace pj {

using u32 = uint32_t;
using u64 = unsigned long long;  // matches HIP's 64-bit atomic overloads
using i64 = int64_t;

constexpr int32_t INT_INF = PJ_INT_INF;

// ---------------------------------------------------------------- errors --
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_error(const std::string& msg);

#define PJ_HIP(expr)                                                                     \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            throw ::pj::Error(e_ == hipErrorOutOfMemory ? PJ_ERR_OOM : PJ_ERR_HIP,       \
                              std::string(#expr) + ": " + hipGetErrorString(e_) +        \
                                  " (" __FILE__ ":" + std::to_string(__LINE__) + ")");   \
    } while (0)

#define PJ_LAUNCH_CHECK() PJ_HIP(hipGetLastError())

// ------------------------------------------------------------ device memory --
// Device allocations of DevBuf. Blocks of 1 GiB and more are kept by a process-wide cache
// when freed and handed out again (devmem.cpp): the partitioned builds allocate and free
// tens of GB of sort temporaries, and a hipMalloc that has to take fresh device memory
// from the driver took seconds for one 17-34 GB block (round 5, the bench's partition legs).
void* dev_alloc(size_t bytes);
void dev_free(void* p, size_t bytes);
size_t dev_trim();  // cached big blocks without a live slice back to the driver; bytes released
size_t dev_free_bytes();  // free device memory of the current device, the cache's idle ranges included

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    explicit DevBuf(size_t count) { alloc(count); }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
        return *this;
    }
    ~DevBuf() { release(); }
    void alloc(size_t count) {
        release();
        n = count;
        if (count) p = static_cast<T*>(dev_alloc(count * sizeof(T)));
    }
    void ensure(size_t count) { if (count > n) alloc(count); }
    void release() {
        if (p) dev_free(p, n * sizeof(T));
        p = nullptr;
        n = 0;
    }
    T* get() const { return p; }
    size_t bytes() const { return n * sizeof(T); }
};

template <typename T>
struct PinnedBuf {
    T* p = nullptr;
    size_t n = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf() { if (p) (void)hipHostFree(p); }
    void alloc(size_t count) {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = count;
        if (count) PJ_HIP(hipHostMalloc(reinterpret_cast<void**>(&p), count * sizeof(T), hipHostMallocDefault));
    }
};

// The automatic light threshold of the weighted solvers (v2 and the weighted partition):
// delta = c(n) x mean weight / mean out-degree, c(n) = 0.1875 log2(n) - 1.875 within
// [2, 3.5]. Round 5 re-swept delta on Kronecker weights 1..255, edgefactor 16
// (profiles/r05/delta_sweep_r5ag.txt): the best delta was 8-10 at s22, 10-11 at s24 and 12
// at s26 (c = 2.25, 2.6, 3.0), against the constant 3.5 (delta 14) of round 1; +38%, +19%
// and +4% GTEPS.
inline double auto_delta(double n, double nnz, double mean_w) {
    const double mean_deg = n > 0 ? nnz / n : 1.0;
    const double c = std::min(3.5, std::max(2.0, 0.1875 * std::log2(std::max(n, 2.0)) - 1.875));
    return std::max(1.0, std::min(65536.0, std::round(c * mean_w / std::max(1.0, mean_deg))));
}

inline unsigned grid_for(i64 work, int per_block, unsigned cap = 256u * 16u) {
    i64 g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > (i64)cap) g = cap;
    return (unsigned)g;
}

// ---------------------------------------------------------------- scan ----
// Exclusive scan of n u32 (or u64) values into out[0..n] (out[n] = total).
// Scratch is managed internally per call-site via ScanWs.
struct ScanWs {
    DevBuf<u64> part;  // block partials of every recursion level
    void ensure(i64 n);
};
void exclusive_scan_u32(const u32* in, u64* out, i64 n, ScanWs& ws, hipStream_t s);
void exclusive_scan_u64(const u64* in, u64* out, i64 n, ScanWs& ws, hipStream_t s);

// ---------------------------------------------------------------- sort ----
// Stable LSD radix sort of (key, value) pairs by key; `bits` = key width to
// sort. Returns through `*kout/*vout` which of the two buffers holds the result.
struct SortWs {
    DevBuf<u32> hist, csum;  // per-tile digit counts [tile][256], per-chunk digit sums [digit][chunk]
    DevBuf<u64> offs, cpre;  // per-tile run starts [tile][256], scanned chunk sums
    ScanWs scan;
};
template <typename V>
void radix_sort_pairs(u32* keys, u32* keys_alt, V* vals, V* vals_alt, i64 n, int bits, SortWs& ws,
                      hipStream_t s, u32** kout, V** vout);

// row_ptr[v] = lower_bound(sorted_keys, v) for v in [0, nv]
template <typename Off>
void csr_bounds(const u32* sorted_keys, i64 nnz, i64 nv, Off* row, hipStream_t s);

// ---------------------------------------------------------------- graph ---
struct Ctx {
    int device = 0;
    hipStream_t stream = nullptr;      // where work is launched (own or external)
    hipStream_t own_stream = nullptr;  // created by pj_create, destroyed by pj_destroy
    int cu_count = 256;
    // pinned staging slots of the file loader (api.cpp read_file_to_device), kept for the
    // ctx's lifetime; freed by pj_destroy
    std::vector<char*> stage;
    std::vector<hipEvent_t> stage_ev;
};

struct BfsWorkHolder;
void delete_bfs_work(BfsWorkHolder* p);
struct BfsWorkDeleter {
    void operator()(BfsWorkHolder* p) const { delete_bfs_work(p); }
};
struct MsWork;
void delete_ms_work(MsWork* p);
struct MsWorkDeleter {
    void operator()(MsWork* p) const { delete_ms_work(p); }
};
struct DeltaWork;
void delete_delta_work(DeltaWork* p);
struct DeltaWorkDeleter {
    void operator()(DeltaWork* p) const { delete_delta_work(p); }
};

// Degree-ordered copy of a graph for the weighted solver (relabel.hip): new
// ids put vertices with in- or out-edges first, by out-degree descending, so
// the distance entries the relaxations hit are dense and the hot ones share
// cache lines. Rows keep their edge order (weight-sorted).
struct Relabeled {
    i64 n_scan = 0;           // vertices with any edge: new ids [0, n_scan)
    DevBuf<u32> perm, inv;    // new -> old, old -> new
    DevBuf<u32> row32;
    DevBuf<u64> row64;
    DevBuf<u32> col;
    DevBuf<uint8_t> w8;       // weights as u8 when every weight fits (the copy's form), else
    DevBuf<u32> w;            // u32 (also widened from w8 on demand: v1, interleaved records)
    DevBuf<int32_t> dist;     // solver distances in new ids
    const void* row_ptr(bool off64) const { return off64 ? (const void*)row64.p : (const void*)row32.p; }
};

struct Graph {
    Ctx* ctx = nullptr;
    i64 n = 0, nnz = 0;
    bool weighted = false, symmetric = false;
    bool off64 = false;  // 64-bit row offsets when nnz >= 2^32
    // CSR (out-edges)
    DevBuf<u32> row32, crow32;
    DevBuf<u64> row64, crow64;
    DevBuf<u32> col, ccol;  // ccol/crow*: CSC (in-edges) for pull steps; alias CSR when symmetric
    DevBuf<u32> w;          // CSR-aligned weights (weighted graphs)
    DevBuf<u32> ccol_hf;    // hub_first: the in-rows ordered highest-degree in-neighbour first (pull_ccol)

    // per-solve workspace (lazily sized)
    DevBuf<int32_t> dist;
    DevBuf<u64> visited;
    DevBuf<u32> qv[2], qdeg[2];
    DevBuf<u64> qbeg[2];
    DevBuf<u64> qoff;
    DevBuf<u64> counters;  // device counters (BfsCounters / DeltaCounters)
    PinnedBuf<u64> hcounters;
    ScanWs scan;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::unique_ptr<BfsWorkHolder, BfsWorkDeleter> bfs_work;
    std::unique_ptr<MsWork, MsWorkDeleter> ms_work;
    std::unique_ptr<DeltaWork, DeltaWorkDeleter> delta_work;
    double mean_weight = -1.0;  // weighted: computed on first delta solve
    long long max_weight = -1;  // weighted: with mean_weight (-1: not computed)
    std::unique_ptr<Relabeled> rl;  // weighted: built on the first delta solve

    // options
    double alpha = 14.0, delta = 0.0;
    double beta = 32.0;  // BFS: pull -> push once the frontier is below n / beta and shrinking (24 until round 6:
                         // 32 with the hub-first pulls, K22 median kernel time 0.190 -> 0.182 ms, web-Google
                         // equal, profiles/r06/bfs_beta_r6aq.txt)
    double pull_vertex = 2.0;  // BFS: push -> pull also when the frontier's out-edges > pull_vertex x the
                               // unvisited vertices (0 = Beamer's rule alone). With hub-first in-rows a
                               // pull probes ~2 in-edges per unvisited vertex, a push pays an atomic per
                               // frontier edge: K22 bench roots 0.2224 -> 0.2007 ms mean kernel time
                               // (1: 0.2006, 0.5: 0.2095, 4: 0.2227; web-Google equal at 1),
                               // profiles/r06/bfs_pull_vertex_r6h.txt
    double pull_factor = 4.0;  // symmetric: pull a band's heavy edges when the heavy edges of unsettled
                               // vertices < pull_factor x the members' heavy edges (0 = never)
    double defer_heavy = 0.002; // v2, symmetric: a heavy push of members holding >= defer_heavy x nnz heavy
                                // edges relaxes only the edges that land in the next band and leaves the
                                // rest to the next heavy step (§4.2; 0 = off)
    double band_width = 0.0;   // v2: width of a band [lo, lo + band_width) (0 = delta, at most delta)
    double tail_delta = -1.0;  // v2: light threshold and band width of the tail (0 = off, < 0 = 64 x delta):
    int tail_after = 1;        // from the first band >= tail_after at which the edges of unsettled
    double tail_frac = 0.2;    // vertices are < tail_frac x nnz (profiles/r01/tail_sweep.txt; 0.1 until
                               // round 5: 0.2 +1% at s22w-s26w with the round-5 delta, delta_sweep_r5ag.txt)
    double light_pull = 6.0;   // v2, symmetric: pull a light round when its frontier's light edges exceed
                               // the light edges of unsettled vertices / light_pull (0 = never; 2 -> 3 at
                               // the end of round 2 with merged rounds: +1%, interleaved A/B; 3 -> 6 late
                               // in round 5 with the cheaper pulls: +0.6%, profiles/r05/sweeps_r5h14.txt)
    double tail_light_pull = 3.0;  // the same rule in the tail's rounds
    int round_log = 0;         // debug: per light round (kind, frontier, light edges) on stderr
    int level_log = 0;         // debug: per BFS level launch (level, direction, frontier, edges, scanned) on stderr
    int force_mode = 0;  // 0 auto, 1 push (top-down) only, 2 pull (bottom-up) from level 0
    int level_batch = 0; // BFS levels enqueued per host check (0 = the previous solve's count, then 2, 4, 8, ...)
    double dense_frac = 0.1; // delta v2: a light round with a frontier above dense_frac x n runs tile-dense (0 = never;
                             // swept 0 / 0.02 / 0.1 / 0.3 on k26w: 0.1 best)
    int light_filter = 1;  // delta v2: skip vertices without light edges in light rounds (hl bitmap)
    int light_pack = 1;    // delta v2: light CSR records packed in 32 bits when they fit (0/1)
    int split_w = 1;       // delta v2: whole-CSR reads as u32 ids + u8 weights when every weight <= 255 (0/1)
    int tail_pull = 1;     // delta v2: light pull rounds allowed in the tail too (round 3: 391 -> 428 GTEPS, once
                           // the tail-entry frontier counts its whole rows, fesplit)
    int spin_sync = 1;     // delta v2: the host spins on a published sequence word instead of a stream sync (0/1)
    int defer_check = 1;   // delta v2: no host check right after a heavy step (0/1)
    int round_gpc = 12;    // delta v2: workgroups per CU of the light-round / hub launches (0 = the heavy
    int hub_gpc = 3;       // kernels' 24); swept (24,24) (6,7) (12,14) (12,7) (12,4) (16,7): (12,4) best; with
                           // spec_round and round_batch 1, hub 3 +0.5% (profiles/r06/round_batch_ab_r6ab.txt)
    int heavy_gpc = 0;     // delta v2: workgroups per CU of the heavy pull (0 = 24; 7-32 swept, 12-32 equal)
    int round_batch = 1; // delta v2: light rounds enqueued per host check at a band's start (at least; 2 until
                         // spec_round: 1 then +1.2%, 3 -2.5%, profiles/r06/round_batch_ab_r6aa.txt / _r6ab.txt)
    int spec_round = 1;  // delta v2: light rounds enqueued behind each check's publish (0-2)
    int batch_streams = 2; // weighted batches (pj_sssp_batch*): solves in flight at once, one stream each
    int grid_per_cu = 0; // BFS level kernel workgroups per CU (0 = auto: 2 below 2^25 entries, else 4)
    int bfs_small = 1;   // BFS: one workgroup runs the levels of small push frontiers (bfs.hip small_levels)
    int hub_first = 1;   // BFS / MS-BFS: pull levels probe a copy of the in-rows ordered highest-degree in-neighbour
                         // first (built at the first solve; K22 0.2305 -> 0.1991 ms median kernel time, pull
                         // probes 21.8M -> 16.2M per 4 roots; web-Google and MS1024 equal or slightly faster,
                         // profiles/r06/bfs_hub_first_r6e.txt)
    int pull_first = 1;  // BFS pull levels: the first two in-neighbours of every row from a dense copy (8 bytes
                         // per vertex, read coalesced) instead of one row-start line per candidate
    int bfs_spare = 0;   // BFS: launches beyond the previous solve's count in the first batch (1 measured
                         // 2-3% slower on K22: the spare launch costs more than the occasional round trip)
    int max_levels = 0;  // debug: truncate the BFS after this many levels (0 = off)
    int ms_width = 0;    // batch BFS: widest pass in 64-source words (0 = 8, i.e. 512 sources;
                         // MS1024 on web-Google: 11.6 ms at 8 against 12.2-14.4 ms at 4; 16
                         // (1024 sources) 3% slower than 8)
    int ms_streams = 2;      // batch BFS: passes in flight at once (one stream + host thread each)
    double ms_alpha = 16.0;  // batch BFS: push levels while the frontier's out-edges < nnz / ms_alpha

    bool have_result = false;
    // weighted: the last solve's distances are still in the solver's ids (R.dist); the first
    // consumer of g.dist gathers them into input ids (delta_materialize)
    bool dist_pending = false;
    i64 pending_source = -1;   // (a source without edges: its 0 is written after the gather)
    i64 last_source = -1;      // source of the single-source result in dist (parent tree)
    bool batch_stats = false;  // stats describe the last pj_sssp_batch
    pj_load_stats load{};      // how the graph was built (pj_graph_load_stats)
    pj_stats stats{};

    const void* row_ptr() const { return off64 ? (const void*)row64.p : (const void*)row32.p; }
    const void* crow_ptr() const {
        if (symmetric) return row_ptr();
        return off64 ? (const void*)crow64.p : (const void*)crow32.p;
    }
    const u32* ccol_ptr() const { return symmetric ? col.p : ccol.p; }
    ~Graph();
};

// Build CSR (+CSC unless symmetric) from device COO (consumed: buffers are
// used as sort scratch). n must already be known.
// Builds g.rl from g's CSR (weighted graphs).
void build_relabeled(Graph& g);
// Loads delta.hip's code object on this host thread (HIP loads a module on the first use
// of one of its kernels, ~2.5 ms for delta.hip), so the relabel can do it behind its copy.
void preload_delta_module();

// Device check of CSR arrays read from a file: row[0] == 0, non-decreasing, row[n] ==
// nnz, every col < n; PJ_ERR_PARSE otherwise (a corrupted cache must not fault a kernel).
void check_csr_device(const void* row, bool off64, const u32* col, i64 n, i64 nnz, hipStream_t s);

void build_graph_from_coo(Graph& g, DevBuf<u32>& src, DevBuf<u32>& dst, DevBuf<u32>* w, i64 nnz,
                          i64 n, bool symmetric);

// ingestion
struct ParseResult {
    i64 nnz = 0;
    i64 max_id = -1;
    i64 bad_line = 0;  // 1-based, 0 = none
    double h2d_ms = 0, parse_ms = 0;
};
// Parses `len` bytes of host text on the device; fills device COO.
ParseResult parse_snap_device(Ctx& ctx, const char* host_text, i64 len, bool weighted,
                              DevBuf<u32>& src, DevBuf<u32>& dst, DevBuf<u32>& w);
// The same from text already on the device (len bytes, zero-padded to padded_text_bytes(len)).
i64 padded_text_bytes(i64 len);
ParseResult parse_device_text(Ctx& ctx, const uint8_t* text, i64 len, bool weighted, DevBuf<u32>& src,
                              DevBuf<u32>& dst, DevBuf<u32>& w);

void generate_webgraph_device(Ctx& ctx, i64 n_ids, i64 n_edges, uint64_t seed, DevBuf<u32>& src,
                              DevBuf<u32>& dst);
void generate_kronecker_device(Ctx& ctx, int scale, int edgefactor, uint64_t seed, bool weighted,
                               DevBuf<u32>& src, DevBuf<u32>& dst, DevBuf<u32>* w);

// solvers
void bfs_solve(Graph& g, i64 source);
// the in-rows the pull levels probe (BFS and MS-BFS): with the hub_first option a copy ordered
// highest in-degree in-neighbour first, built on first use; else the CSC (the CSR if symmetric)
const u32* pull_ccol(Graph& g);
i64 relabeled_id(const Relabeled& R, i64 v, hipStream_t s);  // relabel.hip: inv[v]
void delta_solve(Graph& g, i64 source);
// g.dist in input ids after a delta_solve (a no-op when it already is): every reader of g.dist
// calls it first (enqueued on the ctx stream)
void delta_materialize(Graph& g);
i64 delta_device_bytes(const Graph& g);  // the relabeled copy + delta workspace and solve slots
// Weighted batch with `slots` concurrent solves (delta.hip); on_row(i, device row, stream)
// is called once per source, serialised.
void delta_batch(Graph& g, const i64* sources, int n_src, int slots,
                 const std::function<void(int, const int32_t*, hipStream_t)>& on_row);
void msbfs_solve(Graph& g, const int64_t* sources, int n_src, int32_t* dist_out);
// Batched passes of up to 256 sources; after each pass on_pass(first source
// index, sources in the pass, device rows [ns][n]) runs with the device idle.
using MsPassFn = std::function<void(int, int, const int32_t*)>;
void msbfs_each(Graph& g, const int64_t* sources, int n_src, const MsPassFn& on_pass);
void reach_stats(Graph& g, i64* n_r, i64* m_r);
// shortest-path tree of g.dist (tree.hip)
void parent_tree(Graph& g, i64 source, int64_t* host_out);
void validate_tree(Graph& g, i64 source, const int64_t* host_parent, pj_tree_report* rep);
void debug_bitmaps(Graph& g, u64* vis0, u64* vis1, u64* fnew);

// 1D vertex partition (part.hip)
struct WPart;
void delete_wpart(WPart* p);
WPart* wpart_from_graph(Graph& g, int rank, int world);
WPart* wpart_from_kronecker(Ctx& ctx, int scale, int edgefactor, uint64_t seed, int rank, int world);
WPart* wpart_from_coo(Ctx& ctx, DevBuf<u32>& src, DevBuf<u32>& dst, DevBuf<u32>& w, i64 nnz, i64 n, int rank,
                      int world);
std::vector<WPart*> wparts_from_coo_group(const std::vector<Ctx*>& ctxs, DevBuf<u32>& src, DevBuf<u32>& dst,
                                          DevBuf<u32>& w, i64 nnz, i64 n);
void wpart_info(const WPart& p, i64* out8);
int32_t wpart_begin(WPart& p, i64 source, int32_t delta);
void wpart_select(WPart& p, int32_t lo, int32_t hi, i64* out2);
void wpart_relax(WPart& p, int light, int32_t lo, int32_t hi, i64* counts);
void wpart_pack(WPart& p, u64* send);
void wpart_device_bytes(const WPart& p, i64* out4);
void wpart_apply(WPart& p, const u64* recv, i64 nr, int light, int32_t lo, int32_t hi);
i64 wpart_end_round(WPart& p);
void wpart_reach(WPart& p, i64* out2);
void wpart_copy_dist(WPart& p, int32_t* host);

struct Part;
void delete_part(Part* p);
Part* part_from_kronecker(Ctx& ctx, int scale, int edgefactor, uint64_t seed, int rank, int world);
Part* part_from_coo(Ctx& ctx, DevBuf<u32>& src, DevBuf<u32>& dst, i64 nnz, i64 n, int rank, int world,
                    bool symmetric);
std::vector<Part*> parts_from_coo_group(const std::vector<Ctx*>& ctxs, DevBuf<u32>& src, DevBuf<u32>& dst, i64 nnz,
                                        i64 n, bool symmetric);
void part_info(const Part& p, i64* out);  // n lo hi block bw nnz_local sym off64 rank world nnz_in_local, bytes x4
void part_zmask(Part& p, u64* out_dev);
void part_begin(Part& p, i64 source, const u64* iso, u64* vis, i64* out3);
void part_push(Part& p, int level, u64* vis, u32* packed, i64* counts);
void part_apply(Part& p, int level, u64* vis, const u32* recv, i64 nr);
void part_pull(Part& p, int level, u64* vis);
void part_end_level(Part& p, u64* vis, i64* out3);
void part_reach(Part& p, i64* out2);
void part_copy_dist(Part& p, int32_t* host);
const int32_t* part_dist_device(const Part& p);

}  // namespace pj
