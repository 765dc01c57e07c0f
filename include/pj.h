/*
 * pj.h — C-ABI of libpj, the MI355X-native shortest-path relaxation library.
 *
 * The reference (fagan2888/ParallelJohnson) exposes no library API: its only
 * boundary is the process CLI `parallel_johnson webfile source_node sol_file`
 * (README:9, ParallelJohnson.cpp:294-303) and the internal seam
 * `int parallel_johnson(int argc, char* argv[])` (ParallelJohnson.cpp:286).
 * Each entry point below names the reference code it replaces; the CLI in
 * paralleljohnson_amd/csrc/cli.cpp is the drop-in for the process boundary and
 * is a plain client of this header.
 *
 * Conventions
 *  - Every function returns an int status (PJ_OK = 0, negative on error);
 *    pj_last_error() returns a thread-local message for the last failure.
 *  - Distances are int32; PJ_INT_INF (= the reference's INT_INF, :29) marks
 *    "unreachable", and any hop/weight distance >= PJ_INT_INF is reported as
 *    PJ_INT_INF (reference contract).
 *  - Host buffers are caller-owned; device memory is owned by the handles.
 *  - A pj_ctx is bound to one GPU and is not thread-safe (one thread per ctx).
 *  - No C++ exception crosses this boundary.
 */
#ifndef PJ_H
#define PJ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PJ_INT_INF 100000 /* ParallelJohnson.cpp:29 */

enum pj_status {
    PJ_OK = 0,
    PJ_ERR_ARG = -1,      /* bad argument (null pointer, bad size) */
    PJ_ERR_IO = -2,       /* file could not be written */
    PJ_ERR_PARSE = -3,    /* edge-list line the reference reads as UB (see pj_load_snap) */
    PJ_ERR_HIP = -4,      /* HIP runtime error */
    PJ_ERR_OOM = -5,      /* device or host allocation failed */
    PJ_ERR_RANGE = -6,    /* id / size outside the supported range */
    PJ_ERR_NODEVICE = -7, /* no usable gfx950 device */
    PJ_ERR_STATE = -8,    /* call out of order (e.g. stats before a solve) */
    PJ_ERR_COMM = -9      /* RCCL / multi-GPU error */
};

typedef struct pj_ctx pj_ctx;
typedef struct pj_graph pj_graph;

/* Per-solve statistics of the last pj_sssp* call on a graph. */
typedef struct pj_stats {
    double kernel_ms;        /* device time, dist init -> distances final (HIP events on the ctx stream);
                                the analogue of the reference's timed region :459-462 ... :597-605.
                                Weighted single-source solves end with the distances in the solver's
                                degree-ordered ids; the gather to input ids runs when the result is
                                first read (pj_copy_dist, pj_dist_device, ...) and is not in kernel_ms */
    double wall_ms;          /* host wall time of the call, incl. D2H of dist when requested */
    int64_t levels;          /* BFS levels / delta-stepping buckets processed */
    int64_t td_levels;       /* top-down (push) levels */
    int64_t bu_levels;       /* bottom-up (pull) levels */
    int64_t reached;         /* n_r: vertices with dist < PJ_INT_INF (filled by pj_reach_stats; a unit-weight
                                single-source solve fills it from its levels' counters) */
    int64_t reached_edges;   /* m_r: sum of out-degree over reached vertices (likewise) */
    int64_t relax_rounds;    /* weighted: light/heavy relaxation rounds */
    /* weighted (delta-stepping): the work of the relaxation kernels, counted on the device in
     * every solve -- the analogue of the reference's edge scans (the loop of
     * extract_local_pq :242-275 reads every out-edge of every popped vertex) */
    int64_t scanned_edges;   /* edge records read (packed light CSR, or u32 id + u8 weight) */
    int64_t probes;          /* reads of an edge's other end: its distance, the heavy pull's byte map,
                                or the tail's settled bitmap */
    int64_t work_bytes;      /* the bytes of both as stored (records of 4, 5 or 8 bytes, probes of 4 or 1) */
    int64_t work_by_kernel[4][3]; /* (records, probes, bytes) of the light-round kernel, the light hub
                                     kernel, the heavy pull and the heavy push */
} pj_stats;

/* ---- context ------------------------------------------------------------ */

/* Bind to HIP device `device` (ordinal as HIP sees it). Replaces MPI_Init
 * (:679) + the per-rank setup of parallel_johnson (:291-292). */
int pj_create(int device, pj_ctx** out);
/* Number of visible HIP devices (0 when none). */
int pj_device_count(int* out);
int pj_destroy(pj_ctx* ctx);
/* HIP stream (hipStream_t) all work of this ctx is launched on. */
void* pj_stream(pj_ctx* ctx);
const char* pj_last_error(void);
const char* pj_version(void);
/* A digest of the library's sources and compile flags (16 hex digits): measurements kept in
 * files (profiles/) carry it, so a reader can tell whether they were taken on this build. */
const char* pj_build_id(void);
/* Device blocks of 1 GiB or more that libpj freed stay cached in the process (up to half
 * of the device's memory) and serve later big allocations whole or in slices: a fresh
 * allocation of memory just returned to the driver waits for it to be cleared (seconds
 * for tens of GB). This returns every wholly free cached block to the driver, e.g.
 * before the caller allocates large buffers of its own; *released (may be NULL) = bytes. */
int pj_trim_device_cache(int64_t* released);

/* ---- graph ingestion (replaces read_webgraph :66-105 + coord2csr :117-159) */

/* Parse a SNAP edge-list text file on the GPU and build CSR by a stable radix
 * sort + scan. Line grammar follows the reference exactly: a line is an edge
 * iff its first byte is '0'..'9' (:73, :91); fields are read with
 * `istringstream >> int >> int` semantics (:92-93) — a non-numeric second
 * field reads as 0, extra columns are ignored. N = max id + 1 (:319).
 * With weighted != 0 a third integer column is the edge weight.
 * A missing input file parses as an empty graph (N = 0), as in the reference
 * (no is_open check at :67). Lines the reference turns into undefined
 * behaviour (missing second field, negative or > INT32_MAX-1 ids) fail with
 * PJ_ERR_PARSE; pj_last_error() names the 1-based line number. */
int pj_load_snap(pj_ctx* ctx, const char* path, int weighted, pj_graph** out);
/* Same, from an in-memory text buffer. */
int pj_load_snap_buffer(pj_ctx* ctx, const char* text, int64_t len, int weighted, pj_graph** out);

/* Build a graph from host COO arrays (file order = CSR column order, as the
 * stable counting sort of coord2csr :143-149). n_vertices < 0 means
 * max id + 1. w may be NULL (unit weights, :147). Ids must be in [0, 2^32-2];
 * edge counts may exceed 2^31 (64-bit offsets are used then). */
int pj_load_coo(pj_ctx* ctx, const int64_t* src, const int64_t* dst, const uint32_t* w,
                int64_t nnz, int64_t n_vertices, pj_graph** out);

/* Binary CSR cache (no reference counterpart: the
 * reference re-parses the text on every run, read_webgraph :66-105 +
 * coord2csr :117-159). The file holds the graph's device arrays as they sit in
 * HBM -- a 64-byte header, row offsets (4 or 8 bytes), col, weights when
 * weighted, and the in-edge CSC when the graph is unit-weight and not symmetric -- so loading
 * it is file -> pinned staging -> HBM with no sort. src_size / src_mtime_ns
 * stamp the text the graph came from (-1: none); pj_load_csr_file with an
 * expected stamp other than -1 fails with PJ_ERR_STATE when the file's stamp
 * differs (a stale cache). A missing or unreadable file is PJ_ERR_IO; a bad
 * magic, version or size is PJ_ERR_PARSE, and so is a payload that is not a
 * valid CSR (checked on the device after loading: row[0] = 0, non-decreasing
 * offsets, row[n] = nnz, every column id < n). */
int pj_graph_save(const pj_graph* g, const char* path, int64_t src_size, int64_t src_mtime_ns);
/* pj_load_snap through a CSR cache file: when cache_path (may be NULL) holds a
 * fresh cache of `path` (its size and mtime) in the same weight mode it is
 * loaded instead of parsing; otherwise the text is parsed and, with
 * write_back != 0, the cache is (re)written (a failed write is a warning on
 * stderr, not an error). The CLI's PJ_CSR_CACHE. */
int pj_load_snap_cached(pj_ctx* ctx, const char* path, int weighted, const char* cache_path, int write_back,
                        pj_graph** out);
int pj_load_csr_file(pj_ctx* ctx, const char* path, int64_t expect_src_size, int64_t expect_src_mtime_ns,
                     pj_graph** out);

/* Graph500-style Kronecker generator on the GPU (A,B,C = 0.57,0.19,0.19),
 * 2^scale vertices, edgefactor << scale tuples, labels permuted, every tuple
 * written in both directions (tuple i -> entries 2i, 2i+1). Deterministic in
 * (scale, edgefactor, seed); weighted != 0 gives w = 1 + hash(seed, i) % 255
 * (same for both directions). No reference counterpart (benchmark input). */
int pj_generate_kronecker(pj_ctx* ctx, int scale, int edgefactor, uint64_t seed, int weighted,
                          pj_graph** out);

/* The same Kronecker tuples written as a SNAP text file in generation order
 * (tuple i -> lines 2i and 2i+1, "u\tv[\tw]\n", after two '#' header lines):
 * the text input of the ingestion benchmarks (the reference's read_webgraph
 * :66-105 path at Graph500 sizes). No reference counterpart. */
int pj_kronecker_write_snap(pj_ctx* ctx, int scale, int edgefactor, uint64_t seed, int weighted, const char* path);

/* web-Google-shaped synthetic graph (the SNAP file is not
 * available): n_ids ids (about 95.6% used, the largest always used, so
 * N = n_ids), n_edges directed edges with power-law out- and in-degrees and
 * 30% "same-site" links. Deterministic in (n_ids, n_edges, seed). Benchmark
 * input, no reference counterpart. */
int pj_generate_webgraph(pj_ctx* ctx, int64_t n_ids, int64_t n_edges, uint64_t seed, pj_graph** out);

/* How a graph was built (host wall times of the ingestion phases; 0 where a
 * phase did not run): read_ms = the file into HBM (pj_load_snap: pinned
 * pieces, the read of each overlapped with the H2D copy of the previous;
 * :66-105's getline passes), h2d_ms = a host buffer's copy to the GPU
 * (pj_load_snap_buffer), the GPU parse (line scan + field decode), and the CSR
 * build (radix sort + row offsets, coord2csr :117-159, kernels completed). */
typedef struct pj_load_stats {
    double read_ms, h2d_ms, parse_ms, csr_ms;
    int64_t text_bytes;
} pj_load_stats;
int pj_graph_load_stats(const pj_graph* g, pj_load_stats* out);

int pj_graph_destroy(pj_graph* g);
/* n = number of vertices, nnz = number of CSR entries, weighted = 0/1,
 * symmetric = 1 when the graph is known to equal its transpose. */
int pj_graph_info(const pj_graph* g, int64_t* n, int64_t* nnz, int* weighted, int* symmetric);
/* D2H export of the CSR: row_ptr[n+1] (int64), col[nnz] (int32), w[nnz] or NULL. */
int pj_graph_get_csr(const pj_graph* g, int64_t* row_ptr, int32_t* col, uint32_t* w);
/* Out-degree of vertex v (row_ptr[v+1] - row_ptr[v]). */
int pj_graph_out_degree(const pj_graph* g, int64_t v, int64_t* deg);
/* Pick `n` distinct roots with out-degree >= 1, deterministic in seed
 * (Graph500 root sampling). Returns the count found in *found. */
int pj_sample_roots(const pj_graph* g, uint64_t seed, int n, int64_t* roots, int* found);

/* ---- relaxation (replaces the heap + BSP round loop :466-594) ------------ */

/* Single-source shortest paths from `source` (atoi semantics are the
 * caller's: any int64 is accepted; a source outside [0,n) leaves every
 * distance at PJ_INT_INF, as the reference does). Unit-weight graphs run the
 * direction-optimizing level-synchronous frontier kernels, weighted graphs
 * run delta-stepping. dist_out (host, n int32) may be NULL: the result then
 * stays on the device (pj_copy_dist fetches it). */
int pj_sssp(pj_graph* g, int64_t source, int32_t* dist_out);
/* Copy the last result to the host. Pageable memory goes through pinned
 * staging slots on up to 8 host threads; memory pinned with pj_host_pin is
 * written by one direct DMA copy. */
int pj_copy_dist(pj_graph* g, int32_t* dist_out);
/* Pin (page-lock) host memory for the device -> host copies of pj_copy_dist /
 * pj_sssp, e.g. from a helper thread while the GPU builds the graph; the pages
 * stay pinned until pj_host_unpin (or process exit). No reference counterpart. */
int pj_host_pin(void* p, size_t bytes);
int pj_host_unpin(void* p);
/* Device pointer to the last result (int32[n]); valid until the next solve. */
const int32_t* pj_dist_device(pj_graph* g);
/* Batched multi-source (Johnson-style all-pairs rows): dist_out is n_src x n
 * int32, row i = pj_sssp(g, sources[i]); NULL discards the rows (timing).
 * Unit-weight graphs run up to 512 sources per pass, one bit per source
 * (msbfs.hip; the option ms_width caps the pass at 64 x ms_width); weighted
 * graphs run delta-stepping solves with `batch_streams` (default 2, 1-8) of
 * them in flight at once, each on its own stream and host thread with its own
 * frontiers and counters, the graph shared (delta.hip delta_batch; rows in
 * source order whatever finishes first). Device memory per slot in flight:
 * unit weights ~n x (256 W + 8 W (1 + L)) bytes (a 64 W x n int32 distance block,
 * the reached masks and an archive of L <= 32 levels' W-word masks per vertex, L
 * reduced to keep a slot within 8 GB; ms_streams slots, default 2, all slots within
 * 16 GB); weights ~9.4 n bytes of rows and bitmaps (the heavy pull's n-byte map
 * included) plus ~60 x nnz / 64 bytes of hub queues per
 * extra slot. A slot beyond the first is added only while it takes at most half
 * the free device memory, and a failed allocation leaves the batch on the
 * slots it has (no error). Either way pj_last_stats
 * then describes the whole batch (kernel_ms and levels summed over passes or
 * solves) and pj_copy_dist / pj_reach_stats fail with PJ_ERR_STATE until the
 * next pj_sssp. No reference counterpart: the reference answers one source
 * per run (atoi(argv[2]), :448). */
int pj_sssp_batch(pj_graph* g, const int64_t* sources, int n_src, int32_t* dist_out);
/* The multi-source drop-in: the same batch, with row i written as a sol_file
 * to paths[i] (the bytes of pj_write_sol, i.e. of a single-source run
 * :615-620). Rows are copied to the host in groups and written by a pool of
 * host threads while the GPU computes the next pass. strict as pj_write_sol. */
int pj_sssp_batch_write(pj_graph* g, const int64_t* sources, int n_src, const char* const* paths, int strict);
/* Statistics of the last solve. pj_reach_stats additionally computes
 * reached / reached_edges on the device (not part of kernel_ms). */
int pj_last_stats(const pj_graph* g, pj_stats* out);
int pj_reach_stats(pj_graph* g, pj_stats* out);
/* Tuning knobs: alpha/beta of the direction switch (Beamer), delta for
 * delta-stepping (0 = automatic: c(n) x mean weight / mean out-degree, c(n) =
 * 0.1875 log2(n) - 1.875 within [2, 3.5], swept on Kronecker s22-s26), direction (0 auto, 1 push, 2 pull),
 * bfs_small (one-workgroup levels for small frontiers, 0/1), hub_first (BFS pull levels
 * probe in-rows ordered highest-degree in-neighbour first, 0/1, default 1), pull_first (BFS
 * pull levels take their first two probes from a dense copy of the in-rows' first entries,
 * 0/1, default 1), pull_vertex (BFS: push -> pull also when the frontier's out-edges exceed
 * pull_vertex x the unvisited vertices, default 2, 0 = Beamer's rule alone; applied only with
 * hub-first in-rows), batch_streams
 * (weighted batches: solves in flight, 1-8), defer_heavy (a heavy push of members
 * holding >= defer_heavy x nnz heavy edges relaxes the next band's part only and
 * leaves the rest to the next heavy step; 0 = off, default 0.002), spec_round (delta:
 * light rounds enqueued behind each band-end check, run while the host reads it, 0-2,
 * default 1) and the batch /
 * grid knobs documented in DESIGN.md §4.2b. Returns PJ_ERR_ARG on bad values. */
int pj_set_option(pj_graph* g, const char* key, double value);

/* ---- shortest-path tree (no reference counterpart:
 * the reference writes distances only, output_vector :32-46) --------------- */

/* Parent array of the last pj_sssp on g (host, n int64): parent[v] = the
 * smallest u with an edge u -> v of weight w and dist[u] + w == dist[v],
 * parent[source] = source, -1 where dist[v] = PJ_INT_INF. A function of the
 * distances alone, so every solver path gives the same tree. PJ_ERR_STATE when
 * the last solve was a batch or none ran. */
int pj_parent_tree(pj_graph* g, int64_t* parent_out);

/* Graph500-style validation of a parent array against the graph and the last
 * pj_sssp's distances (which must be from `source`, else PJ_ERR_STATE). Each
 * bad_* field counts violations; all zero = valid. */
typedef struct pj_tree_report {
    int64_t reached;        /* vertices with dist < PJ_INT_INF (the source included) */
    int64_t bad_root;       /* 1 when parent[source] != source or dist[source] != 0 */
    int64_t bad_reach;      /* parent[v] != -1 not exactly where dist[v] < PJ_INT_INF (or out of range) */
    int64_t bad_tree_edge;  /* parent[v] = u with no edge u -> v of dist[u] + w == dist[v] */
    int64_t bad_edge;       /* edges u -> v (dist[u] finite) with dist[v] > min(dist[u] + w, PJ_INT_INF) */
    int64_t bad_cycle;      /* reached vertices whose parent chain does not end at the source */
} pj_tree_report;
int pj_validate_tree(pj_graph* g, int64_t source, const int64_t* parent, pj_tree_report* out);

/* Write a parent array as text: "the parent tree is:\n", then parent[v] per
 * line (-1 for unreached), in vertex order (the sol_file layout). */
int pj_write_parents(const int64_t* parent, int64_t n, const char* path);

/* ---- stream ---------------------------------------------------------------- */

/* Launch all later work of ctx on `stream` (a hipStream_t of the same device,
 * e.g. torch's current stream, so that libpj kernels and RCCL collectives are
 * ordered without host synchronisation). NULL restores the ctx's own stream.
 * The caller keeps ownership of an external stream. */
int pj_set_stream(pj_ctx* ctx, void* stream);

/* ---- 1D vertex partition: one process per GPU -------------
 *
 * Replaces the reference's block distribution nn2rank / get_start_nn
 * (ParallelJohnson.cpp:169-200) and the row scatter :344-410: rank r of world
 * keeps the out-rows (and, for non-symmetric graphs, the in-rows) of the
 * vertex block [lo, hi), lo = r * block, block = ceil(N / world) rounded up
 * to a multiple of 64 (so ranks never share a 64-bit visited word). Column
 * ids stay global. The level loop and the exchange run inside libpj
 * (pj_part_bfs over a pj_comm, below), replacing the reference's per-round
 * MPI_Alltoall(v) and MPI_Allreduce (:522-554, :589-590); the steps are also
 * exported one by one, and pj_part_bfs runs exactly this sequence:
 *
 *   stats = pj_part_begin(source)                     (level 0 = {source})
 *   while sum_ranks(stats.n_f) > 0:
 *     push level:  pj_part_push -> counts[world]; all_to_all_single(ids);
 *                  pj_part_apply(received ids)
 *     pull level:  pj_part_pull (reads the exact global vis snapshot)
 *     stats = pj_part_end_level; all_reduce(stats); all-gather vis slices
 *                  before a pull level (and after one)
 *
 * `vis` (device, world * words_per_rank u64) is the caller-owned replicated
 * visited bitmap of all vertices; slice r (words [r*wpr, (r+1)*wpr)) belongs
 * to rank r. Distances are BFS hops (unit weights, the reference's w = 1,
 * :147); no level assigns a distance >= PJ_INT_INF (the caller stops there). */
typedef struct pj_part pj_part;

typedef struct pj_part_info {
    int64_t n;              /* vertices of the whole graph */
    int64_t lo, hi;         /* owned block [lo, hi) */
    int64_t block;          /* vertices per rank (multiple of 64) */
    int64_t words_per_rank; /* block / 64: u64 words of one vis slice */
    int64_t nnz_local;      /* out-edges of the owned block */
    int64_t nnz_in_local;   /* in-edges of the owned block (== nnz_local if symmetric) */
    int32_t rank, world, symmetric, off64;
    /* device bytes held by this rank: its rows (CSR, and CSC when not symmetric),
     * the O(block) vertex state, the N-bit bitmaps (the level's claimed remote ids,
     * and the engine's replicated visited / isolated masks once pj_part_bfs ran) and
     * the exchange buffers (sized to the largest level's ids sent / received) */
    int64_t bytes_rows, bytes_state, bytes_bitmaps, bytes_exchange;
    /* how the block was built (host wall microseconds, each phase ending at a stream
     * sync): [0] tuple enumeration + owned-entry count, [1] enumeration + write of the
     * owned entries, [2] radix sort of the local COO, [3] CSR bounds, [4] device
     * allocations, [5] per-solve state, [6] total, [7] device frees, [8] the slowest
     * single allocation, [9] its size in MB (not microseconds) */
    int64_t build_us[10];
} pj_part_info;

/* The rank's share of pj_generate_kronecker(scale, edgefactor, seed, unit
 * weights): every rank enumerates the same tuples and keeps its rows. */
int pj_part_generate_kronecker(pj_ctx* ctx, int scale, int edgefactor, uint64_t seed, int rank, int world,
                               pj_part** out);
/* The rank's share of a host COO graph (file order kept inside rows, as
 * coord2csr :143-149). n_vertices < 0 means max id + 1. symmetric != 0 promises
 * the edge list equals its transpose (no in-rows are built). */
int pj_part_load_coo(pj_ctx* ctx, const int64_t* src, const int64_t* dst, int64_t nnz, int64_t n_vertices,
                     int symmetric, int rank, int world, pj_part** out);
/* The rank's share of a SNAP edge-list file (the pj_load_snap grammar, unit
 * weights; N = max id + 1 as :319). Every rank parses the file on its GPU and
 * keeps its rows, so no rank has to scatter (the reference's :344-410). */
int pj_part_load_snap(pj_ctx* ctx, const char* path, int rank, int world, pj_part** out);
/* All ranks of a one-process group at once (ctxs[world], rank r on ctxs[r]; out[world]):
 * the file is parsed ONCE, on ctxs[0]'s GPU, and every rank gets only its block's
 * entries from there (peer copies), then builds its rows -- the reference's rank-0
 * read and scatter (:313-338, :344-410) with the scatter on the device. */
int pj_part_load_snap_group(int world, pj_ctx* const* ctxs, const char* path, pj_part** out);
int pj_part_destroy(pj_part* p);
int pj_part_info_get(const pj_part* p, pj_part_info* out);
/* Copy the rank's isolated-vertex mask (words_per_rank u64, device) to
 * own_words; all-gathered once, it is the `iso` argument of pj_part_begin. */
int pj_part_zmask(pj_part* p, uint64_t* own_words);
/* Start a solve: dist := INF, vis := iso, then the source. stats[3] =
 * (n_f, m_f, frontier vertices with out-edges) of level 0, this rank's share. */
int pj_part_begin(pj_part* p, int64_t source, const uint64_t* iso, uint64_t* vis, int64_t* stats);
/* Top-down expansion of level `level` (this rank's frontier). Owned targets are
 * settled at distance level+1; the others are written to send (device, room for
 * the sum of the counts; world * block u32 always suffices) owner-major,
 * counts[world] (host) per owner. */
int pj_part_push(pj_part* p, int level, uint64_t* vis, uint32_t* send, int64_t* counts);
/* Settle the ids received for this rank after the exchange of a push level. */
int pj_part_apply(pj_part* p, int level, uint64_t* vis, const uint32_t* recv, int64_t n_recv);
/* Bottom-up step of level `level` over the owned block (vis = exact snapshot). */
int pj_part_pull(pj_part* p, int level, uint64_t* vis);
/* Close a level: the new frontier becomes current, the own vis slice is
 * updated; stats[3] as in pj_part_begin. */
int pj_part_end_level(pj_part* p, uint64_t* vis, int64_t* stats);
/* out[2] = (reached vertices, their out-edge sum) of the owned block. */
int pj_part_reach(pj_part* p, int64_t* out);
/* The owned block's distances (hi - lo int32): to the host, or in place. */
int pj_part_copy_dist(pj_part* p, int32_t* dist_out);
const int32_t* pj_part_dist_device(pj_part* p);

/* ---- weighted SSSP over a 1D vertex partition (the
 * delta-stepping variant) ---------------------------------------------------
 *
 * Same block geometry as pj_part_*. Rank r keeps the weighted out-rows of its
 * block, cut from a weighted graph loaded on its GPU (the reference's rank 0
 * builds the whole CSR and scatters row blocks, :344-410; here every rank cuts
 * its own block, nothing is scattered). The band loop runs in libpj
 * (pj_wpart_delta, below), the analogue of the reference's round loop
 * :488-594 with bands of width delta; the steps it runs:
 *
 *   delta = pj_wpart_begin(source, delta or 0 for the default)
 *   lo = 0
 *   loop: pj_wpart_select(lo, lo + delta) -> (count, min dist >= lo)
 *         all_reduce sum(count), min(min): count 0 -> jump lo to the band of
 *         min, or stop when min = INF (the termination test :579-593)
 *         light rounds until all_reduce sum(new frontier) = 0:
 *           pj_wpart_relax(light = 1) -> counts[world] of the queued pairs
 *           (u64 id | cand << 32); all_to_all counts; pj_wpart_pack into a send
 *           buffer of their sum (owner-major); all_to_all_v; pj_wpart_apply(received);
 *           pj_wpart_end_round -> new frontier size on this rank
 *         heavy step: pj_wpart_relax(light = 0); exchange; pj_wpart_apply
 *         lo += delta
 *
 * send and recv are caller-owned device buffers sized to the counts. A relax
 * queues its remote pairs itself (a claim queue that grows with the traffic) and
 * skips the pairs a cache of the pairs already sent shows as useless, so the
 * owner may receive the same id twice in a round (its apply takes the minimum).
 * Distances follow the R9 contract with the graph's integer weights. */
typedef struct pj_wpart pj_wpart;
/* The rank's block of a weighted graph (pj_load_coo / pj_load_snap(weighted) /
 * pj_generate_kronecker(weighted)); the graph may be destroyed afterwards.
 * Memory: the whole graph is resident on the rank's GPU while the block is cut
 * (the unit-weight pj_part_load_* keep only the rank's rows while building). */
int pj_wpart_from_graph(pj_graph* g, int rank, int world, pj_wpart** out);
/* The rank's block of a weighted SNAP file (third column = weight, the
 * pj_load_snap grammar): every rank parses the file on its GPU and keeps only
 * its block's rows, weight-sorted (no whole-graph CSR on any GPU). */
int pj_wpart_load_snap(pj_ctx* ctx, const char* path, int rank, int world, pj_wpart** out);
/* The weighted form of pj_part_load_snap_group: one parse on ctxs[0], each rank's
 * entries (and the degree keys of the per-block order) copied to its GPU. */
int pj_wpart_load_snap_group(int world, pj_ctx* const* ctxs, const char* path, pj_wpart** out);
/* The rank's block of pj_generate_kronecker(scale, edgefactor, seed, weighted = 1):
 * every rank enumerates the generator's tuples on its GPU and keeps only its block's
 * rows (weight-sorted, the same rows as the single-GPU graph's), so the weighted
 * graph never has to fit whole on one device (the reference's split graph,
 * :344-410). The automatic delta uses the whole graph's mean weight on every rank. */
int pj_wpart_generate_kronecker(pj_ctx* ctx, int scale, int edgefactor, uint64_t seed, int rank, int world,
                                pj_wpart** out);
int pj_wpart_destroy(pj_wpart* p);
/* out[8] = (n, lo, hi, block, nnz_local, world, rank, nnz of the whole graph) */
int pj_wpart_info(const pj_wpart* p, int64_t* out);
/* out[4] = this rank's device bytes: its rows; the O(block) vertex state (with the
 * sent-pair cache, block entries); the replicated maps the pulls and the tail
 * all-gather (N bytes, 2N for the tail's 16-bit frontier map, N bits for the
 * settled map: the analogue of the BFS pull's visited bitmap); the claim queue and
 * the exchange buffers, sized to the largest round's pairs. Building a block with
 * the per-block degree order (pj_wpart_generate_kronecker, pj_wpart_from_graph,
 * pj_wpart_load_snap) also holds 8 bytes per vertex of the WHOLE graph for a moment
 * (every vertex's degree and the relabel table of all blocks, which the rank's column
 * ids go through; 20 bytes until round 5), plus 16 bytes per vertex of one block for
 * the block-by-block sort; none of it stays. At world 1 after a single-GPU solve
 * (option "single_gpu") the rows figure includes that solver's copy of the rows, its
 * relabeled copy and its workspace (~14 bytes per entry more). */
int pj_wpart_device_bytes(const pj_wpart* p, int64_t* out);
/* Start a solve from `source` (dist := INF, then the source); delta <= 0 picks
 * the single-GPU default (c(n) x mean weight / mean degree, c(n) = 0.1875 log2(n) -
 * 1.875 within [2, 3.5]: 12 on Kronecker s26 with weights 1..255). *delta_out = delta. */
int pj_wpart_begin(pj_wpart* p, int64_t source, int32_t delta, int32_t* delta_out);
/* Band [lo, hi): frontier := owned vertices with dist in [lo, hi). out[2] =
 * (its size, min owned dist >= lo or PJ_INT_INF). */
int pj_wpart_select(pj_wpart* p, int32_t lo, int32_t hi, int64_t* out);
/* light != 0: the frontier relaxes its light edges (w < delta) and joins the
 * band's members; light == 0: the members relax their heavy edges. counts[o] =
 * the pairs queued for owner o. send must be NULL at world > 1 (PJ_ERR_ARG
 * otherwise: no bound on the pairs is known before the relax, since the queue
 * keeps one pair per improving remote relaxation); the caller sizes its buffer
 * from the counts and calls pj_wpart_pack before any other step of p
 * (PJ_ERR_STATE otherwise: the cache already counts the pairs as sent). The ids
 * are the partition's internal ids (with the per-block degree order,
 * PJ_WP_RELABEL, a block's relabeled ids): only their owner, id / block, is
 * meaningful outside, and pj_wpart_apply on that owner takes them back unchanged. */
int pj_wpart_relax(pj_wpart* p, int light, int32_t lo, int32_t hi, uint64_t* send, int64_t* counts);
/* The pairs of the last pj_wpart_relax (send == NULL), owner-major, into send
 * (room for the sum of its counts). */
int pj_wpart_pack(pj_wpart* p, uint64_t* send);
/* Fold the received candidates into the owned distances (light: those below hi
 * join the next frontier). */
int pj_wpart_apply(pj_wpart* p, const uint64_t* recv, int64_t n_recv, int light, int32_t lo, int32_t hi);
/* The round's new frontier becomes current; *n_f = its size on this rank. */
int pj_wpart_end_round(pj_wpart* p, int64_t* n_f);
/* out[2] = (reached owned vertices, their out-edge sum) */
int pj_wpart_reach(pj_wpart* p, int64_t* out);
/* The owned block's distances (hi - lo int32) to the host. */
int pj_wpart_copy_dist(pj_wpart* p, int32_t* dist_out);

/* ---- multi-GPU transport and partitioned solves ------------
 *
 * A pj_comm is one rank's endpoint of a group: the replacement for the
 * reference's MPI_COMM_WORLD (MPI_Init :679, MPI_Comm_size/rank :291-292) and
 * its collectives. Kinds:
 *  - RCCL, one process per GPU: rank 0 makes an id with pj_comm_unique_id and
 *    the launcher hands it to every rank (pj_comm_create_rank);
 *  - a group in one process, one pj_ctx (and one host thread) per rank
 *    (pj_comm_create_group): PJ_TRANSPORT_RCCL (ncclCommInitAll, one GPU per
 *    rank) or PJ_TRANSPORT_HOST (device copies between the ranks' buffers; ranks
 *    may share a GPU -- the "fake cluster" of SURVEY.md §4.3);
 *  - caller callbacks (pj_comm_create_callbacks), e.g. an MPI program's own
 *    MPI_Allreduce / MPI_Alltoall(v) / MPI_Allgather.
 * Every rank of a group must make the same pj_* calls in the same order. */
typedef struct pj_comm pj_comm;

enum pj_transport { PJ_TRANSPORT_AUTO = 0, PJ_TRANSPORT_RCCL = 1, PJ_TRANSPORT_HOST = 2 };

int pj_comm_unique_id(uint8_t id[128]);
/* id may be NULL only for world == 1 (a one-rank transport without RCCL). */
int pj_comm_create_rank(pj_ctx* ctx, int world, int rank, const uint8_t id[128], pj_comm** out);
/* out[r] is rank r's endpoint, bound to ctxs[r]; AUTO = RCCL when world > 1 and
 * every ctx has its own GPU, else HOST (a single rank: no transport at all). */
int pj_comm_create_group(pj_ctx* const* ctxs, int world, int transport, pj_comm** out);

typedef struct pj_comm_callbacks {
    void* user;
    int rank, world;
    /* each returns 0 on success; vals / counts are host arrays, the buffers are
     * whatever the steps expose (device memory for libpj's own partitions) */
    int (*allreduce)(void* user, int64_t* vals, int k, int is_min);      /* in place, sum or min */
    int (*alltoall_counts)(void* user, const int64_t* send, int64_t* recv); /* world counts each */
    int (*alltoallv)(void* user, const void* send, const int64_t* scounts, void* recv, const int64_t* rcounts,
                     int64_t elem_bytes); /* owner-major segments */
    int (*allgather)(void* user, const void* own, void* all, int64_t bytes); /* all[r*bytes] = rank r's own */
} pj_comm_callbacks;
int pj_comm_create_callbacks(const pj_comm_callbacks* cb, pj_comm** out);
/* kind: "self", "rccl", "host" or "callbacks" */
int pj_comm_info(const pj_comm* c, int* rank, int* world, const char** kind);
/* The group's size and this rank's index as the transport itself reports them -- for RCCL
 * ncclCommCount / ncclCommUserRank of the communicator (the reference's MPI_Comm_size /
 * MPI_Comm_rank, :291-292), the thread group's size for the host transport, 1 for self,
 * the declared world for callbacks -- so that a launcher can prove the group it formed. */
int pj_comm_transport_ranks(const pj_comm* c, int* count, int* index);
int pj_comm_destroy(pj_comm* c);

/* Statistics of one rank's partitioned solve. reached / reached_edges are for
 * the whole graph (summed over the ranks). */
typedef struct pj_part_stats {
    double solve_ms;      /* host wall time of the solve on this rank, device work included
                             (the reference's timed region :459-462 ... :597-605) */
    int64_t levels;       /* BFS levels, or delta-stepping bands */
    int64_t td_levels, bu_levels; /* BFS: push / pull levels; delta-stepping: -, light rounds run as pulls */
    int64_t bands, rounds; /* delta-stepping: non-empty bands, light rounds */
    int64_t reached, reached_edges;
    int64_t sent;         /* ids (BFS) or (id, dist) pairs (delta) this rank sent */
    int32_t delta;        /* delta-stepping: the light threshold the solve started with */
    int32_t heavy_pulls;  /* delta-stepping: heavy steps done by pull (pj_wpart_set_option "pull_factor") */
} pj_part_stats;

/* The partitioned BFS of this rank (part.hip + the level loop of engine.cpp,
 * the analogue of :488-594): every rank of comm calls it with the same source.
 * pj_part_set_option keys: "alpha", "beta" (Beamer), "direction" (0 auto,
 * 1 push, 2 pull), "exchange_cap" (ids per rank and direction the exchange buffers
 * hold; a push level with more goes out in pieces by word range of the owners' slices,
 * each piece its own count exchange, alltoallv and host wait; -1 = max(block / 16,
 * 4096) ids (default), 0 = no cap, else at least 64 ids: smaller caps are
 * PJ_ERR_ARG), "single_gpu" (0/1, default 1: at world 1 the solve is the single-GPU BFS's,
 * bfs.hip on the rank's rows, borrowed for the solve; the stats are its level counters').
 * Every rank must use the same values. */
int pj_part_bfs(pj_part* p, pj_comm* comm, int64_t source, pj_part_stats* st);
int pj_part_set_option(pj_part* p, const char* key, double value);
/* All ranks of a one-process group at once (one host thread per rank);
 * st[world] may be NULL. */
int pj_part_bfs_group(int world, pj_part* const* parts, pj_comm* const* comms, int64_t source, pj_part_stats* st);
/* The whole distance vector (n int32) on this rank (dist_out may be NULL on
 * ranks that do not need it; every rank must call): the MPI_Gatherv of :612-614. */
int pj_part_gather_dist(pj_part* p, pj_comm* comm, int32_t* dist_out);

/* Weighted partitioned solve (delta-stepping, wpart.hip + engine.cpp);
 * delta <= 0 picks the single-GPU default. At world 1 (the rank holds the whole
 * graph) the solve is the single-GPU solver's (delta.hip v2 on the rank's rows) unless
 * option "single_gpu" is 0; the pj_part_stats light-round and band counts are then
 * v2's. */
int pj_wpart_delta(pj_wpart* p, pj_comm* comm, int64_t source, int32_t delta, pj_part_stats* st);
/* pj_wpart_set_option keys: "tail_frac" (switch to the tail threshold once the edges of
 * the vertices not settled yet, over all ranks, drop below tail_frac x all edges; 0 = off;
 * default 0.3 since round 5, profiles/r05/wpart_sweep_r5o.txt) and "tail_mult" (tail
 * threshold and band width = tail_mult x delta,
 * default 64) and "pull_factor" (heavy steps by pull -- the unsettled vertices scan their
 * heavy rows for band members through an all-gathered byte map -- when the unsettled
 * vertices' heavy edges are fewer than pull_factor x the members'; symmetric graphs only;
 * 0 = always push; default 4) and "light_pull" (a light round whose frontier has more light
 * edges than the vertices above the band start / light_pull runs as a pull through an
 * all-gathered frontier map, stopping a row at the frontier's least distance + its weight
 * ("pull_fmin" 1, default); symmetric graphs; 0 = push; default 3 since round 6,
 * profiles/r06/wpart_light_pull_r6l.txt)
 * and "tail_light_pull" (the same rule in the tail's bands, independent of light_pull, the
 * frontier map then 16-bit; 0 = push; default 3). Every rank must use the same values.
 * "single_gpu" (0/1, default 1: the world-1 solve runs delta.hip's v2, see pj_wpart_delta).
 * "grid_per_cu" (this rank only): workgroups per CU of the grid-stride kernels, 1-32, default 8.
 * "queue_shard" (this rank only, any time between steps): the claim queue's shard
 * capacity in pairs from now on, >= 1 (64 shards; it still grows when a round
 * overflows it: tests use small values to run that path). */
int pj_wpart_set_option(pj_wpart* p, const char* key, double value);
int pj_wpart_delta_group(int world, pj_wpart* const* parts, pj_comm* const* comms, int64_t source, int32_t delta,
                         pj_part_stats* st);
int pj_wpart_gather_dist(pj_wpart* p, pj_comm* comm, int32_t* dist_out);

/* The same loops over caller-supplied steps (tests, other backends): the
 * callbacks have the semantics of pj_part_* / pj_wpart_* above, and the
 * buffers (replicated vis / iso: world * words_per_rank u64; zown:
 * words_per_rank u64; send / recv: world * block u32, or u64 for delta) are
 * handed to the transport as they are. */
typedef struct pj_bfs_steps {
    void* user;
    int64_t n, nnz_local, words_per_rank, block;
    int32_t rank, world;
    void *vis, *iso, *zown, *send, *recv;
    int (*zmask)(void* user);                                   /* own isolated words -> zown */
    int (*begin)(void* user, int64_t source, int64_t* st3);
    int (*push)(void* user, int level, int64_t* counts);        /* fills send, counts[world] */
    int (*apply)(void* user, int level, int64_t n_recv);        /* reads recv */
    int (*pull)(void* user, int level);
    int (*end_level)(void* user, int64_t* st3);
} pj_bfs_steps;
int pj_engine_bfs(const pj_bfs_steps* steps, pj_comm* comm, int64_t source, double alpha, double beta, int force,
                  pj_part_stats* st);

typedef struct pj_delta_steps {
    void* user;
    int64_t n;
    int32_t rank, world;
    void *send, *recv;
    int (*begin)(void* user, int64_t source, int32_t delta, int32_t* delta_out);
    int (*select)(void* user, int32_t lo, int32_t hi, int64_t* out2);
    int (*relax)(void* user, int light, int32_t lo, int32_t hi, int64_t* counts);
    int (*apply)(void* user, int64_t n_recv, int light, int32_t lo, int32_t hi);
    int (*end_round)(void* user, int64_t* n_f);
    int (*reach)(void* user, int64_t* out2);
} pj_delta_steps;
int pj_engine_delta(const pj_delta_steps* steps, pj_comm* comm, int64_t source, int32_t delta, pj_part_stats* st);

/* ---- n-GPU handle (SURVEY.md §8b `pj_create(int n_gpus, ...)`) ------------
 *
 * What `mpirun -np P parallel_johnson ...` gives a reference user, as one
 * handle: P ranks in this process (one pj_ctx and one host thread each, rank r
 * on GPU r mod the visible GPUs), the transport between them (pj_comm group:
 * RCCL over xGMI when every rank has its own GPU, device copies otherwise) and
 * the graph in one of two layouts:
 *  - PJ_LAYOUT_PARTITIONED: the reference's 1D vertex partition (nn2rank
 *    :169-200); every rank builds its own rows (no scatter, :344-410); a solve
 *    runs the protocol loops of pj_part_bfs / pj_wpart_delta on all ranks
 *    (exchange :522-554, termination allreduce :589-590) and gathers the
 *    distances to the caller (:612-614);
 *  - PJ_LAYOUT_REPLICATED: every rank holds the whole graph; batches of sources
 *    are sharded over the ranks (source i on rank i mod P), no data-path
 *    collective; a single source runs on rank 0.
 * transport: PJ_TRANSPORT_AUTO / RCCL / HOST as pj_comm_create_group. The
 * handle is driven from one caller thread. */
typedef struct pj_multi pj_multi;
enum pj_layout { PJ_LAYOUT_PARTITIONED = 0, PJ_LAYOUT_REPLICATED = 1 };
typedef struct pj_multi_info_t {
    int64_t n;             /* vertices of the loaded graph (0 before a load) */
    int32_t world;         /* ranks (GPUs) */
    int32_t layout;        /* PJ_LAYOUT_*, -1 before a load */
    int32_t weighted;
    const char* transport; /* "rccl", "host", "self", "replicated" or "none" */
} pj_multi_info_t;

int pj_multi_create(int n_gpus, int transport, pj_multi** out);
int pj_multi_destroy(pj_multi* m);
/* rank r's pj_ctx (owned by the handle) */
int pj_multi_ctx(pj_multi* m, int rank, pj_ctx** out);
/* The pj_load_snap grammar (weighted: third column = weight); replaces any
 * graph loaded before. */
int pj_multi_load_snap(pj_multi* m, const char* path, int weighted, int layout);
/* CSR cache for later replicated loads (pj_load_snap_cached; rank 0 writes it);
 * NULL or "" turns it off. Partitioned loads always parse. */
int pj_multi_set_csr_cache(pj_multi* m, const char* cache_path);
/* pj_generate_kronecker on every rank; partitioned: every rank enumerates the
 * tuples on its GPU and keeps only its block's rows (pj_part_generate_kronecker /
 * pj_wpart_generate_kronecker), so no GPU ever holds the whole graph. */
int pj_multi_generate_kronecker(pj_multi* m, int scale, int edgefactor, uint64_t seed, int weighted, int layout);
/* Rank `rank`'s device bytes of the loaded graph, out[4] = (rows, O(block) vertex
 * state, replicated maps / N-bit bitmaps, exchange buffers): pj_part_info_get's or
 * pj_wpart_device_bytes' four numbers for a partitioned graph; (graph bytes, 0, 0, 0)
 * for a replicated one. */
int pj_multi_device_bytes(const pj_multi* m, int rank, int64_t* out);
int pj_multi_info(const pj_multi* m, pj_multi_info_t* out);
/* One source: dist_out (n int32, host) may be NULL. st (may be NULL): rank 0's
 * counts with solve_ms = the max over ranks (the reference's Time:, :597-605). */
int pj_multi_sssp(pj_multi* m, int64_t source, int32_t* dist_out, pj_part_stats* st);
/* n_src sources -> dist_out[n_src][n] (may be NULL). */
int pj_multi_sssp_batch(pj_multi* m, const int64_t* sources, int n_src, int32_t* dist_out);
/* n_src sources, one sol_file each (paths[i] for sources[i]), each byte-identical
 * to a single-source run (pj_write_sol semantics, strict as there).
 * *solve_ms (may be NULL): device solve time, max over ranks (replicated) or
 * summed over the sources (partitioned). */
int pj_multi_sssp_batch_write(pj_multi* m, const int64_t* sources, int n_src, const char* const* paths, int strict,
                              double* solve_ms);

/* ---- output (replaces output_vector :32-46 + the write at :615-620) ------ */

/* Write the sol_file: "the vector is:\n" then, for v = 0..n-1, the decimal
 * distance or "inf" when it equals PJ_INT_INF, one per line. Like the
 * reference (ofstream without a check, :617), an unopenable path is not an
 * error unless strict != 0. */
int pj_write_sol(const int32_t* dist, int64_t n, const char* path, int strict);
/* Format into a caller buffer; *len_out receives the byte count. With
 * buf == NULL only the length is computed. */
int pj_format_sol(const int32_t* dist, int64_t n, char* buf, int64_t cap, int64_t* len_out);

#ifdef __cplusplus
}
#endif

#endif /* PJ_H */
