// engine.h — the multi-GPU side of libpj (not part of the ABI): the transport
// that replaces the reference's MPI collectives, and the rank-local protocol
// loops that replace its BSP round loop (ParallelJohnson.cpp:488-594).
//
// A rank runs one of the loops (bfs_engine / delta_engine) against
//  - its device steps (BfsSteps / DeltaSteps: part.hip / wpart.hip kernels,
//    or caller callbacks), and
//  - a Comm: RCCL over xGMI (one process per GPU, or one process driving
//    several GPUs from one thread each), device copies between ranks that are
//    threads of one process ("host" transport: several ranks per GPU, the
//    SURVEY.md §4.3 fake cluster), or caller callbacks (e.g. MPI).
#pragma once

#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>

#include "internal.h"

namespace pj {

// ------------------------------------------------------------------ Comm ---
// Collectives of one rank. Device pointers belong to the rank's device and are
// ordered on stream `s` (callback transports get whatever pointers the steps
// expose). Every rank of the group must make the same calls in the same order.
struct Comm {
    int rank = 0, world = 1;
    virtual ~Comm() = default;
    virtual const char* kind() const = 0;
    // the group's size and this rank's index as the transport itself reports them (RCCL:
    // ncclCommCount / ncclCommUserRank of the communicator; the thread group's size; the
    // callbacks' declared world), for a caller to check against the world it launched
    virtual void transport_ranks(int* count, int* index) const {
        *count = world;
        *index = rank;
    }
    // element-wise sum (or min) of k host values over the ranks (:589-590)
    virtual void allreduce(i64* v, int k, bool is_min, hipStream_t s) = 0;
    // recv[q] = what rank q sends to this rank (the counts MPI_Alltoall, :522-523)
    virtual void alltoall_counts(const i64* send, i64* recv, hipStream_t s) = 0;
    // owner-major segments of `elem`-byte items: send[...] holds scount[q] items for
    // rank q in rank order; recv gets rcount[q] items from q in rank order (:553-554)
    virtual void alltoallv(const void* send, const i64* scount, void* recv, const i64* rcount, size_t elem,
                           hipStream_t s) = 0;
    // all[q * bytes ...] := rank q's own bytes (own may alias all + rank * bytes)
    virtual void allgather(const void* own, void* all, size_t bytes, hipStream_t s) = 0;
    // release a group whose peer failed (threads of one process: the host barrier;
    // RCCL: ncclCommAbort, the group's peers abort theirs); no-op elsewhere
    virtual void abort() {}
    // make a host group usable again once every rank has left a failed collective
    virtual void reset() {}
    // wait for the stream (RCCL: polled, so a failed peer ends the wait)
    virtual void sync(hipStream_t s) {
        if (s) PJ_HIP(hipStreamSynchronize(s));
    }
    // Device rows (RCCL): every rank's k-value device row, gathered to the host
    // (world x k values, rank-major) by one collective and one device->host copy.
    // The loops use it for step results that stay on the device (the per-owner
    // counts of a push, the level / band statistics), instead of a host readback
    // by the step plus a host-staged collective: one host wait instead of two.
    virtual bool rows_on_device() const { return false; }
    virtual void allgather_rows_dev(const i64* dev_row, int k, i64* host_all, hipStream_t s) {
        (void)dev_row, (void)k, (void)host_all, (void)s;
        throw Error(PJ_ERR_COMM, "allgather_rows_dev: not supported by this transport");
    }
};

std::unique_ptr<Comm> make_self_comm();
// world ranks in one process, one thread per rank: device copies between the
// ranks' buffers (any devices, several ranks per device allowed)
std::vector<std::unique_ptr<Comm>> make_thread_comms(int world, const std::vector<int>& devices);
// world ranks in one process over RCCL (ncclCommInitAll; distinct devices)
std::vector<std::unique_ptr<Comm>> make_rccl_group(const std::vector<int>& devices);
// one rank of a multi-process RCCL group (ncclCommInitRank)
std::unique_ptr<Comm> make_rccl_rank(int device, int world, int rank, const uint8_t* uid);
void rccl_unique_id(uint8_t* out128);
std::unique_ptr<Comm> make_callback_comm(const pj_comm_callbacks& cb);

// --------------------------------------------------------- device steps ---
// The pj_part_* steps of one rank (include/pj.h) and the buffers they share
// with the transport: vis / iso (world * bw u64, replicated), send / recv (u32
// ids; caller steps: world * block, libpj's steps: sized to the traffic by
// exchange_buffers), zown (bw u64).
struct BfsSteps {
    i64 n = 0, nnz_local = 0, bw = 1, block = 64;
    int rank = 0, world = 1;
    void *vis = nullptr, *iso = nullptr, *zown = nullptr, *send = nullptr, *recv = nullptr;
    virtual ~BfsSteps() = default;
    virtual hipStream_t stream() { return nullptr; }
    virtual void zmask() = 0;  // own isolated-vertex words -> zown
    virtual void begin(i64 source, i64* st3) = 0;
    virtual void push(int level, i64* counts) = 0;
    virtual void apply(int level, i64 n_recv) = 0;
    virtual void pull(int level) = 0;
    virtual void end_level(i64* st3) = 0;
    // Device-resident results (nullptr: host values only). push(level, nullptr)
    // leaves the per-owner counts at counts_dev() (world values); end_level_async()
    // leaves the 5-value level row (n_f, m_f, frontier vertices with edges, -, a
    // nonzero "foreign id received" flag) at stats_dev(), and end_level_finish(own)
    // consumes this rank's row once it is on the host.
    virtual const i64* counts_dev() { return nullptr; }
    virtual const i64* stats_dev() { return nullptr; }
    virtual void end_level_async() {}
    virtual void end_level_finish(const i64* own5) { (void)own5; }
    // Called after a push level's counts are known on every rank, before the exchange:
    // send must then hold the packed ids (nsend of them) and recv room for nrecv. The
    // default (callback steps) keeps the caller's buffers, packed by push itself.
    virtual void exchange_buffers(i64 nsend, i64 nrecv) { (void)nsend, (void)nrecv; }
    // Pieces (optional): a level whose ids exceed exchange_cap() (per rank and direction; 0 =
    // no cap) goes out in K pieces by word range of every owner's slice: piece_counts(k, K)
    // gives the per-owner counts of piece k (its ids stay marked until packed),
    // exchange_buffers(nsend, nrecv) then packs that piece, and each piece is applied.
    virtual i64 exchange_cap() { return 0; }
    virtual void piece_counts(int k, int npieces, i64* counts) { (void)k, (void)npieces, (void)counts; }
};

// The pj_wpart_* steps; send / recv hold u64 (id | cand << 32): world * block for
// caller steps, sized to the traffic by exchange_buffers for libpj's steps.
struct DeltaSteps {
    i64 n = 0;
    int rank = 0, world = 1;
    void *send = nullptr, *recv = nullptr;
    virtual ~DeltaSteps() = default;
    virtual hipStream_t stream() { return nullptr; }
    virtual int32_t begin(i64 source, int32_t delta) = 0;
    virtual void select(int32_t lo, int32_t hi, i64* out2) = 0;
    virtual void relax(int light, int32_t lo, int32_t hi, i64* counts) = 0;
    virtual void apply(i64 n_recv, int light, int32_t lo, int32_t hi) = 0;
    virtual i64 end_round() = 0;
    virtual void reach(i64* out2) = 0;
    // after relax's counts are exchanged, before the alltoallv (as BfsSteps)
    virtual void exchange_buffers(i64 nsend, i64 nrecv) { (void)nsend, (void)nrecv; }
    // Device-resident results (nullptr: host values only): select_async() leaves the
    // row (min pending dist as u64, band size) at select_dev(); end_round_async() leaves
    // the new frontier size at nf_dev(); the finish calls reset the step's counters.
    virtual const i64* select_dev() { return nullptr; }
    virtual const i64* nf_dev() { return nullptr; }
    virtual void select_async(int32_t lo, int32_t hi) { (void)lo, (void)hi; }
    virtual void select_finish() {}
    virtual void end_round_async() {}
    // Tail switch (optional; the defaults disable it): once the out-edges of the vertices
    // not settled below hi, summed over the ranks, drop under tail_frac x all edges, the
    // bands after this one use the light threshold and width tail_delta (64 x delta by
    // default: every edge light, bands of Bellman-Ford rounds). Exact at a band boundary:
    // everything below hi is settled and relaxed. unsettled_edges(hi) returns this rank's
    // sum (-1: not supported, on every rank alike), local_edges() this rank's edges.
    virtual double tail_frac() { return 0.0; }
    virtual int32_t tail_delta(int32_t delta) { return delta; }
    virtual i64 unsettled_edges(int32_t hi) { (void)hi; return -1; }
    virtual i64 local_edges() { return 0; }
    virtual void set_delta(int32_t delta) { (void)delta; }
    // Settled filter of the tail (optional): settled_slice(lo) writes this rank's words of
    // settled_map() (bit v: dist[v] < lo, settled_bytes() bytes at rank x settled_bytes();
    // 64-aligned blocks), the engine all-gathers it once, at the tail switch; the tail's
    // relaxations then skip settled targets without reading their distance.
    virtual void* settled_map() { return nullptr; }
    virtual size_t settled_bytes() { return 0; }
    virtual void settled_slice(int32_t lo) { (void)lo; }
    // Heavy pull (optional; symmetric graphs): instead of the members pushing their heavy
    // edges (relax / exchange / apply), every rank's unsettled vertices scan their own heavy
    // rows for members, read from a replicated byte map (dist - lo of a member, 0xFF
    // otherwise): member_slice() writes this rank's slice of member_map() (member_bytes()
    // bytes at rank x member_bytes()), the engine all-gathers it, heavy_pull() relaxes.
    // heavy_counts(): this rank's (members' heavy edges, unsettled vertices' heavy edges).
    virtual double pull_factor() { return -1.0; }  // -1: no heavy pull (callback steps); 0: off on this rank
    virtual void heavy_counts(int32_t lo, int32_t hi, i64* out2) { (void)lo, (void)hi, out2[0] = out2[1] = 0; }
    virtual void member_slice(int32_t lo, int32_t hi) { (void)lo, (void)hi; }
    virtual void* member_map() { return nullptr; }
    virtual size_t member_bytes() { return 0; }
    virtual void heavy_pull(int32_t lo, int32_t hi) { (void)lo, (void)hi; }
    // Light pull rounds (optional; symmetric graphs): a round whose frontier's light edges
    // exceed the light edges of the vertices above lo / light_pull_factor() runs as a pull:
    // frontier_slice() writes this rank's slice of member_map() (dist - lo of a frontier
    // vertex, 0xFF otherwise), the engine all-gathers it, light_pull() lets every owned vertex
    // above lo scan its light row for frontier vertices and marks the improved ones below hi.
    // light_counts(): this rank's (frontier light edges, light edges of vertices above lo).
    virtual double light_pull_factor() { return -1.0; }
    // the same rule after the tail switch (defaults to light_pull_factor), and the widest band
    // the frontier map can encode (dist - lo per vertex)
    virtual double tail_light_pull_factor() { return light_pull_factor(); }
    virtual int32_t pull_map_width() { return 255; }
    virtual void light_counts(int32_t lo, int32_t hi, i64* out2) { (void)lo, (void)hi, out2[0] = out2[1] = 0; }
    // the least distance of this rank's frontier (after light_counts; INT_INF: none or not
    // counted), and every rank's, min-all-reduced by the loop before a light pull: the pull's
    // rows stop at that minimum + w instead of lo + w (optional: -1 keeps lo)
    virtual i64 frontier_min() { return -1; }
    virtual void set_frontier_min(i64 m) { (void)m; }
    virtual void frontier_slice(int32_t lo, int32_t hi) { (void)lo, (void)hi; }
    virtual void light_pull(int32_t lo, int32_t hi) { (void)lo, (void)hi; }
};

struct BfsParams {
    double alpha = 14.0, beta = 24.0;
    int force = 0;  // 0 auto, 1 push only, 2 pull from level 1 on
    i64 xcap = -1;  // exchange buffer cap in ids per rank and direction (-1: block / 16; 0: none)
};

// The rank-local loops. `iso_ready` says the replicated isolated mask in
// steps.iso is current (it is gathered once per graph and transport).
void bfs_engine(BfsSteps& steps, Comm& comm, i64 source, const BfsParams& prm, bool iso_ready, pj_part_stats* st);
void delta_engine(DeltaSteps& steps, Comm& comm, i64 source, int32_t delta, pj_part_stats* st);

// part.hip / wpart.hip: the GPU implementations (buffers owned by the part)
BfsSteps& part_steps(Part& p);
DeltaSteps& wpart_steps(WPart& p);
bool& part_iso_ready(Part& p, const Comm* comm);
BfsParams& part_params(Part& p);
// the context (device, stream) a part was built on: API entry points bind it first,
// because the per-rank host threads start on device 0
const Ctx& part_ctx(const Part& p);
const Ctx& wpart_ctx(const WPart& p);
int wpart_world(const WPart& p);
// world 1 (option "single_gpu", default on): the solve runs delta.hip's single-GPU solver
bool part_single(const Part& p);  // world 1 with option single_gpu: bfs.hip's solver (part_solve_single)
int& part_single_gpu(Part& p);
void part_solve_single(Part& p, i64 source, pj_part_stats* st);
bool wpart_single(const WPart& p);
int& wpart_single_gpu(WPart& p);
int& wpart_grid_per_cu(WPart& p);  // workgroups per CU of its grid-stride kernels (option "grid_per_cu", default 8)
int& wpart_pull_fmin(WPart& p);  // light pulls' frontier-minimum bound (option "pull_fmin", default 1)
void wpart_solve_single(WPart& p, i64 source, int32_t delta, pj_part_stats* st);
bool wpart_pending(const WPart& p);
void wpart_set_queue_shard(WPart& p, i64 pairs);
double* wpart_tail_params(WPart& p);  // [0] tail_frac, [1] tail_mult (pj_wpart_set_option)
double& wpart_pull_factor(WPart& p);  // heavy pull rule (pj_wpart_set_option "pull_factor")
double& wpart_light_pull(WPart& p);   // light pull rule (pj_wpart_set_option "light_pull")
double& wpart_tail_light_pull(WPart& p);  // its tail form ("tail_light_pull")
// every rank's slice of dist, gathered (n int32 to host; NULL: gather only)
void part_gather_dist(Part& p, Comm& comm, int32_t* out);
void wpart_gather_dist(WPart& p, Comm& comm, int32_t* out);

}  // namespace pj
