// comm.cpp — the transports behind pj_comm (engine.h): the analogue of the
// reference's MPI_COMM_WORLD collectives (ParallelJohnson.cpp:344-406 setup,
// :522-554 per-round Alltoall + Alltoallv, :589-590 Allreduce, :612 Gatherv).
//
//  - RcclComm: RCCL over xGMI. librccl is opened at run time (dlopen), so
//    libpj loads on hosts without it and a single-GPU run never touches it.
//    Variable-size exchanges are grouped ncclSend/ncclRecv (one peer per xGMI
//    link, no ring), counts and bitmaps go through ncclAllGather, termination
//    counts through ncclAllReduce.
//  - ThreadComm: the ranks are threads of one process; each rank pulls its
//    segments from the peers' device buffers (hipMemcpyPeerAsync, or a D2D copy
//    on a shared device) between two host barriers. Several ranks may share a
//    GPU (the fake cluster of SURVEY.md §4.3).
//  - CallbackComm: the caller's functions (e.g. MPI, or gloo in the CPU tests).
#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <chrono>
#include <thread>

#include <rccl/rccl.h>

#include "engine.h"

namespace pj {

// ------------------------------------------------------------------ self ---
namespace {

void copy_on(void* dst, int ddev, const void* src, int sdev, size_t bytes, hipStream_t s) {
    if (!bytes || dst == src) return;
    if (ddev == sdev || ddev < 0 || sdev < 0) PJ_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s));
    else PJ_HIP(hipMemcpyPeerAsync(dst, ddev, src, sdev, bytes, s));
}

struct SelfComm final : Comm {
    const char* kind() const override { return "self"; }
    void allreduce(i64*, int, bool, hipStream_t) override {}
    void alltoall_counts(const i64* send, i64* recv, hipStream_t) override { recv[0] = send[0]; }
    void alltoallv(const void* send, const i64* scount, void* recv, const i64*, size_t elem, hipStream_t s) override {
        copy_on(recv, -1, send, -1, (size_t)scount[0] * elem, s);
    }
    void allgather(const void* own, void* all, size_t bytes, hipStream_t s) override {
        copy_on(all, -1, own, -1, bytes, s);
    }
};

}  // namespace

std::unique_ptr<Comm> make_self_comm() { return std::make_unique<SelfComm>(); }

// ---------------------------------------------------------------- threads ---
namespace {

struct ThreadGroup {
    int world;
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<int> arrived{0};
    std::atomic<u64> gen{0};
    std::atomic<bool> failed{false};
    std::vector<i64> red;                 // world x k allreduce slots (k > kslot)
    std::vector<const void*> ptr;         // per rank: published buffer
    std::vector<const i64*> cnt;          // per rank: published host counts
    std::vector<int> dev;                 // per rank: device
    // two banks of world x kslot slots for the one-barrier allreduce / count exchange: the
    // collectives alternate banks, and a bank is written again only after every rank has
    // passed the barrier of the collective in between, so after it has read the bank
    int kslot;
    std::vector<i64> bank[2];
    explicit ThreadGroup(int w) : world(w), ptr((size_t)w), cnt((size_t)w), dev((size_t)w, -1), kslot(std::max(8, w)) {
        bank[0].assign((size_t)w * (size_t)kslot, 0);
        bank[1].assign((size_t)w * (size_t)kslot, 0);
    }

    // Spins for up to ~200 us before it sleeps on the condition variable: a collective step
    // of the band loop waits for its peer for tens of microseconds, and a futex wake-up costs
    // about as much again per barrier (round 5: 7 barriers per light round over the host
    // transport, 4 since the one-barrier allreduce and count exchange). The ranks are threads of one process on a CPU share of >= 16 cores.
    void barrier() {
        if (failed.load(std::memory_order_acquire))
            throw Error(PJ_ERR_COMM, "a peer rank of the thread group failed");
        const u64 g = gen.load(std::memory_order_acquire);
        if (arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == world) {
            arrived.store(0, std::memory_order_relaxed);
            gen.store(g + 1, std::memory_order_release);
            { std::lock_guard<std::mutex> lk(mu); }  // (a sleeper sees the new generation or is notified)
            cv.notify_all();
            return;
        }
        const auto t0 = std::chrono::steady_clock::now();
        for (int spin = 0; gen.load(std::memory_order_acquire) == g; ++spin) {
            if (failed.load(std::memory_order_acquire))
                throw Error(PJ_ERR_COMM, "a peer rank of the thread group failed");
            if ((spin & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return gen.load(std::memory_order_acquire) != g || failed.load(); });
                break;
            }
        }
        if (gen.load(std::memory_order_acquire) == g && failed.load())
            throw Error(PJ_ERR_COMM, "a peer rank of the thread group failed");
    }
    void abort() {
        failed.store(true, std::memory_order_release);
        { std::lock_guard<std::mutex> lk(mu); }
        cv.notify_all();
    }
    // after every rank has left the failed collective (the caller joined the rank threads)
    void reset() {
        std::lock_guard<std::mutex> lk(mu);
        failed.store(false);
        arrived.store(0);
    }
};

struct ThreadComm final : Comm {
    std::shared_ptr<ThreadGroup> g;
    int device = -1;
    u64 seq = 0;  // slot collectives so far (the same on every rank): the bank of the next one
    const char* kind() const override { return "host"; }
    void transport_ranks(int* count, int* index) const override {
        *count = g->world;
        *index = rank;
    }

    void allreduce(i64* v, int k, bool is_min, hipStream_t) override {
        if (k <= g->kslot) {  // one barrier: publish into this collective's bank, then reduce
            i64* b = g->bank[seq++ & 1].data();
            const size_t K = (size_t)g->kslot;
            std::copy(v, v + k, b + (size_t)rank * K);
            g->barrier();
            for (int j = 0; j < k; ++j) {
                i64 a = b[(size_t)j];
                for (int q = 1; q < world; ++q) {
                    const i64 x = b[(size_t)q * K + (size_t)j];
                    a = is_min ? std::min(a, x) : a + x;
                }
                v[j] = a;
            }
            return;
        }
        {
            std::lock_guard<std::mutex> lk(g->mu);
            if (g->red.size() < (size_t)world * (size_t)k) g->red.resize((size_t)world * (size_t)k);
        }
        g->barrier();  // every rank sized the slots
        std::copy(v, v + k, g->red.begin() + (ptrdiff_t)rank * k);
        g->barrier();
        for (int j = 0; j < k; ++j) {
            i64 a = g->red[(size_t)j];
            for (int q = 1; q < world; ++q) {
                const i64 b = g->red[(size_t)q * (size_t)k + (size_t)j];
                a = is_min ? std::min(a, b) : a + b;
            }
            v[j] = a;
        }
        g->barrier();  // the slots are free again
    }

    void alltoall_counts(const i64* send, i64* recv, hipStream_t) override {
        i64* b = g->bank[seq++ & 1].data();  // (kslot >= world)
        const size_t K = (size_t)g->kslot;
        std::copy(send, send + world, b + (size_t)rank * K);
        g->barrier();
        for (int q = 0; q < world; ++q) recv[q] = b[(size_t)q * K + (size_t)rank];
    }

    void alltoallv(const void* send, const i64* scount, void* recv, const i64* rcount, size_t elem,
                   hipStream_t s) override {
        PJ_HIP(hipStreamSynchronize(s));  // the send segments are complete
        g->ptr[(size_t)rank] = send;
        g->cnt[(size_t)rank] = scount;
        g->dev[(size_t)rank] = device;
        g->barrier();
        size_t roff = 0;
        for (int q = 0; q < world; ++q) {
            const i64* sc = g->cnt[(size_t)q];
            size_t displ = 0;  // where rank q's segment for this rank starts
            for (int o = 0; o < rank; ++o) displ += (size_t)sc[o];
            if ((i64)sc[rank] != rcount[q]) throw Error(PJ_ERR_COMM, "alltoallv: counts disagree");
            copy_on(static_cast<char*>(recv) + roff * elem, device,
                    static_cast<const char*>(g->ptr[(size_t)q]) + displ * elem, g->dev[(size_t)q],
                    (size_t)sc[rank] * elem, s);
            roff += (size_t)sc[rank];
        }
        PJ_HIP(hipStreamSynchronize(s));
        g->barrier();  // every peer has read this rank's send buffer
    }

    void allgather(const void* own, void* all, size_t bytes, hipStream_t s) override {
        PJ_HIP(hipStreamSynchronize(s));
        g->ptr[(size_t)rank] = own;
        g->dev[(size_t)rank] = device;
        g->barrier();
        for (int q = 0; q < world; ++q)
            copy_on(static_cast<char*>(all) + (size_t)q * bytes, device, g->ptr[(size_t)q], g->dev[(size_t)q], bytes,
                    s);
        PJ_HIP(hipStreamSynchronize(s));
        g->barrier();
    }

    void abort() override { g->abort(); }
    void reset() override {
        g->reset();
        seq = 0;
    }
};

}  // namespace

std::vector<std::unique_ptr<Comm>> make_thread_comms(int world, const std::vector<int>& devices) {
    if (world < 1 || (int)devices.size() != world) throw Error(PJ_ERR_ARG, "thread comm: one device per rank");
    auto grp = std::make_shared<ThreadGroup>(world);
    std::vector<std::unique_ptr<Comm>> out;
    for (int r = 0; r < world; ++r) {
        auto c = std::make_unique<ThreadComm>();
        c->rank = r;
        c->world = world;
        c->g = grp;
        c->device = devices[(size_t)r];
        out.push_back(std::move(c));
    }
    return out;
}

// ------------------------------------------------------------------ RCCL ---
namespace {

struct RcclApi {
    void* h = nullptr;
    decltype(&ncclGetUniqueId) getUniqueId = nullptr;
    decltype(&ncclCommInitRank) commInitRank = nullptr;
    decltype(&ncclCommInitAll) commInitAll = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclAllReduce) allReduce = nullptr;
    decltype(&ncclAllGather) allGather = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) groupStart = nullptr;
    decltype(&ncclGroupEnd) groupEnd = nullptr;
    decltype(&ncclGetErrorString) errorString = nullptr;
    decltype(&ncclCommAbort) commAbort = nullptr;
    decltype(&ncclCommGetAsyncError) getAsyncError = nullptr;
    decltype(&ncclCommCount) commCount = nullptr;
    decltype(&ncclCommUserRank) commUserRank = nullptr;
};

const RcclApi& rccl() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        // an RCCL already in the process (e.g. PyTorch's) is reused by SONAME
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return;
        api.h = h;
#define PJ_SYM(field, name) api.field = reinterpret_cast<decltype(api.field)>(dlsym(h, #name))
        PJ_SYM(getUniqueId, ncclGetUniqueId);
        PJ_SYM(commInitRank, ncclCommInitRank);
        PJ_SYM(commInitAll, ncclCommInitAll);
        PJ_SYM(commDestroy, ncclCommDestroy);
        PJ_SYM(allReduce, ncclAllReduce);
        PJ_SYM(allGather, ncclAllGather);
        PJ_SYM(send, ncclSend);
        PJ_SYM(recv, ncclRecv);
        PJ_SYM(groupStart, ncclGroupStart);
        PJ_SYM(groupEnd, ncclGroupEnd);
        PJ_SYM(errorString, ncclGetErrorString);
        PJ_SYM(commAbort, ncclCommAbort);
        PJ_SYM(getAsyncError, ncclCommGetAsyncError);
        PJ_SYM(commCount, ncclCommCount);
        PJ_SYM(commUserRank, ncclCommUserRank);
#undef PJ_SYM
    });
    if (!api.h || !api.getUniqueId || !api.commInitRank || !api.commInitAll || !api.allReduce || !api.allGather ||
        !api.send || !api.recv || !api.groupStart || !api.groupEnd || !api.commDestroy || !api.errorString ||
        !api.commAbort || !api.getAsyncError || !api.commCount || !api.commUserRank)
        throw Error(PJ_ERR_COMM, "RCCL (librccl.so.1) is not available");
    return api;
}

void nccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw Error(PJ_ERR_COMM, std::string(what) + ": " + rccl().errorString(r));
}

// Failure state shared by the ranks of one process's RCCL group (ncclCommInitAll):
// a rank that fails raises it, and every peer waiting on a collective aborts its
// own communicator, so its blocked kernels exit instead of hanging the group.
struct RcclGroupState {
    std::atomic<bool> failed{false};
};

struct RcclComm final : Comm {
    ncclComm_t c = nullptr;
    int device = 0;
    bool aborted = false;
    std::shared_ptr<RcclGroupState> grp;  // null for one rank of a multi-process group
    DevBuf<i64> scratch;  // allreduce values / all-gathered count rows
    PinnedBuf<i64> host;
    const char* kind() const override { return "rccl"; }
    void transport_ranks(int* count, int* index) const override {
        usable();
        nccl_check(rccl().commCount(c, count), "ncclCommCount");
        nccl_check(rccl().commUserRank(c, index), "ncclCommUserRank");
    }

    void init_buffers() {
        PJ_HIP(hipSetDevice(device));
        const size_t cap = std::max<size_t>(64, (size_t)world * (size_t)(world + 8));
        scratch.alloc(cap);
        host.alloc(cap);
    }
    ~RcclComm() override {
        if (c && !aborted) (void)rccl().commDestroy(c);
    }
    void usable() const {
        if (aborted) throw Error(PJ_ERR_COMM, "the RCCL communicator was aborted after a rank failure");
    }
    void abort_local() {
        if (c && !aborted) {
            aborted = true;
            (void)rccl().commAbort(c);
        }
    }
    void abort() override {
        if (grp) grp->failed = true;
        abort_local();
    }
    // stream completion, polled so a peer's failure (group flag) or an RCCL async
    // error ends the wait: hipStreamSynchronize would block forever on a dead peer
    void wait(hipStream_t s) {
        const RcclApi& api = rccl();
        for (int spin = 0;; ++spin) {
            const hipError_t e = hipStreamQuery(s);
            if (e == hipSuccess) return;
            if (e != hipErrorNotReady) PJ_HIP(e);
            ncclResult_t ae = ncclSuccess;
            if (api.getAsyncError(c, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
                abort_local();
                throw Error(PJ_ERR_COMM, std::string("RCCL async error: ") + api.errorString(ae));
            }
            if (grp && grp->failed) {
                abort_local();
                throw Error(PJ_ERR_COMM, "a peer rank of the RCCL group failed");
            }
            if (spin > 2000) std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    }

    void allreduce(i64* v, int k, bool is_min, hipStream_t s) override {
        usable();
        if ((size_t)k > scratch.n) throw Error(PJ_ERR_ARG, "allreduce: too many values");
        std::copy(v, v + k, host.p);
        PJ_HIP(hipMemcpyAsync(scratch.p, host.p, sizeof(i64) * (size_t)k, hipMemcpyHostToDevice, s));
        nccl_check(rccl().allReduce(scratch.p, scratch.p, (size_t)k, ncclInt64, is_min ? ncclMin : ncclSum, c, s),
                   "ncclAllReduce");
        PJ_HIP(hipMemcpyAsync(host.p, scratch.p, sizeof(i64) * (size_t)k, hipMemcpyDeviceToHost, s));
        wait(s);
        std::copy(host.p, host.p + k, v);
    }

    void alltoall_counts(const i64* send, i64* recv, hipStream_t s) override {
        usable();
        // row r of a world x world matrix per rank; in place: own row at offset rank * world
        i64* rows = scratch.p;
        std::copy(send, send + world, host.p);
        PJ_HIP(hipMemcpyAsync(rows + (size_t)rank * world, host.p, sizeof(i64) * (size_t)world, hipMemcpyHostToDevice,
                              s));
        nccl_check(rccl().allGather(rows + (size_t)rank * world, rows, (size_t)world, ncclInt64, c, s),
                   "ncclAllGather(counts)");
        PJ_HIP(hipMemcpyAsync(host.p, rows, sizeof(i64) * (size_t)world * world, hipMemcpyDeviceToHost, s));
        wait(s);
        for (int q = 0; q < world; ++q) recv[q] = host.p[(size_t)q * world + rank];
    }

    void alltoallv(const void* send, const i64* scount, void* recv, const i64* rcount, size_t elem,
                   hipStream_t s) override {
        usable();
        const char* sb = static_cast<const char*>(send);
        char* rb = static_cast<char*>(recv);
        size_t so = 0, ro = 0, self_s = 0, self_r = 0;
        const RcclApi& api = rccl();
        nccl_check(api.groupStart(), "ncclGroupStart");
        for (int q = 0; q < world; ++q) {
            const size_t sbytes = (size_t)scount[q] * elem, rbytes = (size_t)rcount[q] * elem;
            if (q == rank) {
                self_s = so;
                self_r = ro;
            } else {
                if (sbytes) nccl_check(api.send(sb + so, sbytes, ncclUint8, q, c, s), "ncclSend");
                if (rbytes) nccl_check(api.recv(rb + ro, rbytes, ncclUint8, q, c, s), "ncclRecv");
            }
            so += sbytes;
            ro += rbytes;
        }
        nccl_check(api.groupEnd(), "ncclGroupEnd");
        copy_on(rb + self_r, device, sb + self_s, device, (size_t)scount[rank] * elem, s);
        wait(s);  // any later host wait of the steps is then on local work only
    }

    void allgather(const void* own, void* all, size_t bytes, hipStream_t s) override {
        usable();
        nccl_check(rccl().allGather(own, all, bytes, ncclUint8, c, s), "ncclAllGather");
        wait(s);
    }
    // the loops' own stream waits after a collective (end of a solve, gathers)
    void sync(hipStream_t s) override { wait(s); }

    bool rows_on_device() const override { return true; }
    void allgather_rows_dev(const i64* dev_row, int k, i64* host_all, hipStream_t s) override {
        usable();
        if (k < 1 || (size_t)world * (size_t)k > scratch.n) throw Error(PJ_ERR_ARG, "allgather_rows_dev: row too long");
        nccl_check(rccl().allGather(dev_row, scratch.p, (size_t)k, ncclInt64, c, s), "ncclAllGather(rows)");
        PJ_HIP(hipMemcpyAsync(host.p, scratch.p, sizeof(i64) * (size_t)world * (size_t)k, hipMemcpyDeviceToHost, s));
        wait(s);
        std::copy(host.p, host.p + (size_t)world * (size_t)k, host_all);
    }
};

}  // namespace

void rccl_unique_id(uint8_t* out128) {
    static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id is 128 bytes");
    ncclUniqueId id;
    nccl_check(rccl().getUniqueId(&id), "ncclGetUniqueId");
    std::memcpy(out128, &id, sizeof(id));
}

std::unique_ptr<Comm> make_rccl_rank(int device, int world, int rank, const uint8_t* uid) {
    auto c = std::make_unique<RcclComm>();
    c->rank = rank;
    c->world = world;
    c->device = device;
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    PJ_HIP(hipSetDevice(device));
    nccl_check(rccl().commInitRank(&c->c, world, id, rank), "ncclCommInitRank");
    c->init_buffers();
    return c;
}

std::vector<std::unique_ptr<Comm>> make_rccl_group(const std::vector<int>& devices) {
    const int world = (int)devices.size();
    std::vector<int> sorted = devices;
    std::sort(sorted.begin(), sorted.end());
    if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end())
        throw Error(PJ_ERR_COMM, "RCCL needs one GPU per rank (use the host transport to share a GPU)");
    std::vector<ncclComm_t> cs((size_t)world);
    nccl_check(rccl().commInitAll(cs.data(), world, devices.data()), "ncclCommInitAll");
    auto grp = std::make_shared<RcclGroupState>();
    std::vector<std::unique_ptr<Comm>> out;
    for (int r = 0; r < world; ++r) {
        auto c = std::make_unique<RcclComm>();
        c->rank = r;
        c->world = world;
        c->device = devices[(size_t)r];
        c->c = cs[(size_t)r];
        c->grp = grp;
        c->init_buffers();
        out.push_back(std::move(c));
    }
    return out;
}

// -------------------------------------------------------------- callbacks ---
namespace {

struct CallbackComm final : Comm {
    pj_comm_callbacks cb;
    const char* kind() const override { return "callbacks"; }
    static void ok(int rc, const char* what) {
        if (rc != 0) throw Error(PJ_ERR_COMM, std::string("transport callback ") + what + " failed");
    }
    void allreduce(i64* v, int k, bool is_min, hipStream_t s) override {
        if (s) PJ_HIP(hipStreamSynchronize(s));
        ok(cb.allreduce(cb.user, v, k, is_min ? 1 : 0), "allreduce");
    }
    void alltoall_counts(const i64* send, i64* recv, hipStream_t s) override {
        if (s) PJ_HIP(hipStreamSynchronize(s));
        ok(cb.alltoall_counts(cb.user, send, recv), "alltoall_counts");
    }
    void alltoallv(const void* send, const i64* scount, void* recv, const i64* rcount, size_t elem,
                   hipStream_t s) override {
        if (s) PJ_HIP(hipStreamSynchronize(s));
        ok(cb.alltoallv(cb.user, send, scount, recv, rcount, (int64_t)elem), "alltoallv");
    }
    void allgather(const void* own, void* all, size_t bytes, hipStream_t s) override {
        if (s) PJ_HIP(hipStreamSynchronize(s));
        ok(cb.allgather(cb.user, own, all, (int64_t)bytes), "allgather");
    }
};

}  // namespace

std::unique_ptr<Comm> make_callback_comm(const pj_comm_callbacks& cb) {
    if (!cb.allreduce || !cb.alltoall_counts || !cb.alltoallv || !cb.allgather || cb.world < 1 || cb.rank < 0 ||
        cb.rank >= cb.world)
        throw Error(PJ_ERR_ARG, "pj_comm_create_callbacks: missing callback or bad rank/world");
    auto c = std::make_unique<CallbackComm>();
    c->cb = cb;
    c->rank = cb.rank;
    c->world = cb.world;
    return c;
}

}  // namespace pj
