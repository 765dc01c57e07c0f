// devmem.cpp — DevBuf's device allocations, with a process-wide cache of big blocks.
//
// A block of 1 GiB or more that is freed is kept (up to a third of the device's memory)
// and handed out again to a later request of at most its size and at least 4/9 of it, on
// the same device (a world-2 build's blocks fit in a world-1 build's, about twice their
// size). Reason (round 5, bench.py's partition legs): the partitioned builds allocate and free tens of GB of sort temporaries per rank, and the one hipMalloc per
// build that had to take fresh memory from the driver took 2.7-5.2 s for a 17-34 GB block
// (profiles/r05: the build phases' slowest allocation); from the cache it is free. A
// request that fails with the cache holding blocks empties the cache and tries again, so
// the cache never costs an allocation that would otherwise succeed.
#include <mutex>
#include <unordered_map>
#include <vector>

#include "internal.h"

namespace pj {

namespace {

constexpr size_t BIG = size_t(1) << 30;

struct BigCache {
    std::mutex mu;
    struct Blk {
        int dev;
        void* p;
        size_t bytes;
    };
    std::vector<Blk> free_blocks;                // cached, not in use
    std::unordered_map<void*, Blk> live;         // big blocks in use (their real size)
    size_t cached = 0;
    size_t cap(int dev) {
        size_t fr = 0, tot = 0;
        (void)dev;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 0;
        return tot / 3;
    }
    void flush() {  // (mu held)
        for (auto& b : free_blocks) (void)hipFree(b.p);
        free_blocks.clear();
        cached = 0;
    }
};

BigCache& cache() {
    static BigCache* c = new BigCache();  // (never destroyed: no teardown-order issues at exit)
    return *c;
}

}  // namespace

void* dev_alloc(size_t bytes) {
    void* p = nullptr;
    if (bytes < BIG) {
        PJ_HIP(hipMalloc(&p, bytes));
        return p;
    }
    int dev = 0;
    PJ_HIP(hipGetDevice(&dev));
    BigCache& c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    size_t best = (size_t)-1;
    for (size_t i = 0; i < c.free_blocks.size(); ++i) {
        const auto& b = c.free_blocks[i];
        if (b.dev == dev && b.bytes >= bytes && b.bytes <= bytes / 4 * 9 &&
            (best == (size_t)-1 || b.bytes < c.free_blocks[best].bytes))
            best = i;
    }
    if (best != (size_t)-1) {
        const BigCache::Blk b = c.free_blocks[best];
        c.free_blocks.erase(c.free_blocks.begin() + (std::ptrdiff_t)best);
        c.cached -= b.bytes;
        c.live[b.p] = b;
        return b.p;
    }
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess && !c.free_blocks.empty()) {
        (void)hipGetLastError();
        c.flush();
        e = hipMalloc(&p, bytes);
    }
    PJ_HIP(e);
    c.live[p] = BigCache::Blk{dev, p, bytes};
    return p;
}

void dev_free(void* p, size_t bytes) {
    if (!p) return;
    if (bytes < BIG) {
        (void)hipFree(p);
        return;
    }
    BigCache& c = cache();
    {
        std::lock_guard<std::mutex> lk(c.mu);
        auto it = c.live.find(p);
        if (it != c.live.end()) {
            const BigCache::Blk b = it->second;
            c.live.erase(it);
            if (c.cached + b.bytes <= c.cap(b.dev)) {
                c.free_blocks.push_back(b);
                c.cached += b.bytes;
                return;
            }
        }
    }
    (void)hipFree(p);
}

}  // namespace pj
