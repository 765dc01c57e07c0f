// devmem.cpp — DevBuf's device allocations, with a process-wide cache of big blocks.
//
// Reason (round 5, bench.py's partition legs): the partitioned builds allocate and free
// tens of GB of sort temporaries per rank, and a hipMalloc that takes memory the driver
// has just had back from a hipFree waits for that memory to be cleared (2.7-5.2 s for a
// 17-34 GB block, ~6 GB/s; profiles/r05: the build phases' slowest allocation). Memory
// that stays allocated in the process skips that.
//
// So a block of 1 GiB or more is not returned to the driver when DevBuf frees it: it stays
// cached (up to half of the device's memory; past that the least recently freed wholly
// free blocks go back first) and is handed out again, whole or in slices,
// to later requests on the same device. A request takes the smallest free range that holds
// it and leaves the rest of the range free (a world-2 build's two ranks take the two halves
// of a block a world-1 build freed); a freed slice merges with its free neighbours. A libpj
// allocation (big or small) that fails while the cache holds blocks returns every wholly free
// block to the driver and tries again, so the cache never costs libpj an allocation that
// would otherwise succeed; the free-memory estimates that size libpj's optional buffers
// (batch slots) count the cache's idle bytes as free (dev_free_bytes). Other allocators in the
// same process (e.g. torch) do not see the cached blocks: such callers trim the cache first
// (pj_trim_device_cache). A big free synchronizes the block's device first, as hipFree does: work still
// in flight on any stream may use the memory, and the next owner of a slice may be another
// stream (another rank's, or another batch slot's).
#include <algorithm>
#include <cstdlib>
#include <iterator>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "internal.h"

namespace pj {

namespace {

constexpr size_t BIG = size_t(1) << 30;
constexpr size_t ALIGN = 4096;            // slice boundaries
constexpr size_t SLACK = size_t(2) << 20;  // a fresh block's extra bytes: two slices whose sizes
                                           // add up to its request still fit after rounding

struct Blk {  // one hipMalloc'ed block: its free ranges (offset -> bytes) and live slices
    int dev;
    char* base;
    size_t bytes;
    std::map<size_t, size_t> free_ranges;
    int live;
    unsigned long long stamp;  // when a slice of it was last freed
};

struct BigCache {
    std::mutex mu;
    std::vector<Blk*> blocks;
    std::unordered_map<void*, std::pair<Blk*, size_t>> live;  // slice -> (its block, its bytes)
    size_t held = 0;                                           // bytes of all blocks
    unsigned long long clock = 0;

    static size_t cap() {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 0;
        return tot / 2;
    }
    void release(Blk* b) {  // (mu held; b has no live slice)
        (void)hipFree(b->base);
        held -= b->bytes;
        blocks.erase(std::find(blocks.begin(), blocks.end(), b));
        delete b;
    }
    void flush() {  // every wholly free block back to the driver (mu held)
        std::vector<Blk*> idle;
        for (Blk* b : blocks)
            if (b->live == 0) idle.push_back(b);
        for (Blk* b : idle) release(b);
    }
    void* take(Blk* b, std::map<size_t, size_t>::iterator it, size_t bytes) {
        const size_t off = it->first, len = it->second;
        b->free_ranges.erase(it);
        const size_t want = (bytes + ALIGN - 1) / ALIGN * ALIGN;
        size_t taken = len;
        if (len > want && len - want >= ALIGN) {  // the rest of the range stays free
            b->free_ranges[off + want] = len - want;
            taken = want;
        }
        b->live++;
        char* p = b->base + off;
        live[p] = {b, taken};
        return p;
    }
};

BigCache& cache() {
    static BigCache* c = new BigCache();  // (never destroyed: no teardown-order issues at exit)
    return *c;
}

// test hook: with PJ_DEVMEM_POISON set, every allocation (a cached slice, or a small block the
// driver may hand back from a recent free) starts full of 0xFF, so that a buffer relying on the
// zeroed pages of fresh driver memory, or a kernel reading words its pass never wrote, shows up
// (tests/test_partition.py, tests/test_gpu_parity.py); a device-wide wait after it: the memset
// runs on the null stream, which does not order against libpj's non-blocking streams
void poison(void* p, size_t bytes) {
    if (p && bytes && std::getenv("PJ_DEVMEM_POISON")) {
        PJ_HIP(hipMemset(p, 0xFF, bytes));
        PJ_HIP(hipDeviceSynchronize());
    }
}

}  // namespace

void* dev_alloc(size_t bytes) {
    void* p = nullptr;
    if (bytes < BIG) {
        hipError_t e = hipMalloc(&p, bytes);
        if (e != hipSuccess) {  // the cache's idle blocks back to the driver, then once more
            (void)hipGetLastError();
            BigCache& c = cache();
            std::lock_guard<std::mutex> lk(c.mu);
            if (c.held > 0) {
                c.flush();
                e = hipMalloc(&p, bytes);
            }
        }
        PJ_HIP(e);
        poison(p, bytes);
        return p;
    }
    int dev = 0;
    PJ_HIP(hipGetDevice(&dev));
    BigCache& c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    Blk* bb = nullptr;  // best fit: the smallest free range that holds the request
    std::map<size_t, size_t>::iterator bi;
    for (Blk* b : c.blocks) {
        if (b->dev != dev) continue;
        for (auto it = b->free_ranges.begin(); it != b->free_ranges.end(); ++it)
            if (it->second >= bytes && (!bb || it->second < bi->second)) {
                bb = b;
                bi = it;
            }
    }
    if (bb) {
        void* q = c.take(bb, bi, bytes);
        poison(q, bytes);
        return q;
    }
    const size_t bb_bytes = (bytes + SLACK - 1) / SLACK * SLACK + SLACK;
    hipError_t e = hipMalloc(&p, bb_bytes);
    if (e != hipSuccess && c.held > 0) {
        (void)hipGetLastError();
        c.flush();
        e = hipMalloc(&p, bb_bytes);
    }
    PJ_HIP(e);
    Blk* b = new Blk{dev, static_cast<char*>(p), bb_bytes, {}, 1, 0};
    c.blocks.push_back(b);
    c.held += bb_bytes;
    c.live[p] = {b, bb_bytes};
    return p;
}

void dev_free(void* p, size_t bytes) {
    if (!p) return;
    if (bytes < BIG) {
        (void)hipFree(p);
        return;
    }
    BigCache& c = cache();
    int bdev = -1;
    {
        std::lock_guard<std::mutex> lk(c.mu);
        auto it = c.live.find(p);
        if (it == c.live.end()) {  // (not from dev_alloc's big path; DevBuf never does this)
            (void)hipFree(p);
            return;
        }
        bdev = it->second.first->dev;
    }
    {  // (hipFree's implicit synchronization, on the block's device)
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (cur != bdev) (void)hipSetDevice(bdev);
        (void)hipDeviceSynchronize();
        if (cur != bdev && cur >= 0) (void)hipSetDevice(cur);
    }
    std::lock_guard<std::mutex> lk(c.mu);
    auto it = c.live.find(p);
    Blk* b = it->second.first;
    size_t off = (size_t)(static_cast<char*>(p) - b->base), len = it->second.second;
    c.live.erase(it);
    b->live--;
    auto nx = b->free_ranges.lower_bound(off);  // merge with the free neighbours
    if (nx != b->free_ranges.end() && nx->first == off + len) {
        len += nx->second;
        nx = b->free_ranges.erase(nx);
    }
    if (nx != b->free_ranges.begin()) {
        auto pv = std::prev(nx);
        if (pv->first + pv->second == off) {
            off = pv->first;
            len += pv->second;
            b->free_ranges.erase(pv);
        }
    }
    b->free_ranges[off] = len;
    b->stamp = ++c.clock;
    const size_t cap = BigCache::cap();
    if (c.held > cap) {  // over the cap: wholly free blocks back to the driver, least recent first
        std::vector<Blk*> idle;
        for (Blk* x : c.blocks)
            if (x->live == 0) idle.push_back(x);
        std::sort(idle.begin(), idle.end(), [](const Blk* x, const Blk* y) { return x->stamp < y->stamp; });
        for (Blk* x : idle) {
            if (c.held <= cap) break;
            c.release(x);
        }
    }
}

size_t dev_free_bytes() {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fr;
    BigCache& c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    for (const Blk* b : c.blocks)
        if (b->dev == dev)
            for (const auto& r : b->free_ranges) fr += r.second;
    return fr;
}

size_t dev_trim() {
    BigCache& c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    const size_t before = c.held;
    c.flush();
    return before - c.held;
}

}  // namespace pj
