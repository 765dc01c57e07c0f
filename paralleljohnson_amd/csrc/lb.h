// lb.h — edge-balanced ("load-balanced search") mapping of frontier edges to
// frontier slots. The frontier is a queue of vertices with out-degree >= 1
// and qoff = exclusive scan of their degrees; a workgroup takes a tile of TILE
// consecutive edges, finds the first slot with one global binary search,
// stages the <= TILE+1 slot offsets it can touch in LDS, and every lane maps
// its edge to a slot with a binary search in LDS. A hub row is thereby split
// over as many workgroups as it has tiles of edges.
#pragma once

#include "devutil.h"

namespace pj {

template <int TILE>
struct LbShared {
    u64 off[TILE + 1];
    u64 s0;
};

// Collective (whole block). After return: sh.off[0..ns) = qoff[s0..s0+ns).
template <int TILE>
__device__ __forceinline__ void lb_tile_load(const u64* __restrict__ qoff, u64 nq, u64 e0, LbShared<TILE>& sh,
                                             u64& s0, u32& ns) {
    if (threadIdx.x < WAVE) {
        // last slot with qoff[slot] <= e0, by a 64-ary search of wave 0: each step
        // probes 64 evenly spaced slots at once (one load latency per 64x
        // narrowing instead of one per halving; qoff[0] = 0 <= e0)
        const int lane = threadIdx.x;
        u64 lo = 0, hi = nq;  // answer in [lo, hi)
        while (hi - lo > 1) {
            const u64 step = (hi - lo + WAVE - 1) / WAVE;
            const u64 p = lo + (u64)lane * step;
            const bool ok = p < hi && qoff[p] <= e0;
            const u64 m = __ballot(ok);  // a prefix of the lanes (qoff ascends); lane 0 is set
            const u64 j = (u64)(63 - __clzll((long long)m));
            const u64 nlo = lo + j * step;
            hi = min(hi, nlo + step);
            lo = nlo;
        }
        if (lane == 0) sh.s0 = lo;
    }
    __syncthreads();
    s0 = sh.s0;
    ns = (u32)min(nq - s0, (u64)TILE);  // every slot holds >= 1 edge
    for (u32 i = threadIdx.x; i < ns; i += blockDim.x) sh.off[i] = qoff[s0 + i];
    __syncthreads();
}

template <int TILE>
__device__ __forceinline__ u32 lb_find(const LbShared<TILE>& sh, u32 ns, u64 e) {
    u32 lo = 0, hi = ns - 1;
    while (lo < hi) {
        const u32 mid = (lo + hi + 1) >> 1;
        if (sh.off[mid] <= e) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

}  // namespace pj
