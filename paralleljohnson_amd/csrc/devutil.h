// devutil.h — wave64 / block helpers shared by the kernels (gfx950: wave = 64 lanes).
#pragma once

#include <hip/hip_runtime.h>

#include "internal.h"

namespace pj {

constexpr int WAVE = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }
__device__ __forceinline__ u64 lanemask_lt() { return (1ull << lane_id()) - 1ull; }

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T x) {
    const int lane = lane_id();
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        T y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    return x;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

template <typename T>
__device__ __forceinline__ T wave_max(T x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        T y = __shfl_xor(x, off, 64);
        x = y > x ? y : x;
    }
    return x;
}

// Exclusive scan across a block of NW waves; lds must hold NW values.
template <int NW, typename T>
__device__ __forceinline__ T block_excl_scan(T x, T* lds, T& total) {
    const int lane = lane_id(), wid = wave_id();
    T incl = wave_incl_scan(x);
    if (lane == 63) lds[wid] = incl;
    __syncthreads();
    T wp = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        T v = lds[w];
        if (w < wid) wp += v;
        tot += v;
    }
    __syncthreads();
    total = tot;
    return wp + incl - x;
}

template <int NW, typename T>
__device__ __forceinline__ T block_sum(T x, T* lds) {
    T s = wave_sum(x);
    if (lane_id() == 0) lds[wave_id()] = s;
    __syncthreads();
    T tot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) tot += lds[w];
    __syncthreads();
    return tot;
}

// position of the r-th set bit (0-based) of w; r < popcount(w)
__device__ __forceinline__ u32 select_bit(u64 w, u32 r) {
    u32 base = 0;
#pragma unroll
    for (int half = 32; half >= 8; half >>= 1) {
        const u64 lo = w & ((1ull << half) - 1ull);
        const u32 c = (u32)__popcll(lo);
        if (r >= c) {
            r -= c;
            w >>= half;
            base += half;
        } else {
            w = lo;
        }
    }
    for (u32 k = 0; k < 8; ++k) {
        if ((w >> k) & 1ull) {
            if (r == 0) return base + k;
            --r;
        }
    }
    return base;
}

// Wave-aggregated append: one atomic per wave for all lanes with pred set.
// Returns this lane's slot (valid only when pred).
__device__ __forceinline__ u64 wave_append(bool pred, u64* counter) {
    const u64 m = __ballot(pred);
    u64 base = 0;
    if (m) {
        const int leader = __ffsll((long long)m) - 1;
        if (lane_id() == leader) base = atomicAdd(counter, (u64)__popcll(m));
        base = __shfl(base, leader, 64);
    }
    return base + (u64)__popcll(m & lanemask_lt());
}

}  // namespace pj
