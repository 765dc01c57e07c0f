// kron.h — the Graph500-style Kronecker tuple generator shared by the
// single-GPU builder (graph.hip) and the partitioned builder (part.hip), so
// both see exactly the same edge list. Spec in DESIGN.md; restated
// independently in oracle/pj_oracle.c (pjo_kronecker) for the tests.
#pragma once

#include "devutil.h"

namespace pj {

__device__ __forceinline__ u64 splitmix64(u64 x) {
    u64 z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

inline u64 splitmix64_h(u64 x) {
    u64 z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Label permutation: an invertible mix on [0, 2^scale).
struct PermKeys {
    u64 mask, k1, k2, c1;
    int sh;
};

inline PermKeys make_perm_keys(int scale, u64 seed) {
    PermKeys pk;
    pk.mask = scale >= 64 ? ~0ull : ((1ull << scale) - 1);
    pk.k1 = splitmix64_h(seed ^ 0x243F6A8885A308D3ull) | 1ull;
    pk.k2 = splitmix64_h(seed ^ 0x13198A2E03707344ull) | 1ull;
    pk.c1 = splitmix64_h(seed ^ 0xA4093822299F31D0ull);
    pk.sh = (scale + 1) / 2;
    return pk;
}

__device__ __forceinline__ u64 kperm(u64 x, const PermKeys& p) {
    x = (x * p.k1 + p.c1) & p.mask;
    x ^= x >> p.sh;
    x = (x * p.k2) & p.mask;
    x ^= x >> p.sh;
    x = (x * p.k1 + (p.c1 >> 7)) & p.mask;
    return x;
}

// Tuple i: (pu, pv) permuted endpoints; entries 2i = pu->pv, 2i+1 = pv->pu.
__device__ __forceinline__ void kron_tuple(int scale, u64 seed, const PermKeys& pk, u64 i, u32& pu, u32& pv) {
    const u32 TA = 2448131358u, TAB = 3264175144u, TABC = 4080218931u;  // 0.57, 0.76, 0.95 of 2^32
    u64 u = 0, v = 0;
    for (int l = 0; l < scale; ++l) {
        const u32 r = (u32)(splitmix64(seed ^ ((i << 6) | (u64)l)) >> 32);
        const u64 bu = r >= TAB;
        const u64 bv = (r >= TA && r < TAB) || r >= TABC;
        u = (u << 1) | bu;
        v = (v << 1) | bv;
    }
    pu = 0;
    pv = 0;
    if (scale > 0) {
        pu = (u32)kperm(u, pk);
        pv = (u32)kperm(v, pk);
    }
}

// Weight of tuple i (both directions): 1 + hash mod 255, or 1 when unweighted.
__device__ __forceinline__ u32 kron_weight(u64 seed, u64 i, bool weighted) {
    return weighted ? 1u + (u32)(splitmix64(seed ^ 0x5851F42D4C957F2Dull ^ i) % 255ull) : 1u;
}

}  // namespace pj
