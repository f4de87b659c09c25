// philox.h -- Philox4x32-10 (Random123 / rocRAND constants) for device code,
// and the simulation's draw helpers.  Each simulated process has its own
// sequential stream (seed, vertex, kind); draw j is counter {vertex, j_lo,
// kind, j_hi} under key {seed_lo, seed_hi} (DESIGN.md "RNG").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace psim {

enum RngKind : uint32_t { KIND_WORKLOAD = 1, KIND_RM = 2, KIND_AE = 3, KIND_HV = 4, KIND_SCAMP = 5, KIND_CAUSAL = 6 };

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
        k.x += 0x9E3779B9u;
        k.y += 0xBB67AE85u;
    }
    return c;
}

// Draw j (u64) of the stream of process (v, kind): Philox counter
// {v, j_lo, kind, j_hi}, the first two words (HyParView, SCAMP and Demers).
__device__ __forceinline__ uint64_t draw64(uint2 key, uint32_t v, uint32_t kind, uint64_t j) {
    const uint4 r = philox4x32_10(make_uint4(v, (uint32_t)j, kind, (uint32_t)(j >> 32)), key);
    return (uint64_t)r.x | ((uint64_t)r.y << 32);
}

// Demers select_random_sublist(lists:usort(Members), 2) over members 0..n-1
// (n >= 2), the call whose first draw is draw j of process (v, kind): the
// first two of shuffle/1 = sort of {rand:uniform(), N}.  Faithful up to
// kDmFaithfulMax members (one draw per member in list order, the two
// smallest (draw >> 11, member)); above it the same distribution -- a
// uniform ordered pair of distinct members -- from 2 draws.  The process's
// counter advances by dm_draws_per_call(n) per call (oracle/demers.c).
constexpr uint32_t kDmFaithfulMax = 1024;   // = the C restatement's DM_FAITHFUL_MAX
__host__ __device__ inline uint64_t dm_draws_per_call(uint32_t n) { return n <= kDmFaithfulMax ? n : 2u; }

__device__ __forceinline__ uint2 select2(uint2 key, uint32_t v, uint32_t kind, uint32_t n, uint64_t j) {
    if (n <= kDmFaithfulMax) {
        uint64_t k0 = ~0ull, k1 = ~0ull;
        uint32_t i0 = 0, i1 = 0;
        for (uint32_t i = 0; i < n; i++) {
            const uint64_t k = draw64(key, v, kind, j + i) >> 11;
            if (k < k0) {
                k1 = k0;
                i1 = i0;
                k0 = k;
                i0 = i;
            } else if (k < k1) {
                k1 = k;
                i1 = i;
            }
        }
        return make_uint2(i0, i1);
    }
    const uint32_t i1 = (uint32_t)__umul64hi(draw64(key, v, kind, j), (uint64_t)n);
    uint32_t i2 = (uint32_t)__umul64hi(draw64(key, v, kind, j + 1), (uint64_t)(n - 1));
    if (i2 >= i1) i2++;
    return make_uint2(i1, i2);
}

}  // namespace psim
