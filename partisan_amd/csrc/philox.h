// philox.h -- Philox4x32-10 (Random123 / rocRAND constants) for device code,
// and the simulation's draw helpers.  Streams are addressed by counter
// {vertex, event, kind, 0} under key {seed_lo, seed_hi} (DESIGN.md "RNG").
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

// select_random_sublist(lists:usort(Members), 2) over members 0..n-1: the
// first two of a uniformly random shuffle = a uniform ordered pair of
// distinct members.  Returns the pair; p.y is meaningless when n == 1.
__device__ __forceinline__ uint2 sample2(uint2 key, uint32_t v, uint32_t event, uint32_t kind, uint32_t n) {
    const uint4 r = philox4x32_10(make_uint4(v, event, kind, 0u), key);
    const uint64_t r0 = (uint64_t)r.x | ((uint64_t)r.y << 32);
    const uint64_t r1 = (uint64_t)r.z | ((uint64_t)r.w << 32);
    const uint32_t i1 = (uint32_t)__umul64hi(r0, (uint64_t)n);
    uint32_t i2 = n > 1 ? (uint32_t)__umul64hi(r1, (uint64_t)(n - 1)) : 0u;
    if (i2 >= i1) i2++;
    return make_uint2(i1, i2);
}

}  // namespace psim
