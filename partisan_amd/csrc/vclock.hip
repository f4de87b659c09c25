// vclock.hip -- partisan_vclock (src/partisan_vclock.erl:58-198) on dense
// lanes for gfx950: one wave per clock, one lane per actor (64 actors).
//
// Lane value 0 = actor absent, c + 1 = counter c.  With that encoding every
// reference predicate becomes a plain lane-wise integer operation:
//   descends(A, B)  (:63-73)  <=> for all lanes  A >= B
//       (an actor of B absent from A fails even when B's counter is 0, Q22:
//        B stores 1 there, A stores 0)
//   dominates(A, B) (:75-77)  <=> descends(A, B) and not descends(B, A)
//   merge([A, B])   (:102-129) = lane-wise max (absent < any present)
//   increment(N, A) (:140-153): lane N := max(A[N], 1) + 1
//   get_counter(N, A) (:132-137) = A[N] - 1, 0 when absent
//   equal(A, B)     (:163-164)  <=> A == B lane-wise (sorted sets)
//   glb(A, B)       (:183-198)  = lane-wise min: an actor absent from
//       either clock (0) drops out, else the smaller counter
//   subtract_dots(D, C) (:85-99): dot lane k survives iff present and
//       get_counter(k, C) < its counter, i.e. D[k] > max(C[k], 1)
// Clocks are compared as sorted sets (equal/2 sorts, Q23), which is the only
// order a dense form has.
#include "psim_internal.h"
#include "../../include/psim.h"

namespace psim {

namespace {

constexpr int kWavesPerBlock = kBlock / 64;

__global__ __launch_bounds__(kBlock) void vc_kernel(int op, const uint32_t* __restrict__ a,
                                                    const uint32_t* __restrict__ b,
                                                    const uint32_t* __restrict__ actor,
                                                    uint32_t* __restrict__ out, uint8_t* __restrict__ outb,
                                                    size_t n) {
    const size_t c = size_t(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (c >= n) return;                               // whole wave leaves together
    const size_t i = c * PSIM_VC_LANES + lane;
    const uint32_t sa = a[i];
    switch (op) {
    case 0: {  // descends
        const uint32_t sb = b[i];
        const bool d = __all(sa >= sb);
        if (lane == 0) outb[c] = d;
        break;
    }
    case 1: {  // dominates
        const uint32_t sb = b[i];
        const bool ab = __all(sa >= sb);
        const bool ba = __all(sb >= sa);
        if (lane == 0) outb[c] = ab && !ba;
        break;
    }
    case 2: {  // merge
        const uint32_t sb = b[i];
        out[i] = sa > sb ? sa : sb;
        break;
    }
    case 3: {  // increment
        const uint32_t who = actor[c];
        out[i] = lane == who ? (sa > 1u ? sa : 1u) + 1u : sa;
        break;
    }
    case 4: {  // equal
        const bool e = __all(sa == b[i]);
        if (lane == 0) outb[c] = e;
        break;
    }
    case 5: {  // glb
        const uint32_t sb = b[i];
        out[i] = sa < sb ? sa : sb;
        break;
    }
    case 6: {  // subtract_dots(A = dots, B = clock)
        const uint32_t sb = b[i];
        out[i] = sa > (sb > 1u ? sb : 1u) ? sa : 0u;
        break;
    }
    case 7: {  // get_counter: out[c] = counter of actor[c] in A (one word per clock)
        const uint32_t x = __shfl(sa, (int)actor[c], 64);
        if (lane == 0) out[c] = x ? x - 1u : 0u;
        break;
    }
    default:
        break;
    }
}

}  // namespace

hipError_t launch_vc(int op, const uint32_t* a, const uint32_t* b, const uint32_t* actor, uint32_t* out,
                     uint8_t* outb, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const size_t blocks = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL(vc_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, op, a, b, actor, out, outb, n);
    return hipGetLastError();
}

}  // namespace psim
