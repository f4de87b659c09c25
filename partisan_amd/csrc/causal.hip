// causal.hip -- causal delivery (src/partisan_causality_backend.erl) over
// dense 64-lane vector clocks, one wavefront per vertex: lane k of the
// wave holds the clock entry of emitter actor k, so descends / dominates
// are one compare + one ballot, merge is one max, increment one add.
//
// Messages are never materialised.  Emitter k's broadcast at the end of
// round r is recorded once as its clock (base[r % W][k][*]); the message to
// vertex v carries that clock with lane k raised by rank(v) + 1 (emit/4
// increments the sender's entry once per destination, :176-177), and its
// order-buffer entry is the clock of k's previous emission to v, i.e. the
// same construction at k's previous broadcast round.  Arrival rounds are a
// Philox function of (v, r, k), so every receiver enumerates its own
// arrivals.  What remains per vertex is its clock and its buffer of
// undelivered (k, r) pairs (buffered_messages, in list order).
#include "psim_internal.h"
#include "philox.h"

namespace psim {

namespace {

constexpr uint32_t kWavesPerBlock = kBlock / 64;

__device__ __forceinline__ uint32_t emitter_id(uint32_t k, uint32_t n, uint32_t m) {
    return (uint32_t)(((unsigned long long)k * n) / m);
}
// index k of the emitter whose actor is v, or -1
__device__ __forceinline__ int emitter_index(uint32_t v, uint32_t n, uint32_t m) {
    const uint32_t k = (uint32_t)(((unsigned long long)v * m + n - 1) / n);   // ceil(v m / n)
    return (k < m && emitter_id(k, n, m) == v) ? (int)k : -1;
}
// arrival delay of emitter k's round-r message to v (1..dmax)
__device__ __forceinline__ uint32_t delay_of(uint2 key, uint32_t v, uint32_t r, uint32_t k, uint32_t dmax) {
    const uint4 x = philox4x32_10(make_uint4(v, r, KIND_CAUSAL, k), key);
    return 1u + (uint32_t)__umul64hi((unsigned long long)x.x | ((unsigned long long)x.y << 32), dmax);
}

struct Wave {
    const CsArgs* a;
    uint32_t v, lane, c, self, nb;
    int ke;
    uint32_t* sbuf;
    uint32_t received, delivered, checks, err;
};

// internal_receive_message/2 (:309-344) + deliver/5 (:265-300) for (k, r)
__device__ bool try_deliver(Wave& w, uint32_t k, uint32_t r) {
    const CsArgs& a = *w.a;
    if (a.t - r >= kCsWindow - 1 || (r > a.period && a.t - (r - a.period) >= kCsWindow - 1)) w.err |= 2u;
    const uint32_t e = emitter_id(k, a.n_global, a.m);
    const uint32_t rank = w.v - (w.v > e ? 1u : 0u);
    if (r > a.period) {                                   // orddict:find(MyNode, IncomingOrderBuffer) -> {ok, Dep}
        uint32_t dl = a.base[((r - a.period) % kCsWindow) * kCsLanes * kCsLanes + k * kCsLanes + w.lane];
        if (w.lane == k) dl += rank + 1u;
        w.checks++;
        // dominates(Local, Dep) = descends(Local, Dep) andalso not descends(Dep, Local)
        const bool d1 = __ballot(!(dl == 0u || w.c >= dl)) == 0ull;
        const bool d2 = __ballot(!(w.c == 0u || dl >= w.c)) == 0ull && w.self == 0u;
        if (!(d1 && !d2)) return false;
    }
    uint32_t ml = a.base[(r % kCsWindow) * kCsLanes * kCsLanes + k * kCsLanes + w.lane];
    if (w.lane == k) ml += rank + 1u;
    w.c = max(w.c, ml);                                   // merge([LocalClock, MessageClock])
    if (w.ke >= 0) { if (w.lane == (uint32_t)w.ke) w.c += 1u; }   // increment(MyNode, ...)
    else w.self += 1u;
    w.delivered++;
    return true;
}

// one lists:foldl over the buffer snapshot; delivered entries leave the
// buffer, the others keep their order
__device__ void fold(Wave& w) {
    const uint32_t n0 = w.nb;
    uint32_t keep = 0;
    for (uint32_t i = 0; i < n0; i++) {
        const uint32_t e = w.sbuf[i];
        __builtin_amdgcn_wave_barrier();
        if (!try_deliver(w, e >> 24, e & 0xFFFFFFu)) {
            if (w.lane == 0) w.sbuf[keep] = e;
            keep++;
        }
        __builtin_amdgcn_wave_barrier();
    }
    w.nb = keep;
}

__global__ __launch_bounds__(kBlock) void cs_round_kernel(CsArgs a) {
    __shared__ uint32_t sbuf[kWavesPerBlock][kCsBufCap];
    __shared__ unsigned long long red[kWavesPerBlock][4];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t lv = blockIdx.x * kWavesPerBlock + wv;
    Wave w;
    w.received = w.delivered = w.checks = w.err = 0;
    w.nb = 0;
    if (lv < a.n) {
        w.a = &a;
        w.v = a.v_lo + lv;
        w.lane = lane;
        w.sbuf = sbuf[wv];
        w.c = a.clk[(size_t)lv * kCsLanes + lane];
        w.self = a.self[lv];
        w.ke = emitter_index(w.v, a.n_global, a.m);
        w.nb = a.nbuf[lv];
        for (uint32_t i = lane; i < w.nb; i += 64) w.sbuf[i] = a.buf[(size_t)lv * kCsBufCap + i];
        __builtin_amdgcn_wave_barrier();
        // arrivals of round t: lane k marks bit d if k's round-(t-d) message lands now
        uint32_t am = 0;
        if (lane < a.m && emitter_id(lane, a.n_global, a.m) != w.v)
            for (uint32_t d = 1; d <= a.dmax && d < a.t; d++) {
                const uint32_t r = a.t - d;
                if (r % a.period == lane % a.period && delay_of(a.key, w.v, r, lane, a.dmax) == d) am |= 1u << d;
            }
        // receive_message (:205-220) in (src, seq) order: emitter id, then oldest round first
        for (;;) {
            const unsigned long long any = __ballot(am != 0u);
            if (!any) break;
            const uint32_t k = (uint32_t)__ffsll((long long)any) - 1u;
            const uint32_t mk = __shfl(am, (int)k, 64);
            const uint32_t d = 31u - __clz(mk);
            if (lane == k) am &= ~(1u << d);
            w.received++;
            if (w.nb >= kCsBufCap) { w.err |= 1u; continue; }
            if (lane == 0) w.sbuf[w.nb] = (k << 24) | (a.t - d);
            w.nb++;
            __builtin_amdgcn_wave_barrier();
            fold(w);
        }
        if (a.redeliver && a.t % a.redeliver == 0) fold(w);   // handle_info(deliver) (:233-248)
        a.clk[(size_t)lv * kCsLanes + lane] = w.c;
        if (lane == 0) {
            a.self[lv] = w.self;
            a.nbuf[lv] = w.nb;
            a.delivered[lv] += w.delivered;
        }
        for (uint32_t i = lane; i < w.nb; i += 64) a.buf[(size_t)lv * kCsBufCap + i] = w.sbuf[i];
    }
    if (lane == 0) {
        red[wv][0] = w.received;
        red[wv][1] = w.delivered;
        red[wv][2] = w.checks;
        red[wv][3] = ((unsigned long long)w.err << 32) | w.nb;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        unsigned long long s = 0, e = 0;
        for (uint32_t i = 0; i < kWavesPerBlock; i++) {
            if (threadIdx.x == 3) { s += red[i][3] & 0xFFFFFFFFull; e |= red[i][3] >> 32; }
            else s += red[i][threadIdx.x];
        }
        unsigned long long* st = a.stats + (blockIdx.x & (kStatShards - 1)) * kCsNStat;
        if (s) atomicAdd(&st[1 + threadIdx.x], s);
        if (e) atomicOr(&st[5], e);
    }
}

// end of round t: emitters due to broadcast record their clock, then
// advance their own entry by one per destination (N - 1 emits)
__global__ void cs_broadcast_kernel(CsArgs a) {
    const uint32_t k = blockIdx.x, lane = threadIdx.x;
    if (k >= a.m || a.t % a.period != k % a.period) return;
    const uint32_t e = emitter_id(k, a.n_global, a.m);
    if (e < a.v_lo || e >= a.v_lo + a.n) return;
    uint32_t* ce = a.clk + (size_t)(e - a.v_lo) * kCsLanes;
    const uint32_t x = ce[lane];
    a.base[(a.t % kCsWindow) * kCsLanes * kCsLanes + k * kCsLanes + lane] = x;
    if (lane == k) {
        const unsigned long long nx = (unsigned long long)x + (a.n_global - 1);
        if (nx > 0xFFFFFFFFull) atomicOr(&a.stats[5], 4ull);
        ce[lane] = (uint32_t)nx;
        atomicAdd(&a.stats[6], (unsigned long long)(a.n_global - 1));
    }
}

}  // namespace

hipError_t launch_cs_round(const CsArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(cs_round_kernel, dim3((a.n + kWavesPerBlock - 1) / kWavesPerBlock), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_cs_broadcast(const CsArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(cs_broadcast_kernel, dim3(a.m), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace psim
