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

// Watch of a buffered entry: the cheapest condition that must change before
// its dependency check can pass again.  A failed `dominates` leaves either a
// lane j with Local[j] < Dep[j] (recheck once Local[j] >= Dep[j]: the clock
// only grows) or Local == Dep (recheck after the next delivery, the only thing
// that changes the clock).  Entries loaded at the start of a round are
// unchecked.  A fold visits every entry in list order exactly as
// lists:foldl does; an entry whose watch still holds is not deliverable, so
// skipping its full check changes nothing but the work (it still counts as
// one dependency check).
constexpr uint32_t kWatchAny = 64;      // Local == Dep: recheck after a delivery
constexpr uint32_t kWatchNone = 65;     // not checked this round

struct Wave {
    const CsArgs* a;
    uint32_t v, lane, c, self, nb;
    uint32_t eid;                       // lane k: emitter_id(k)
    int ke;
    uint32_t* sbuf;                     // entries (k << 24 | round), list order
    uint32_t* wj;                       // watch lane / kWatchAny / kWatchNone
    uint32_t* wx;                       // watch value (clock entry or delivery count)
    // while nb <= 64 the buffer lives in registers, entry l at lane l
    uint32_t rent, rjw, rxw;
    unsigned long long pend;            // register entries whose watch no longer holds
    uint32_t inreg;                     // 1 while the buffer is in registers
    bool old_any;                       // a loaded entry is older than the clock window
    uint32_t received, delivered, checks, err;
};

// the clocks entry (k, r) is checked against, at this lane: the message's
// (ml) and its order-buffer dependency's (dl, only used when r > period)
struct Clocks { uint32_t ml, dl; };
__device__ __forceinline__ Clocks load_clocks(const Wave& w, uint32_t k, uint32_t r) {
    const CsArgs& a = *w.a;
    const uint32_t e = (uint32_t)__builtin_amdgcn_readlane((int)w.eid, (int)k);
    const uint32_t raise = w.lane == k ? w.v - (w.v > e ? 1u : 0u) + 1u : 0u;
    const uint32_t* row = a.base + k * kCsLanes + w.lane;
    Clocks q;
    q.ml = row[(r % kCsWindow) * kCsLanes * kCsLanes] + raise;
    q.dl = r > a.period ? row[((r - a.period) % kCsWindow) * kCsLanes * kCsLanes] + raise : 0u;
    return q;
}

// a wave-uniform value, moved to a scalar register (the compiler cannot
// always prove uniformity through the fold's loops)
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

// internal_receive_message/2 (:309-344) + deliver/5 (:265-300) for (k, r);
// on failure (jw, xw) is the entry's new watch
__device__ bool try_deliver(Wave& w, uint32_t r, const Clocks& q, uint32_t& jw, uint32_t& xw) {
    const CsArgs& a = *w.a;
    bool ok = true;
    if (r > a.period) {                                   // orddict:find(MyNode, IncomingOrderBuffer) -> {ok, Dep}
        const uint32_t dl = q.dl;
        w.checks = uni(w.checks + 1u);
        // dominates(Local, Dep) = descends(Local, Dep) andalso not descends(Dep, Local)
        const unsigned long long f1 = __ballot(!(dl == 0u || w.c >= dl));
        const unsigned long long f2 = __ballot(!(w.c == 0u || dl >= w.c));
        if (f1) {
            jw = uni((uint32_t)__ffsll((long long)f1) - 1u);
            xw = uni((uint32_t)__builtin_amdgcn_readlane((int)dl, (int)jw));
            ok = false;
        } else if (f2 == 0ull && w.self == 0u) {
            jw = kWatchAny;
            xw = w.delivered;
            ok = false;
        }
    }
    if (ok) {
        w.c = max(w.c, q.ml);                             // merge([LocalClock, MessageClock])
        if (w.ke >= 0) w.c += w.lane == (uint32_t)w.ke ? 1u : 0u;   // increment(MyNode, ...)
        else w.self = uni(w.self + 1u);
        w.delivered = uni(w.delivered + 1u);
    }
    return ok;
}

// the fold over one 64-entry slice (lane l holds the slice's entry l; lanes
// outside `vmask` hold none): every entry in list order, full dependency
// checks only where the watch no longer holds; returns the delivered lanes
__device__ unsigned long long fold_slice(Wave& w, uint32_t ent, uint32_t& jw, uint32_t& xw,
                                         unsigned long long vmask) {
    const bool valid = (vmask >> w.lane) & 1ull;
    unsigned long long gone = 0, seen = 0;
    uint32_t from = 0;                                    // first lane not yet visited
    for (;;) {
        const uint32_t cj = (uint32_t)__shfl((int)w.c, (int)(jw & 63u), 64);
        const bool cand = (jw == kWatchNone) | ((jw == kWatchAny) & (w.delivered > xw)) | ((jw < 64u) & (cj >= xw));
        const unsigned long long m = __ballot(valid & cand) & (~0ull << from);
        if (!m) break;
        const uint32_t l = uni((uint32_t)__ffsll((long long)m) - 1u);
        const uint32_t e = uni((uint32_t)__builtin_amdgcn_readlane((int)ent, (int)l));
        uint32_t nj = 0, nx = 0;
        seen |= 1ull << l;
        if (try_deliver(w, e & 0xFFFFFFu, load_clocks(w, e >> 24, e & 0xFFFFFFu), nj, nx)) gone |= 1ull << l;
        else {
            jw = w.lane == l ? nj : jw;
            xw = w.lane == l ? nx : xw;
        }
        if (l == 63u) break;
        from = l + 1u;
    }
    w.checks = uni(w.checks + (uint32_t)__popcll(vmask & ~seen));   // watched entries: checks that cannot pass
    return gone;
}

__device__ __forceinline__ unsigned long long first_n(uint32_t n) { return n >= 64u ? ~0ull : (1ull << n) - 1ull; }
__device__ __forceinline__ unsigned long long uni64(unsigned long long x) {
    return ((unsigned long long)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x);
}

// the register entries whose watch no longer holds (clock or delivery count moved)
__device__ __forceinline__ unsigned long long pending(const Wave& w) {
    const uint32_t cj = (uint32_t)__shfl((int)w.c, (int)(w.rjw & 63u), 64);
    const bool cand = (w.rjw == kWatchNone) | ((w.rjw == kWatchAny) & (w.delivered > w.rxw)) |
                      ((w.rjw < 64u) & (cj >= w.rxw));
    return uni64(__ballot(cand) & first_n(w.nb));
}

// the fold over the register entries: only pending entries are checked;
// the pending set is recomputed after each delivery (the only event that
// moves the clock), so a fold in which nothing is delivered costs one check
// per pending entry
__device__ void fold_reg(Wave& w) {
    const uint32_t n0 = uni(w.nb);
    if (n0 == 0u) return;
    if (uni64(w.pend) == 1ull << (n0 - 1u)) {
        // the common fold: only the entry just appended can pass (the others'
        // watches hold); it leaves from the end, so nothing moves
        const uint32_t l = n0 - 1u;
        const uint32_t e = uni((uint32_t)__builtin_amdgcn_readlane((int)w.rent, (int)l));
        uint32_t nj = 0, nx = 0;
        w.checks = uni(w.checks + l);
        if (try_deliver(w, e & 0xFFFFFFu, load_clocks(w, e >> 24, e & 0xFFFFFFu), nj, nx)) {
            w.nb = l;
            w.pend = pending(w);
        } else {
            w.rjw = w.lane == l ? nj : w.rjw;
            w.rxw = w.lane == l ? nx : w.rxw;
            w.pend = 0ull;
        }
        return;
    }
    unsigned long long gone = 0;
    uint32_t tried = 0;
    unsigned long long m = uni64(w.pend);
    while (m) {
        const uint32_t l = uni((uint32_t)__ffsll((long long)m) - 1u);
        const uint32_t e = uni((uint32_t)__builtin_amdgcn_readlane((int)w.rent, (int)l));
        uint32_t nj = 0, nx = 0;
        tried++;
        if (try_deliver(w, e & 0xFFFFFFu, load_clocks(w, e >> 24, e & 0xFFFFFFu), nj, nx)) {
            gone |= 1ull << l;
            w.pend = uni64(pending(w) & ~gone);
        } else {
            w.rjw = w.lane == l ? nj : w.rjw;
            w.rxw = w.lane == l ? nx : w.rxw;
            w.pend = uni64(w.pend & ~(1ull << l));
        }
        if (l == 63u) break;
        m = uni64(w.pend & (~0ull << (l + 1u)));
    }
    w.checks = uni(w.checks + n0 - tried);                // watched entries: checks that cannot pass
    if (!gone) return;
    const uint32_t nk = uni(n0 - (uint32_t)__popcll(gone));
    if (gone != 1ull << (n0 - 1u)) {
        // compact: kept entries to the front in order, the rest behind them
        // (a permutation of the 64 lanes, so ds_permute moves every value)
        const unsigned long long kept = first_n(n0) & ~gone, lt = (1ull << w.lane) - 1ull;
        const uint32_t o = 4u * ((kept >> w.lane) & 1ull ? (uint32_t)__popcll(kept & lt)
                                                          : nk + (uint32_t)__popcll(~kept & lt));
        w.rent = (uint32_t)__builtin_amdgcn_ds_permute((int)o, (int)w.rent);
        w.rjw = (uint32_t)__builtin_amdgcn_ds_permute((int)o, (int)w.rjw);
        w.rxw = (uint32_t)__builtin_amdgcn_ds_permute((int)o, (int)w.rxw);
        const uint32_t pb = (uint32_t)__builtin_amdgcn_ds_permute((int)o, (int)((w.pend >> w.lane) & 1ull));
        w.nb = nk;
        w.pend = uni64(__ballot(pb != 0u) & first_n(nk));
    } else {
        w.nb = nk;                                        // the last entry left: nothing moves
    }
}

// one lists:foldl over the buffer snapshot; delivered entries leave the
// buffer, the others keep their order.  An old entry is visited by every
// fold, so the window error is raised by the first fold of the round.
__device__ void fold(Wave& w) {
    if (w.old_any) w.err = uni(w.err | 2u);
    if (uni(w.inreg)) {
        fold_reg(w);
        return;
    }
    const uint32_t n0 = uni(w.nb);
    uint32_t keep = 0;
    for (uint32_t s0 = 0; s0 < n0; s0 = uni(s0 + 64u)) {
        const uint32_t i = s0 + w.lane;
        uint32_t ent = 0, jw = kWatchNone, xw = 0;
        if (i < n0) { ent = w.sbuf[i]; jw = w.wj[i]; xw = w.wx[i]; }
        const unsigned long long vmask = __ballot(i < n0);
        const unsigned long long kept = vmask & ~fold_slice(w, ent, jw, xw, vmask);
        if ((kept >> w.lane) & 1ull) {
            const uint32_t o = keep + (uint32_t)__popcll(kept & ((1ull << w.lane) - 1ull));
            w.sbuf[o] = ent;
            w.wj[o] = jw;
            w.wx[o] = xw;
        }
        keep = uni(keep + (uint32_t)__popcll(kept));
        __builtin_amdgcn_wave_barrier();
    }
    w.nb = keep;
    if (keep <= 64u) {                                    // back to registers
        w.inreg = 1u;
        w.rent = w.lane < keep ? w.sbuf[w.lane] : 0u;
        w.rjw = w.lane < keep ? w.wj[w.lane] : kWatchNone;
        w.rxw = w.lane < keep ? w.wx[w.lane] : 0u;
        w.pend = pending(w);
        __builtin_amdgcn_wave_barrier();
    }
}

// append a received entry at the end of the buffer
__device__ void append(Wave& w, uint32_t e) {
    w.nb = uni(w.nb);
    w.inreg = uni(w.inreg);
    if (w.inreg && w.nb == 64u) {                         // spill the registers
        w.sbuf[w.lane] = w.rent;
        w.wj[w.lane] = w.rjw;
        w.wx[w.lane] = w.rxw;
        w.inreg = 0u;
    }
    if (w.inreg) {
        if (w.lane == w.nb) { w.rent = e; w.rjw = kWatchNone; }
        w.pend = uni64(w.pend | (1ull << w.nb));
    } else if (w.lane == 0) {
        w.sbuf[w.nb] = e;
        w.wj[w.nb] = kWatchNone;
    }
    w.nb = uni(w.nb + 1u);
    __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(kBlock) void cs_round_kernel(CsArgs a) {
    __shared__ uint32_t sbuf[kWavesPerBlock][kCsBufCap];
    __shared__ uint32_t wj[kWavesPerBlock][kCsBufCap];
    __shared__ uint32_t wx[kWavesPerBlock][kCsBufCap];
    __shared__ unsigned long long red[kWavesPerBlock][4];
    // wave-uniform values are read into scalar registers explicitly, so the
    // fold's control flow stays scalar (no exec-mask bookkeeping)
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const uint32_t lv = blockIdx.x * kWavesPerBlock + wv;
    Wave w;
    w.received = w.delivered = w.checks = w.err = 0;
    w.nb = 0;
    if (lv < a.n) {
        w.a = &a;
        w.v = a.v_lo + lv;
        w.lane = lane;
        w.sbuf = sbuf[wv];
        w.wj = wj[wv];
        w.wx = wx[wv];
        w.c = a.clk[(size_t)lv * kCsLanes + lane];
        w.self = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.self[lv]);
        w.eid = lane < a.m ? emitter_id(lane, a.n_global, a.m) : 0xFFFFFFFFu;
        w.ke = (int)uni((uint32_t)emitter_index(w.v, a.n_global, a.m));
        w.nb = uni(a.nbuf[lv]);
        w.inreg = w.nb <= 64u ? 1u : 0u;
        w.rent = 0;
        w.rjw = kWatchNone;
        w.rxw = 0;
        w.pend = w.inreg ? first_n(w.nb) : 0ull;
        bool old = false;
        for (uint32_t i = lane; i < w.nb; i += 64) {
            const uint32_t e = a.buf[(size_t)lv * kCsBufCap + i], r0 = e & 0xFFFFFFu;
            old |= (a.t - r0 >= kCsWindow - 1) | ((r0 > a.period) & (a.t - (r0 - a.period) >= kCsWindow - 1));
            if (w.inreg) w.rent = e;
            else {
                w.sbuf[i] = e;
                w.wj[i] = kWatchNone;
            }
        }
        w.old_any = __ballot(old) != 0ull;
        __builtin_amdgcn_wave_barrier();
        // arrivals of round t: lane k marks bit d if k's round-(t-d) message lands now
        uint32_t am = 0;
        if (lane < a.m && w.eid != w.v) {
            const uint32_t ph = lane % a.period;
            for (uint32_t d = 1; d <= a.dmax && d < a.t; d++) {
                const uint32_t r = a.t - d;
                if (r % a.period == ph && delay_of(a.key, w.v, r, lane, a.dmax) == d) am |= 1u << d;
            }
        }
        // receive_message (:205-220) in (src, seq) order: emitter id, then oldest round first
        for (;;) {
            const unsigned long long any = __ballot(am != 0u);
            if (!any) break;
            const uint32_t k = uni((uint32_t)__ffsll((long long)any) - 1u);
            const uint32_t d = uni(31u - __clz((uint32_t)__builtin_amdgcn_readlane((int)am, (int)k)));
            if (lane == k) am &= ~(1u << d);
            w.received = uni(w.received + 1u);
            if (w.nb >= kCsBufCap) { w.err = uni(w.err | 1u); continue; }
            append(w, (k << 24) | (a.t - d));
            fold(w);
        }
        if (a.redeliver && a.t % a.redeliver == 0) fold(w);   // handle_info(deliver) (:233-248)
        a.clk[(size_t)lv * kCsLanes + lane] = w.c;
        if (lane == 0) {
            a.self[lv] = w.self;
            a.nbuf[lv] = w.nb;
            a.delivered[lv] += w.delivered;
        }
        if (w.inreg) {
            if (lane < w.nb) a.buf[(size_t)lv * kCsBufCap + lane] = w.rent;
        } else {
            for (uint32_t i = lane; i < w.nb; i += 64) a.buf[(size_t)lv * kCsBufCap + i] = w.sbuf[i];
        }
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
