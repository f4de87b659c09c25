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
// that changes the clock).  A watch is (ja, x): ja = 4 j, the ds_bpermute
// address of clock lane j, and the entry is rechecked once c[j] >= x; ja =
// kWatchAny rechecks once the delivery count reaches x.  An unchecked entry
// (loaded at the start of the round, or just received) has (0, 0), which
// always holds; register lanes past the buffer hold (kWatchAny, kNever),
// which never does.  A fold visits every entry in list order exactly as
// lists:foldl does; an entry whose watch is closed is not deliverable, so
// skipping its full check changes nothing but the work (it still counts as
// one dependency check).
constexpr uint32_t kWatchAny = 256u;
constexpr uint32_t kNever = 0xFFFFFFFFu;

struct Wave {
    const CsArgs* a;
    uint32_t v, lane, c, self, nb;
    uint32_t rk;                        // lane k: raise of emitter k's messages to v (rank(v) + 1)
    uint32_t inc;                       // 1 at v's own emitter lane: a delivery increments it
    uint32_t self_inc;                  // 1 when v is no emitter: a delivery increments its own entry
    uint32_t* sbuf;                     // entries (k << 24 | round), list order
    uint32_t* wj;                       // watch address
    uint32_t* wx;                       // watch threshold
    // while nb <= 64 the buffer lives in registers, entry l at lane l
    uint32_t rent, rja, rxw;
    unsigned long long pend;            // register entries whose watch is open
    uint32_t inreg;                     // 1 while the buffer is in registers
    uint32_t received, delivered, checks, err;
#ifdef CS_PROF
    uint32_t pf, pt;                    // diagnostics: fast-path arrivals, general-fold checks
#endif
};

// a wave-uniform value, moved to a scalar register (the compiler cannot
// always prove uniformity through the fold's loops)
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ unsigned long long uni64(unsigned long long x) {
    return ((unsigned long long)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x);
}
// lane l of `old` replaced by the wave-uniform x (a compare shared by the
// writes to one lane and a v_cndmask each: VALU, where the scalar unit is the
// busier one)
__device__ __forceinline__ uint32_t wlane(uint32_t x, uint32_t l, uint32_t old) {
    return (uint32_t)(threadIdx.x & 63u) == l ? x : old;
}
__device__ __forceinline__ unsigned long long first_n(uint32_t n) { return n >= 64u ? ~0ull : (1ull << n) - 1ull; }

__device__ __forceinline__ bool watch_open(const Wave& w, uint32_t ja, uint32_t x) {
    const uint32_t cj = (uint32_t)__builtin_amdgcn_ds_bpermute((int)ja, (int)w.c);
    return (ja == kWatchAny ? w.delivered : cj) >= x;
}

// the base-clock rows entry (k, r) is checked against, at this lane: the
// message's (round r) and its order-buffer dependency's (round r - period;
// only used when r > period, so an earlier round's slot is harmless)
struct Rows { uint32_t ml, dl; };
__device__ __forceinline__ Rows load_rows(const Wave& w, uint32_t e) {
    const CsArgs& a = *w.a;
    // the row offsets in vector registers: the scalar unit is the busier pipe
    // (round r's slot at (r % 64) * 4096 words, emitter k's row at k * 64)
    uint32_t ev = e;
    asm volatile("" : "+v"(ev));
    const uint32_t kk = (ev >> 18) & 0xFC0u;
    const uint32_t im = ((ev & 63u) << 12) | kk, id = (((ev - a.period) & 63u) << 12) | kk;
    Rows q;
    q.ml = a.base[im + w.lane];
    q.dl = a.base[id + w.lane];
    return q;
}

// internal_receive_message/2 (:309-344) + deliver/5 (:265-300) for entry e
// whose rows are q; on failure (ja, x) is the entry's new watch
__device__ __forceinline__ bool try_deliver(Wave& w, uint32_t e, const Rows& q, uint32_t& ja, uint32_t& x) {
    const uint32_t k = e >> 24, r = e & 0xFFFFFFu;
    const uint32_t rs = w.lane == k ? w.rk : 0u;          // lane k raised by rank(v) + 1
    if (r > w.a->period) {                                // orddict:find(MyNode, IncomingOrderBuffer) -> {ok, Dep}
        const uint32_t dl = q.dl + rs;
        w.checks++;
        // dominates(Local, Dep) = descends(Local, Dep) andalso not descends(Dep, Local)
        const unsigned long long f1 = __ballot(w.c < dl);
        if (f1) {
            const uint32_t j = (uint32_t)__builtin_ctzll(f1);
            ja = 4u * j;
            x = (uint32_t)__builtin_amdgcn_readlane((int)dl, (int)j);
            return false;
        }
        if (w.self == 0u && __ballot(dl < w.c) == 0ull) {
            ja = kWatchAny;
            x = w.delivered + 1u;
            return false;
        }
    }
    w.c = max(w.c, q.ml + rs) + w.inc;                    // merge([LocalClock, MessageClock]), increment(MyNode, ...)
    w.self += w.self_inc;
    w.delivered++;
    return true;
}


// the register entries whose watch is open
__device__ __forceinline__ unsigned long long pending(const Wave& w) {
    return uni64(__ballot(watch_open(w, w.rja, w.rxw)));
}

// receive_message + the fold it triggers when the buffer is in registers
// with room and no entry's watch is open, so that only the entry just
// received can pass (try_deliver and fold_reg's fast path for that case):
// the dependency check is branch-free, then one uniform branch on its
// outcome -- a delivery leaves lane l as it was (lanes past the buffer never
// open) and recomputes the open set, a failure appends the entry with its
// watch.  The entry's own dependency check was counted with the round's
// arrivals (Wave::checks, kernel).  Returns whether the next arrival can
// take this path too.
__device__ __forceinline__ bool arrive_fast(Wave& w, uint32_t e, const Rows& q) {
#ifdef CS_PROF
    w.pf++;
#endif
    const uint32_t l = w.nb;
    const uint32_t k = e >> 24, r = e & 0xFFFFFFu;
    const uint32_t rs = w.lane == k ? w.rk : 0u;
    const uint32_t ml = q.ml + rs, dl = q.dl + rs;
    w.checks += l;                                        // the others' watches hold: checks that cannot pass
    if (r > w.a->period) {
        // dominates(Local, Dep) fails on a lane below Dep ...
        const unsigned long long f1 = __ballot(w.c < dl);
        if (f1) {
            const uint32_t j = (uint32_t)__builtin_ctzll(f1);
            const uint32_t xj = (uint32_t)__builtin_amdgcn_readlane((int)dl, (int)j);
            const bool me = w.lane == l;
            w.rent = me ? e : w.rent;
            w.rja = me ? 4u * j : w.rja;
            w.rxw = me ? xj : w.rxw;
            w.nb = l + 1u;
            return w.nb < 64u;
        }
        // ... or on Local == Dep (no lane above it either, no own-actor entry outside the 64 lanes)
        if (w.self == 0u && __ballot(dl < w.c) == 0ull) {
            const bool me = w.lane == l;
            w.rent = me ? e : w.rent;
            w.rja = me ? kWatchAny : w.rja;
            w.rxw = me ? w.delivered + 1u : w.rxw;
            w.nb = l + 1u;
            return w.nb < 64u;
        }
    }
    w.c = max(w.c, ml) + w.inc;                           // merge + increment(MyNode)
    w.self += w.self_inc;
    w.delivered++;
    if (l == 0u) return true;
    w.pend = pending(w);
    return w.pend == 0ull;
}

// A fold's dependency check of register entry l (entry e, rows q), as
// try_deliver with nested uniform branches: deliver it (the lane is freed,
// the open set recomputed) or give it its new watch (it leaves the open set)
__device__ __forceinline__ bool try_lane(Wave& w, uint32_t l, uint32_t e, const Rows& q) {
    const uint32_t k = e >> 24, r = e & 0xFFFFFFu;
    const uint32_t rs = w.lane == k ? w.rk : 0u;
    const uint32_t dl = q.dl + rs;
    const bool me = w.lane == l;
    if (r > w.a->period) {
        w.checks++;
        const unsigned long long f1 = __ballot(w.c < dl);
        if (f1) {
            const uint32_t j = (uint32_t)__builtin_ctzll(f1);
            const uint32_t xj = (uint32_t)__builtin_amdgcn_readlane((int)dl, (int)j);
            w.rja = me ? 4u * j : w.rja;
            w.rxw = me ? xj : w.rxw;
            w.pend &= ~(1ull << l);
            return false;
        }
        if (w.self == 0u && __ballot(dl < w.c) == 0ull) {
            w.rja = me ? kWatchAny : w.rja;
            w.rxw = me ? w.delivered + 1u : w.rxw;
            w.pend &= ~(1ull << l);
            return false;
        }
    }
    w.c = max(w.c, q.ml + rs) + w.inc;
    w.self += w.self_inc;
    w.delivered++;
    w.rja = me ? kWatchAny : w.rja;
    w.rxw = me ? kNever : w.rxw;
    w.pend = pending(w);
    return true;
}

// the fold over the register entries: only open entries are checked; the
// open set is recomputed after each delivery (the only event that moves the
// clock), so a fold in which nothing is delivered costs one check per open
// entry.  (he, hq): the entry just appended and its rows, loaded ahead.
__device__ void fold_reg(Wave& w, bool hinted, uint32_t he, const Rows& hq) {
    const uint32_t n0 = uni(w.nb);
    if (n0 == 0u) return;
    const uint32_t last = n0 - 1u;
    if (w.pend == 1ull << last) {
        // the common fold: only the entry just appended can pass (the others'
        // watches hold); it leaves from the end, so nothing moves
        const uint32_t e = hinted ? he : uni((uint32_t)__builtin_amdgcn_readlane((int)w.rent, (int)last));
        const Rows q = hinted ? hq : load_rows(w, e);
        w.checks += last;
        if (try_lane(w, last, e, q)) w.nb = last;
        return;
    }
    unsigned long long gone = 0;
    uint32_t tried = 0;
    unsigned long long m = w.pend;
    while (m) {
        const uint32_t l = (uint32_t)__builtin_ctzll(m);
        const uint32_t e = uni((uint32_t)__builtin_amdgcn_readlane((int)w.rent, (int)l));
        const Rows q = hinted && l == last ? hq : load_rows(w, e);
        tried++;
#ifdef CS_PROF
        w.pt++;
#endif
        if (try_lane(w, l, e, q)) gone |= 1ull << l;
        if (l == 63u) break;
        m = w.pend & (~0ull << (l + 1u));
    }
    w.checks += n0 - tried;                               // watched entries: checks that cannot pass
    if (!gone) return;
    const uint32_t nk = n0 - (uint32_t)__popcll(gone);
    if (gone != 1ull << last) {
        // compact: kept entries to the front in order, the rest behind them
        // (a permutation of the 64 lanes, so ds_permute moves every value)
        const unsigned long long kept = first_n(n0) & ~gone, lt = (1ull << w.lane) - 1ull;
        const uint32_t o = 4u * ((kept >> w.lane) & 1ull ? (uint32_t)__popcll(kept & lt)
                                                          : nk + (uint32_t)__popcll(~kept & lt));
        w.rent = (uint32_t)__builtin_amdgcn_ds_permute((int)o, (int)w.rent);
        w.rja = (uint32_t)__builtin_amdgcn_ds_permute((int)o, (int)w.rja);
        w.rxw = (uint32_t)__builtin_amdgcn_ds_permute((int)o, (int)w.rxw);
        w.nb = nk;
        w.pend = pending(w);                              // removed lanes hold (kWatchAny, kNever)
    } else {
        w.nb = nk;                                        // the last entry left: nothing moves
    }
}

// the fold over one 64-entry slice of the LDS buffer (lane l holds the
// slice's entry l; lanes outside `vmask` hold none): every entry in list
// order, full dependency checks only where the watch is open; returns the
// delivered lanes
__device__ unsigned long long fold_slice(Wave& w, uint32_t ent, uint32_t& jw, uint32_t& xw,
                                         unsigned long long vmask) {
    const bool valid = (vmask >> w.lane) & 1ull;
    unsigned long long gone = 0, seen = 0;
    uint32_t from = 0;                                    // first lane not yet visited
    for (;;) {
        const bool open = watch_open(w, jw, xw);         // every lane takes part in the ds_bpermute
        const unsigned long long m = __ballot(valid & open) & (~0ull << from);
        if (!m) break;
        const uint32_t l = (uint32_t)__builtin_ctzll(m);
        const uint32_t e = uni((uint32_t)__builtin_amdgcn_readlane((int)ent, (int)l));
        uint32_t ja = 0, x = 0;
        seen |= 1ull << l;
        if (try_deliver(w, e, load_rows(w, e), ja, x)) gone |= 1ull << l;
        else {
            jw = wlane(ja, l, jw);
            xw = wlane(x, l, xw);
        }
        if (l == 63u) break;
        from = l + 1u;
    }
    w.checks += (uint32_t)__popcll(vmask & ~seen);       // watched entries: checks that cannot pass
    return gone;
}

// one lists:foldl over the buffer snapshot; delivered entries leave the
// buffer, the others keep their order
__device__ void fold(Wave& w, bool hinted, uint32_t he, const Rows& hq) {
    if (w.inreg) {
        fold_reg(w, hinted, he, hq);
        return;
    }
    const uint32_t n0 = w.nb;
    uint32_t keep = 0;
    for (uint32_t s0 = 0; s0 < n0; s0 += 64u) {
        const uint32_t i = s0 + w.lane;
        uint32_t ent = 0, jw = kWatchAny, xw = kNever;
        if (i < n0) { ent = w.sbuf[i]; jw = w.wj[i]; xw = w.wx[i]; }
        const unsigned long long vmask = __ballot(i < n0);
        const unsigned long long kept = vmask & ~fold_slice(w, ent, jw, xw, vmask);
        if ((kept >> w.lane) & 1ull) {
            const uint32_t o = keep + (uint32_t)__popcll(kept & ((1ull << w.lane) - 1ull));
            w.sbuf[o] = ent;
            w.wj[o] = jw;
            w.wx[o] = xw;
        }
        keep += (uint32_t)__popcll(kept);
        __builtin_amdgcn_wave_barrier();
    }
    w.nb = keep;
    if (keep <= 64u) {                                    // back to registers
        w.inreg = 1u;
        w.rent = w.lane < keep ? w.sbuf[w.lane] : 0u;
        w.rja = w.lane < keep ? w.wj[w.lane] : kWatchAny;
        w.rxw = w.lane < keep ? w.wx[w.lane] : kNever;
        w.pend = pending(w);
        __builtin_amdgcn_wave_barrier();
    }
}

// append a received entry, unchecked, at the end of the buffer
__device__ __forceinline__ void append(Wave& w, uint32_t e) {
    if (w.inreg && w.nb == 64u) {                         // spill the registers
        w.sbuf[w.lane] = w.rent;
        w.wj[w.lane] = w.rja;
        w.wx[w.lane] = w.rxw;
        w.inreg = 0u;
    }
    if (w.inreg) {
        w.rent = wlane(e, w.nb, w.rent);
        w.rja = wlane(0u, w.nb, w.rja);
        w.rxw = wlane(0u, w.nb, w.rxw);
        w.pend |= 1ull << w.nb;
    } else if (w.lane == 0) {
        w.sbuf[w.nb] = e;
        w.wj[w.nb] = 0u;
        w.wx[w.nb] = 0u;
    }
    w.nb++;
    __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(kBlock) void cs_round_kernel(CsArgs a) {
    __shared__ uint32_t sbuf[kWavesPerBlock][kCsBufCap];
    __shared__ uint32_t wj[kWavesPerBlock][kCsBufCap];
    __shared__ uint32_t wx[kWavesPerBlock][kCsBufCap];
    __shared__ uint32_t alist[kWavesPerBlock][3][64];
    __shared__ unsigned long long red[kWavesPerBlock][6];
    // wave-uniform values are read into scalar registers explicitly, so the
    // fold's control flow stays scalar (no exec-mask bookkeeping)
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const uint32_t lv = blockIdx.x * kWavesPerBlock + wv;
    Wave w;
    w.received = w.delivered = w.checks = w.err = 0;
#ifdef CS_PROF
    w.pf = w.pt = 0;
#endif
    w.nb = 0;
    if (lv < a.n) {
        w.a = &a;
        w.v = a.v_lo + lv;
        w.lane = lane;
        w.sbuf = sbuf[wv];
        w.wj = wj[wv];
        w.wx = wx[wv];
        w.c = a.clk[(size_t)lv * kCsLanes + lane];
        w.self = uni(a.self[lv]);
        const uint32_t eid = lane < a.m ? emitter_id(lane, a.n_global, a.m) : 0xFFFFFFFFu;
        const int ke = (int)uni((uint32_t)emitter_index(w.v, a.n_global, a.m));
        w.rk = w.v - (w.v > eid ? 1u : 0u) + 1u;
        w.inc = ke >= 0 && lane == (uint32_t)ke ? 1u : 0u;
        w.self_inc = ke < 0 ? 1u : 0u;
        w.nb = uni(a.nbuf[lv]);
        w.inreg = w.nb <= 64u ? 1u : 0u;
        w.rent = 0;
        w.rja = w.lane < w.nb ? 0u : kWatchAny;           // loaded entries are unchecked
        w.rxw = w.lane < w.nb ? 0u : kNever;
        w.pend = w.inreg ? first_n(w.nb) : 0ull;
        bool old = false;
        for (uint32_t i = lane; i < w.nb; i += 64) {
            const uint32_t e = a.buf[(size_t)lv * kCsBufCap + i], r0 = e & 0xFFFFFFu;
            old |= (a.t - r0 >= kCsWindow - 1) | ((r0 > a.period) & (a.t - (r0 - a.period) >= kCsWindow - 1));
            if (w.inreg) w.rent = e;
            else {
                w.sbuf[i] = e;
                w.wj[i] = 0u;
                w.wx[i] = 0u;
            }
        }
        const bool old_any = __ballot(old) != 0ull;
        __builtin_amdgcn_wave_barrier();
        // arrivals of round t: lane k marks bit d if k's round-(t-d) message lands now
        uint32_t am = 0;
        if (a.dring) {
            // the delay of k's round-(t-1) message is drawn now and kept in
            // its 4-bit slot (r % 8) until it lands: one draw per message
            uint32_t* rp = a.dring + (size_t)lv * kCsLanes + lane;
            uint32_t ring = *rp;
            if (lane < a.m && eid != w.v && a.t >= 2u) {
                const uint32_t r = a.t - 1u, sh = 4u * (r % 8u);
                const uint32_t dv = r % a.period == lane % a.period ? delay_of(a.key, w.v, r, lane, a.dmax) : 0u;
                ring = (ring & ~(0xFu << sh)) | (dv << sh);
                for (uint32_t d = 1; d <= a.dmax && d < a.t; d++)
                    if (((ring >> (4u * ((a.t - d) % 8u))) & 0xFu) == d) am |= 1u << d;
                *rp = ring;
            }
        } else if (lane < a.m && eid != w.v) {
            const uint32_t ph = lane % a.period;
            for (uint32_t d = 1; d <= a.dmax && d < a.t; d++) {
                const uint32_t r = a.t - d;
                if (r % a.period == ph && delay_of(a.key, w.v, r, lane, a.dmax) == d) am |= 1u << d;
            }
        }
        // receive_message (:205-220) in (src, seq) order: emitter id, then
        // oldest round first.  Arrival i sits at position pre(k) + (bits of
        // lane k above d); the list is staged 64 arrivals at a time.
        uint32_t pre = 0, total = 0, nchk = 0;
        for (uint32_t d = 1; d <= a.dmax; d++) {
            const unsigned long long b = __ballot((am >> d) & 1u);
            pre += __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
            total += (uint32_t)__popcll(b);
            if (a.t - d > a.period) nchk += (uint32_t)__popcll(b);   // arrivals with a dependency to check
        }
        // each arrival's own first dependency check (orddict:find ... {ok, Dep})
        // is counted here; the folds count every other check
        w.checks += nchk;
        // the staged list: entry (k << 24 | r) and the word offsets of its
        // two base rows (message round r, dependency round r - period), so
        // the per-arrival loads take scalar offsets (buffer loads, soffset)
        uint32_t* al = alist[wv][0];
        uint32_t* am_ = alist[wv][1];
        uint32_t* ad = alist[wv][2];
        auto chunk = [&](uint32_t base, uint32_t& lm, uint32_t& ld) -> uint32_t {
            for (uint32_t d = 1; d <= a.dmax; d++) {
                if ((am >> d) & 1u) {
                    const uint32_t p = pre + (uint32_t)__popc(am >> (d + 1u)) - base;
                    if (p < 64u) {
                        const uint32_t r = a.t - d;
                        al[p] = (lane << 24) | r;
                        am_[p] = 4u * (((r % kCsWindow) * kCsLanes + lane) * kCsLanes);
                        ad[p] = 4u * ((((r - a.period) % kCsWindow) * kCsLanes + lane) * kCsLanes);
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            const uint32_t x = al[lane];
            lm = am_[lane];
            ld = ad[lane];
            __builtin_amdgcn_wave_barrier();
            return x;
        };
        const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)a.base, (short)0, (int)(kCsWindow * kCsLanes * kCsLanes * 4), 0x00020000);
        const int lane4 = (int)(4u * lane);
        auto rows_at = [&](uint32_t j, uint32_t lm, uint32_t ld) {
            Rows q;
            q.ml = __builtin_amdgcn_raw_buffer_load_b32(brs, lane4, __builtin_amdgcn_readlane((int)lm, (int)j), 0);
            q.dl = __builtin_amdgcn_raw_buffer_load_b32(brs, lane4, __builtin_amdgcn_readlane((int)ld, (int)j), 0);
            return q;
        };
        bool folded = false;
        w.received = total;                               // receive_message for every arrival
        if (total) {
            uint32_t lm = 0, ld = 0;
            uint32_t lst = chunk(0, lm, ld);
            uint32_t ecur = uni((uint32_t)__builtin_amdgcn_readlane((int)lst, 0));
            Rows qcur = rows_at(0, lm, ld);
            uint32_t i = 0;
            // each step loads the next arrival's entry and rows ahead of handling the current one
            auto next = [&](uint32_t& en, Rows& qn) {
                if (i + 1u < total) {
                    const uint32_t j = (i + 1u) & 63u;
                    if (j == 0u) lst = chunk(i + 1u, lm, ld);
                    en = uni((uint32_t)__builtin_amdgcn_readlane((int)lst, (int)j));
                    qn = rows_at(j, lm, ld);
                }
            };
            while (i < total) {
                // a run of arrivals on the fast path, two per iteration so
                // that the rows loaded ahead alternate between two register
                // sets instead of being copied
                if (w.inreg && w.nb < 64u && w.pend == 0ull) {
                    uint32_t eb = 0;
                    Rows qb = qcur;
                    folded = true;
                    for (;;) {
                        eb = 0;
                        qb = qcur;
                        next(eb, qb);
                        const bool c1 = arrive_fast(w, ecur, qcur);
                        i++;
                        if (!c1 || i >= total) {
                            ecur = eb;
                            qcur = qb;
                            break;
                        }
                        ecur = 0;
                        qcur = qb;
                        next(ecur, qcur);
                        const bool c2 = arrive_fast(w, eb, qb);
                        i++;
                        if (!c2 || i >= total) break;
                    }
                }
                if (i >= total) break;
                uint32_t enext = 0;
                Rows qnext = qcur;
                next(enext, qnext);
                // the fold below counts this entry's check itself (none on overflow)
                w.checks -= (ecur & 0xFFFFFFu) > a.period ? 1u : 0u;
                if (w.nb >= a.bufcap) {
                    w.err |= 1u;
                } else {
                    append(w, ecur);
                    fold(w, true, ecur, qcur);
                    folded = true;
                }
                ecur = enext;
                qcur = qnext;
                i++;
            }
        }
        if (a.redeliver && a.t % a.redeliver == 0) {     // handle_info(deliver) (:233-248)
            fold(w, false, 0u, Rows{0u, 0u});
            folded = true;
        }
        // an old entry is visited by every fold, so the window error is
        // raised by the first fold of the round
        if (old_any && folded) w.err |= 2u;
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
#ifdef CS_PROF
        red[wv][4] = w.pf;
        red[wv][5] = w.pt;
#endif
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
#ifdef CS_PROF
    if (threadIdx.x == 4 || threadIdx.x == 5) {
        unsigned long long s = 0;
        for (uint32_t i = 0; i < kWavesPerBlock; i++) s += red[i][threadIdx.x];
        unsigned long long* st = a.stats + (blockIdx.x & (kStatShards - 1)) * kCsNStat;
        if (s) atomicAdd(&st[threadIdx.x == 4 ? 0 : 7], s);
    }
#endif
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
