// plumtree.hip -- CDNA4 (gfx950) kernels for one round of Partisan's Plumtree
// (src/partisan_plumtree_broadcast.erl) with the heartbeat handler
// (src/partisan_plumtree_backend.erl) as Mod.
//
// Formulation (DESIGN.md "Plumtree kernel"):
//   * one thread per vertex, grid-stride; a vertex is visited when its inbox
//     flag is set or when the lazy tick fires and it holds outstanding rows;
//   * the inbox of v is one 32-bit word per peer slot of v: a FIFO of up to
//     four 3-bit message kinds, the reading round's tag and the 12-bit Round
//     carried by broadcast / i_have (psim_internal.h).  Each word is written
//     by exactly one sender per round, so there are no atomics on the data
//     path and the result never depends on arrival order; a consumed word is
//     left in place (its tag goes stale), so a message costs one store;
//   * slots are sorted by peer id, so walking them in order IS the schedule's
//     (src id, src emission seq) order; per-slot FIFO order is the sender's
//     emission order;
//   * outgoing words are composed after the inbox walk: for each peer slot s
//     the sender emitted, in order, the replies to s's messages and (at most
//     once per heartbeat) the eager push -- before the replies when s comes
//     after the slot that delivered the heartbeat, after them otherwise --
//     and finally the lazy-tick i_have;
//   * counters are reduced per wave with shuffles, per workgroup in LDS, and
//     added to one of 64 shards so atomics never pile onto one address.
#include "psim_internal.h"
#include <algorithm>
#include <type_traits>
#include "../../include/psim.h"

namespace psim {

namespace {

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));   // 16-byte vector for non-temporal access

__device__ __forceinline__ bool bit_alive(const uint32_t* __restrict__ alive, uint32_t v) {
    return (alive[v >> 5] >> (v & 31)) & 1u;
}

// Per-thread counters.  Message kinds are packed 12 bits each into one
// 64-bit word (a thread emits < 4096 messages per round: <= 4 candidate
// vertices x 32 slots x 4 messages) so that no counter is indexed at run
// time (that would spill the array to scratch).
struct Ctr {
    unsigned long long kinds;   // field t (t = 1..5) at bits [12(t-1), 12t): 60 bits, no field truncated
    uint32_t deliv, active, senders, degsum, ost_delta, live_delta, overflow, words;
    __device__ __forceinline__ void zero() {
        kinds = 0; deliv = active = senders = degsum = ost_delta = live_delta = overflow = words = 0;
    }
    __device__ __forceinline__ void kind(uint32_t t) { kinds += 1ull << (12 * (t - 1)); }
    __device__ __forceinline__ unsigned long long get(int i) const {
        switch (i) {
        case 1: case 2: case 3: case 4: case 5: return (kinds >> (12 * (i - 1))) & 0xFFFull;
        case S_DELIV: return deliv;
        case S_ACTIVE: return active;
        case S_SENDERS: return senders;
        case S_DEGSUM: return degsum;
        case S_OST_DELTA: return (unsigned long long)(long long)(int32_t)ost_delta;
        case S_LIVE_DELTA: return (unsigned long long)(long long)(int32_t)live_delta;
        case S_OVERFLOW: return overflow;
        case S_WORDS: return words;
        default: return 0;
        }
    }
};

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

// Reduce the per-thread counters of a workgroup and add them to a shard.
__device__ __forceinline__ void flush_counters(const Ctr& c, unsigned long long* __restrict__ stats,
                                               int* ost_total, uint32_t* msgs = nullptr, int* hold_d = nullptr) {
    __shared__ unsigned long long red[kBlock / 64][kNStat];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int i = 1; i < kNStat; i++) {
        unsigned long long x = c.get(i);
        if (i == S_OVERFLOW) {
            // OR-reduce the flag bits
            unsigned long long y = x;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) y |= __shfl_xor(y, off, 64);
            x = y;
        } else {
            x = wave_sum(x);
        }
        if (lane == 0) red[wv][i] = x;
    }
    __syncthreads();
    // shard by the workgroup's x and y index: the forest's lanes (blockIdx.y)
    // must not all add into shard 0
    const uint32_t sh = (blockIdx.x + blockIdx.y) & (kStatShards - 1);
    if (threadIdx.x < kNStat && threadIdx.x >= 1) {
        const int i = threadIdx.x;
        unsigned long long s = 0;
        if (i == S_OVERFLOW) {
            for (int w = 0; w < kBlock / 64; w++) s |= red[w][i];
            if (s) atomicOr(&stats[sh * kNStat + i], s);
        } else {
            for (int w = 0; w < kBlock / 64; w++) s += red[w][i];
            if (s) atomicAdd(&stats[sh * kNStat + i], s);
            if (s && i == S_OST_DELTA && ost_total) atomicAdd(ost_total, (int)(long long)s);
            if (s && i == S_OST_DELTA && hold_d) atomicAdd(hold_d, (int)(long long)s);   // kMcntHoldD ring
        }
    }
    if (msgs && threadIdx.x == 0) {          // this round's messages into its count shard (PtArgs::mcnt)
        unsigned long long m = 0;
        for (int k = 1; k <= 5; k++)
            for (int w = 0; w < kBlock / 64; w++) m += red[w][k];
        if (m) atomicAdd(msgs, (uint32_t)m);
    }
}

// After flush_counters (whose barrier orders the LDS counts): the
// workgroup's per-delay message counts into the round's stats row tail.
template <bool kFault>
__device__ __forceinline__ void flush_delays(const PtArgs& a);

// Append the nibble FIFO `f` to (fifo, n); count kinds (kCount).
template <bool kCount>
__device__ __forceinline__ void fifo_append(uint32_t& fifo, uint32_t& n, uint32_t f, Ctr& c) {
    while (f) {
        const uint32_t t = f & 7u;
        f >>= kKindBits;
        if (n < 4) fifo |= t << (kKindBits * n);
        else if (kCount) c.overflow |= 1u;
        n++;
        if (kCount) c.kind(t);
    }
}

// Hand the word for sender slot e to its receiver: a local receiver slot
// (rev[e] is a global slot id) plus its group flag, or -- receiver on another
// shard -- the staging word of the sender slot, packed by pt_compact_kernel.
// Omission faults (prop_partisan_crash_fault_model.erl:117-196): the word
// over sender slot e is sent (counted) and lost.
__device__ __forceinline__ bool omitted(const PtArgs& a, uint32_t e) {
    return a.omit && ((a.omit[e >> 5] >> (e & 31)) & 1u);
}

// Delay faults (psim_set_delays): the word over sender slot e goes to the
// ring slot of the round that reads it, 1 + dly[e] rounds on, tagged with
// that round; `hist` counts the messages per delay (the host keeps the
// arrivals pending, so a delayed message keeps the run from ending).
__device__ __forceinline__ uint32_t word_msgs(uint32_t w) {
    const uint32_t f = w & kFifoMask;
    return __popc((f | (f >> 1) | (f >> 2)) & 0x249u);   // non-zero 3-bit kinds
}

__device__ __forceinline__ void put_delayed(const PtArgs& a, uint32_t e, uint32_t ls, uint32_t u, uint32_t w,
                                            unsigned long long* hist) {
    const uint32_t d = a.dly[e];
    const uint32_t k = (a.rpos + d) & (kRing - 1);
    w = (w & ~(0xFFu << kTagShift)) | (((a.wtag + d) & 0xFFu) << kTagShift);
    a.ring[size_t(k) * a.ed + ls] = w;
    a.pring[size_t(k) * a.ngrp + (u >> kGroupShift)] = 1;
    atomicAdd(&hist[d], (unsigned long long)word_msgs(w));
}

// ... and, receiver on another shard, to the staging ring slot of the round
// whose exchange carries it (the round before its arrival), tagged with the
// arrival round; the receiving shard's ingest puts it in its inbox ring.
__device__ __forceinline__ void put_delayed_remote(const PtArgs& a, uint32_t e, uint32_t w, unsigned long long* hist) {
    const uint32_t d = a.dly[e];
    const uint32_t k = (a.rpos + kRing - 1u + d) & (kRing - 1);
    w = (w & ~(0xFFu << kTagShift)) | (((a.wtag + d) & 0xFFu) << kTagShift);
    a.srg[size_t(k) * a.ed + e] = w;
    atomicAdd(&hist[d], (unsigned long long)word_msgs(w));
}

// The round kernels' per-delay message counts (LDS, flushed once per workgroup).
__device__ __forceinline__ unsigned long long* delay_hist() {
    __shared__ unsigned long long dh[kRing];
    return dh;
}

// Group flag of receiver group g (mark: 0 = none, the next round reads every
// group; 1 = flag; 2 = flag + worklist).  Mode 2 claims the flag with an
// atomicOr on its 4-byte word; the sender that set it appends g to this
// workgroup's LDS list (`wl`, flushed by wl_flush) or, past its capacity or
// without one, straight to the round's worklist shard.  The flags stay
// authoritative: a reader takes the list only when it is complete.
constexpr uint32_t kWlLds = 256;
struct WlLds {
    uint32_t n;
    uint32_t g[kWlLds];
};

__device__ __forceinline__ void wl_push_global(const PtArgs& a, uint32_t g) {
    const uint32_t sh = blockIdx.x & 63u;
    const uint32_t pos = atomicAdd(&a.wlcnt[a.m_w * 64 + sh], 1u);
    if (pos < a.wl_cap) a.wl_nxt[size_t(sh) * a.wl_cap + pos] = g;
}

__device__ __forceinline__ void mark_group(const PtArgs& a, uint32_t g, uint32_t mark, WlLds* wl) {
    if (mark == 1) {
        a.pend_nxt[g] = 1;
    } else if (mark == 2) {
        const uint32_t bit = 1u << (8 * (g & 3u));
        if (atomicOr(reinterpret_cast<uint32_t*>(a.pend_nxt) + (g >> 2), bit) & bit) return;   // already listed
        const uint32_t k = wl ? atomicAdd(&wl->n, 1u) : kWlLds;
        if (k < kWlLds) wl->g[k] = g;
        else wl_push_global(a, g);
    }
}

// End of a mark-2 round in a workgroup: its LDS list into the worklist shard
// (one atomicAdd per workgroup).  Uniform call; contains barriers.
__device__ __forceinline__ void wl_flush(const PtArgs& a, WlLds* wl) {
    __shared__ uint32_t wbase;
    __syncthreads();
    const uint32_t k = min(wl->n, kWlLds), sh = blockIdx.x & 63u;
    if (threadIdx.x == 0) wbase = k ? atomicAdd(&a.wlcnt[a.m_w * 64 + sh], k) : 0u;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < k; i += kBlock)
        if (wbase + i < a.wl_cap) a.wl_nxt[size_t(sh) * a.wl_cap + wbase + i] = wl->g[i];
}

template <bool kFault = true>
__device__ __forceinline__ void deliver_word(const PtArgs& a, uint32_t e, uint32_t w,
                                             unsigned long long* hist = nullptr, uint32_t mark = 1,
                                             WlLds* wl = nullptr) {
    if (kFault && omitted(a, e)) return;
    const uint32_t u = a.col[e] - a.v_lo;
    if (u < a.n) {
        if (kFault && a.dly) {
            put_delayed(a, e, a.rev[e] - a.slot_base, u, w, hist ? hist : delay_hist());
            return;
        }
        a.in_nxt[a.rev[e] - a.slot_base] = w;
        mark_group(a, u >> kGroupShift, mark, wl);
    } else if (kFault && a.srg) {
        put_delayed_remote(a, e, w, hist ? hist : delay_hist());
    } else {
        a.stage[e] = w;
    }
}

// A vertex's Plumtree state while it handles one round (both engines).
struct VSt {
    uint32_t eager, lazy, outst, outst0, myround, rseq, ep;
    uint32_t push_mask, push_pos;   // eager_push of this round: targets, delivering slot
    int32_t live_delta;
    bool rcv;
};

// `mb`: memb[v] when the caller already loaded it (vload issues it with the
// state record), else it is read here on an epoch mismatch.
__device__ __forceinline__ void vst_load(const PtArgs& a, uint32_t v, const uint4& st, VSt& x,
                                         const uint32_t* mb = nullptr) {
    x.eager = st.x;
    x.lazy = st.y;
    x.outst = x.outst0 = st.z;
    x.myround = st.w & 0xFFFFu;
    x.rseq = (st.w >> 16) & 0xFFu;
    x.ep = st.w >> 24;
    if (x.ep != a.epoch8) {     // all_peers/3 (:1278-1282): no map entry -> common sets
        x.eager = mb ? *mb : a.memb[v];   // common_eagers = Members -- self
        x.lazy = 0;             // common_lazys = [] (start_link/0 :253-254)
        x.ep = a.epoch8;
    }
    x.rcv = x.rseq == a.mono8;
    x.push_mask = 0;
    x.push_pos = 0xFFFFFFFFu;
    x.live_delta = 0;
}

// handle_cast of the messages of one inbox word (slot s of the vertex whose
// row starts at rs); returns the FIFO of replies sent back over s.
// `peer(q)`: the peer id of slot q (global col by default; the ELL kernel
// passes the ids it already holds in registers).
template <class Peer>
__device__ __forceinline__ uint32_t pt_word(const PtArgs& a, uint32_t s, uint32_t w, VSt& x, Ctr& c, Peer peer) {
    const uint32_t b = 1u << s;
    uint32_t f = w & kFifoMask;
    const uint32_t rnd = w >> kRoundShift;
    uint32_t r = 0, rn = 0;
    while (f) {
        const uint32_t t = f & 7u;
        f >>= kKindBits;
        uint32_t reply = 0;
        switch (t) {
        case PSIM_MSG_BROADCAST:           // handle_cast :571-578
            if (!x.rcv) {                  // merge/2 -> true; handle_broadcast(true) :852-857
                x.rcv = true;
                x.rseq = a.mono8;
                x.myround = rnd + 1;
                if (x.myround > kMaxRound) { c.overflow |= 2u; x.myround = kMaxRound; }
                c.deliv++;
                x.eager |= b;              // add_eager(From, Root)
                x.lazy &= ~b;
                x.push_mask = x.eager & ~b;  // eager_push(.., Round+1, Root, From)
                x.push_pos = s;
                if (x.outst) c.overflow |= 4u;
                {                          // schedule_lazy_push(.., Round+1, Root, From)
                    uint32_t add = x.lazy & ~b & ~x.outst;
                    x.outst |= x.lazy & ~b;
                    while (add) {
                        const uint32_t q = __ffs(add) - 1;
                        add &= add - 1;
                        x.live_delta += bit_alive(a.alive, peer(q));
                    }
                }
            } else {                       // handle_broadcast(false) :843-850
                x.eager &= ~b;             // add_lazy(From, Root)
                x.lazy |= b;
                reply = PSIM_MSG_PRUNE;
            }
            break;
        case PSIM_MSG_PRUNE:               // :580-584
            x.eager &= ~b;
            x.lazy |= b;
            break;
        case PSIM_MSG_IHAVE:               // :586-590 -> handle_ihave/7 :861-876
            if (x.rcv) {
                reply = PSIM_MSG_IGNORED;
            } else {
                reply = PSIM_MSG_GRAFT;
                x.eager |= b;
                x.lazy &= ~b;
            }
            break;
        case PSIM_MSG_IGNORED:             // :592-598 ack_outstanding/5
            if (x.outst & b) {
                x.outst &= ~b;
                x.live_delta -= bit_alive(a.alive, peer(s));
            }
            break;
        case PSIM_MSG_GRAFT:               // :600-605 -> handle_graft/7 :880-906
            if (x.rcv) {                   // Mod:graft -> {ok, M}
                x.eager |= b;
                x.lazy &= ~b;
                reply = PSIM_MSG_BROADCAST;  // same Round (Q3)
            }                              // {error, not_found}: logged only
            break;
        default:
            break;
        }
        if (reply) {
            if (rn < 4) r |= reply << (kKindBits * rn);
            else c.overflow |= 1u;
            rn++;
        }
    }
    return r;
}

__device__ __forceinline__ uint32_t pt_word(const PtArgs& a, uint32_t rs, uint32_t s, uint32_t w, VSt& x, Ctr& c) {
    return pt_word(a, s, w, x, c, [&](uint32_t q) { return a.col[rs + q]; });
}

// lazy tick: send_lazy/0 (:992-1019), connected peers only, rows persist
__device__ __forceinline__ uint32_t pt_ihave(const PtArgs& a, uint32_t rs, const VSt& x) {
    uint32_t ihave = 0;
    if (a.tick && x.outst) {
        uint32_t m = x.outst;
        while (m) {
            const uint32_t q = __ffs(m) - 1;
            m &= m - 1;
            if (bit_alive(a.alive, a.col[rs + q])) ihave |= 1u << q;
        }
    }
    return ihave;
}

// The word sent over slot s this round (0 = nothing): the replies r to s's
// messages and the eager push -- before them when s comes after the slot
// that delivered the heartbeat, after them otherwise -- then the i_have.
template <bool kCount>
__device__ __forceinline__ uint32_t pt_out(uint32_t s, uint32_t r, const VSt& x, uint32_t ihave, uint32_t wtag,
                                           Ctr& c) {
    const uint32_t b = 1u << s;
    if (!r && !((x.push_mask | ihave) & b)) return 0u;
    uint32_t fifo = 0, n = 0;
    const bool p = (x.push_mask & b) != 0;
    if (p && s > x.push_pos) fifo_append<kCount>(fifo, n, PSIM_MSG_BROADCAST, c);
    fifo_append<kCount>(fifo, n, r, c);
    if (p && s < x.push_pos) fifo_append<kCount>(fifo, n, PSIM_MSG_BROADCAST, c);
    if (ihave & b) fifo_append<kCount>(fifo, n, PSIM_MSG_IHAVE, c);
    return fifo | (wtag << kTagShift) | (x.myround << kRoundShift);
}

// pt_out for replies of at most one message (every reply of a flood's
// single-message words): the FIFO assembled with selects -- push before the
// reply on slots after the delivering one, after it on slots before, then the
// i_have; at most three entries, so no overflow -- and the kinds counted in
// one add, instead of fifo_append's per-kind walk.
template <bool kCount>
__device__ __forceinline__ uint32_t pt_out1(uint32_t s, uint32_t r, const VSt& x, uint32_t ihave, uint32_t wtag,
                                            Ctr& c) {
    const uint32_t b = 1u << s;
    const bool p = (x.push_mask & b) != 0, ih = (ihave & b) != 0;
    const uint32_t k1 = p && s > x.push_pos ? (uint32_t)PSIM_MSG_BROADCAST : 0u;
    const uint32_t k3 = p && s < x.push_pos ? (uint32_t)PSIM_MSG_BROADCAST : 0u;
    const uint32_t k4 = ih ? (uint32_t)PSIM_MSG_IHAVE : 0u;
    uint32_t fifo = k1, n = k1 ? 1u : 0u;
    fifo |= r << (kKindBits * n);
    n += r ? 1u : 0u;
    fifo |= k3 << (kKindBits * n);
    n += k3 ? 1u : 0u;
    fifo |= k4 << (kKindBits * n);
    if (kCount)
        c.kinds += (p ? 1ull : 0ull) + (r ? 1ull << (12 * (r - 1u)) : 0ull) + (ih ? 1ull << 24 : 0ull);
    return (fifo | k4) ? fifo | (wtag << kTagShift) | (x.myround << kRoundShift) : 0u;
}

// Write back the state record and the outstanding flag; returns the change
// in "holds outstanding rows" (-1, 0, +1).
__device__ __forceinline__ int vst_store(const PtArgs& a, uint32_t v, const uint4& st, const VSt& x, Ctr& c) {
    const uint32_t nw = x.myround | (x.rseq << 16) | (x.ep << 24);
    if (x.eager != st.x || x.lazy != st.y || x.outst != st.z || nw != st.w) {
        u32x4_t q = {x.eager, x.lazy, x.outst, nw};
        __builtin_nontemporal_store(q, reinterpret_cast<u32x4_t*>(a.vs) + v);
    }
    c.live_delta += (uint32_t)x.live_delta;
    if ((x.outst0 != 0) != (x.outst != 0)) {
        a.ost[v] = x.outst != 0;
        c.ost_delta += x.outst != 0 ? 1u : 0xFFFFFFFFu;
        return x.outst != 0 ? 1 : -1;
    }
    return 0;
}

// Slot-scatter engine: one vertex, one round.  `rep` is this thread's LDS
// column (stride kBlock) for the reply FIFOs of its slots.  `pend`: the
// vertex's 16-vertex group was flagged (it may have words); `due`: the lazy
// tick fires and it holds outstanding rows.
// Fast path for rows of <= kFastDeg slots (every HyParView active view):
// the same clauses in the same slot order, with the row held in registers so
// that a vertex costs three dependent global round trips (row pointers ->
// inbox words -> state + neighbour ids + reverse slots), not one or two per
// slot.  The sparse and middle rounds of a flood are bound by exactly that
// chain (a workgroup holds few active vertices, each walked by one thread).
constexpr uint32_t kFastDeg = 8;

// ELL layout (a.ell = row width W <= kFastDeg, single GPU): slot s of v is
// v*W + s, so the inbox words are loaded without first reading rowp -- two
// dependent round trips per vertex instead of three; padding slots (col =
// kNoPeer) never carry a word, a mask bit or an outgoing message.
// kLdsWords: the round kernel already gathered the vertex's live inbox words
// into LDS (pt_round_ell_body) and `lw` points at them.
// kCap (>= deg): the register arrays' size.  The ELL kernel is instantiated
// per row-width class (4 / 6 / 8, and 5 for rows of exactly 5 slots without
// faults: HyParView's active view) so a row holds as few slots in registers
// as it has: fewer VGPRs (kCap 6 spilled 3 to scratch once the pair words
// joined the mask path), one slot fewer in every unrolled loop.
// Streaming loads: the inbox words a round sweeps are read once and are stale
// after it, so the sweep loads them non-temporally and they do not displace
// the lines the round scatters its own words into (2.43 -> 2.33 ms per 10M
// flood, profiles/r02/experiments/ab_nt_loads.txt).  Rows and state records
// are re-read every round: non-temporal loads of those were slower or
// neutral (profiles/r02/experiments/ab_nt_*.txt).
template <bool kNt, class T>
__device__ __forceinline__ T ld_stream(const T* p) {
    if constexpr (kNt) return __builtin_nontemporal_load(p);
    else return *p;
}
constexpr bool kNtRows = false;
constexpr bool kNtSweep = true;
constexpr bool kNtState = false;

#ifndef PSIM_W5_CONST
#define PSIM_W5_CONST 1        // A/B knob: 0 = the 5-slot kernel reads the row width at run time
#endif
#ifndef PSIM_OUT_MASKS
#define PSIM_OUT_MASKS 1       // A/B knob: 0 = the flood's output words through pt_out1 slot by slot
#endif
#ifndef PSIM_MARK1_LOOP
#define PSIM_MARK1_LOOP 1      // A/B knob: 0 = flag rounds share the run-time-mark candidate loop with list rounds
#endif
#ifndef PSIM_VLOAD_ONE_REGION
#define PSIM_VLOAD_ONE_REGION 1   // A/B knob: 0 = one predicated load per slot
#endif

template <uint32_t kCap>
struct VLoad {
    uint4 st;
    uint32_t aw;
    uint32_t cl[kCap], rv[kCap];
    bool rows;   // cl / rv were loaded
    bool has_mb; // mb = memb[v] was loaded with the rest
    uint32_t mb;
};

// `rows` false: the vertex's words hold only prunes and no row is due, so it
// sends nothing and never tests a peer's liveness -- its peer ids and
// reverse slots (2 x 4 B per slot, most of a sparse round's row bytes) are
// not loaded.
template <uint32_t kCap, bool kNtSt = kNtState>
__device__ __forceinline__ void vload(const PtArgs& a, uint32_t v, uint32_t rs, uint32_t deg, VLoad<kCap>& L,
                                      bool rows = true) {
    L.aw = a.alive[(a.v_lo + v) >> 5];
    // common_eagers, needed when the vertex has no map entry for the root (a
    // fresh tree: every vertex's first round after reset_peers): loaded with
    // the state, not after it -- one dependent round trip less per vertex
    L.mb = a.memb[v];
    L.has_mb = true;
    if constexpr (kNtSt) {
        const u32x4_t q = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(a.vs) + v);
        L.st = make_uint4(q.x, q.y, q.z, q.w);
    } else {
        L.st = a.vs[v];
    }
    L.rows = rows;
    if (a.ecol) {                // ELL packed rows: half the row bytes
        const uint32_t W = a.ell;
        uint32_t p[kCap];
        if (PSIM_VLOAD_ONE_REGION) {
            // one divergent region for the whole row (a region per slot cost
            // an exec save / restore and a branch per slot)
#pragma unroll
            for (uint32_t s = 0; s < kCap; s++) p[s] = 0u;
            if (rows) {
#pragma unroll
                for (uint32_t s = 0; s < kCap; s++) p[s] = s < deg ? ld_stream<kNtRows>(a.ecol + rs + s) : 0u;
            }
        } else {
#pragma unroll
            for (uint32_t s = 0; s < kCap; s++) p[s] = (rows && s < deg) ? ld_stream<kNtRows>(a.ecol + rs + s) : 0u;
        }
#pragma unroll
        for (uint32_t s = 0; s < kCap; s++) {
            L.cl[s] = p[s] == kNoPeer ? kNoPeer : p[s] >> 3;
            L.rv[s] = p[s] == kNoPeer ? 0u : (p[s] >> 3) * W + (p[s] & 7u);
        }
        return;
    }
#pragma unroll
    for (uint32_t s = 0; s < kCap; s++) {
        L.cl[s] = (rows && s < deg) ? a.col[rs + s] : 0u;
        L.rv[s] = (rows && s < deg) ? a.rev[rs + s] : 0u;
    }
}

// Does the FIFO of w hold a kind other than PSIM_MSG_PRUNE?  (3-bit fields:
// non-zero and != 2.)
__device__ __forceinline__ bool word_non_prune(uint32_t w) {
    const uint32_t f = w & kFifoMask, g = f ^ 0x492u;   // 0x492: PRUNE in every field
    return ((f | (f >> 1) | (f >> 2)) & (g | (g >> 1) | (g >> 2)) & 0x249u) != 0;
}

// What happens to a local receiver u after its word over slot s was stored:
// the round kernels flag its group (and list it in a sparse round).
// Mark 2 (flag + worklist) claims a flag with a RETURNING atomicOr: the
// claims of a vertex's words are all issued before any result is used, so the
// vertex waits for one atomic round trip instead of one per word (a wave's
// dependent random memory operations are what a sparse round costs).
// kMark: the round's mark when the caller resolved it at compile time (it is
// uniform over a launch: RoundMode::mark), -1 = read `mark` at run time.  A
// dense round (mark 0) then stores its words and nothing else -- no flag
// store, no branch per slot, and the flag / worklist pointers need no
// registers in the candidate loop (they were spilled to VGPR lanes and
// reloaded with v_readlane per word: VERDICT r4 #4).
template <uint32_t kCap, int kMark = -1>
struct GroupSink {
    const PtArgs& a;
    uint32_t mark;
    WlLds* wl;
    uint32_t m = 0;
    uint32_t g[kCap];
    __device__ __forceinline__ void word(uint32_t s, uint32_t u) {
        if constexpr (kMark == 0) {
            return;
        } else if constexpr (kMark == 1) {
            a.pend_nxt[u >> kGroupShift] = 1;
            return;
        } else if constexpr (kMark == -1) {
            if (mark != 2) {
                mark_group(a, u >> kGroupShift, mark, wl);
                return;
            }
        }
        g[s] = u >> kGroupShift;
        m |= 1u << s;
    }
    uint32_t old[kCap];
    // the claims of a vertex, issued together after its word stores (issuing
    // them before the stores, so their results do not wait behind the stores
    // in vmcnt, measured neutral in round 4: profiles/r04/experiments)
    __device__ __forceinline__ void issue() {
        if constexpr (kMark == 0 || kMark == 1) return;
        if (!m) return;
#pragma unroll
        for (uint32_t s = 0; s < kCap; s++)
            old[s] = ((m >> s) & 1u)
                         ? atomicOr(reinterpret_cast<uint32_t*>(a.pend_nxt) + (g[s] >> 2), 1u << (8 * (g[s] & 3u)))
                         : 0u;
    }
    __device__ __forceinline__ void done() {
        if constexpr (kMark == 0 || kMark == 1) return;
        if (!m) return;
#pragma unroll
        for (uint32_t s = 0; s < kCap; s++) {
            if (!((m >> s) & 1u) || (old[s] & (1u << (8 * (g[s] & 3u))))) continue;   // not sent / already listed
            const uint32_t k = wl ? atomicAdd(&wl->n, 1u) : kWlLds;
            if (k < kWlLds) wl->g[k] = g[s];
            else wl_push_global(a, g[s]);
        }
    }
};

// Returns the change in "holds outstanding rows" (vst_store).
// kLocal: one GPU, not sharded (no staging of remote words, v_lo = slot_base
// = 0) -- the store of a word is the store, with no receiver-range test.
template <bool kFault, uint32_t kCap, class Sink, bool kLocal = false>
__device__ __forceinline__ int pt_vertex_core(const PtArgs& a, uint32_t v, uint32_t rs, uint32_t deg,
                                              const uint32_t (&w)[kCap], const VLoad<kCap>& L, Ctr& c, Sink& sink) {
    const uint32_t aw = L.aw;
    const uint4 st = L.st;
    const uint32_t(&cl)[kCap] = L.cl;
    const uint32_t(&rv)[kCap] = L.rv;
    if (!((aw >> ((a.v_lo + v) & 31)) & 1u)) return 0;   // a dead vertex receives nothing
    c.active++;
    VSt x;
    vst_load(a, v, st, x, L.has_mb ? &L.mb : nullptr);
    auto peer = [&](uint32_t q) {                        // ids from the registers (select chain)
        uint32_t id = 0;
#pragma unroll
        for (uint32_t k = 0; k < kCap; k++) id = k == q ? cl[k] : id;
        return L.rows ? id : a.col[rs + q];
    };
    uint32_t r[kCap];
    // A flood's words carry a broadcast, a prune, or both (a sender's prune
    // reply and its eager push over the same slot, in either order): those
    // vertices take pt_word's clauses over slot masks at once, in the same
    // slot order -- prunes below the first broadcast (and a prune ahead of it
    // in its own word), its delivery (handle_broadcast(true)), then the later
    // broadcasts' prunes and the later prunes (set operations on distinct
    // slots commute; within a later slot both leave the peer lazy) -- instead
    // of a divergent per-slot FIFO walk.  Any other word: the general walk.
    constexpr uint32_t kBP = PSIM_MSG_BROADCAST | (PSIM_MSG_PRUNE << kKindBits);   // [broadcast, prune]
    constexpr uint32_t kPB = PSIM_MSG_PRUNE | (PSIM_MSG_BROADCAST << kKindBits);   // [prune, broadcast]
    uint32_t bm = 0, pm = 0, om = 0, rep = 0;        // rep: slots answering a broadcast with a prune
#pragma unroll
    for (uint32_t s = 0; s < kCap; s++) {
        const uint32_t f = w[s] & kFifoMask;
        const bool pair = f == kBP || f == kPB;
        const bool b = f == PSIM_MSG_BROADCAST || pair;
        const bool p = f == PSIM_MSG_PRUNE || pair;
        bm |= (b ? 1u : 0u) << s;
        pm |= (p ? 1u : 0u) << s;
        om |= (f != 0u && !b && !p ? 1u : 0u) << s;
    }
    if (om == 0u) {
        if (!x.rcv && bm) {
            const uint32_t s0 = (uint32_t)__ffs(bm) - 1u, b0 = 1u << s0;
            uint32_t w0 = 0;
#pragma unroll
            for (uint32_t k = 0; k < kCap; k++) w0 = k == s0 ? w[k] : w0;
            // the delivering word's own prune counts as earlier when it came first
            const uint32_t pre = (pm & (b0 - 1u)) | ((w0 & kFifoMask) == kPB ? b0 : 0u);
            x.eager &= ~pre;
            x.lazy |= pre;
            x.rcv = true;                                // merge/2 -> true; handle_broadcast(true) :852-857
            x.rseq = a.mono8;
            x.myround = (w0 >> kRoundShift) + 1u;
            if (x.myround > kMaxRound) { c.overflow |= 2u; x.myround = kMaxRound; }
            c.deliv++;
            x.eager |= b0;                               // add_eager(From, Root)
            x.lazy &= ~b0;
            x.push_mask = x.eager & ~b0;                 // eager_push(.., Round+1, Root, From)
            x.push_pos = s0;
            if (x.outst) c.overflow |= 4u;
            uint32_t add = x.lazy & ~b0 & ~x.outst;      // schedule_lazy_push(.., Round+1, Root, From)
            x.outst |= x.lazy & ~b0;
            while (add) {
                const uint32_t q = __ffs(add) - 1;
                add &= add - 1;
                x.live_delta += bit_alive(a.alive, peer(q));
            }
            const uint32_t later = (bm & ~b0) | (pm & ~pre);
            x.eager &= ~later;                           // add_lazy(From, Root) / prune
            x.lazy |= later;
            rep = bm & ~b0;
        } else {
            x.eager &= ~(bm | pm);
            x.lazy |= bm | pm;
            rep = x.rcv ? bm : 0u;                       // handle_broadcast(false) :843-850
        }
#pragma unroll
        for (uint32_t s = 0; s < kCap; s++) r[s] = ((rep >> s) & 1u) ? PSIM_MSG_PRUNE : 0u;
    } else
    {
#pragma unroll
        for (uint32_t s = 0; s < kCap; s++) r[s] = w[s] ? pt_word(a, s, w[s], x, c, peer) : 0u;
    }
    uint32_t ihave = 0;                                  // pt_ihave over the registers
    if (a.tick && x.outst) {
        // rows held but not due cannot happen (ost mirrors them); still, never test id 0's liveness
#pragma unroll
        for (uint32_t s = 0; s < kCap; s++)
            if ((x.outst >> s) & 1u)
                ihave |= (bit_alive(a.alive, L.rows ? cl[s] : a.col[rs + s]) ? 1u : 0u) << s;
    }
    bool sent = false;
    uint32_t wo[kCap];
    uint32_t nstored = 0;
    if (PSIM_OUT_MASKS && om == 0u) {
        // The flood's words (every reply a prune): each slot's FIFO from the
        // push / reply / i_have masks -- [push, prune] after the delivering
        // slot, [prune, push] before it, then the i_have -- and the kinds
        // counted once per vertex by popcount instead of per slot (pt_out1).
        const uint32_t dm = deg >= 32u ? ~0u : (1u << deg) - 1u;
        const uint32_t pu = x.push_mask & dm, re = rep & dm, ih = ihave & dm;
        const uint32_t hi = x.push_pos >= 31u ? 0u : ~0u << (x.push_pos + 1u);   // slots after the delivering one
        const uint32_t hdr = (x.myround << kRoundShift) | (a.wtag << kTagShift);
#pragma unroll
        for (uint32_t s = 0; s < kCap; s++) {
            const uint32_t b = 1u << s;
            const bool p = (pu & b) != 0u, r1 = (re & b) != 0u, i1 = (ih & b) != 0u;
            const uint32_t n = (p ? 1u : 0u) + (r1 ? 1u : 0u);
            const uint32_t first = p && (!r1 || (hi & b)) ? (uint32_t)PSIM_MSG_BROADCAST
                                 : r1 ? (uint32_t)PSIM_MSG_PRUNE : 0u;
            const uint32_t second = p && r1 ? ((hi & b) ? (uint32_t)PSIM_MSG_PRUNE : (uint32_t)PSIM_MSG_BROADCAST) : 0u;
            const uint32_t fifo = first | (second << kKindBits) | (i1 ? (uint32_t)PSIM_MSG_IHAVE << (kKindBits * n) : 0u);
            wo[s] = fifo ? fifo | hdr : 0u;
            sent |= fifo != 0u;
            if (kFault && wo[s] && omitted(a, rs + s)) wo[s] = 0u;   // sent (counted) and lost
            nstored += wo[s] != 0u ? 1u : 0u;
        }
        c.kinds += (unsigned long long)__popc(pu) + ((unsigned long long)__popc(re) << 12) +
                   ((unsigned long long)__popc(ih) << 24);
    } else {
#pragma unroll
        for (uint32_t s = 0; s < kCap; s++) {
            wo[s] = s >= deg ? 0u : r[s] < 8u ? pt_out1<true>(s, r[s], x, ihave, a.wtag, c)
                                               : pt_out<true>(s, r[s], x, ihave, a.wtag, c);
            sent |= wo[s] != 0u;
            if (kFault && wo[s] && omitted(a, rs + s)) wo[s] = 0u;   // sent (counted) and lost
            nstored += wo[s] != 0u ? 1u : 0u;
        }
    }
    c.words += nstored;
    if constexpr (kLocal && !kFault) {
#pragma unroll
        for (uint32_t s = 0; s < kCap; s++) {
            if (!wo[s]) continue;
            a.in_nxt[rv[s]] = wo[s];
            sink.word(s, cl[s]);
        }
    } else
#pragma unroll
    for (uint32_t s = 0; s < kCap; s++) {
        if (!wo[s]) continue;
        const uint32_t u = cl[s] - a.v_lo;
        if (kFault && a.dly && u < a.n) {
            put_delayed(a, rs + s, rv[s] - a.slot_base, u, wo[s], delay_hist());
        } else if (u < a.n) {
            a.in_nxt[rv[s] - a.slot_base] = wo[s];
            sink.word(s, u);
        } else if (kFault && a.srg) {
            put_delayed_remote(a, rs + s, wo[s], delay_hist());
        } else {
            a.stage[rs + s] = wo[s];
        }
    }
    sink.issue();
    sink.done();
    if (sent) {
        c.senders++;
        uint32_t d = deg;
        if (a.ell) {                                     // true degree: the non-padding slots
            d = 0;
#pragma unroll
            for (uint32_t s = 0; s < kCap; s++) d += (s < deg && cl[s] != kNoPeer) ? 1u : 0u;
        }
        c.degsum += d;
    }
    return vst_store(a, v, st, x, c);
}

template <bool kFault, uint32_t kCap, int kMark = -1, bool kLocal = false>
__device__ __forceinline__ void pt_vertex_core(const PtArgs& a, uint32_t v, uint32_t rs, uint32_t deg,
                                               const uint32_t (&w)[kCap], const VLoad<kCap>& L, Ctr& c, uint32_t mark,
                                               WlLds* wl) {
    GroupSink<kCap, kMark> sink{a, mark, wl};
    (void)pt_vertex_core<kFault, kCap, GroupSink<kCap, kMark>, kLocal>(a, v, rs, deg, w, L, c, sink);
}

template <bool kFault, bool kLdsWords = false, uint32_t kCap = kFastDeg, int kMark = -1, bool kLocal = false>
__device__ __forceinline__ void pt_vertex_fast(const PtArgs& a, uint32_t v, uint32_t rs, uint32_t deg, bool pend,
                                               bool due, Ctr& c, const uint32_t* lw = nullptr, uint32_t mark = 1,
                                               WlLds* wl = nullptr) {
    uint32_t w[kCap];
    uint32_t any = 0;
    bool rows = due;
#pragma unroll
    for (uint32_t s = 0; s < kCap; s++) {
        if (kLdsWords) {
            w[s] = (pend && s < deg) ? lw[s] : 0u;
        } else {
            w[s] = (pend && s < deg) ? a.in_cur[rs + s] : 0u;
            if (!live_word(w[s], a.ctag)) w[s] = 0u;   // stale: consumed in an earlier round
        }
        any |= w[s];
        rows |= word_non_prune(w[s]);
    }
    pend = any != 0;
    if (!pend && !due) return;
    VLoad<kCap> L;
    vload(a, v, rs, deg, L, rows);
    pt_vertex_core<kFault, kCap, kMark, kLocal>(a, v, rs, deg, w, L, c, mark, wl);
}

template <bool kFault>
__device__ __forceinline__ void flush_delays(const PtArgs& a) {
    if (!kFault || !a.dly) return;
    const uint32_t t = threadIdx.x;
    if (t < kRing) {
        const unsigned long long x = delay_hist()[t];
        if (x) atomicAdd(&a.dhist[t], x);
    }
}

template <bool kFault>
__device__ __forceinline__ void pt_vertex(const PtArgs& a, uint32_t v, bool pend, bool due, uint16_t* rep,
                                          Ctr& c, uint32_t mark) {
    if (a.ell) {
        pt_vertex_fast<kFault>(a, v, v * a.ell, a.ell, pend, due, c, nullptr, mark);
        return;
    }
    const uint32_t rs = a.rowp[v];
    const uint32_t deg = a.rowp[v + 1] - rs;
    if (deg <= kFastDeg) {
        pt_vertex_fast<kFault>(a, v, rs, deg, pend, due, c, nullptr, mark);
        return;
    }
    if (pend) {
        bool any = false;
        for (uint32_t s = 0; s < deg; s++) any |= live_word(a.in_cur[rs + s], a.ctag);
        pend = any;
    }
    if (!pend && !due) return;
    if (!bit_alive(a.alive, a.v_lo + v)) return;   // a dead vertex receives nothing: its words go stale
    c.active++;
    const uint4 st = a.vs[v];
    VSt x;
    vst_load(a, v, st, x);
    if (pend) {
        for (uint32_t s = 0; s < deg; s++) {
            const uint32_t w = a.in_cur[rs + s];
            uint32_t r = 0;
            if (live_word(w, a.ctag)) r = pt_word(a, rs, s, w, x, c);
            rep[s * kBlock] = (uint16_t)r;
        }
    }
    const uint32_t ihave = pt_ihave(a, rs, x);
    bool sent = false;
    for (uint32_t s = 0; s < deg; s++) {
        const uint32_t w = pt_out<true>(s, pend ? rep[s * kBlock] : 0u, x, ihave, a.wtag, c);
        if (!w) continue;
        deliver_word<kFault>(a, rs + s, w, nullptr, mark);
        c.words += (kFault && omitted(a, rs + s)) ? 0u : 1u;
        sent = true;
    }
    if (sent) {
        c.senders++;
        c.degsum += deg;
    }
    vst_store(a, v, st, x, c);
}

// A workgroup owns kChunkV consecutive vertices.  Each thread looks at 4 of
// them: their group flag (set by any sender to the group) and, on a tick
// round while some vertex holds outstanding rows, their outstanding byte.
// Candidates are compacted into an LDS list and spread over the threads.
// The counts of the last two rounds (PtArgs::mcnt): wave 0 sums the 64
// shards; block 0 zeroes the slot of the round after next.  Returns false
// when the round is a no-op (nothing was sent, no row is due).
struct RoundMode {
    uint32_t mark;   // this round's senders: 0 = no group flags, 1 = flags, 2 = flags + worklist
    bool all_in;     // the last round wrote no flags: every group is read
    bool list_in;    // the last round's worklist is complete: read its groups, not the flags
    bool rows_due;   // the lazy tick fires and some vertex held rows when the round started
};

// This round's change in row holders (kMcntHoldD ring slot m_w), or null without counts.
__device__ __forceinline__ int* hold_delta(const PtArgs& a) {
    return a.mcnt ? reinterpret_cast<int*>(a.mcnt + kMcntHoldD + a.m_w) : nullptr;
}

// wl_off (ELL kernel): [65] prefix of the worklist shards this round reads.
// Every decision below is taken from values written by EARLIER launches, so
// all workgroups of this launch agree: the running holder count
// (*ost_total) moves while the launch runs, and a workgroup that read it
// after another had flushed used to pick the flags while the others read the
// list -- a listed vertex that gained rows this round was then visited again
// as "due" and sent a second i_have (the 1M world-2 mismatch of round 2).
// The group-flag mode of round R's senders from the counts of rounds R-1
// (prev) and R-2 (prev2) -- round_counts and the sharded ingest of R's remote
// words take it from the same numbers.  PSIM_FF_GROWING 1 would keep a round
// after the peak (prev < prev2: a 10M flood's round 14, 2.45M words after
// 19.3M) flagging, so that the round after it reads the flagged groups
// instead of sweeping the whole inbox (round 15: 613k receivers): measured a
// loss (the flag stores cost round 14 more than round 15 saves).
#ifndef PSIM_FF_GROWING
#define PSIM_FF_GROWING 0      // A/B knob: 1 = flag-free only while the count grows (measured: round 14 +15-20 us
                               // of flag stores, round 15 -3..-8 us; profiles/r06/experiments/ab_group_shift.txt)
#endif
__device__ __forceinline__ uint32_t round_mark(const PtArgs& a, uint32_t prev, uint32_t prev2) {
    if (prev >= a.dense && (prev >= prev2 || !PSIM_FF_GROWING)) return a.force_flags ? 1u : 0u;
    return (a.wl_nxt && prev < a.wl_thr) ? 2u : 1u;
}

__device__ __forceinline__ bool round_counts(const PtArgs& a, RoundMode& m, uint32_t* wl_off = nullptr) {
    __shared__ uint32_t cnt2[6];
    m.mark = 1;
    m.all_in = m.list_in = false;
    if (!a.mcnt) {
        // no counts: flag mode only, every workgroup reads its own chunks'
        // row bytes, which no other workgroup writes -- a stale total is harmless
        m.rows_due = a.tick && *a.ost_total > 0;
        return true;
    }
    const uint32_t t = threadIdx.x;
    if (t == 0) {                                         // holders at the start of this round
        const int hold = int(a.mcnt[kMcntHold + a.m_r]) + int(a.mcnt[kMcntHoldD + a.m_s]);
        cnt2[3] = uint32_t(hold);
        // an abandoned pipelined interval (PtArgs::spec), loaded with the counts
        cnt2[4] = a.spec ? a.spec[0] : 0u;
        cnt2[5] = a.mcnt[kMcntFF + a.m_s];               // the last round wrote no group flags
    }
    if (t < 64) {
        uint32_t c1 = a.mcnt[a.m_s * 64 + t], c2 = a.mcnt[a.m_r * 64 + t];
        uint32_t l = a.wl_cur ? a.wlcnt[a.m_s * 64 + t] : 0u;
        const bool ovf = __ballot(l > a.wl_cap) != 0ull;   // a shard overflowed: the flags are read
        l = min(l, a.wl_cap);
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(l, off, 64);
            if (t >= (uint32_t)off) l += y;
        }
        if (wl_off) {
            wl_off[t + 1] = l;
            if (t == 0) wl_off[0] = 0;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            c1 += __shfl_xor(c1, off, 64);
            c2 += __shfl_xor(c2, off, 64);
        }
        if (t == 0) { cnt2[0] = c1; cnt2[1] = c2; cnt2[2] = ovf; }
    }
    __syncthreads();
    // nothing of an abandoned interval runs, not even the rings' upkeep below
    if (cnt2[4]) return false;
    const uint32_t prev = cnt2[0], prev2 = cnt2[1];
    const uint32_t mark = round_mark(a, prev, prev2);
    if (blockIdx.x == 0) {        // (no workgroup of this launch reads these slots)
        if (t == 0) {
            a.mcnt[kMcntHold + a.m_s] = cnt2[3];          // = holders at the end of round R-1
            a.mcnt[kMcntHoldD + a.m_z] = 0u;              // the round after next adds into it
            a.mcnt[kMcntFF + a.m_w] = mark == 0u ? 1u : 0u;   // a no-op round sends nothing: 0
        }
        if (t < 64) {                                     // the round after next starts empty
            a.mcnt[a.m_z * 64 + t] = 0;
            if (a.wl_cur) a.wlcnt[a.m_z * 64 + t] = 0;
        }
    }
    const bool rows_due = a.tick && int(cnt2[3]) > 0;
    m.rows_due = rows_due;
    // nothing was sent last round and no row is due: every vertex is idle
    // (no inbox flag can be set), so the whole round is a no-op
    if (prev == 0 && !rows_due) return false;
    // many senders expected (and the flood still growing): no group flags this round; few: flags + worklist
    m.mark = mark;
    m.all_in = cnt2[5] != 0u;                          // the last round wrote none: every group is read
    // the last round's senders listed every group they flagged (the same
    // test on the same count) and no row is due: only the listed groups
    m.list_in = wl_off && a.wl_cur && prev2 < a.dense && prev2 < a.wl_thr && !cnt2[2] && !rows_due;
    return true;
}

// kFault: omission faults installed (psim_set_omissions); the common case
// compiles without the per-word bitmap test.
template <bool kFault>
__device__ __forceinline__ void pt_round_body(const PtArgs& a) {
    __shared__ uint16_t rep[kMaxDeg * kBlock];
    __shared__ uint16_t cand[kChunkV];           // (vertex - base) << 2 | pend << 1 | due: 12 bits
    static_assert(kChunkV == 4 * kBlock && (kChunkV << 2) <= 65536, "candidate encoding");
    __shared__ uint32_t ncand;
    const uint32_t t = threadIdx.x;
    RoundMode md;
    if (!round_counts(a, md)) return;
    const bool all_in = md.all_in;
    const uint32_t base = blockIdx.x * kChunkV;
    if (t == 0) ncand = 0;
    if (kFault && a.dly && t < kRing) delay_hist()[t] = 0;
    __syncthreads();
    const uint32_t v0 = base + 4 * t;
    uint32_t pmask = 0, dmask = 0;
    if (v0 < a.n) {
        const uint32_t g = v0 >> kGroupShift;
        const bool lead = (t & ((1u << (kGroupShift - 2)) - 1)) == 0;   // threads of a group share the byte
        if (all_in) {
            // flags a forced-flag round left (PtArgs::force_flags) are cleared too, or a
            // later worklist round would find the claim bit set and not list the group
            pmask = 0xFu;
            if (lead) a.pend_cur[g] = 0;
        } else if (a.pend_cur[g]) {
            pmask = 0xFu;
            if (lead) a.pend_cur[g] = 0;
        }
        if (md.rows_due) {
            uint32_t w;
            if (v0 + 4 <= a.n) w = *reinterpret_cast<const uint32_t*>(a.ost + v0);
            else { w = 0; for (uint32_t i = 0; v0 + i < a.n; i++) w |= uint32_t(a.ost[v0 + i]) << (8 * i); }
            for (int i = 0; i < 4; i++) dmask |= ((w >> (8 * i)) & 0xFFu) ? (1u << i) : 0u;
        }
        if (v0 + 4 > a.n) {
            const uint32_t valid = (1u << (a.n - v0)) - 1u;
            pmask &= valid;
            dmask &= valid;
        }
    }
    const uint32_t m = pmask | dmask;
    if (m) {
        const uint32_t off = atomicAdd(&ncand, (uint32_t)__popc(m));
        uint32_t k = off;
        for (int i = 0; i < 4; i++)
            if (m & (1u << i)) cand[k++] = (uint16_t)(((4 * t + i) << 2) | (((pmask >> i) & 1u) << 1) | ((dmask >> i) & 1u));
    }
    __syncthreads();
    const uint32_t nc = ncand;
    if (nc == 0) return;                          // uniform: idle chunk
    Ctr c;
    c.zero();
    for (uint32_t i = t; i < nc; i += kBlock) {
        const uint32_t x = cand[i];
        pt_vertex<kFault>(a, base + (x >> 2), (x >> 1) & 1u, x & 1u, &rep[t], c, md.mark);
    }
    flush_counters(c, a.stats, a.ost_total, a.mcnt ? a.mcnt + a.m_w * 64 + (blockIdx.x & 63) : nullptr,
                   hold_delta(a));
    flush_delays<kFault>(a);
}

template <bool kFault>
__global__ __launch_bounds__(kBlock) void pt_round_kernel(PtArgs a) {
    pt_round_body<kFault>(a);
}

// ELL rows (a.ell = W): the workgroup first reads the inbox words of every
// flagged 16-vertex group of its chunk with ALL its threads -- consecutive
// words, one coalesced sweep (a group's words are 16 W consecutive words) --
// keeps the live ones in LDS and marks the vertices that have any; only those
// (and, on a tick round, the vertices holding outstanding rows) are handed to
// threads, which then need one round trip (state, peer ids, reverse slots)
// instead of a per-vertex dependent load of words that are mostly stale
// (a flagged group typically has one or two receivers in the sparse rounds).
// kEllChunk vertices per workgroup (kVpt per thread): the words buffer is
// kEllChunk * W * 4 bytes of LDS, which is what bounds workgroups per CU.
constexpr uint32_t kEllChunk = 1024;   // 512 / 256 / 2048 measured slower
constexpr uint32_t kVpt = kEllChunk / kBlock;
static_assert(kVpt >= 1 && kVpt <= 8 && kEllChunk % 32 == 0 && (kEllChunk << 2) <= 65536,
              "ELL chunk: 1-8 vertices per thread, candidates fit 16 bits");

// A chunk whose flagged groups are at least kFullQuarters / 4 of its groups
// is read whole (the contiguous sweep below): the unflagged groups' words are
// stale (a live word always has its group flagged), so reading them is only
// bandwidth.  A/B knob PSIM_FULL_QUARTERS (4 = only chunks with every group
// flagged).
#ifndef PSIM_FULL_QUARTERS
#define PSIM_FULL_QUARTERS 4
#endif
constexpr uint32_t kFullQuarters = PSIM_FULL_QUARTERS;

// x / W for x < 2^13 and 1 <= W <= 8: x * ceil(2^18 / W) >> 18 (the rounding
// error stays below 2^13 / 2^18 of one, under the 1/8 a fraction of x/W
// leaves to the next integer)
__device__ __forceinline__ uint32_t div_w(uint32_t x, uint32_t wmag) { return (x * wmag) >> 18; }

// Diagnostic build (-DPSIM_PHASE_PROF=1, tools/phase_probe.py): workgroup 0
// of every ELL round launch clocks its phases on the 100 MHz real-time
// counter -- entry, counts read, first chunk's group list, sweep, candidates,
// candidate loop, all chunks, counters flushed -- into g_phase[launch][8].
#ifndef PSIM_PHASE_PROF
#define PSIM_PHASE_PROF 0
#endif
#if PSIM_PHASE_PROF
constexpr uint32_t kPhaseRecs = 4096;
__device__ unsigned long long g_phase[kPhaseRecs][8];
__device__ uint32_t g_phase_n;
struct PhaseClock {
    unsigned long long t[8] = {};
    bool on;
    __device__ PhaseClock() : on(blockIdx.x == 0 && threadIdx.x == 0) {}
    __device__ __forceinline__ void mark(int i) { if (on) t[i] = (unsigned long long)wall_clock64(); }
    __device__ __forceinline__ void flush() {
        if (!on) return;
        const uint32_t k = g_phase_n;
        if (k < kPhaseRecs)
            for (int i = 0; i < 8; i++) g_phase[k][i] = t[i];
        g_phase_n = k + 1u;
        on = false;
    }
};
#else
struct PhaseClock {
    __device__ __forceinline__ void mark(int) {}
    __device__ __forceinline__ void flush() {}
};
#endif

template <bool kFault, uint32_t kCap, bool kLocal = false>
__device__ __forceinline__ void pt_round_ell_body(const PtArgs& a) {
    static_assert(kEllChunk * kEllMax <= (1u << 13), "div_w is exact below 2^13");
    PhaseClock ph;
    ph.mark(0);
    extern __shared__ __attribute__((aligned(16))) uint32_t wbuf[];   // [kEllChunk * W] the live words of the groups read
    __shared__ uint32_t actm[kEllChunk / 32];          // vertices with live words
    __shared__ uint32_t duem[kEllChunk / 32];          // vertices holding outstanding rows on a tick round
    __shared__ uint16_t cand[kEllChunk];
    __shared__ uint8_t glist[kEllChunk >> kGroupShift];   // flag mode: chunk-local groups to read
    __shared__ uint32_t gl[kEllChunk >> kGroupShift];     // list mode: global groups to read
    __shared__ uint32_t wl_off[65];
    __shared__ WlLds wl;
    __shared__ uint32_t ncand, ngrp;
    constexpr uint32_t kGroups = kEllChunk >> kGroupShift, kGV = 1u << kGroupShift;
    const uint32_t t = threadIdx.x;
    RoundMode md;
    if (!round_counts(a, md, wl_off)) {
        ph.flush();
        return;
    }
    ph.mark(1);
    // the 5-slot instantiation runs rows of exactly 5 slots (launch_pt_round):
    // a compile-time row width folds every per-slot "s < deg" test, the row
    // offsets v * W and the sweep's division
    const uint32_t W = (kCap == 5 && PSIM_W5_CONST) ? 5u : a.ell;
    const bool list = md.list_in;
    // The grid is the chip's resident workgroups (PtArgs::ell_grid), each
    // looping over chunks c = blockIdx.x, + gridDim.x, ...: a chunk is 1024
    // consecutive vertices, or in list mode (sparse rounds) entries [64 c,
    // 64 c + 64) of the groups the last round listed -- so a sparse round
    // costs one dispatch of the resident grid, not of n / 1024 workgroups
    // whose LDS must be allocated before each can find it has nothing to do.
    // list mode: the listed groups are spread over the resident workgroups (gpc groups per chunk,
    // PtArgs::wl_gpc or total / min(grid, wl_wgs)): a chunk of 64 groups loaded one CU with ~64
    // receivers' random loads per dependent step, and one CU sustains only ~0.45 G random loads/s
    // (tools/mb_latency.hip); spread over all 1,280, a round of 1-20k groups paid every busy
    // workgroup's fixed costs (counts, claims, counter flushes) -- 256 measured best
    const uint32_t total = wl_off[64];
    const uint32_t lwg = a.wl_wgs ? min(a.wl_wgs, gridDim.x) : gridDim.x;
    const uint32_t gpc = !list ? kGroups
                       : a.wl_gpc ? min(a.wl_gpc, kGroups)
                                  : max(1u, min(kGroups, (total + lwg - 1) / lwg));
    const uint32_t nchunks = list ? (total + gpc - 1) / gpc : (a.n + kEllChunk - 1) / kEllChunk;
    if (blockIdx.x >= nchunks) {                       // uniform
        ph.flush();
        return;
    }
    if (t == 0) wl.n = 0;
    if (kFault && a.dly && t < kRing) delay_hist()[t] = 0;
    Ctr c;
    c.zero();
    const uint32_t nW = a.n * W;                       // words that exist
    const uint32_t gw = kGV * W;
    // x / W by one multiply (a runtime divide is a ~20-instruction sequence,
    // and the sweep divided once per quad and once per live word)
    const uint32_t wmag = ((1u << 18) + W - 1u) / W;
    for (uint32_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
        const uint32_t base = ch * kEllChunk;
        const uint32_t nv = list ? 0u : min(kEllChunk, a.n - base);
        if (t < kEllChunk / 32) {
            actm[t] = 0;
            duem[t] = 0;
        }
        if (t == 0) ncand = ngrp = 0;
        __syncthreads();
        if (list) {
            const uint32_t idx = ch * gpc + t;
            if (t < gpc && idx < total) {
                uint32_t lo = 0, hi = 64;              // shard: wl_off[lo] <= idx < wl_off[lo + 1]
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (wl_off[mid] <= idx) lo = mid; else hi = mid;
                }
                const uint32_t g = a.wl_cur[size_t(lo) * a.wl_cap + (idx - wl_off[lo])];
                gl[t] = g;
                a.pend_cur[g] = 0;
            }
            if (t == 0) ngrp = min(gpc, total - ch * gpc);
        } else {
            if (t < kGroups && t * kGV < nv) {
                const uint32_t g = (base >> kGroupShift) + t;
                if (md.all_in) {
                    a.pend_cur[g] = 0;                 // a forced-flag round's flags (see pt_round_body)
                    glist[atomicAdd(&ngrp, 1u)] = (uint8_t)t;
                } else if (a.pend_cur[g]) {
                    a.pend_cur[g] = 0;
                    glist[atomicAdd(&ngrp, 1u)] = (uint8_t)t;
                }
            }
            if (md.rows_due && kVpt * t < nv) {
                const uint32_t v0 = base + kVpt * t;
                uint32_t d = 0;
                for (uint32_t i = 0; i < kVpt; i++)
                    if (v0 + i < a.n && a.ost[v0 + i]) d |= 1u << i;
                if (d) atomicOr(&duem[(kVpt * t) >> 5], d << ((kVpt * t) & 31));
            }
        }
        __syncthreads();
        if (ch == blockIdx.x) ph.mark(2);
        const uint32_t ng = ngrp;
        // group slot i of this chunk: LDS words at pos(i) * gw, first vertex gv(i)
        auto pos = [&](uint32_t i) -> uint32_t { return list ? i : uint32_t(glist[i]); };
        auto gv = [&](uint32_t i) -> uint32_t {
            return list ? gl[i] << kGroupShift : base + (uint32_t(glist[i]) << kGroupShift);
        };
        auto keep = [&](uint32_t lwi, uint32_t w) {      // LDS word = group slot vertex * W + slot
            if (!live_word(w, a.ctag)) w = 0u;
            wbuf[lwi] = w;
            if (w) {
                const uint32_t lv = div_w(lwi, wmag);
                atomicOr(&actm[lv >> 5], 1u << (lv & 31));
            }
        };
        // A chunk whose 64 groups are all read (every dense round: all_in, or
        // every flag set) holds its words contiguously, in LDS as in HBM: the
        // sweep is a straight copy of kEllChunk W words, quad k of the chunk to
        // LDS quad k, and which vertices hold live words is read back from LDS
        // by the candidate pass -- no per-word group lookup, division or LDS
        // atomic (the general sweep below spends ~100 VALU per quad on those).
        const bool full = !list && ng * 4u >= kGroups * kFullQuarters && nv == kEllChunk &&
                          (reinterpret_cast<uintptr_t>(a.in_cur) & 15u) == 0;   // uniform
        if (full) {
            constexpr uint32_t kSweepF = (kEllChunk * kCap / 4 + kBlock - 1) / kBlock;   // W <= kCap
            const u32x4_t* src = reinterpret_cast<const u32x4_t*>(a.in_cur + size_t(base) * W);
            static_assert(kEllChunk == 4 * kBlock, "quad k * kBlock + t exists iff k < W");
            u32x4_t wv[kSweepF];
#pragma unroll
            for (uint32_t k = 0; k < kSweepF; k++) {     // k < W: uniform
                const u32x4_t z = {0u, 0u, 0u, 0u};
                wv[k] = k < W ? ld_stream<kNtSweep>(src + k * kBlock + t) : z;
            }
#pragma unroll
            for (uint32_t k = 0; k < kSweepF; k++) {
                const uint32_t q = k * kBlock + t;
                if (k >= W) continue;
                u32x4_t x = wv[k];
                x.x = live_word(x.x, a.ctag) ? x.x : 0u;
                x.y = live_word(x.y, a.ctag) ? x.y : 0u;
                x.z = live_word(x.z, a.ctag) ? x.z : 0u;
                x.w = live_word(x.w, a.ctag) ? x.w : 0u;
                reinterpret_cast<u32x4_t*>(wbuf)[q] = x;
            }
        } else if ((reinterpret_cast<uintptr_t>(a.in_cur) & 15u) == 0) {   // group g's words start at 4 kGV W g bytes
            // A group's kGV W words (kGV >= 4) start on a 16-byte boundary: read them as
            // quads, kSweepU quads per thread in flight before any is used (the
            // word-at-a-time loop waited out one load latency per word).
            constexpr uint32_t kSweepU = 8;   // a dense round's 5 quads per thread all in flight at once
            const uint32_t gq = gw >> 2, nq = ng * gq;
            for (uint32_t q0 = 0; q0 < nq; q0 += kBlock * kSweepU) {
                uint4 wv[kSweepU];
                uint32_t li[kSweepU], gi[kSweepU];
#pragma unroll
                for (uint32_t k = 0; k < kSweepU; k++) {
                    const uint32_t q = q0 + k * kBlock + t;
                    // group slot i = q / gq, gq = kGV W / 4 quads: (4 q / kGV) / W
                    const uint32_t i = div_w((q << 2) >> kGroupShift, wmag), r = (q - i * gq) * 4u;
                    li[k] = q < nq ? pos(i) * gw + r : 0xFFFFFFFFu;
                    gi[k] = q < nq ? gv(i) * W + r : nW;
                    if (gi[k] + 4 <= nW) {
                        const u32x4_t q = ld_stream<kNtSweep>(reinterpret_cast<const u32x4_t*>(a.in_cur + gi[k]));
                        wv[k] = make_uint4(q.x, q.y, q.z, q.w);
                    } else {
                        wv[k] = make_uint4(0, 0, 0, 0);
                    }
                }
#pragma unroll
                for (uint32_t k = 0; k < kSweepU; k++) {
                    if (gi[k] >= nW) continue;
                    if (gi[k] + 4 <= nW) {
                        keep(li[k], wv[k].x);
                        keep(li[k] + 1, wv[k].y);
                        keep(li[k] + 2, wv[k].z);
                        keep(li[k] + 3, wv[k].w);
                    } else {
                        for (uint32_t j = 0; gi[k] + j < nW; j++) keep(li[k] + j, a.in_cur[gi[k] + j]);   // the tail
                    }
                }
            }
        } else
        {
            for (uint32_t q = t; q < ng * gw; q += kBlock) {
                const uint32_t i = q / gw, r = q % gw;
                if (gv(i) * W + r < nW) keep(pos(i) * gw + r, a.in_cur[gv(i) * W + r]);
            }
        }
        __syncthreads();
        if (ch == blockIdx.x) ph.mark(3);
        {
            constexpr uint32_t kMask = (1u << kVpt) - 1u;
            const uint32_t v4 = kVpt * t;
            uint32_t am = (actm[v4 >> 5] >> (v4 & 31)) & kMask;
            if (full) {                                  // live words read back from LDS
                am = 0;
#pragma unroll
                for (uint32_t i = 0; i < kVpt; i++) {
                    uint32_t o = 0;
#pragma unroll
                    for (uint32_t s = 0; s < kCap; s++)
                        if (s < W) o |= wbuf[(v4 + i) * W + s];
                    am |= (o != 0u ? 1u : 0u) << i;
                }
            }
            const uint32_t dm = (duem[v4 >> 5] >> (v4 & 31)) & kMask;
            const uint32_t m = am | dm;
            if (m) {
                uint32_t k = atomicAdd(&ncand, (uint32_t)__popc(m));
                for (uint32_t i = 0; i < kVpt; i++)
                    if (m & (1u << i))
                        cand[k++] = (uint16_t)(((v4 + i) << 2) | (((am >> i) & 1u) << 1) | ((dm >> i) & 1u));
            }
        }
        __syncthreads();
        if (ch == blockIdx.x) ph.mark(4);
        const uint32_t nc = ncand;
        // the round's mark is uniform over the launch: the dense rounds' (mark 0,
        // no flags) get a candidate loop of their own
        auto cand_loop = [&](auto mk) {
            constexpr int M = decltype(mk)::value;
            for (uint32_t i = t; i < nc; i += kBlock) {
                const uint32_t x = cand[i], lv = x >> 2;
                const uint32_t v = list ? (gl[lv >> kGroupShift] << kGroupShift) + (lv & (kGV - 1u)) : base + lv;
                pt_vertex_fast<kFault, true, kCap, M, kLocal && M == 0>(a, v, v * W, W, (x >> 1) & 1u, x & 1u, c,
                                                                        &wbuf[lv * W], md.mark, &wl);
            }
        };
        const uint32_t mark = __builtin_amdgcn_readfirstlane(md.mark);
        if (mark == 0) cand_loop(std::integral_constant<int, 0>{});
#if PSIM_MARK1_LOOP
        else if (mark == 1) cand_loop(std::integral_constant<int, 1>{});   // flags only: no claims, no list
#endif
        else cand_loop(std::integral_constant<int, -1>{});
        __syncthreads();                               // LDS (cand, wbuf, gl) is reused by the next chunk
        if (ch == blockIdx.x) ph.mark(5);
    }
    ph.mark(6);
    if (md.mark == 2) wl_flush(a, &wl);
    flush_counters(c, a.stats, a.ost_total, a.mcnt ? a.mcnt + a.m_w * 64 + (blockIdx.x & 63) : nullptr,
                   hold_delta(a));
    flush_delays<kFault>(a);
    ph.mark(7);
    ph.flush();
}

template <bool kFault, uint32_t kCap, bool kLocal>
// At least 5 waves per SIMD (<= 96 VGPRs): the LDS holds 5-6 workgroups per
// CU at W = 5-6, and the contiguous sweep's quads in flight would otherwise
// take the kernel to 99 VGPRs, 4 waves (no spills at 96).
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(5))) void pt_round_ell_kernel(PtArgs a) {
    pt_round_ell_body<kFault, kCap, kLocal>(a);
}

// Multi-root rounds: one launch runs the round of every
// non-quiescent heartbeat lane, blockIdx.y = lane, each lane's arguments in
// device memory -- the lanes' sparse rounds share the chip instead of
// following each other launch by launch.
template <bool kFault>
__global__ __launch_bounds__(kBlock) void pt_round_lanes_kernel(const PtArgs* __restrict__ args) {
    pt_round_body<kFault>(args[blockIdx.y]);
}

template <bool kFault, uint32_t kCap, bool kLocal>
__global__ __launch_bounds__(kBlock) void pt_round_ell_lanes_kernel(const PtArgs* __restrict__ args) {
    pt_round_ell_body<kFault, kCap, kLocal>(args[blockIdx.y]);
}

// ---------------------------------------------------------------------------
// The forest (FoArgs, psim_internal.h): lane L's arguments
// are lane 0's shifted by L slices -- built in registers from one kernel
// argument block, so a round over 10^4 roots uploads nothing per lane.
__device__ __forceinline__ uint32_t fo_slot(const FoArgs& f, uint32_t lane) { return f.slot ? f.slot[lane] : lane; }

__device__ __forceinline__ PtArgs fo_lane(const FoArgs& f, uint32_t lane) {
    PtArgs a = f.a;
    const uint32_t sl = fo_slot(f, lane);               // the lane's root's records (parked roots: FoArgs::slot)
    a.vs += sl * f.s_vs;
    a.in_cur += lane * f.s_in;
    a.in_nxt += lane * f.s_in;
    a.pend_cur += lane * f.s_pend;
    a.pend_nxt += lane * f.s_pend;
    a.ost += lane * f.s_ost;
    a.ost_total += 4 * lane;
    if (a.mcnt) {
        a.mcnt += size_t(lane) * kMcntLane;
        if (a.wlcnt) a.wlcnt = a.mcnt + 256;
    }
    if (a.stage) a.stage += lane * f.s_stage;           // sharded forest: the lane's staged remote words
    if (a.dly) {                                         // delay faults: the lane's inbox ring (s_in / s_pend
        a.ring += lane * f.s_in;                         // are the ring strides then, forest_args)
        a.pring += lane * f.s_pend;
    }
    if (a.wl_cur) a.wl_cur = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(a.wl_cur) + lane * f.s_pend);
    if (a.wl_nxt) a.wl_nxt = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(a.wl_nxt) + lane * f.s_pend);
    const uint2 li = f.info[sl];
    a.mono8 = li.x;
    a.root = li.y;
    return a;
}

template <bool kFault, uint32_t kCap, bool kLocal>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(5))) void pt_forest_ell_kernel(FoArgs f) {
    pt_round_ell_body<kFault, kCap, kLocal>(fo_lane(f, f.lane0 + blockIdx.y));   // kLocal: one GPU
}

template <bool kFault>
__global__ __launch_bounds__(kBlock) void pt_forest_kernel(FoArgs f) {
    pt_round_body<kFault>(fo_lane(f, f.lane0 + blockIdx.y));
}

// ---------------------------------------------------------------------------
// Binned engine (single GPU).  A round is two launches:
//   pb_route_kernel: the records emitted last round sit in coarse receiver
//     bins (2^cv_shift vertices); each workgroup moves <= kRouteK of one
//     coarse bin's records into its fine bins (2^fv_shift vertices) --
//     an LDS histogram, one atomicAdd per fine bin, contiguous runs out;
//   pb_round_kernel: a workgroup owns one fine bin: it drops the bin's
//     records into an LDS copy of the bin's receiver slots (the same words
//     the slot-scatter engine keeps in HBM), runs every vertex of the bin
//     through the shared handlers, and appends its outgoing words as
//     {receiver slot, word} records to the coarse bins of the next round
//     (histogram, one atomicAdd per coarse bin, contiguous runs).
// Each bin region is the bin's receiver-slot range, which bounds its record
// count (a receiver slot has one sender and gets <= 1 word per round), so no
// region can overflow.  Random 4-byte scatters into HBM become appends of
// 8-byte records in runs plus LDS scatters.
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(kBlock) void pb_route_kernel(PtArgs a) {
    __shared__ uint32_t fsb[kCoarseMax + 1];
    __shared__ uint32_t hist[kCoarseMax];
    __shared__ uint32_t base[kCoarseMax];
    constexpr uint32_t kPer = kRouteK / kBlock;
    const uint32_t t = threadIdx.x;
    const uint32_t G = 1u << (a.cv_shift - a.fv_shift);
    const uint32_t total = a.nc * kCoarseShards * a.chunks;
    for (uint32_t blk = blockIdx.x; blk < total; blk += gridDim.x) {
        const uint32_t cs = blk / a.chunks, j = blk - cs * a.chunks;
        const uint32_t c = cs / kCoarseShards;
        const uint32_t nrec = a.cnt_c_cur[cs];
        const uint32_t lo = j * kRouteK;
        if (lo >= nrec) continue;                     // uniform
        const uint32_t hi = min(nrec, lo + kRouteK);
        const uint32_t f0 = c * G;
        const uint32_t ng = min(G, a.nf - f0);
        for (uint32_t g = t; g <= ng; g += kBlock) fsb[g] = a.fslot[f0 + g];
        for (uint32_t g = t; g < ng; g += kBlock) hist[g] = 0;
        const uint32_t cb = a.csub[cs];
        uint2 r[kPer];
#pragma unroll
        for (uint32_t q = 0; q < kPer; q++) {
            const uint32_t i = lo + t + q * kBlock;
            if (i < hi) r[q] = a.rec_c[cb + i];
        }
        __syncthreads();
        uint32_t fb[kPer];
#pragma unroll
        for (uint32_t q = 0; q < kPer; q++) {
            const uint32_t i = lo + t + q * kBlock;
            fb[q] = 0xFFFFFFFFu;
            if (i < hi) {
                uint32_t l = 0, h = ng;               // fsb[l] <= slot < fsb[h]
                while (h - l > 1) {
                    const uint32_t m = (l + h) >> 1;
                    if (fsb[m] <= r[q].x) l = m; else h = m;
                }
                fb[q] = l;
                atomicAdd(&hist[l], 1u);
            }
        }
        __syncthreads();
        for (uint32_t g = t; g < ng; g += kBlock) {
            const uint32_t k = hist[g];
            if (k) base[g] = fsb[g] + atomicAdd(&a.cnt_f[f0 + g], k);
            hist[g] = 0;
        }
        __syncthreads();
        bool bad = false;
#pragma unroll
        for (uint32_t q = 0; q < kPer; q++)
            if (fb[q] != 0xFFFFFFFFu) {
                const uint32_t pos = base[fb[q]] + atomicAdd(&hist[fb[q]], 1u);
                if (pos < fsb[fb[q] + 1]) a.rec_f[pos] = r[q];   // a region holds its slots' words
                else bad = true;
            }
        if (bad) atomicOr(&a.stats[S_OVERFLOW], 8ull);
        __syncthreads();                              // LDS reuse by the next chunk
    }
}

__global__ __launch_bounds__(kBlock) void pb_round_kernel(PtArgs a) {
    constexpr uint32_t kVPer = kBinVMax / kBlock;
    __shared__ uint32_t words[kBinSlots];            // the bin's receiver slots, then the replies
    __shared__ uint32_t rpc[kBinVMax + 1];           // row starts of the bin's vertices
    __shared__ uint16_t cand[kBinVMax];              // bin-local vertex | 0x8000 = has words
    __shared__ uint32_t hist[kCoarseMax];
    __shared__ uint32_t base[kCoarseMax];
    __shared__ uint32_t ncand;
    __shared__ int obd;
    const uint32_t t = threadIdx.x;
    // the coarse counts route read this round are free for the round after next
    for (uint32_t i = blockIdx.x * kBlock + t; i < a.nc * kCoarseShards; i += gridDim.x * kBlock)
        a.cnt_c_cur[i] = 0;
    Ctr c;
    c.zero();
    bool any_bin = false;
    for (uint32_t f = blockIdx.x; f < a.nf; f += gridDim.x) {
        uint32_t nrec = a.cnt_f[f];
        const bool due = a.tick && a.obin[f] != 0;
        if (nrec == 0 && !due) continue;              // uniform: idle bin
        any_bin = true;
        const uint32_t v0 = f << a.fv_shift;
        const uint32_t nv = min(1u << a.fv_shift, a.n - v0);
        const uint32_t sb = a.fslot[f], ns = a.fslot[f + 1] - sb;
        for (uint32_t i = t; i <= nv; i += kBlock) rpc[i] = a.rowp[v0 + i] - sb;
        for (uint32_t i = t; i < ns; i += kBlock) words[i] = 0;
        for (uint32_t i = t; i < a.nc; i += kBlock) hist[i] = 0;
        if (t == 0) { obd = 0; ncand = 0; }
        if (nrec > ns) {                              // cannot happen: one word per receiver slot
            nrec = ns;
            c.overflow |= 8u;
        }
        uint2 rr[4];
#pragma unroll
        for (uint32_t q = 0; q < 4; q++)              // the first records are in flight during the zeroing
            if (t + q * kBlock < nrec) rr[q] = a.rec_f[sb + t + q * kBlock];
        __syncthreads();
        if (t == 0 && nrec) a.cnt_f[f] = 0;           // consumed (route of the next round adds again)
#pragma unroll
        for (uint32_t q = 0; q < 4; q++)
            if (t + q * kBlock < nrec) words[rr[q].x - sb] = rr[q].y;
        for (uint32_t i = t + 4 * kBlock; i < nrec; i += kBlock) {
            const uint2 r = a.rec_f[sb + i];
            words[r.x - sb] = r.y;
        }
        __syncthreads();
        // candidates: vertices with words, and (tick) vertices holding rows
#pragma unroll
        for (uint32_t k = 0; k < kVPer; k++) {
            const uint32_t lv = t + k * kBlock;
            if (lv >= nv) continue;
            uint32_t any = 0;
            for (uint32_t i = rpc[lv]; i < rpc[lv + 1]; i++) any |= words[i];
            if (any || (due && a.ost[v0 + lv]))
                cand[atomicAdd(&ncand, 1u)] = (uint16_t)(lv | (any ? 0x8000u : 0u));
        }
        __syncthreads();
        const uint32_t nk = ncand;
        // handle: replies are written over the words
        VSt x[kVPer];
        uint32_t ihave[kVPer], lvk[kVPer];
        bool send[kVPer];
        int od = 0;
#pragma unroll
        for (uint32_t k = 0; k < kVPer; k++) {
            send[k] = false;
            ihave[k] = 0;
            lvk[k] = 0;
            const uint32_t i = t + k * kBlock;
            if (i >= nk) continue;
            const uint32_t cv = cand[i];
            const uint32_t lv = cv & 0x7FFFu;
            const bool pend = (cv & 0x8000u) != 0;
            const uint32_t v = v0 + lv;
            lvk[k] = lv;
            if (!bit_alive(a.alive, v)) continue;     // a dead vertex drops its words
            c.active++;
            const uint32_t ls = rpc[lv], deg = rpc[lv + 1] - ls, rs = sb + ls;
            const uint4 st = a.vs[v];
            vst_load(a, v, st, x[k]);
            if (pend)
                for (uint32_t s = 0; s < deg; s++) {
                    const uint32_t w = words[ls + s];
                    if (w) words[ls + s] = pt_word(a, rs, s, w, x[k], c);
                }
            ihave[k] = pt_ihave(a, rs, x[k]);
            od += vst_store(a, v, st, x[k], c);
            send[k] = true;
        }
        if (od) atomicAdd(&obd, od);
        // emit, pass 1: records per coarse bin of the next round
#pragma unroll
        for (uint32_t k = 0; k < kVPer; k++) {
            if (!send[k]) continue;
            const uint32_t ls = rpc[lvk[k]], deg = rpc[lvk[k] + 1] - ls, rs = sb + ls;
            for (uint32_t s = 0; s < deg; s++)
                if (pt_out<false>(s, words[ls + s], x[k], ihave[k], a.wtag, c) && !omitted(a, rs + s))
                    atomicAdd(&hist[a.col[rs + s] >> a.cv_shift], 1u);
        }
        __syncthreads();
        const uint32_t sh = f & (kCoarseShards - 1);     // this bin's sub-region of every coarse bin
        for (uint32_t i = t; i < a.nc; i += kBlock) {
            const uint32_t k = hist[i];
            if (k) base[i] = a.csub[i * kCoarseShards + sh] + atomicAdd(&a.cnt_c_nxt[i * kCoarseShards + sh], k);
            hist[i] = 0;
        }
        if (t == 0 && obd) a.obin[f] += (uint32_t)obd;
        __syncthreads();
        // pass 2: the records
#pragma unroll
        for (uint32_t k = 0; k < kVPer; k++) {
            if (!send[k]) continue;
            const uint32_t ls = rpc[lvk[k]], deg = rpc[lvk[k] + 1] - ls, rs = sb + ls;
            bool sent = false;
            for (uint32_t s = 0; s < deg; s++) {
                const uint32_t w = pt_out<true>(s, words[ls + s], x[k], ihave[k], a.wtag, c);
                if (!w) continue;
                sent = true;
                if (omitted(a, rs + s)) continue;
                const uint32_t cb = a.col[rs + s] >> a.cv_shift;
                const uint32_t pos = base[cb] + atomicAdd(&hist[cb], 1u);
                if (pos < a.csub[cb * kCoarseShards + sh + 1]) a.rec_c[pos] = make_uint2(a.rev[rs + s], w);
                else c.overflow |= 8u;
                c.words++;                            // one record per word
            }
            if (sent) {
                c.senders++;
                c.degsum += deg;
            }
        }
        __syncthreads();                              // LDS reuse by the next bin
    }
    if (__syncthreads_or(any_bin)) flush_counters(c, a.stats, a.ost_total);
}

// The origin's {broadcast, Id, Payload, Mod} cast (:565-569): eager_push/4
// and schedule_lazy_push/3 with Round 0, Root = From = the origin; the
// backend already did add_timestamp (backend :341-368).
__device__ __forceinline__ void pt_origin_body(const PtArgs& a) {
    const uint32_t v = a.root;   // local index of the origin (only its owner launches this)
    PtArgs ao = a;               // listed groups count as the round the next round reads as previous
    ao.m_w = a.m_s;
    const uint32_t rs = a.ell ? v * a.ell : a.rowp[v];
    const uint32_t deg = a.ell ? a.ell : a.rowp[v + 1] - rs;   // ELL padding: no mask bits
    const uint4 st = a.vs[v];
    uint32_t eager = st.x, lazy = st.y, outst = st.z;
    uint32_t ep = st.w >> 24;
    if (ep != a.epoch8) { eager = a.memb[v]; lazy = 0; ep = a.epoch8; }
    unsigned long long add_live = 0, flags = 0;
    if (outst) flags |= 4u;
    const uint32_t outst0 = outst;
    uint32_t nmsg = 0, nword = 0;
    for (uint32_t s = 0; s < deg; s++) {
        const uint32_t b = 1u << s;
        const uint32_t e = rs + s;
        if (eager & b) {
            nword += omitted(a, e) ? 0u : 1u;
            if (omitted(a, e)) {
                // sent and lost
            } else if (a.rec_c) {                    // binned: a record for the next route
                const uint32_t cs = (a.col[e] >> a.cv_shift) * kCoarseShards + ((v >> a.fv_shift) & (kCoarseShards - 1));
                a.rec_c[a.csub[cs] + atomicAdd(&a.cnt_c_nxt[cs], 1u)] =
                    make_uint2(a.rev[e], PSIM_MSG_BROADCAST | (a.wtag << kTagShift));
            } else {
                deliver_word(ao, e, PSIM_MSG_BROADCAST | (a.wtag << kTagShift), a.dhist,  // Round 0
                             a.wl_nxt ? 2u : 1u);
            }
            nmsg++;
        }
        if ((lazy & b) && !(outst & b)) {
            outst |= b;
            add_live += bit_alive(a.alive, a.col[e]);
        }
    }
    a.vs[v] = make_uint4(eager, lazy, outst, 0u | (a.mono8 << 16) | (ep << 24));
    if ((outst0 != 0) != (outst != 0)) {
        a.ost[v] = 1;
        if (a.obin) a.obin[v >> a.fv_shift] += 1u;
        atomicAdd(&a.stats[S_OST_DELTA], 1ull);
        atomicAdd(a.ost_total, 1);
        if (int* d = hold_delta(ao)) atomicAdd(d, 1);   // a change of the round before the next one
    }
    if (add_live) atomicAdd(&a.stats[S_LIVE_DELTA], add_live);
    if (nmsg) atomicAdd(&a.stats[PSIM_MSG_BROADCAST], (unsigned long long)nmsg);
    if (nword) atomicAdd(&a.stats[S_WORDS], (unsigned long long)nword);
    if (nmsg && a.mcnt) atomicAdd(&a.mcnt[a.m_s * 64], nmsg);   // read by the next round
    if (flags) atomicOr(&a.stats[S_OVERFLOW], flags);
}

// One root's origin by the 64 lanes of a wave, lane s on peer slot s (rows of
// <= 64 slots: every row, kMaxDeg = 32): its pushes are issued together, where
// pt_origin_body walks the slots one after another (a store, a flag claim and
// a list push per slot, each waiting on the last: ~14 us of the step).  The
// same counts and state as pt_origin_body; worklist and bin record order
// differ, which no consumer reads.
__device__ __forceinline__ void pt_origin_wave(const PtArgs& a) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t v = a.root;
    PtArgs ao = a;
    ao.m_w = a.m_s;
    const uint32_t rs = a.ell ? v * a.ell : a.rowp[v];
    const uint32_t deg = a.ell ? a.ell : a.rowp[v + 1] - rs;
    const uint4 st = a.vs[v];
    uint32_t eager = st.x, lazy = st.y, outst = st.z;
    uint32_t ep = st.w >> 24;
    if (ep != a.epoch8) { eager = a.memb[v]; lazy = 0; ep = a.epoch8; }
    const uint32_t outst0 = outst;
    const uint32_t b = lane < 32u ? 1u << lane : 0u;
    bool sent = false, stored = false, live = false;
    if (lane < deg) {
        const uint32_t e = rs + lane;
        if (eager & b) {
            sent = true;
            if (!omitted(a, e)) {
                stored = true;
                if (a.rec_c) {                           // binned: a record for the next route
                    const uint32_t cs = (a.col[e] >> a.cv_shift) * kCoarseShards + ((v >> a.fv_shift) & (kCoarseShards - 1));
                    a.rec_c[a.csub[cs] + atomicAdd(&a.cnt_c_nxt[cs], 1u)] =
                        make_uint2(a.rev[e], PSIM_MSG_BROADCAST | (a.wtag << kTagShift));
                } else {
                    deliver_word(ao, e, PSIM_MSG_BROADCAST | (a.wtag << kTagShift), a.dhist,   // Round 0
                                 a.wl_nxt ? 2u : 1u);
                }
            }
        }
        if ((lazy & b) && !(outst & b)) live = bit_alive(a.alive, a.col[e]);
    }
    const uint32_t nmsg = (uint32_t)__popcll(__ballot(sent)), nword = (uint32_t)__popcll(__ballot(stored));
    const unsigned long long add_live = (unsigned long long)__popcll(__ballot(live));
    const uint32_t dm = deg >= 32u ? ~0u : (1u << deg) - 1u;
    outst |= lazy & dm;                                  // schedule_lazy_push: a row per lazy peer
    if (lane != 0) return;
    unsigned long long flags = outst0 ? 4ull : 0ull;
    a.vs[v] = make_uint4(eager, lazy, outst, 0u | (a.mono8 << 16) | (ep << 24));
    if ((outst0 != 0) != (outst != 0)) {
        a.ost[v] = 1;
        if (a.obin) a.obin[v >> a.fv_shift] += 1u;
        atomicAdd(&a.stats[S_OST_DELTA], 1ull);
        atomicAdd(a.ost_total, 1);
        if (int* d = hold_delta(ao)) atomicAdd(d, 1);
    }
    if (add_live) atomicAdd(&a.stats[S_LIVE_DELTA], add_live);
    if (nmsg) atomicAdd(&a.stats[PSIM_MSG_BROADCAST], (unsigned long long)nmsg);
    if (nword) atomicAdd(&a.stats[S_WORDS], (unsigned long long)nword);
    if (nmsg && a.mcnt) atomicAdd(&a.mcnt[a.m_s * 64], nmsg);
    if (flags) atomicOr(&a.stats[S_OVERFLOW], flags);
}

// prep != 0: first the fills the host used to enqueue before an origin, by
// this block -- the stats row (prep words) zeroed, the lane's count area
// zeroed and its hold ring seeded with `hold` (psim_host.hip seed_hold_ring)
// -- one launch instead of four
__global__ void pt_origin_kernel(PtArgs a, uint32_t prep, uint32_t hold) {
    if (blockIdx.x != 0) return;
    if (a.spec) {
        // pipelined: run only if the previous heartbeat ended exactly at its
        // predicted last round (PtArgs::spec); the host reads the decision
        const uint32_t t = threadIdx.x & 63u, rl = a.spec_rl & 3u, rp = (rl + 3u) & 3u;
        unsigned long long last = threadIdx.x < 64 ? a.mcnt[rl * 64 + t] : 0u;
        unsigned long long before = threadIdx.x < 64 ? a.mcnt[rp * 64 + t] : 0u;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            last += __shfl_xor(last, off, 64);
            before += __shfl_xor(before, off, 64);
        }
        const int holders = int(a.mcnt[kMcntHold + rp]) + int(a.mcnt[kMcntHoldD + rl]);
        const bool run = last == 0ull && before != 0ull && holders == 0;
        if (threadIdx.x == 0) {
            a.spec[0] = run ? 0u : 1u;
            a.spec[1] = run ? 1u : 2u;
        }
        if (!run) return;
    }
    if (prep) {
        for (uint32_t i = threadIdx.x; i < prep; i += blockDim.x) a.stats[i] = 0ull;
        if (a.mcnt)
            for (uint32_t i = threadIdx.x; i < kMcntLane; i += blockDim.x) a.mcnt[i] = i == kMcntHold + a.m_r ? hold : 0u;
        __threadfence();
        __syncthreads();
    }
    if (threadIdx.x >= 64) return;
    pt_origin_wave(a);
}

// The fills before a chunk of rounds (psim_host.hip drive): its stats rows
// zeroed and every lane's hold ring seeded, in one launch.
__global__ __launch_bounds__(kBlock) void pt_prep_kernel(PtPrep p) {
    const uint64_t i0 = blockIdx.x * uint64_t(kBlock) + threadIdx.x, st = uint64_t(gridDim.x) * kBlock;
    for (uint64_t i = i0; i < p.nz; i += st) p.z[i] = 0ull;
    if (i0 < p.k) {
        *p.hold[i0] = p.hv[i0];
        *p.holdd[i0] = 0u;
    }
}

// The forest's origins: one thread per heartbeat, each on its own lane.
__global__ __launch_bounds__(64) void fo_origin_kernel(FoArgs f, const uint32_t* __restrict__ lanes, uint32_t k) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i < k) pt_origin_body(fo_lane(f, lanes[i]));
}

// A lane is busy while its last round (count slot `slot`, origins included)
// sent messages or some vertex holds rows of its heartbeat.
__global__ __launch_bounds__(64) void fo_busy_kernel(FoArgs f, const uint32_t* __restrict__ lanes, uint32_t k,
                                                     uint32_t slot, uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= k) return;
    const uint32_t lane = lanes[i];
    const uint32_t* m = f.a.mcnt + size_t(lane) * kMcntLane + slot * 64;
    uint32_t msgs = 0;
    for (int q = 0; q < 64; q++) msgs += m[q];
    out[i] = (msgs != 0u || f.a.ost_total[4 * lane] != 0) ? 1u : 0u;
}

__global__ __launch_bounds__(kBlock) void fo_seed_kernel(FoArgs f) {
    const uint32_t lane = blockIdx.x * kBlock + threadIdx.x;
    if (lane >= f.nl) return;
    uint32_t* m = f.a.mcnt + size_t(lane) * kMcntLane;
    m[kMcntHold + f.a.m_r] = uint32_t(f.a.ost_total[4 * lane]);
    m[kMcntHoldD + f.a.m_s] = 0u;
}

// (state slot, vertex) pairs, flattened: slot i of slots[] (or slot i itself)
__global__ __launch_bounds__(kBlock) void fo_renorm_kernel(FoArgs f, const uint32_t* __restrict__ slots, uint32_t k) {
    const unsigned long long total = (unsigned long long)k * f.a.n;
    const unsigned long long stride = (unsigned long long)gridDim.x * kBlock;
    for (unsigned long long x = blockIdx.x * (unsigned long long)kBlock + threadIdx.x; x < total; x += stride) {
        const uint32_t i = uint32_t(x / f.a.n), v = uint32_t(x % f.a.n);
        const uint32_t sl = slots ? slots[i] : i;
        const uint32_t mono8 = f.info[sl].x;
        uint4* vs = f.a.vs + sl * f.s_vs;
        uint4 st = vs[v];
        uint32_t rseq = (st.w >> 16) & 0xFFu, ep = st.w >> 24;
        if (rseq != mono8) rseq = (mono8 - 1u) & 0xFFu;
        if (ep != f.a.epoch8) ep = (f.a.epoch8 - 1u) & 0xFFu;
        st.w = (st.w & 0xFFFFu) | (rseq << 16) | (ep << 24);
        vs[v] = st;
    }
}

__global__ __launch_bounds__(kBlock) void fo_count_live_kernel(FoArgs f, unsigned long long* out) {
    const PtArgs& a = f.a;
    const unsigned long long total = (unsigned long long)f.nl * a.n;
    const unsigned long long stride = (unsigned long long)gridDim.x * kBlock;
    unsigned long long cnt = 0;
    for (unsigned long long x = blockIdx.x * (unsigned long long)kBlock + threadIdx.x; x < total; x += stride) {
        const uint32_t lane = uint32_t(x / a.n), v = uint32_t(x % a.n);
        if (!a.ost[lane * f.s_ost + v] || !bit_alive(a.alive, a.v_lo + v)) continue;
        uint32_t m = a.vs[fo_slot(f, lane) * f.s_vs + v].z;
        const uint32_t rs = a.ell ? v * a.ell : a.rowp[v];
        while (m) {
            const uint32_t q = __ffs(m) - 1;
            m &= m - 1;
            cnt += bit_alive(a.alive, a.col[rs + q]);
        }
    }
    cnt = wave_sum(cnt);
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(out, cnt);
}

__global__ __launch_bounds__(kBlock) void fo_forget_kernel(FoArgs f, uint32_t v) {
    const uint32_t sl = blockIdx.x * kBlock + threadIdx.x;   // every root's records, parked or not
    if (sl >= f.ns) return;
    uint4* p = f.a.vs + sl * f.s_vs + v;
    uint4 st = *p;
    st.w = (st.w & 0xFF00FFFFu) | (((f.info[sl].x - 1u) & 0xFFu) << 16);
    *p = st;
}

// Outstanding rows to live peers, counted densely (after psim_set_alive).
__global__ __launch_bounds__(kBlock) void pt_count_live_kernel(PtArgs a, unsigned long long* out) {
    unsigned long long cnt = 0;
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t v = blockIdx.x * kBlock + threadIdx.x; v < a.n; v += stride) {
        if (!a.ost[v] || !bit_alive(a.alive, a.v_lo + v)) continue;
        uint32_t m = a.vs[v].z;
        const uint32_t rs = a.ell ? v * a.ell : a.rowp[v];
        while (m) {
            const uint32_t q = __ffs(m) - 1;
            m &= m - 1;
            cnt += bit_alive(a.alive, a.col[rs + q]);
        }
    }
    cnt = wave_sum(cnt);
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(out, cnt);
}

// psim_trace_hash: order-independent digests (sums of splitmix64 mixes).
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Per vertex: the psim_get_plumtree view (eager / lazy resolved through the
// tree epoch, outstanding mask, recv_round) -> out[0]; delivered -> out[2].
__global__ __launch_bounds__(kBlock) void pt_hash_state_kernel(PtArgs a, uint32_t has_serial, uint32_t root_local,
                                                               unsigned long long* out) {
    unsigned long long sum = 0, cnt = 0;
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t v = blockIdx.x * kBlock + threadIdx.x; v < a.n; v += stride) {
        const uint4 st = a.vs[v];
        const bool cur = (st.w >> 24) == a.epoch8;
        const uint32_t e = cur ? st.x : a.memb[v], l = cur ? st.y : 0u;
        const bool got = has_serial && ((st.w >> 16) & 0xFFu) == a.mono8;
        const uint32_t rr = !got ? 0xFFFFu : (v == root_local ? 0xFFFEu : ((st.w & 0xFFFFu) - 1u) & 0xFFFFu);
        const unsigned long long g = a.v_lo + v;
        sum += mix64(mix64(mix64(st.z) ^ ((unsigned long long)e << 32 | l)) ^ (g << 32 | rr));
        cnt += got;
    }
    sum = wave_sum(sum);
    cnt = wave_sum(cnt);
    if ((threadIdx.x & 63) == 0) {
        if (sum) atomicAdd(&out[0], sum);
        if (cnt) atomicAdd(&out[2], cnt);
    }
}

// In-flight words of the slot-scatter engine (one per receiver slot) -> out[1],
// keyed by the ABI (CSR) slot id in both layouts.
__global__ __launch_bounds__(kBlock) void pt_hash_words_kernel(PtArgs a, unsigned long long E, unsigned long long* out) {
    unsigned long long sum = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * kBlock;
    for (unsigned long long i = blockIdx.x * kBlock + threadIdx.x; i < E; i += stride) {
        const uint32_t w = a.in_cur[i];
        if (!live_word(w, a.ctag)) continue;
        const unsigned long long e = a.ell ? a.rowp[i / a.ell] + i % a.ell : i;   // ELL -> CSR slot id
        sum += mix64(((a.abi_slot_base + e) << 32) | abi_word(w));
    }
    sum = wave_sum(sum);
    if ((threadIdx.x & 63) == 0 && sum) atomicAdd(&out[1], sum);
}

// ... and of the binned engine (records waiting in the coarse sub-regions).
__global__ __launch_bounds__(kBlock) void pb_hash_records_kernel(PtArgs a, unsigned long long* out) {
    unsigned long long sum = 0;
    for (uint32_t cs = blockIdx.x; cs < a.nc * kCoarseShards; cs += gridDim.x) {
        const uint32_t k = a.cnt_c_cur[cs], b = a.csub[cs];
        for (uint32_t i = threadIdx.x; i < k; i += kBlock) {
            const uint2 r = a.rec_c[b + i];
            sum += mix64(((unsigned long long)r.x << 32) | abi_word(r.y));
        }
    }
    sum = wave_sum(sum);
    if ((threadIdx.x & 63) == 0 && sum) atomicAdd(&out[1], sum);
}

// Re-base the 8-bit Monotonic / epoch tags so they cannot alias after wrap.
__global__ __launch_bounds__(kBlock) void pt_renorm_kernel(PtArgs a) {
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t v = blockIdx.x * kBlock + threadIdx.x; v < a.n; v += stride) {
        uint4 st = a.vs[v];
        uint32_t rseq = (st.w >> 16) & 0xFFu, ep = st.w >> 24;
        if (rseq != a.mono8) rseq = (a.mono8 - 1u) & 0xFFu;
        if (ep != a.epoch8) ep = (a.epoch8 - 1u) & 0xFFu;
        st.w = (st.w & 0xFFFFu) | (rseq << 16) | (ep << 24);
        a.vs[v] = st;
    }
}

// Zero inbox words whose round tag is not among the `span` rounds from
// `keep` on (stale ones, before a tag could repeat): one pass over a buffer
// every <= 256 rounds.  span = 1 for the double buffer, kRing - 1 for the
// delay ring (words up to kRing - 1 rounds ahead are in flight).
__device__ __forceinline__ uint32_t scrub_word(uint32_t x, uint32_t keep, uint32_t span) {
    return ((word_tag(x) - keep) & 0xFFu) < span ? x : 0u;
}

__global__ __launch_bounds__(kBlock) void pt_scrub_kernel(uint4* __restrict__ w, unsigned long long n4, uint32_t keep,
                                                          uint32_t span) {
    const unsigned long long stride = (unsigned long long)gridDim.x * kBlock;
    for (unsigned long long i = blockIdx.x * kBlock + threadIdx.x; i < n4; i += stride) {
        uint4 x = w[i];
        const uint4 y = make_uint4(scrub_word(x.x, keep, span), scrub_word(x.y, keep, span),
                                   scrub_word(x.z, keep, span), scrub_word(x.w, keep, span));
        if (y.x != x.x || y.y != x.y || y.z != x.z || y.w != x.w) w[i] = y;
    }
}

__global__ void pt_scrub_tail_kernel(uint32_t* __restrict__ w, unsigned long long lo, unsigned long long n,
                                     uint32_t keep, uint32_t span) {
    const unsigned long long i = lo + threadIdx.x;
    if (i < n) w[i] = scrub_word(w[i], keep, span);
}

// Pack the staged cross-shard words into (global receiver slot, word)
// records, one region per destination shard.  A workgroup owns <= 1024
// entries of ONE destination's remote-slot list (blk = {rank, start, len}),
// so it reserves its run with a single atomicAdd.  Record order inside a
// region is irrelevant: every receiver slot has one writer per round.
// send_base null (the in-library record exchange of sparse rounds): region d
// starts at record (d - [d > self]) * cap and holds at most cap records; a
// region that would overflow is reported (S_OVERFLOW bit 0x200), never
// written past.
__global__ __launch_bounds__(kBlock) void pt_compact_kernel(PtArgs a, const uint32_t* __restrict__ rem,
                                                            const uint4* __restrict__ blk,
                                                            const uint32_t* __restrict__ send_base,
                                                            uint32_t* __restrict__ cursor, uint2* __restrict__ out,
                                                            uint32_t cap, uint32_t self) {
    __shared__ uint32_t wsum_[kBlock / 64];
    __shared__ uint32_t base;
    const uint4 b = blk[blockIdx.x];
    const uint32_t t = threadIdx.x;
    uint32_t e[4], w[4], cnt = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t j = 4 * t + i;
        w[i] = 0;
        e[i] = 0;
        if (j < b.z) {
            e[i] = rem[b.y + j];
            w[i] = a.stage[e[i]];
            if (w[i]) { a.stage[e[i]] = 0; cnt++; }
        }
    }
    // workgroup exclusive scan of cnt
    const uint32_t lane = t & 63, wv = t >> 6;
    uint32_t x = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= (uint32_t)off) x += y;
    }
    if (lane == 63) wsum_[wv] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (int i = 0; i < kBlock / 64; i++) {
        if (i < (int)wv) pre += wsum_[i];
        tot += wsum_[i];
    }
    if (t == 0) {
        base = tot ? atomicAdd(&cursor[b.x], tot) : 0u;
        if (tot && base + tot > cap) atomicOr(&a.stats[S_OVERFLOW], 0x200ull);
    }
    __syncthreads();
    const uint32_t rbase = send_base ? send_base[b.x] : (b.x - (b.x > self ? 1u : 0u)) * cap;
    uint32_t pos = base + pre + x - cnt;                // within the region
#pragma unroll
    for (int i = 0; i < 4; i++)
        if (w[i]) {
            if (pos < cap) out[rbase + pos] = make_uint2(a.rev[e[i]], w[i]);
            pos++;
        }
}

// Scatter records received from other shards into the local receiver slots.
// Sharded rounds with per-round counts (psim_shard_run): the words received
// count as messages of the round that sent them (PtArgs::mcnt slot m_w), so
// the next round's no-op test and flag-free decision see remote senders too.
__device__ __forceinline__ void ingest_count(const PtArgs& a, uint32_t c) {
    if (!a.mcnt) return;
    const unsigned long long s = wave_sum((unsigned long long)c);
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(&a.mcnt[a.m_w * 64 + (blockIdx.x & 63)], (uint32_t)s);
}

// The group-flag mode of the round whose words an ingest delivers: the same
// decision its local senders took (round_counts), from the same count, so a
// flag-free round's remote words set no flag either and a listed round's are
// listed.  Without counts: flags.  Uniform call (barrier).
__device__ __forceinline__ uint32_t ingest_mark(const PtArgs& a) {
    if (!a.mcnt) return 1u;
    __shared__ uint32_t pm[2];
    if (threadIdx.x < 64) {
        uint32_t c = a.mcnt[a.m_s * 64 + threadIdx.x], c2 = a.mcnt[a.m_r * 64 + threadIdx.x];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            c += __shfl_xor(c, off, 64);
            c2 += __shfl_xor(c2, off, 64);
        }
        if (threadIdx.x == 0) { pm[0] = c; pm[1] = c2; }
    }
    __syncthreads();
    return round_mark(a, pm[0], pm[1]);
}

__global__ __launch_bounds__(kBlock) void pt_ingest_kernel(PtArgs a, const uint2* __restrict__ rec, uint32_t nrec,
                                                           const uint32_t* __restrict__ slot2v) {
    const uint32_t mark = ingest_mark(a);
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const uint2 r = i < nrec ? rec[i] : make_uint2(0u, 0u);
    if (r.y) {                                          // else padding of a fixed-size record region
        const uint32_t ls = r.x - a.slot_base;
        a.in_nxt[ls] = r.y;
        mark_group(a, slot2v[ls] >> kGroupShift, mark, nullptr);
    }
    ingest_count(a, r.y ? 1u : 0u);
}

// Dense exchange (no counts, no host sync): word i of the send buffer is the
// staged word of the i-th remote slot in the static order of psim_shard_layout
// (zero when nothing was sent over that slot this round).
__global__ __launch_bounds__(kBlock) void pt_pack_dense_kernel(PtArgs a, const uint32_t* __restrict__ rem, uint32_t nrem,
                                                               uint32_t* __restrict__ send) {
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < nrem; i += stride) {
        const uint32_t e = rem[i];
        const uint32_t w = a.stage[e];
        send[i] = w;
        if (w) a.stage[e] = 0;
    }
}

// ... and word i of the receive buffer feeds local receiver slot recv_map[i].
__global__ __launch_bounds__(kBlock) void pt_ingest_dense_kernel(PtArgs a, const uint32_t* __restrict__ recv,
                                                                 const uint32_t* __restrict__ recv_map, uint32_t nrecv,
                                                                 const uint32_t* __restrict__ slot2v) {
    const uint32_t mark = ingest_mark(a);
    const uint32_t stride = gridDim.x * kBlock;
    uint32_t c = 0;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < nrecv; i += stride) {
        const uint32_t w = recv[i];
        if (!w) continue;
        const uint32_t ls = recv_map[i];
        a.in_nxt[ls] = w;
        mark_group(a, slot2v[ls] >> kGroupShift, mark, nullptr);
        c++;
    }
    ingest_count(a, c);
}

// Sharded forest: every lane's dense regions in one
// all-to-all-v.  Region d of the send buffer holds, lane after lane, each
// lane's words for shard d in psim_shard_layout order: word i (region d of
// the single-lane layout, base sb[d]) of lane L sits at
// sb[d] nl + L (sb[d+1] - sb[d]) + i - sb[d]; the receive side the same over
// the recv layout.  blockIdx.y = lane - f.lane0.
__device__ __forceinline__ uint64_t fo_region_pos(const uint64_t* b, uint32_t world, uint32_t i, uint32_t lane,
                                                  uint32_t nl) {
    uint32_t d = 0;
    while (d + 1 < world && b[d + 1] <= i) d++;       // world <= 64; regions in rank order
    return b[d] * nl + uint64_t(lane) * (b[d + 1] - b[d]) + (i - b[d]);
}

__global__ __launch_bounds__(kBlock) void fo_pack_dense_kernel(FoArgs f, const uint32_t* __restrict__ rem,
                                                               uint32_t nrem, const uint64_t* __restrict__ sb,
                                                               uint32_t world, uint32_t* __restrict__ send) {
    __shared__ uint64_t b[65];
    if (threadIdx.x <= world) b[threadIdx.x] = sb[threadIdx.x];
    __syncthreads();
    const uint32_t lane = f.lane0 + blockIdx.y;
    const PtArgs a = fo_lane(f, lane);
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < nrem; i += stride) {
        const uint32_t e = rem[i];
        const uint32_t w = a.stage[e];
        send[fo_region_pos(b, world, i, lane, f.nl)] = w;
        if (w) a.stage[e] = 0;
    }
}

// fixed_mark >= 0: the group-flag mode of the words' round is given (the
// origins' pushes: flags + list), else the ingest's own decision (ingest_mark)
__global__ __launch_bounds__(kBlock) void fo_ingest_dense_kernel(FoArgs f, const uint32_t* __restrict__ recv,
                                                                 const uint32_t* __restrict__ recv_map, uint32_t nrecv,
                                                                 const uint64_t* __restrict__ rb, uint32_t world,
                                                                 const uint32_t* __restrict__ slot2v, int fixed_mark) {
    __shared__ uint64_t b[65];
    if (threadIdx.x <= world) b[threadIdx.x] = rb[threadIdx.x];
    const uint32_t lane = f.lane0 + blockIdx.y;
    const PtArgs a = fo_lane(f, lane);
    const uint32_t mark = fixed_mark >= 0 ? uint32_t(fixed_mark) : ingest_mark(a);   // (barrier inside)
    __syncthreads();
    const uint32_t stride = gridDim.x * kBlock;
    uint32_t c = 0;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < nrecv; i += stride) {
        const uint32_t w = recv[fo_region_pos(b, world, i, lane, f.nl)];
        if (!w) continue;
        const uint32_t ls = recv_map[i];
        a.in_nxt[ls] = w;
        mark_group(a, slot2v[ls] >> kGroupShift, mark, nullptr);
        c++;
    }
    ingest_count(a, c);
}

uint32_t grid_chunks(uint32_t n) { return (n + kChunkV - 1) / kChunkV; }
uint32_t grid_ell(uint32_t n) { return (n + kEllChunk - 1) / kEllChunk; }


uint32_t grid_for(uint32_t n) {
    uint32_t g = (n + kBlock - 1) / kBlock;
    if (g > 8192) g = 8192;     // grid-stride beyond 32 blocks per CU
    return g ? g : 1;
}

}  // namespace

// Workgroups of the ELL round kernel for W-slot rows the chip holds at once
// (LDS-bound: the words buffer is kEllChunk W 4 bytes): the kernel's grid.
uint32_t ell_round_grid(uint32_t W, int device) {
    int cus = 0, o0 = 0, o1 = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) return 0;
    const size_t lds = size_t(kEllChunk) * W * 4;
    const auto k0 = W <= 4 ? pt_round_ell_kernel<false, 4, false> : W <= 6 ? pt_round_ell_kernel<false, 6, false>
                                                                    : pt_round_ell_kernel<false, 8, false>;
    const auto k1 = W <= 4 ? pt_round_ell_kernel<true, 4, false> : W <= 6 ? pt_round_ell_kernel<true, 6, false>
                                                                   : pt_round_ell_kernel<true, 8, false>;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o0, k0, kBlock, lds) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&o1, k1, kBlock, lds) != hipSuccess)
        return 0;
    const int o = std::min(o0, o1);
    return o > 0 ? uint32_t(cus) * uint32_t(o) : 0u;
}

hipError_t launch_pt_round(const PtArgs& a, hipStream_t s) {
    if (a.rec_c) {
        const uint32_t nr = a.nc * kCoarseShards * a.chunks;
        hipLaunchKernelGGL(pb_route_kernel, dim3(nr < 2048u ? nr : 2048u), dim3(kBlock), 0, s, a);
        hipLaunchKernelGGL(pb_round_kernel, dim3(a.nf < 4096u ? a.nf : 4096u), dim3(kBlock), 0, s, a);
        return hipGetLastError();
    }
    if (a.ell) {
        const size_t lds = size_t(kEllChunk) * a.ell * 4;
        const bool f = a.omit || a.dly;
        // kLocal: one GPU, not sharded (no staging ring, no staged remote words)
        const bool loc = !a.stage && !a.srg;
        // rows of exactly 5 slots (HyParView's active view, the bench overlay):
        // a kernel unrolled for 5, not 6 -- one slot fewer in every per-slot loop
        const auto k = a.ell <= 4 ? (f ? pt_round_ell_kernel<true, 4, false>
                                       : loc ? pt_round_ell_kernel<false, 4, true> : pt_round_ell_kernel<false, 4, false>)
                     : a.ell == 5 && !f ? (loc ? pt_round_ell_kernel<false, 5, true> : pt_round_ell_kernel<false, 5, false>)
                     : a.ell <= 6 ? (f ? pt_round_ell_kernel<true, 6, false>
                                       : loc ? pt_round_ell_kernel<false, 6, true> : pt_round_ell_kernel<false, 6, false>)
                                  : (f ? pt_round_ell_kernel<true, 8, false>
                                       : loc ? pt_round_ell_kernel<false, 8, true> : pt_round_ell_kernel<false, 8, false>);
        hipLaunchKernelGGL(k, dim3(a.ell_grid ? min(a.ell_grid, grid_ell(a.n)) : grid_ell(a.n)), dim3(kBlock), lds, s,
                           a);
        return hipGetLastError();
    }
    if (a.omit || a.dly)
        hipLaunchKernelGGL(pt_round_kernel<true>, dim3(grid_chunks(a.n)), dim3(kBlock), 0, s, a);
    else
        hipLaunchKernelGGL(pt_round_kernel<false>, dim3(grid_chunks(a.n)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_pt_round_lanes(const PtArgs* d_args, const PtArgs& a0, uint32_t nlanes, hipStream_t s) {
    const dim3 grid(grid_chunks(a0.n), nlanes);
    if (a0.ell) {
        const uint32_t gx = a0.ell_grid ? std::max<uint32_t>(1u, a0.ell_grid / nlanes) : grid_ell(a0.n);
        const dim3 grid(std::min(gx, grid_ell(a0.n)), nlanes);
        const size_t lds = size_t(kEllChunk) * a0.ell * 4;
        const bool f = a0.omit || a0.dly;
        const bool loc = !a0.stage && !a0.srg;
        const auto k = a0.ell <= 4 ? (f ? pt_round_ell_lanes_kernel<true, 4, false>
                                        : loc ? pt_round_ell_lanes_kernel<false, 4, true>
                                              : pt_round_ell_lanes_kernel<false, 4, false>)
                     : a0.ell <= 6 ? (f ? pt_round_ell_lanes_kernel<true, 6, false>
                                        : loc ? pt_round_ell_lanes_kernel<false, 6, true>
                                              : pt_round_ell_lanes_kernel<false, 6, false>)
                                   : (f ? pt_round_ell_lanes_kernel<true, 8, false>
                                        : loc ? pt_round_ell_lanes_kernel<false, 8, true>
                                              : pt_round_ell_lanes_kernel<false, 8, false>);
        hipLaunchKernelGGL(k, grid, dim3(kBlock), lds, s, d_args);
        return hipGetLastError();
    }
    if (a0.omit || a0.dly)
        hipLaunchKernelGGL(pt_round_lanes_kernel<true>, grid, dim3(kBlock), 0, s, d_args);
    else
        hipLaunchKernelGGL(pt_round_lanes_kernel<false>, grid, dim3(kBlock), 0, s, d_args);
    return hipGetLastError();
}

hipError_t launch_fo_round(FoArgs f, uint32_t gx, hipStream_t s) {
    const PtArgs& a0 = f.a;
    const bool flt = a0.omit || a0.dly;
    const uint32_t nl = f.nl;
    for (uint32_t l0 = 0; l0 < nl; l0 += 65535u) {
        f.lane0 = l0;
        const uint32_t ny = std::min<uint32_t>(65535u, nl - l0);
        if (a0.ell) {
            // resident workgroups spread over the lanes, at least one per lane
            const uint32_t g = gx ? gx : std::max<uint32_t>(1u, (a0.ell_grid ? a0.ell_grid : 1536u) / ny);
            const dim3 grid(std::min(g, grid_ell(a0.n)), ny);
            const size_t lds = size_t(kEllChunk) * a0.ell * 4;
            const bool loc = a0.stage == nullptr;        // sharded forests stage remote words per lane
            const auto k = a0.ell <= 4 ? (flt ? pt_forest_ell_kernel<true, 4, false>
                                              : loc ? pt_forest_ell_kernel<false, 4, true> : pt_forest_ell_kernel<false, 4, false>)
                         : a0.ell <= 6 ? (flt ? pt_forest_ell_kernel<true, 6, false>
                                              : loc ? pt_forest_ell_kernel<false, 6, true> : pt_forest_ell_kernel<false, 6, false>)
                                       : (flt ? pt_forest_ell_kernel<true, 8, false>
                                              : loc ? pt_forest_ell_kernel<false, 8, true> : pt_forest_ell_kernel<false, 8, false>);
            hipLaunchKernelGGL(k, grid, dim3(kBlock), lds, s, f);
        } else {
            const dim3 grid(grid_chunks(a0.n), ny);
            if (flt) hipLaunchKernelGGL(pt_forest_kernel<true>, grid, dim3(kBlock), 0, s, f);
            else hipLaunchKernelGGL(pt_forest_kernel<false>, grid, dim3(kBlock), 0, s, f);
        }
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_fo_origin(const FoArgs& f, const uint32_t* lanes, uint32_t k, hipStream_t s) {
    if (!k) return hipSuccess;
    hipLaunchKernelGGL(fo_origin_kernel, dim3((k + 63) / 64), dim3(64), 0, s, f, lanes, k);
    return hipGetLastError();
}

hipError_t launch_fo_busy(const FoArgs& f, const uint32_t* lanes, uint32_t k, uint32_t slot, uint32_t* out,
                          hipStream_t s) {
    if (!k) return hipSuccess;
    hipLaunchKernelGGL(fo_busy_kernel, dim3((k + 63) / 64), dim3(64), 0, s, f, lanes, k, slot, out);
    return hipGetLastError();
}

hipError_t launch_fo_seed(const FoArgs& f, hipStream_t s) {
    if (!f.nl || !f.a.mcnt) return hipSuccess;
    hipLaunchKernelGGL(fo_seed_kernel, dim3((f.nl + kBlock - 1) / kBlock), dim3(kBlock), 0, s, f);
    return hipGetLastError();
}

hipError_t launch_fo_renorm(const FoArgs& f, const uint32_t* slots, uint32_t k, hipStream_t s) {
    if (!k || !f.a.n) return hipSuccess;
    const unsigned long long total = (unsigned long long)k * f.a.n;
    const uint32_t g = uint32_t(std::min<unsigned long long>(65535ull * 8, (total + kBlock - 1) / kBlock));
    hipLaunchKernelGGL(fo_renorm_kernel, dim3(g), dim3(kBlock), 0, s, f, slots, k);
    return hipGetLastError();
}

hipError_t launch_fo_count_live(const FoArgs& f, unsigned long long* out, hipStream_t s) {
    if (!f.nl || !f.a.n) return hipSuccess;
    const unsigned long long total = (unsigned long long)f.nl * f.a.n;
    const uint32_t g = uint32_t(std::min<unsigned long long>(65535ull * 8, (total + kBlock - 1) / kBlock));
    hipLaunchKernelGGL(fo_count_live_kernel, dim3(g), dim3(kBlock), 0, s, f, out);
    return hipGetLastError();
}

hipError_t launch_fo_forget(const FoArgs& f, uint32_t v, hipStream_t s) {
    if (!f.ns) return hipSuccess;
    hipLaunchKernelGGL(fo_forget_kernel, dim3((f.ns + kBlock - 1) / kBlock), dim3(kBlock), 0, s, f, v);
    return hipGetLastError();
}

hipError_t launch_pt_prep(const PtPrep& p, hipStream_t s) {
    const uint64_t b = (p.nz + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(pt_prep_kernel, dim3(uint32_t(b < 1 ? 1 : b > 64 ? 64 : b)), dim3(kBlock), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_pt_origin(const PtArgs& a, hipStream_t s, uint32_t prep, uint32_t hold) {
    hipLaunchKernelGGL(pt_origin_kernel, dim3(1), dim3(64), 0, s, a, prep, hold);
    return hipGetLastError();
}

hipError_t launch_pt_count_live(const PtArgs& a, unsigned long long* out, hipStream_t s) {
    hipLaunchKernelGGL(pt_count_live_kernel, dim3(grid_for(a.n)), dim3(kBlock), 0, s, a, out);
    return hipGetLastError();
}

hipError_t launch_pt_compact(const PtArgs& a, const uint32_t* rem, const uint4* blk, uint32_t nblk,
                             const uint32_t* send_base, uint32_t* cursor, uint2* out, hipStream_t s, uint32_t cap,
                             uint32_t self) {
    if (nblk == 0) return hipSuccess;
    hipLaunchKernelGGL(pt_compact_kernel, dim3(nblk), dim3(kBlock), 0, s, a, rem, blk, send_base, cursor, out, cap,
                       self);
    return hipGetLastError();
}

hipError_t launch_pt_ingest(const PtArgs& a, const uint2* rec, uint32_t nrec, const uint32_t* slot2v, hipStream_t s) {
    if (nrec == 0) return hipSuccess;
    hipLaunchKernelGGL(pt_ingest_kernel, dim3((nrec + kBlock - 1) / kBlock), dim3(kBlock), 0, s, a, rec, nrec, slot2v);
    return hipGetLastError();
}

hipError_t launch_pt_pack_dense(const PtArgs& a, const uint32_t* rem, uint32_t nrem, uint32_t* send, hipStream_t s) {
    if (nrem == 0) return hipSuccess;
    hipLaunchKernelGGL(pt_pack_dense_kernel, dim3(grid_for(nrem)), dim3(kBlock), 0, s, a, rem, nrem, send);
    return hipGetLastError();
}

hipError_t launch_fo_pack_dense(FoArgs f, const uint32_t* rem, uint32_t nrem, const uint64_t* sb, uint32_t world,
                                uint32_t* send, hipStream_t s) {
    if (nrem == 0 || f.nl == 0) return hipSuccess;
    const uint32_t gx = std::max<uint32_t>(1u, std::min<uint32_t>(grid_for(nrem), 4096u / std::min(f.nl, 4096u)));
    for (uint32_t l0 = 0; l0 < f.nl; l0 += 65535u) {
        f.lane0 = l0;
        hipLaunchKernelGGL(fo_pack_dense_kernel, dim3(gx, std::min<uint32_t>(65535u, f.nl - l0)), dim3(kBlock), 0, s, f,
                           rem, nrem, sb, world, send);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_fo_ingest_dense(FoArgs f, const uint32_t* recv, const uint32_t* recv_map, uint32_t nrecv,
                                  const uint64_t* rb, uint32_t world, const uint32_t* slot2v, int fixed_mark,
                                  hipStream_t s) {
    if (nrecv == 0 || f.nl == 0) return hipSuccess;
    const uint32_t gx = std::max<uint32_t>(1u, std::min<uint32_t>(grid_for(nrecv), 4096u / std::min(f.nl, 4096u)));
    for (uint32_t l0 = 0; l0 < f.nl; l0 += 65535u) {
        f.lane0 = l0;
        hipLaunchKernelGGL(fo_ingest_dense_kernel, dim3(gx, std::min<uint32_t>(65535u, f.nl - l0)), dim3(kBlock), 0, s,
                           f, recv, recv_map, nrecv, rb, world, slot2v, fixed_mark);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_pt_ingest_dense(const PtArgs& a, const uint32_t* recv, const uint32_t* recv_map, uint32_t nrecv,
                                  const uint32_t* slot2v, hipStream_t s) {
    if (nrecv == 0) return hipSuccess;
    hipLaunchKernelGGL(pt_ingest_dense_kernel, dim3(grid_for(nrecv)), dim3(kBlock), 0, s, a, recv, recv_map, nrecv,
                       slot2v);
    return hipGetLastError();
}

hipError_t launch_pt_hash(const PtArgs& a, uint32_t has_serial, uint32_t root_local, unsigned long long E,
                          unsigned long long* out, hipStream_t s) {
    hipLaunchKernelGGL(pt_hash_state_kernel, dim3(grid_for(a.n)), dim3(kBlock), 0, s, a, has_serial, root_local, out);
    if (a.rec_c)
        hipLaunchKernelGGL(pb_hash_records_kernel, dim3(1024), dim3(kBlock), 0, s, a, out);
    else if (E)
        hipLaunchKernelGGL(pt_hash_words_kernel, dim3(2048), dim3(kBlock), 0, s, a, E, out);
    return hipGetLastError();
}

hipError_t launch_pt_scrub(uint32_t* words, uint64_t n, uint32_t keep, uint32_t span, hipStream_t s) {
    if (!words || !n) return hipSuccess;
    const unsigned long long n4 = n / 4;    // hipMalloc'd buffers: 16-byte aligned
    if (n4) {
        const unsigned long long g = std::min<unsigned long long>((n4 + kBlock - 1) / kBlock, 8192ull);
        hipLaunchKernelGGL(pt_scrub_kernel, dim3((uint32_t)g), dim3(kBlock), 0, s, reinterpret_cast<uint4*>(words),
                           n4, keep, span);
    }
    if (n % 4)
        hipLaunchKernelGGL(pt_scrub_tail_kernel, dim3(1), dim3(64), 0, s, words, n4 * 4, (unsigned long long)n, keep, span);
    return hipGetLastError();
}

hipError_t launch_pt_renorm(const PtArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(pt_renorm_kernel, dim3(grid_for(a.n)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace psim

#if PSIM_PHASE_PROF
// diagnostic build only (not in include/psim.h): the phase records so far,
// [launch][8] real-time ticks (100 MHz); the record count restarts at zero
extern "C" int psim_debug_phases(unsigned long long* out, uint32_t cap, uint32_t* n) {
    uint32_t k = 0;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(&k, HIP_SYMBOL(psim::g_phase_n), 4) != hipSuccess) return -1;
    k = k < psim::kPhaseRecs ? k : psim::kPhaseRecs;
    const uint32_t c = k < cap ? k : cap;
    if (c && hipMemcpyFromSymbol(out, HIP_SYMBOL(psim::g_phase), size_t(c) * 8 * 8) != hipSuccess) return -1;
    const uint32_t z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(psim::g_phase_n), &z, 4) != hipSuccess) return -1;
    *n = c;
    return 0;
}
#endif
