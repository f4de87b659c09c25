// hyparview.hip -- HyParView view maintenance
// (src/partisan_hyparview_peer_service_manager.erl) as gfx950 kernels.
//
// Messages are fixed 64-byte records in an HBM queue.  One round:
//   hv_count   -- histogram of destinations (atomicAdd)
//   hv_scan    -- exclusive scan of the histogram (3-phase, deterministic)
//   hv_scatter -- bucket message indices by destination
//   hv_process -- one thread per vertex: sort its bucket by (src, emission
//                 seq) -- the schedule's order -- and run the handle_message
//                 clauses in sequence, then the timers due this round.
// Emission appends to the next queue with atomicAdd; the slot a message
// lands in never matters because the next round re-sorts by (src, seq).
// Each vertex has its own Philox stream (kind 4) whose counter is the
// process's draw index, so draws follow Erlang's sequential consumption.
#include "psim_internal.h"
#include "philox.h"
#include "../../include/psim.h"

namespace psim {

namespace {

enum { HV_JOIN = 1, HV_NEIGHBOR, HV_FORWARD_JOIN, HV_DISCONNECT, HV_NEIGHBOR_REQUEST, HV_NEIGHBOR_REJECTED,
       HV_NEIGHBOR_ACCEPTED, HV_SHUFFLE, HV_SHUFFLE_REPLY };

__device__ __forceinline__ bool alive_of(const HvArgs& a, uint32_t v) { return (a.alive[v >> 5] >> (v & 31)) & 1u; }

// ---------------------------------------------------------------- one wave per vertex
// A vertex is handled by a whole wavefront.  Every control decision is
// wave-uniform (the same on all 64 lanes: message fields, view sizes, draws),
// so the clauses run without divergence; the lanes hold the views -- lane i
// the i-th active (i < 8) and passive (i < 32) id, in `sets` order -- and the
// set operations of the reference (ordsets add / del / member, pick_random's
// filter, the exchange list's usort) are ballots, popcounts and shuffles.
// Nothing is indexed at run time from a private array, so nothing spills.
constexpr uint32_t kHvStage = 32;   // records a wave stages in LDS before one reservation
struct W {
    const HvArgs* a;
    uint32_t* stage;               // this wave's LDS staging: kHvStage records of 16 dwords
    uint32_t* nstage;              // records staged (wave-uniform, in registers of the caller)
    uint32_t v;
    uint32_t A, P;                 // this lane's active / passive view element
    uint32_t na, np;
    uint32_t nsent, nrecv, seq;
    uint64_t draws;
    uint64_t k0, k1, k2;           // messages sent by kind: 16-bit fields, kinds 1-3 / 4-7 / 8-9 (no indexed array)
    uint32_t ndraw, err;
};
__device__ __forceinline__ void count_kind(W& c, uint32_t t) {
    const uint64_t inc = 1ull << (16 * (t & 3));
    if (t < 4) c.k0 += inc; else if (t < 8) c.k1 += inc; else c.k2 += inc;
}
__device__ __forceinline__ uint32_t kind_count(uint64_t k0, uint64_t k1, uint64_t k2, uint32_t t) {
    const uint64_t w = t < 4 ? k0 : (t < 8 ? k1 : k2);
    return (uint32_t)((w >> (16 * (t & 3))) & 0xFFFFull);
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// index of the k-th (0-based) set bit of m (m has > k set bits)
__device__ __forceinline__ uint32_t kth_bit(uint64_t m, uint32_t k) {
    uint32_t lo = 0, hi = 64;                         // smallest i with popc(m & ((2 << i) - 1)) > k
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((uint32_t)__popcll(m & ((1ull << mid) - 1ull)) > k) hi = mid; else lo = mid;
    }
    return lo;
}

__device__ __forceinline__ uint64_t draw64(W& c) {
    const uint4 r = philox4x32_10(make_uint4(c.v, (uint32_t)c.draws, KIND_HV, (uint32_t)(c.draws >> 32)), c.a->key);
    c.draws++;
    c.ndraw++;
    return (uint64_t)r.x | ((uint64_t)r.y << 32);
}
// draws whose values nothing uses (shuffle/2's sort keys of a list that is
// only truncated): the counter-based stream just moves on
__device__ __forceinline__ void skip_draws(W& c, uint32_t k) {
    c.draws += k;
    c.ndraw += k;
}
__device__ __forceinline__ uint32_t uniform(W& c, uint32_t n) {   // rand:uniform(N), N >= 1
    return 1u + (uint32_t)__umul64hi(draw64(c), (uint64_t)n);
}

// ordsets over a lane-distributed sorted list (x = this lane's element, n valid)
__device__ __forceinline__ bool l_has(uint32_t x, uint32_t n, uint32_t q) { return ballot(lane_id() < n && x == q) != 0; }
__device__ __forceinline__ void l_add(uint32_t& x, uint32_t& n, uint32_t q) {
    if (l_has(x, n, q)) return;
    const uint32_t l = lane_id();
    const uint32_t pos = (uint32_t)__popcll(ballot(l < n && x < q));
    const uint32_t prev = __shfl(x, l ? l - 1 : 0, 64);
    if (l > pos && l <= n) x = prev;
    else if (l == pos) x = q;
    n++;
}
__device__ __forceinline__ void l_del(uint32_t& x, uint32_t& n, uint32_t q) {
    const uint32_t l = lane_id();
    const uint64_t keep = ballot(l < n && x != q);
    const uint32_t k = (uint32_t)__popcll(keep);
    const uint32_t src = l < k ? kth_bit(keep, l) : l;
    const uint32_t y = __shfl(x, src, 64);
    x = l < k ? y : 0xFFFFFFFFu;
    n = k;
}
// the element at position i (uniform i < n)
__device__ __forceinline__ uint32_t l_at(uint32_t x, uint32_t i) { return uni(__shfl(x, i, 64)); }

// id maps (sent_message_map / recv_message_map, unbounded maps in the
// reference): one global open-addressing table per map, key (v << 32 | peer),
// value {epoch, cnt}.  Only vertex v inserts or reads keys of v, so a key is
// never raced; distinct vertices share probe chains through atomicCAS on the
// empty key.  Nothing is ever deleted, so a find that meets an empty slot is
// a definite miss.  The wave probes 64 consecutive slots per load.
constexpr unsigned long long kEmpty = ~0ull;
constexpr uint32_t kProbeMax = 256;
struct IdMap { unsigned long long* key; uint2* val; uint32_t mask; };
__device__ __forceinline__ uint32_t hslot(unsigned long long k, uint32_t mask) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33;
    return (uint32_t)k & mask;
}
// Map words are read at device scope (past this CU's L1): a key or value may
// have been written by another lane of this wave (its lane 0) or claimed by
// another wave since this CU last cached the line.
__device__ __forceinline__ unsigned long long key_at(const IdMap& m, uint32_t i) {
    return __hip_atomic_load(&m.key[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint2 val_at(const IdMap& m, uint32_t i) {
    const unsigned long long x =
        __hip_atomic_load(reinterpret_cast<unsigned long long*>(&m.val[i]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_uint2((uint32_t)x, (uint32_t)(x >> 32));
}
__device__ __forceinline__ bool mget(const IdMap& m, uint32_t v, uint32_t p, uint2& out) {
    const unsigned long long k = ((unsigned long long)v << 32) | p;
    const uint32_t h = hslot(k, m.mask);
    for (uint32_t t = 0; t < kProbeMax; t += 64) {
        const uint32_t i = (h + t + lane_id()) & m.mask;
        const unsigned long long x = key_at(m, i);
        const uint64_t hit = ballot(x == k), emp = ballot(x == kEmpty);
        const uint64_t any = hit | emp;
        if (any) {
            const uint32_t f = (uint32_t)__ffsll((long long)any) - 1;
            if (!((hit >> f) & 1ull)) return false;
            const uint2 val = val_at(m, (h + t + f) & m.mask);
            out = make_uint2(uni(val.x), uni(val.y));
            return true;
        }
    }
    return false;
}
__device__ __forceinline__ void mput(W& c, const IdMap& m, uint32_t& n, uint32_t p, uint32_t e, uint32_t cnt) {
    const unsigned long long k = ((unsigned long long)c.v << 32) | p;
    const uint32_t h = hslot(k, m.mask);
    uint32_t t = 0;
    while (t < kProbeMax) {
        const uint32_t i = (h + t + lane_id()) & m.mask;
        const unsigned long long x = (t + lane_id() < kProbeMax) ? key_at(m, i) : 0ull;
        const uint64_t cand = ballot(t + lane_id() < kProbeMax && (x == k || x == kEmpty));
        if (!cand) { t += 64; continue; }
        const uint32_t f = (uint32_t)__ffsll((long long)cand) - 1;
        const uint32_t slot = (h + t + f) & m.mask;
        bool mine = true;
        if (uni((uint32_t)(__shfl((uint32_t)(x == kEmpty), f, 64)))) {   // empty: claim it
            unsigned long long old = 0;
            if (lane_id() == 0) old = atomicCAS(&m.key[slot], kEmpty, k);
            const uint32_t lo = uni((uint32_t)old), hi = uni((uint32_t)(old >> 32));
            old = ((unsigned long long)hi << 32) | lo;
            if (old == kEmpty) n++;
            else mine = old == k;                       // another vertex took it: probe on
        }
        if (mine) {
            if (lane_id() == 0)
                __hip_atomic_store(reinterpret_cast<unsigned long long*>(&m.val[slot]),
                                   (unsigned long long)e | ((unsigned long long)cnt << 32), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        t += f + 1;
    }
    c.err |= 2u;
}
__device__ __forceinline__ IdMap sent_map(const W& c) { return IdMap{c.a->skey, c.a->sval, c.a->map_mask}; }
__device__ __forceinline__ IdMap recv_map(const W& c) { return IdMap{c.a->rkey, c.a->rval, c.a->map_mask}; }

// A message under construction: uniform header fields plus the exchange list
// held one element per lane (x, nx).
struct Out {
    uint32_t type, ttl, prio, nx, peer, epoch, did_e, did_c;
    uint32_t x;
};
__device__ __forceinline__ Out out_msg(uint32_t type) {
    Out o;
    o.type = type; o.ttl = 0; o.prio = 0; o.nx = 0; o.peer = 0; o.epoch = 0; o.did_e = 0; o.did_c = 0; o.x = 0;
    return o;
}
// The wave's staged records go to the queue with ONE reservation (lane 0's
// atomicAdd) and a coalesced copy: where a record lands never matters, the
// next round re-sorts each bucket by (src, seq).  One atomic per message on
// the queue counter was the round's bound (~0.8M serialised atomics).
__device__ __forceinline__ uint32_t flush_stage(const HvArgs& a, uint32_t* stage, uint32_t ns) {
    if (ns == 0) return 0;
    __builtin_amdgcn_wave_barrier();
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(a.nout, ns);
    base = uni(base);
    uint32_t err = 0;
    uint32_t fit = ns;
    if (base >= a.out_cap) { fit = 0; err = 1u; }
    else if (base + ns > a.out_cap) { fit = a.out_cap - base; err = 1u; }
    uint32_t* out = reinterpret_cast<uint32_t*>(a.out + base);
    for (uint32_t k = lane_id(); k < fit * 16; k += 64) out[k] = stage[k];
    __builtin_amdgcn_wave_barrier();
    return err;
}

// emission: the 64-byte record written into the wave's LDS stage by lanes
// 0..15 (one dword each)
__device__ __forceinline__ void emit(W& c, uint32_t dst, const Out& o) {
    if (dst >= c.a->n) { c.err |= 16u; return; }
    count_kind(c, o.type);
    const uint32_t seq = c.seq++;
    if (*c.nstage == kHvStage) {
        c.err |= flush_stage(*c.a, c.stage, *c.nstage);
        *c.nstage = 0;
    }
    const uint32_t pos = (*c.nstage)++;
    const uint32_t l = lane_id();
    uint32_t w = 0;
    switch (l) {
    case 0: w = o.type | (o.ttl << 8) | (o.prio << 16) | (o.nx << 24); break;
    case 1: w = c.v; break;
    case 2: w = dst; break;
    case 3: w = seq; break;
    case 4: w = o.peer; break;
    case 5: w = o.epoch; break;
    case 6: w = o.did_e; break;
    case 7: w = o.did_c; break;
    default: break;
    }
    const uint32_t xv = __shfl(o.x, (l - 8) & 63, 64);
    if (l >= 8 && l < 16) w = (l - 8 < o.nx) ? xv : 0u;
    if (l < 16) c.stage[pos * 16 + l] = w;
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ bool alive_w(W& c, uint32_t p) {
    if (p >= c.a->n) { c.err |= 16u; return false; }      // not a vertex id: reported, never dereferenced
    return alive_of(*c.a, p);
}

// pick_random(View, Omit) (:2291-2301) over a lane-distributed view; false =
// undefined (no draw, Q13)
__device__ __forceinline__ bool pick_random(W& c, uint32_t view, uint32_t nv, uint32_t o0, uint32_t o1, uint32_t o2,
                                            uint32_t& out) {
    const uint64_t ok = ballot(lane_id() < nv && view != o0 && view != o1 && view != o2);
    const uint32_t k = (uint32_t)__popcll(ok);
    if (k == 0) return false;
    const uint32_t idx = uniform(c, k) - 1;
    out = l_at(view, kth_bit(ok, idx));
    return true;
}

// select_peers_for_exchange/1 (:2324-2333): shuffle/2 draws one float per
// element (Q8); the list is usort([Myself | k_active of Active ++ k_passive of
// Passive]), returned lane-distributed
__device__ __forceinline__ uint32_t select_exchange(W& c, uint32_t& ex) {
    skip_draws(c, c.na + c.np);
    const uint32_t l = lane_id();
    const uint32_t ka = min(c.na, c.a->cfg.shuffle_k_active), kp = min(c.np, c.a->cfg.shuffle_k_passive);
    const uint32_t av = __shfl(c.A, (l - 1) & 63, 64), pv = __shfl(c.P, (l - 1 - ka) & 63, 64);
    const uint32_t cand = l == 0 ? c.v : (l <= ka ? av : pv);
    const uint32_t nc = 1 + ka + kp;
    const bool valid = l < nc;
    // keep the first occurrence of each id; rank = number of kept ids below it
    // (every shuffle runs with all lanes active: a lane that is switched off
    // in a branch cannot be read)
    bool keep = valid;
    for (uint32_t j = 0; j < nc; j++) {
        const uint32_t y = __shfl(cand, j, 64);
        if (j < l && y == cand) keep = false;
    }
    uint32_t rank = 0;
    for (uint32_t j = 0; j < nc; j++) {
        const uint32_t y = __shfl(cand, j, 64), kj = __shfl((uint32_t)keep, j, 64);
        rank += (kj && y < cand) ? 1u : 0u;
    }
    const uint64_t km = ballot(keep && valid);
    const uint32_t n = (uint32_t)__popcll(km);
    // lane t takes the kept candidate of rank t
    uint32_t got = 0xFFFFFFFFu;
    for (uint32_t j = 0; j < nc; j++) {
        const uint32_t rj = __shfl(rank, j, 64), cj = __shfl(cand, j, 64);
        if (((km >> j) & 1ull) && rj == l) got = cj;
    }
    ex = got;
    return n;
}

__device__ __forceinline__ void get_current_id(W& c, uint32_t p, uint32_t& e, uint32_t& cnt) {   // :2618-2627
    uint2 r;
    if (mget(recv_map(c), c.v, p, r)) { e = r.x; cnt = r.y; }
    else { e = 1; cnt = 0; }
}
__device__ __forceinline__ bool is_addable_did(W& c, uint32_t ie, uint32_t ic, uint32_t p) {       // :2652-2665
    uint2 r;
    if (!mget(sent_map(c), c.v, p, r)) return true;
    if (ie > r.x) return true;
    if (ie == r.x) return ic >= r.y;
    return false;
}
__device__ __forceinline__ bool is_addable_epoch(W& c, uint32_t pe, uint32_t p) {                  // :2667-2674
    uint2 r;
    return !mget(sent_map(c), c.v, p, r) || pe >= r.x;
}
__device__ __forceinline__ bool is_valid_disconnect(W& c, uint32_t ie, uint32_t ic, uint32_t p) {  // :2639-2650
    uint2 r;
    if (!mget(recv_map(c), c.v, p, r)) return true;
    if (ie > r.x) return true;
    return ic > r.y;
}

__device__ __forceinline__ void add_to_passive(W& c, uint32_t p) {                                 // :2418-2449
    if (p == c.v || l_has(c.A, c.na, p) || l_has(c.P, c.np, p)) return;
    if (c.np >= c.a->cfg.passive_max_size) {
        uint32_t r;
        if (pick_random(c, c.P, c.np, c.v, c.v, c.v, r)) l_del(c.P, c.np, r);
    }
    l_add(c.P, c.np, p);
}

__device__ __forceinline__ void drop_random_active(W& c) {                                         // :2476-2525
    uint32_t r;
    if (!pick_random(c, c.A, c.na, c.v, c.v, c.v, r)) return;
    l_del(c.A, c.na, r);
    add_to_passive(c, r);
    const IdMap m = sent_map(c);
    uint2 prev;
    uint32_t ne = 1, nc = 1;
    if (mget(m, c.v, r, prev)) {                                                     // get_next_id/3
        if (prev.x != 1u) { c.err |= 4u; return; }                                    // case_clause
        nc = prev.y + 1;
    }
    mput(c, m, c.nsent, r, ne, nc);
    if (alive_w(c, r)) {
        Out o = out_msg(HV_DISCONNECT);
        o.peer = c.v; o.did_e = ne; o.did_c = nc;
        emit(c, r, o);
    }
}

__device__ __forceinline__ void add_to_active(W& c, uint32_t p) {                                  // :2344-2410
    if (p == c.v || l_has(c.A, c.na, p)) return;
    l_del(c.P, c.np, p);
    if (c.na >= c.a->cfg.active_max_size) drop_random_active(c);
    l_add(c.A, c.na, p);
}

// merge_exchange/2 (:2569-2576): usort(Exchange) minus self and active, each
// added to the passive view in order
__device__ __forceinline__ void merge_exchange(W& c, uint32_t ex, uint32_t nx) {
    const uint32_t l = lane_id();
    uint32_t to = 0xFFFFFFFFu, k = 0;
    for (uint32_t i = 0; i < nx; i++) {
        const uint32_t y = l_at(ex, i);
        if (y != c.v && !l_has(c.A, c.na, y)) l_add(to, k, y);
    }
    (void)l;
    for (uint32_t i = 0; i < k; i++) add_to_passive(c, l_at(to, i));
}

__device__ __forceinline__ void promote_peer(W& c, uint32_t p) {                                   // :2675-2697
    uint32_t ex;
    const uint32_t nx = select_exchange(c, ex);
    uint32_t e, cnt;
    get_current_id(c, p, e, cnt);
    if (!alive_w(c, p)) return;
    Out o = out_msg(HV_NEIGHBOR_REQUEST);
    o.peer = c.v; o.prio = 1; o.did_e = e; o.did_c = cnt; o.nx = nx; o.x = ex;
    emit(c, p, o);
}

__device__ __forceinline__ void send_neighbor(W& c, uint32_t p) {
    uint32_t e, cnt;
    get_current_id(c, p, e, cnt);
    Out o = out_msg(HV_NEIGHBOR);
    o.peer = c.v; o.did_e = e; o.did_c = cnt;
    emit(c, p, o);
}

// one received message (uniform header m*, exchange list mx one per lane)
struct In {
    uint32_t type, ttl, prio, nx, src, peer, epoch, did_e, did_c;
    uint32_t x;
};

__device__ __forceinline__ void handle(W& c, const In& m) {
    const uint32_t P = m.peer;
    switch (m.type) {
    case HV_JOIN:                                                                   // :1234-1338
        if (is_addable_epoch(c, m.epoch, P) && !l_has(c.A, c.na, P) && alive_w(c, P)) {
            add_to_active(c, P);
            send_neighbor(c, P);
            for (uint32_t i = 0; i < c.na; i++) {
                const uint32_t q = l_at(c.A, i);
                if (q == c.v || q == P || !alive_w(c, q)) continue;
                Out o = out_msg(HV_FORWARD_JOIN);
                o.peer = P; o.epoch = m.epoch; o.ttl = c.a->cfg.active_rwl;
                emit(c, q, o);
            }
        }
        break;
    case HV_NEIGHBOR:                                                               // :1340-1379
        if (is_addable_did(c, m.did_e, m.did_c, P) && alive_w(c, P)) add_to_active(c, P);
        break;
    case HV_FORWARD_JOIN: {                                                         // :1381-1563
        const uint32_t S = m.src;
        if (m.ttl == 0 || c.na == 1) {
            if (is_addable_epoch(c, m.epoch, P) && !l_has(c.A, c.na, P) && alive_w(c, P)) {
                add_to_active(c, P);
                send_neighbor(c, P);
            }
        } else {
            const uint32_t A0 = c.A, na0 = c.na, P0 = c.P, np0 = c.np;
            if (m.ttl == c.a->cfg.passive_rwl) add_to_passive(c, P);
            uint32_t r;
            if (!pick_random(c, A0, na0, S, c.v, P, r)) {
                if (is_addable_epoch(c, m.epoch, P) && !l_has(A0, na0, P)) {
                    if (alive_w(c, P)) {
                        add_to_active(c, P);
                        send_neighbor(c, P);
                    } else {                                   // `false -> State0`
                        c.np = np0;
                        c.P = P0;
                    }
                }
            } else if (alive_w(c, r)) {
                Out o = out_msg(HV_FORWARD_JOIN);
                o.peer = P; o.epoch = m.epoch; o.ttl = m.ttl - 1;
                emit(c, r, o);
            }
        }
        break;
    }
    case HV_DISCONNECT: {                                                           // :1565-1617
        if (!is_valid_disconnect(c, m.did_e, m.did_c, P)) break;
        const uint32_t P0 = c.P, np0 = c.np;
        l_del(c.A, c.na, P);
        add_to_passive(c, P);
        mput(c, recv_map(c), c.nrecv, P, m.did_e, m.did_c);
        if (c.na == 1) {
            uint32_t r;
            if (pick_random(c, P0, np0, c.v, P, P, r)) promote_peer(c, r);
        }
        break;
    }
    case HV_NEIGHBOR_REQUEST: {                                                     // :1619-1711
        uint32_t ack;
        const uint32_t nack = select_exchange(c, ack);
        if (!m.prio && c.na >= c.a->cfg.active_max_size) {
            c.err |= 8u;                                       // 2-tuple neighbor_rejected: no clause
        } else if (is_addable_did(c, m.did_e, m.did_c, P)) {
            if (alive_w(c, P)) {
                uint32_t e, cnt;
                get_current_id(c, P, e, cnt);
                Out o = out_msg(HV_NEIGHBOR_ACCEPTED);
                o.peer = c.v; o.did_e = e; o.did_c = cnt; o.nx = nack; o.x = ack;
                emit(c, P, o);
                add_to_active(c, P);
            }
        } else if (alive_w(c, P)) {
            Out o = out_msg(HV_NEIGHBOR_REJECTED);
            o.peer = c.v; o.nx = nack; o.x = ack;
            emit(c, P, o);
        }
        merge_exchange(c, m.x, m.nx);
        break;
    }
    case HV_NEIGHBOR_REJECTED:                                                      // :1713-1724
        merge_exchange(c, m.x, m.nx);
        break;
    case HV_NEIGHBOR_ACCEPTED:                                                      // :1726-1748
        if (is_addable_did(c, m.did_e, m.did_c, P)) add_to_active(c, P);
        merge_exchange(c, m.x, m.nx);
        break;
    case HV_SHUFFLE_REPLY:                                                          // :1750-1752
        merge_exchange(c, m.x, m.nx);
        break;
    case HV_SHUFFLE: {                                                              // :1754-1798
        const uint32_t S = P;
        if (m.ttl > 0 && c.na > 1) {
            uint32_t r;
            if (pick_random(c, c.A, c.na, S, c.v, c.v, r) && alive_w(c, r)) {
                Out o = out_msg(HV_SHUFFLE);
                o.peer = c.v; o.ttl = m.ttl - 1; o.nx = m.nx; o.x = m.x;
                emit(c, r, o);
            }
        } else {
            skip_draws(c, c.np);                                      // shuffle(Passive, |Exchange|)
            const uint32_t k = c.np < m.nx ? c.np : m.nx;
            if (alive_w(c, S)) {
                Out o = out_msg(HV_SHUFFLE_REPLY);
                o.peer = c.v; o.nx = k; o.x = c.P;
                emit(c, S, o);
            }
            merge_exchange(c, m.x, m.nx);
        }
        break;
    }
    default:
        break;
    }
}


__device__ __forceinline__ uint32_t n_in(const HvArgs& a) { const uint32_t k = *a.nin; return k < a.out_cap ? k : a.out_cap; }

constexpr uint32_t kStrideBlocks = 1024;   // grid of the grid-stride message kernels

__global__ __launch_bounds__(kBlock) void hv_count(HvArgs a) {
    const uint32_t k = n_in(a);
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < k; i += kStrideBlocks * kBlock)
        atomicAdd(&a.cnt[a.in[i].dst], 1u);
}

// exclusive scan of cnt[0..n) into off[0..n], off[n] = total (3 phases)
__global__ __launch_bounds__(kBlock) void hv_scan_blocks(HvArgs a) {
    __shared__ uint32_t ws[kBlock / 64];
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t x0 = i < a.n ? a.cnt[i] : 0u;
    uint32_t x = x0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) ws[wv] = x;
    __syncthreads();
    uint32_t pre = 0;
    for (uint32_t w = 0; w < wv; w++) pre += ws[w];
    if (i < a.n) a.off[i] = pre + x - x0;
    if (threadIdx.x == kBlock - 1) a.bsum[blockIdx.x] = pre + x;
}
// one workgroup of 1024: each thread scans a contiguous run of block sums
__global__ __launch_bounds__(1024) void hv_scan_sums(HvArgs a, uint32_t nb) {
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x, per = (nb + 1023) / 1024;
    const uint32_t lo = t * per, hi = min(nb, lo + per);
    uint32_t s = 0;
    for (uint32_t b = lo; b < hi; b++) s += a.bsum[b];
    part[t] = s;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {      // Hillis-Steele over 1024 partials
        const uint32_t y = t >= o ? part[t - o] : 0u;
        __syncthreads();
        part[t] += y;
        __syncthreads();
    }
    uint32_t run = part[t] - s;
    for (uint32_t b = lo; b < hi; b++) { const uint32_t x = a.bsum[b]; a.bsum[b] = run; run += x; }
    if (t == 1023) a.off[a.n] = part[1023];
}
__global__ __launch_bounds__(kBlock) void hv_scan_add(HvArgs a) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < a.n) a.off[i] += a.bsum[blockIdx.x];
}

__global__ __launch_bounds__(kBlock) void hv_scatter(HvArgs a) {
    const uint32_t k = n_in(a);
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < k; i += kStrideBlocks * kBlock) {
        const uint32_t d = a.in[i].dst;
        a.idx[a.off[d] + atomicAdd(&a.cur[d], 1u)] = i;
    }
}

// Small overlays (C2: 10k peers, one join per round): a round's bucketing --
// counts, exclusive scan, scatter -- by ONE workgroup with the counts in LDS,
// instead of two fills and five launches that each cost a few microseconds
// of a round moving a handful of messages.  The same off[] and the same
// indices per bucket (their order within a bucket is free: hv_process sorts
// each bucket by (src, seq)).
constexpr uint32_t kHvSmallN = 12288;                // 48 KB of LDS counts
__global__ __launch_bounds__(1024) void hv_bucket_small(HvArgs a) {
    __shared__ uint32_t c[kHvSmallN];
    __shared__ uint32_t ws[1024 / 64];
    const uint32_t t = threadIdx.x, n = a.n, k = n_in(a);
    for (uint32_t i = t; i < n; i += 1024) c[i] = 0;
    __syncthreads();
    for (uint32_t i = t; i < k; i += 1024) atomicAdd(&c[a.in[i].dst], 1u);
    __syncthreads();
    // exclusive scan: thread t sums its run of counts, the runs' sums are
    // scanned over the workgroup, then each run is written out
    const uint32_t per = (n + 1023) / 1024, lo = min(n, t * per), hi = min(n, lo + per);
    uint32_t s = 0;
    for (uint32_t i = lo; i < hi; i++) s += c[i];
    const uint32_t lane = t & 63, wv = t >> 6;
    uint32_t x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) ws[wv] = x;
    __syncthreads();
    uint32_t pre = 0;
    for (uint32_t w = 0; w < wv; w++) pre += ws[w];
    uint32_t run = pre + x - s;
    for (uint32_t i = lo; i < hi; i++) {
        const uint32_t y = c[i];
        c[i] = run;                                   // the bucket's cursor
        a.off[i] = run;
        run += y;
    }
    if (t == 1023) a.off[n] = pre + x;
    __syncthreads();
    for (uint32_t i = t; i < k; i += 1024) a.idx[atomicAdd(&c[a.in[i].dst], 1u)] = i;
}

constexpr uint32_t kHvWaves = kBlock / 64;

// the message with index i, fields made wave-uniform, x[] one per lane
__device__ __forceinline__ In load_msg(const HvArgs& a, uint32_t i) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a.in + i);
    const uint32_t l = lane_id();
    const uint32_t mine = l < 16 ? w[l] : 0u;
    In m;
    const uint32_t h = uni(__shfl(mine, 0, 64));
    m.type = h & 0xFFu; m.ttl = (h >> 8) & 0xFFu; m.prio = (h >> 16) & 0xFFu; m.nx = h >> 24;
    m.src = uni(__shfl(mine, 1, 64));
    m.peer = uni(__shfl(mine, 4, 64));
    m.epoch = uni(__shfl(mine, 5, 64));
    m.did_e = uni(__shfl(mine, 6, 64));
    m.did_c = uni(__shfl(mine, 7, 64));
    const uint32_t xv = __shfl(mine, (8 + l) & 63, 64);
    m.x = l < m.nx ? xv : 0xFFFFFFFFu;
    return m;
}

// One wave per vertex: a wave takes a.group consecutive vertices at a time,
// keeps those with messages (or every live one on a timer round), and runs
// each of them with all its lanes.  The vertices of a group run one after
// another (each a chain of dependent loads and draws), so the group shrinks
// until a timer round -- where every live vertex runs -- has about as many
// waves as the chip holds (hv_group): at 10k vertices 64-vertex groups made
// 157 waves of 64 vertices each.
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void hv_process(HvArgs a) {
    __shared__ uint32_t stage_all[kHvWaves][kHvStage * 16];
    const uint32_t l = lane_id();
    const uint32_t gw = blockIdx.x * kHvWaves + (threadIdx.x >> 6), nw = gridDim.x * kHvWaves;
    uint32_t* stage = stage_all[threadIdx.x >> 6];
    uint32_t nstage = 0;
    uint32_t err = 0;
    const uint32_t G = a.group;
    for (uint32_t base = gw * G; base < a.n; base += nw * G) {
        uint64_t k0 = 0, k1 = 0, k2 = 0;     // this group's counters (flushed per group: no field overflows)
        uint32_t ndraw = 0, nproc = 0, act1 = 0;
        const uint32_t u = base + l;
        bool want = false;
        if (l < G && u < a.n && alive_of(a, u)) {
            // a random_promotion-only round leaves a vertex with >= active_min_size
            // active peers and an empty inbox untouched (no draw, no send)
            want = (a.timers & 2u) || a.off[u + 1] > a.off[u] ||
                   ((a.timers & 1u) && a.head[u].na < a.cfg.active_min_size);
        }
        uint64_t todo = ballot(want);
        while (todo) {
            const uint32_t j = (uint32_t)__ffsll((long long)todo) - 1;
            todo &= todo - 1;
            W c;
            c.a = &a;
            c.stage = stage;
            c.nstage = &nstage;
            c.v = base + j;
            const uint32_t v = c.v;
            const HvHead h = a.head[v];
            c.na = uni(h.na); c.np = uni(h.np); c.nsent = uni(h.nsent); c.nrecv = uni(h.nrecv); c.seq = uni(h.seq);
            c.draws = ((uint64_t)uni((uint32_t)(h.draws >> 32)) << 32) | uni((uint32_t)h.draws);
            c.A = l < 8 ? a.act[(size_t)v * 8 + l] : 0xFFFFFFFFu;
            c.P = l < 32 ? a.pas[(size_t)v * 32 + l] : 0xFFFFFFFFu;
            if (l >= c.na) c.A = 0xFFFFFFFFu;
            if (l >= c.np) c.P = 0xFFFFFFFFu;
            const uint32_t A_in = c.A, P_in = c.P, na_in = c.na, np_in = c.np, ns_in = c.nsent, nr_in = c.nrecv,
                           seq_in = c.seq;
            const uint64_t dr_in = c.draws;
            c.k0 = c.k1 = c.k2 = 0;
            c.ndraw = 0;
            c.err = 0;
            const uint32_t lo = uni(a.off[v]), hi = uni(a.off[v + 1]), nb = hi - lo;
            // the bucket in (src, seq) order: a rank sort over the wave --
            // in registers for <= 64 messages, 64 keys at a time for more --
            // then the messages handled in order, the next one's record loaded
            // while the current one is handled
            uint32_t sorted = 0;
            const uint32_t* order = nullptr;
            if (nb <= 64) {
                const uint32_t mi = l < nb ? a.idx[lo + l] : 0u;
                uint32_t src = 0xFFFFFFFFu, sq = 0xFFFFFFFFu;
                if (l < nb) { src = a.in[mi].src; sq = a.in[mi].seq; }
                uint32_t rank = 0;
                for (uint32_t q = 0; q < nb; q++) {
                    const uint32_t s2 = __shfl(src, q, 64), q2 = __shfl(sq, q, 64);
                    rank += (s2 < src || (s2 == src && q2 < sq)) ? 1u : 0u;
                }
                // lane r holds the index of the message of rank r
                sorted = __builtin_amdgcn_ds_permute((l < nb ? rank : l) * 4, (int)mi);
            } else {
                for (uint32_t oc = 0; oc < nb; oc += 64) {
                    const uint32_t me = oc + l < nb ? a.idx[lo + oc + l] : 0u;
                    uint64_t mk = ~0ull;
                    if (oc + l < nb) mk = ((uint64_t)a.in[me].src << 32) | a.in[me].seq;
                    uint32_t rank = 0;
                    for (uint32_t kc = 0; kc < nb; kc += 64) {
                        const uint32_t oi = kc + l < nb ? a.idx[lo + kc + l] : 0u;
                        uint64_t ok = ~0ull;
                        if (kc + l < nb) ok = ((uint64_t)a.in[oi].src << 32) | a.in[oi].seq;
                        const uint32_t klo = (uint32_t)ok, khi = (uint32_t)(ok >> 32);
                        const uint32_t lim = min(64u, nb - kc);
                        for (uint32_t q = 0; q < lim; q++) {
                            const uint64_t y = ((uint64_t)__shfl(khi, q, 64) << 32) | __shfl(klo, q, 64);
                            rank += y < mk ? 1u : 0u;
                        }
                    }
                    if (oc + l < nb) a.idx2[lo + rank] = me;
                }
                __threadfence_block();
                order = a.idx2 + lo;
            }
            if (nb) {
                In cur = load_msg(a, order ? uni(order[0]) : uni(__shfl(sorted, 0, 64)));
                for (uint32_t q = 0; q < nb; q++) {
                    In nxt = cur;
                    if (q + 1 < nb) nxt = load_msg(a, order ? uni(order[q + 1]) : uni(__shfl(sorted, q + 1, 64)));
                    handle(c, cur);
                    cur = nxt;
                }
            }
            nproc += nb;
            act1++;
            if (a.timers & 1u) {                                   // random_promotion (:1046-1067)
                if (c.na < a.cfg.active_min_size) {
                    uint32_t r;
                    if (pick_random(c, c.P, c.np, v, v, v, r)) promote_peer(c, r);
                }
            }
            if (a.timers & 2u) {                                   // passive_view_maintenance (:1078-1111)
                uint32_t ex;
                const uint32_t nx = select_exchange(c, ex);
                uint32_t r;
                if (pick_random(c, c.A, c.na, v, v, v, r) && alive_w(c, r)) {
                    Out o = out_msg(HV_SHUFFLE);
                    o.peer = v; o.ttl = a.cfg.active_rwl; o.nx = nx; o.x = ex;
                    emit(c, r, o);
                }
            }
            // write back only what changed
            if (ballot(l < 8 && c.A != A_in)) {
                if (l < 8) a.act[(size_t)v * 8 + l] = l < c.na ? c.A : 0xFFFFFFFFu;
            }
            if (ballot(l < 32 && c.P != P_in)) {
                if (l < 32) a.pas[(size_t)v * 32 + l] = l < c.np ? c.P : 0xFFFFFFFFu;
            }
            if (l == 0 && (c.na != na_in || c.np != np_in || c.nsent != ns_in || c.nrecv != nr_in || c.seq != seq_in ||
                           c.draws != dr_in)) {
                HvHead nh;
                nh.na = (uint8_t)c.na; nh.np = (uint8_t)c.np; nh.nsent = (uint16_t)c.nsent; nh.nrecv = (uint16_t)c.nrecv;
                nh.seq = c.seq; nh.draws = c.draws;
                a.head[v] = nh;
            }
            ndraw += c.ndraw;
            err |= c.err;
            k0 += c.k0;
            k1 += c.k1;
            k2 += c.k2;
        }
        // counters: wave-uniform, one atomic per group and counter
        if (l == 0 && act1) {
#pragma unroll
            for (uint32_t t = 1; t < 10; t++) {
                const uint32_t x = kind_count(k0, k1, k2, t);
                if (x) atomicAdd(&a.stats[t], (unsigned long long)x);
            }
            if (ndraw) atomicAdd(&a.stats[10], (unsigned long long)ndraw);
            if (nproc) atomicAdd(&a.stats[12], (unsigned long long)nproc);
            atomicAdd(&a.stats[13], (unsigned long long)act1);
        }
    }
    err |= flush_stage(a, stage, nstage);
    if (l == 0 && err) atomicOr(&a.stats[11], (unsigned long long)err);
}

// handle_cast({join, Peer}) (:999-1016) at v[i]: connect + {join, Myself, Tag, Epoch};
// the v[i] are distinct (checked by the host), so each thread owns its seq
__global__ __launch_bounds__(kBlock) void hv_join_kernel(HvArgs a, const uint32_t* __restrict__ vv,
                                                         const uint32_t* __restrict__ cc, uint32_t k) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= k) return;
    const uint32_t v = vv[i], contact = cc[i];
    if (!alive_of(a, contact)) return;
    HvHead h = a.head[v];
    const uint32_t pos = atomicAdd(a.nout, 1u);
    if (pos >= a.out_cap) { atomicOr(&a.stats[11], 1ull); return; }
    HvMsg* m = &a.out[pos];
    m->type = HV_JOIN; m->src = v; m->dst = contact; m->seq = h.seq++;
    m->peer = v; m->epoch = 1; m->ttl = 0; m->prio = 0; m->did_e = 0; m->did_c = 0; m->nx = 0;
    a.head[v] = h;
}

__global__ __launch_bounds__(kBlock) void hv_init_kernel(HvArgs a) {
    const uint32_t v = blockIdx.x * kBlock + threadIdx.x;
    if (v >= a.n) return;
    HvHead h;
    h.na = 1; h.np = 0; h.nsent = 0; h.nrecv = 0; h.seq = 0; h.draws = 0;   // init/1: Active = {self}
    a.head[v] = h;
    a.act[(size_t)v * 8] = v;
    for (uint32_t i = 1; i < 8; i++) a.act[(size_t)v * 8 + i] = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < 32; i++) a.pas[(size_t)v * 32 + i] = 0xFFFFFFFFu;
}

inline uint32_t nblk(uint32_t n) { return (n + kBlock - 1) / kBlock; }
// hv_process: vertices per wave -- the smallest power of two that leaves at
// most kHvWaveTarget waves, so that a timer round at 10k vertices runs 1250
// waves of 8 vertices (0.082 ms per C2 round against 0.247 with groups of
// 64 and 0.136 with groups of 2: each wave also pays its staging flush and
// counter atomics) and one above 128k vertices keeps groups of 64 (groups of
// 8 measured 2.4x slower at 1M, where the chip is full anyway)
constexpr uint32_t kHvWaveTarget = 2048;
inline uint32_t hv_group(uint32_t n) {
    uint32_t g = 1;
    while (g < 64 && uint64_t(g) * kHvWaveTarget < n) g <<= 1;
    return g;
}
// grid-striding beyond 64K workgroups
inline uint32_t hv_blocks(uint32_t n, uint32_t group) {
    const uint32_t groups = (n + group - 1) / group;
    const uint32_t b = (groups + kHvWaves - 1) / kHvWaves;
    return b < 1 ? 1 : (b > 65535 ? 65535 : b);
}

}  // namespace

hipError_t launch_hv_init(const HvArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(hv_init_kernel, dim3(nblk(a.n)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_hv_join(const HvArgs& a, const uint32_t* v, const uint32_t* contact, uint32_t k, hipStream_t s) {
    if (k) hipLaunchKernelGGL(hv_join_kernel, dim3(nblk(k)), dim3(kBlock), 0, s, a, v, contact, k);
    return hipGetLastError();
}

// one round: bucket the input messages by destination, then process
hipError_t launch_hv_round(const HvArgs& a, hipStream_t s) {
    if (a.n <= kHvSmallN) {
        hipLaunchKernelGGL(hv_bucket_small, dim3(1), dim3(1024), 0, s, a);
    } else {
        hipError_t e;
        if ((e = hipMemsetAsync(a.cnt, 0, size_t(a.n) * 4, s)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(a.cur, 0, size_t(a.n) * 4, s)) != hipSuccess) return e;
        hipLaunchKernelGGL(hv_count, dim3(kStrideBlocks), dim3(kBlock), 0, s, a);
        hipLaunchKernelGGL(hv_scan_blocks, dim3(nblk(a.n)), dim3(kBlock), 0, s, a);
        hipLaunchKernelGGL(hv_scan_sums, dim3(1), dim3(1024), 0, s, a, nblk(a.n));
        hipLaunchKernelGGL(hv_scan_add, dim3(nblk(a.n)), dim3(kBlock), 0, s, a);
        hipLaunchKernelGGL(hv_scatter, dim3(kStrideBlocks), dim3(kBlock), 0, s, a);
    }
    HvArgs b = a;
    b.group = hv_group(a.n);
    hipLaunchKernelGGL(hv_process, dim3(hv_blocks(a.n, b.group)), dim3(kBlock), 0, s, b);
    return hipGetLastError();
}

}  // namespace psim
