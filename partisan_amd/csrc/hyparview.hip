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

// ---------------------------------------------------------------- context
struct Ctx {
    const HvArgs* a;
    uint32_t v;
    uint32_t act[8], na;
    uint32_t pas[32], np;
    uint32_t nsent, nrecv;
    uint32_t seq;
    uint64_t draws;
    uint32_t sent_cnt[10];
    uint32_t ndraw, err;
};

__device__ uint64_t draw64(Ctx& c) {
    const uint4 r = philox4x32_10(make_uint4(c.v, (uint32_t)c.draws, KIND_HV, (uint32_t)(c.draws >> 32)), c.a->key);
    c.draws++;
    c.ndraw++;
    return (uint64_t)r.x | ((uint64_t)r.y << 32);
}
__device__ __forceinline__ uint32_t uniform(Ctx& c, uint32_t n) {   // rand:uniform(N), N >= 1
    return 1u + (uint32_t)__umul64hi(draw64(c), (uint64_t)n);
}

__device__ __forceinline__ bool has(const uint32_t* s, uint32_t n, uint32_t x) {
    for (uint32_t i = 0; i < n; i++)
        if (s[i] == x) return true;
    return false;
}
__device__ __forceinline__ void sadd(uint32_t* s, uint32_t& n, uint32_t x) {
    if (has(s, n, x)) return;
    uint32_t i = n;
    while (i > 0 && s[i - 1] > x) { s[i] = s[i - 1]; i--; }
    s[i] = x;
    n++;
}
__device__ __forceinline__ void sdel(uint32_t* s, uint32_t& n, uint32_t x) {
    uint32_t k = 0;
    for (uint32_t i = 0; i < n; i++)
        if (s[i] != x) s[k++] = s[i];
    n = k;
}

// id maps (sent_message_map / recv_message_map, unbounded maps in the
// reference): one global open-addressing table per map, key (v << 32 | peer),
// value {epoch, cnt}.  Only vertex v inserts or reads keys of v, so a key is
// never raced; distinct vertices share probe chains through atomicCAS on the
// empty key.  Nothing is ever deleted, so a find that meets an empty slot is
// a definite miss.
constexpr unsigned long long kEmpty = ~0ull;
constexpr uint32_t kProbeMax = 256;
struct IdMap { unsigned long long* key; uint2* val; uint32_t mask; };
__device__ __forceinline__ uint32_t hslot(unsigned long long k, uint32_t mask) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33;
    return (uint32_t)k & mask;
}
__device__ bool mget(const IdMap& m, uint32_t v, uint32_t p, uint2& out) {
    const unsigned long long k = ((unsigned long long)v << 32) | p;
    uint32_t i = hslot(k, m.mask);
    for (uint32_t t = 0; t < kProbeMax; t++, i = (i + 1) & m.mask) {
        const unsigned long long x = m.key[i];
        if (x == k) { out = m.val[i]; return true; }
        if (x == kEmpty) return false;
    }
    return false;
}
__device__ void mput(Ctx& c, const IdMap& m, uint32_t& n, uint32_t p, uint32_t e, uint32_t cnt) {
    const unsigned long long k = ((unsigned long long)c.v << 32) | p;
    uint32_t i = hslot(k, m.mask);
    for (uint32_t t = 0; t < kProbeMax; t++, i = (i + 1) & m.mask) {
        unsigned long long x = m.key[i];
        if (x == kEmpty) {
            x = atomicCAS(&m.key[i], kEmpty, k);
            if (x == kEmpty) { n++; x = k; }
        }
        if (x == k) { m.val[i] = make_uint2(e, cnt); return; }
    }
    c.err |= 2u;
}
__device__ __forceinline__ IdMap sent_map(const Ctx& c) { return IdMap{c.a->skey, c.a->sval, c.a->map_mask}; }
__device__ __forceinline__ IdMap recv_map(const Ctx& c) { return IdMap{c.a->rkey, c.a->rval, c.a->map_mask}; }

__device__ HvMsg* emit(Ctx& c, uint32_t dst, uint32_t type) {
    const uint32_t pos = atomicAdd(c.a->nout, 1u);
    c.sent_cnt[type]++;
    if (pos >= c.a->out_cap) { c.err |= 1u; return nullptr; }
    HvMsg* m = &c.a->out[pos];
    m->type = type;
    m->src = c.v;
    m->dst = dst;
    m->seq = c.seq++;
    m->peer = 0; m->epoch = 0; m->ttl = 0; m->prio = 0; m->did_e = 0; m->did_c = 0; m->nx = 0;
    return m;
}

// pick_random(View, Omit) (:2291-2301); returns false = undefined (no draw, Q13)
__device__ bool pick_random(Ctx& c, const uint32_t* view, uint32_t nv, const uint32_t* om, uint32_t no, uint32_t& out) {
    uint32_t k = 0;
    for (uint32_t i = 0; i < nv; i++)
        if (!has(om, no, view[i])) k++;
    if (k == 0) return false;
    uint32_t idx = uniform(c, k) - 1;
    for (uint32_t i = 0; i < nv; i++)
        if (!has(om, no, view[i])) {
            if (idx == 0) { out = view[i]; return true; }
            idx--;
        }
    return false;
}

// select_peers_for_exchange/1 (:2324-2333); shuffle/2 draws one float per element (Q8)
__device__ uint32_t select_exchange(Ctx& c, uint32_t* out) {
    for (uint32_t i = 0; i < c.na + c.np; i++) (void)draw64(c);
    uint32_t n = 0;
    sadd(out, n, c.v);
    for (uint32_t i = 0; i < c.na && i < c.a->cfg.shuffle_k_active; i++) sadd(out, n, c.act[i]);
    for (uint32_t i = 0; i < c.np && i < c.a->cfg.shuffle_k_passive; i++) sadd(out, n, c.pas[i]);
    return n;
}

__device__ void get_current_id(Ctx& c, uint32_t p, uint32_t& e, uint32_t& cnt) {   // :2618-2627
    uint2 r;
    if (mget(recv_map(c), c.v, p, r)) { e = r.x; cnt = r.y; }
    else { e = 1; cnt = 0; }
}
__device__ bool is_addable_did(Ctx& c, uint32_t ie, uint32_t ic, uint32_t p) {       // :2652-2665
    uint2 r;
    if (!mget(sent_map(c), c.v, p, r)) return true;
    if (ie > r.x) return true;
    if (ie == r.x) return ic >= r.y;
    return false;
}
__device__ bool is_addable_epoch(Ctx& c, uint32_t pe, uint32_t p) {                  // :2667-2674
    uint2 r;
    return !mget(sent_map(c), c.v, p, r) || pe >= r.x;
}
__device__ bool is_valid_disconnect(Ctx& c, uint32_t ie, uint32_t ic, uint32_t p) {  // :2639-2650
    uint2 r;
    if (!mget(recv_map(c), c.v, p, r)) return true;
    if (ie > r.x) return true;
    return ic > r.y;
}

__device__ void add_to_passive(Ctx& c, uint32_t p) {                                 // :2418-2449
    if (p == c.v || has(c.act, c.na, p) || has(c.pas, c.np, p)) return;
    if (c.np >= c.a->cfg.passive_max_size) {
        uint32_t r;
        const uint32_t om[1] = {c.v};
        if (pick_random(c, c.pas, c.np, om, 1, r)) sdel(c.pas, c.np, r);
    }
    sadd(c.pas, c.np, p);
}

__device__ void drop_random_active(Ctx& c) {                                         // :2476-2525
    uint32_t r;
    const uint32_t om[1] = {c.v};
    if (!pick_random(c, c.act, c.na, om, 1, r)) return;
    sdel(c.act, c.na, r);
    add_to_passive(c, r);
    const IdMap m = sent_map(c);
    uint2 prev;
    uint32_t ne = 1, nc = 1;
    if (mget(m, c.v, r, prev)) {                                                     // get_next_id/3
        if (prev.x != 1u) { c.err |= 4u; return; }                                    // case_clause
        nc = prev.y + 1;
    }
    mput(c, m, c.nsent, r, ne, nc);
    if (alive_of(*c.a, r)) {
        HvMsg* x = emit(c, r, HV_DISCONNECT);
        if (x) { x->peer = c.v; x->did_e = ne; x->did_c = nc; }
    }
}

__device__ void add_to_active(Ctx& c, uint32_t p) {                                  // :2344-2410
    if (p == c.v || has(c.act, c.na, p)) return;
    sdel(c.pas, c.np, p);
    if (c.na >= c.a->cfg.active_max_size) drop_random_active(c);
    sadd(c.act, c.na, p);
}

__device__ void merge_exchange(Ctx& c, const uint32_t* ex, uint32_t nx) {            // :2569-2576
    uint32_t to[kHvX + 1], k = 0;
    for (uint32_t i = 0; i < nx; i++)
        if (ex[i] != c.v && !has(c.act, c.na, ex[i])) sadd(to, k, ex[i]);
    for (uint32_t i = 0; i < k; i++) add_to_passive(c, to[i]);
}

__device__ void promote_peer(Ctx& c, uint32_t p) {                                   // :2675-2697
    uint32_t ex[kHvX];
    const uint32_t nx = select_exchange(c, ex);
    uint32_t e, cnt;
    get_current_id(c, p, e, cnt);
    if (!alive_of(*c.a, p)) return;
    HvMsg* x = emit(c, p, HV_NEIGHBOR_REQUEST);
    if (!x) return;
    x->peer = c.v; x->prio = 1; x->did_e = e; x->did_c = cnt; x->nx = nx;
    for (uint32_t i = 0; i < nx; i++) x->x[i] = ex[i];
}

__device__ void send_neighbor(Ctx& c, uint32_t p) {
    uint32_t e, cnt;
    get_current_id(c, p, e, cnt);
    HvMsg* x = emit(c, p, HV_NEIGHBOR);
    if (x) { x->peer = c.v; x->did_e = e; x->did_c = cnt; }
}

__device__ void handle(Ctx& c, const HvMsg& m) {
    const uint32_t P = m.peer;
    switch (m.type) {
    case HV_JOIN:                                                                   // :1234-1338
        if (is_addable_epoch(c, m.epoch, P) && !has(c.act, c.na, P) && alive_of(*c.a, P)) {
            add_to_active(c, P);
            send_neighbor(c, P);
            for (uint32_t i = 0; i < c.na; i++) {
                const uint32_t q = c.act[i];
                if (q == c.v || q == P || !alive_of(*c.a, q)) continue;
                HvMsg* f = emit(c, q, HV_FORWARD_JOIN);
                if (f) { f->peer = P; f->epoch = m.epoch; f->ttl = c.a->cfg.active_rwl; }
            }
        }
        break;
    case HV_NEIGHBOR:                                                               // :1340-1379
        if (is_addable_did(c, m.did_e, m.did_c, P) && alive_of(*c.a, P)) add_to_active(c, P);
        break;
    case HV_FORWARD_JOIN: {                                                         // :1381-1563
        const uint32_t S = m.src;
        if (m.ttl == 0 || c.na == 1) {
            if (is_addable_epoch(c, m.epoch, P) && !has(c.act, c.na, P) && alive_of(*c.a, P)) {
                add_to_active(c, P);
                send_neighbor(c, P);
            }
        } else {
            uint32_t act0[8], na0 = c.na, pas0[32], np0 = c.np;
            for (uint32_t i = 0; i < 8; i++) act0[i] = c.act[i];
            for (uint32_t i = 0; i < np0; i++) pas0[i] = c.pas[i];
            if (m.ttl == c.a->cfg.passive_rwl) add_to_passive(c, P);
            const uint32_t om[3] = {S, c.v, P};
            uint32_t r;
            if (!pick_random(c, act0, na0, om, 3, r)) {
                if (is_addable_epoch(c, m.epoch, P) && !has(act0, na0, P)) {
                    if (alive_of(*c.a, P)) {
                        add_to_active(c, P);
                        send_neighbor(c, P);
                    } else {                                   // `false -> State0`
                        c.np = np0;
                        for (uint32_t i = 0; i < np0; i++) c.pas[i] = pas0[i];
                    }
                }
            } else if (alive_of(*c.a, r)) {
                HvMsg* f = emit(c, r, HV_FORWARD_JOIN);
                if (f) { f->peer = P; f->epoch = m.epoch; f->ttl = m.ttl - 1; }
            }
        }
        break;
    }
    case HV_DISCONNECT: {                                                           // :1565-1617
        if (!is_valid_disconnect(c, m.did_e, m.did_c, P)) break;
        uint32_t pas0[32], np0 = c.np;
        for (uint32_t i = 0; i < np0; i++) pas0[i] = c.pas[i];
        sdel(c.act, c.na, P);
        add_to_passive(c, P);
        mput(c, recv_map(c), c.nrecv, P, m.did_e, m.did_c);
        if (c.na == 1) {
            const uint32_t om[2] = {c.v, P};
            uint32_t r;
            if (pick_random(c, pas0, np0, om, 2, r)) promote_peer(c, r);
        }
        break;
    }
    case HV_NEIGHBOR_REQUEST: {                                                     // :1619-1711
        uint32_t ack[kHvX];
        const uint32_t nack = select_exchange(c, ack);
        if (!m.prio && c.na >= c.a->cfg.active_max_size) {
            c.err |= 8u;                                       // 2-tuple neighbor_rejected: no clause
        } else if (is_addable_did(c, m.did_e, m.did_c, P)) {
            if (alive_of(*c.a, P)) {
                uint32_t e, cnt;
                get_current_id(c, P, e, cnt);
                HvMsg* x = emit(c, P, HV_NEIGHBOR_ACCEPTED);
                if (x) {
                    x->peer = c.v; x->did_e = e; x->did_c = cnt; x->nx = nack;
                    for (uint32_t i = 0; i < nack; i++) x->x[i] = ack[i];
                }
                add_to_active(c, P);
            }
        } else if (alive_of(*c.a, P)) {
            HvMsg* x = emit(c, P, HV_NEIGHBOR_REJECTED);
            if (x) {
                x->peer = c.v; x->nx = nack;
                for (uint32_t i = 0; i < nack; i++) x->x[i] = ack[i];
            }
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
            const uint32_t om[2] = {S, c.v};
            uint32_t r;
            if (pick_random(c, c.act, c.na, om, 2, r) && alive_of(*c.a, r)) {
                HvMsg* f = emit(c, r, HV_SHUFFLE);
                if (f) {
                    f->peer = c.v; f->ttl = m.ttl - 1; f->nx = m.nx;
                    for (uint32_t i = 0; i < m.nx; i++) f->x[i] = m.x[i];
                }
            }
        } else {
            for (uint32_t i = 0; i < c.np; i++) (void)draw64(c);     // shuffle(Passive, |Exchange|)
            const uint32_t k = c.np < m.nx ? c.np : m.nx;
            if (alive_of(*c.a, S)) {
                HvMsg* f = emit(c, S, HV_SHUFFLE_REPLY);
                if (f) {
                    f->peer = c.v; f->nx = k;
                    for (uint32_t i = 0; i < k; i++) f->x[i] = c.pas[i];
                }
            }
            merge_exchange(c, m.x, m.nx);
        }
        break;
    }
    default:
        break;
    }
}

__device__ __forceinline__ bool msg_less(const HvMsg& x, const HvMsg& y) {
    return x.src < y.src || (x.src == y.src && x.seq < y.seq);
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

__global__ __launch_bounds__(kBlock) void hv_process(HvArgs a) {
    const uint32_t v = blockIdx.x * kBlock + threadIdx.x;
    uint32_t ndraw = 0, err = 0, nproc = 0, act1 = 0;
    uint32_t sent[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (v < a.n) {
        const uint32_t lo = a.off[v], hi = a.off[v + 1];
        const bool up = alive_of(a, v);
        if (up && (hi > lo || a.timers)) {
            Ctx c;
            c.a = &a;
            c.v = v;
            const HvHead h = a.head[v];
            c.na = h.na; c.np = h.np; c.nsent = h.nsent; c.nrecv = h.nrecv; c.seq = h.seq; c.draws = h.draws;
            for (uint32_t i = 0; i < 8; i++) c.act[i] = a.act[(size_t)v * 8 + i];
            for (uint32_t i = 0; i < 32; i++) c.pas[i] = a.pas[(size_t)v * 32 + i];
            for (int i = 0; i < 10; i++) c.sent_cnt[i] = 0;
            c.ndraw = 0;
            c.err = 0;
            // sort the bucket by (src, seq): insertion sort of indices
            for (uint32_t i = lo + 1; i < hi; i++) {
                const uint32_t x = a.idx[i];
                const HvMsg& mx = a.in[x];
                uint32_t j = i;
                while (j > lo && msg_less(mx, a.in[a.idx[j - 1]])) { a.idx[j] = a.idx[j - 1]; j--; }
                a.idx[j] = x;
            }
            for (uint32_t i = lo; i < hi; i++) handle(c, a.in[a.idx[i]]);
            nproc = hi - lo;
            act1 = 1;
            if (a.timers & 1u) {                                   // random_promotion (:1046-1067)
                if (c.na < a.cfg.active_min_size) {
                    const uint32_t om[1] = {v};
                    uint32_t r;
                    if (pick_random(c, c.pas, c.np, om, 1, r)) promote_peer(c, r);
                }
            }
            if (a.timers & 2u) {                                   // passive_view_maintenance (:1078-1111)
                uint32_t ex[kHvX];
                const uint32_t nx = select_exchange(c, ex);
                const uint32_t om[1] = {v};
                uint32_t r;
                if (pick_random(c, c.act, c.na, om, 1, r) && alive_of(a, r)) {
                    HvMsg* f = emit(c, r, HV_SHUFFLE);
                    if (f) {
                        f->peer = v; f->ttl = a.cfg.active_rwl; f->nx = nx;
                        for (uint32_t i = 0; i < nx; i++) f->x[i] = ex[i];
                    }
                }
            }
            for (uint32_t i = 0; i < 8; i++) a.act[(size_t)v * 8 + i] = i < c.na ? c.act[i] : 0xFFFFFFFFu;
            for (uint32_t i = 0; i < 32; i++) a.pas[(size_t)v * 32 + i] = i < c.np ? c.pas[i] : 0xFFFFFFFFu;
            HvHead nh;
            nh.na = c.na; nh.np = c.np; nh.nsent = c.nsent; nh.nrecv = c.nrecv; nh.seq = c.seq; nh.draws = c.draws;
            a.head[v] = nh;
            ndraw = c.ndraw;
            err = c.err;
            for (int i = 0; i < 10; i++) sent[i] = c.sent_cnt[i];
        }
    }
    // counters: one atomic per wave per counter
    unsigned long long vals[14];
    for (int i = 1; i < 10; i++) vals[i] = sent[i];
    vals[10] = ndraw;
    vals[11] = 0;
    vals[12] = nproc;
    vals[13] = act1;
    for (int i = 1; i <= 13; i++) {
        if (i == 11) continue;
        unsigned long long x = vals[i];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
        if ((threadIdx.x & 63) == 0 && x) atomicAdd(&a.stats[i], x);
    }
    unsigned long long e = err;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) e |= __shfl_xor(e, o, 64);
    if ((threadIdx.x & 63) == 0 && e) atomicOr(&a.stats[11], e);
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
    hipError_t e;
    if ((e = hipMemsetAsync(a.cnt, 0, size_t(a.n) * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(a.cur, 0, size_t(a.n) * 4, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(hv_count, dim3(kStrideBlocks), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(hv_scan_blocks, dim3(nblk(a.n)), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(hv_scan_sums, dim3(1), dim3(1024), 0, s, a, nblk(a.n));
    hipLaunchKernelGGL(hv_scan_add, dim3(nblk(a.n)), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(hv_scatter, dim3(kStrideBlocks), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(hv_process, dim3(nblk(a.n)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace psim
