// ptdyn.hip -- configuration C3: the Plumtree server
// (src/partisan_plumtree_broadcast.erl) with the heartbeat handler, over the
// churning SCAMP v2 membership of scamp.hip, one gfx950 thread per vertex.
//
// Unlike the static-overlay engine (plumtree.hip), a vertex's peers change
// every round, so its Plumtree state is a small peer table (<= kPdTab ids)
// with one 128-bit mask per set over it: all_members, common_eagers,
// common_lazys and the root's eager and lazy sets (present iff the root's map
// entry exists).  The outstanding ETS rows {Peer, {Id, Mod, Round, Root}} are
// a per-vertex list in insertion order (several heartbeats may be in flight:
// a row of an older one is still re-announced), and the backend's timestamp
// ISet for the root is a 64-heartbeat window bitmap.  Messages are 24 B records in a queue bucketed by
// destination and sorted by (src, seq) per vertex, as in the SCAMP engine.
// A round, after the SCAMP round it follows:
//   1. the {update, Members} casts the manager fired this round
//      (partisan_plumtree_broadcast.erl:607-639), in order, as the set
//      deltas scamp.hip recorded: a new member -> common_eagers U New and
//      reset_peers/4 (:1320-1328); a removed one -> neighbors_down/2
//      (:910-951), which also deletes its outstanding rows;
//   2. the inbox (handle_cast clauses :565-605);
//   3. the lazy tick (every round): i_have to every outstanding peer that
//      is connected (:992-1030).
// A send needs a connection (partisan:cast_message -> do_send_message):
// the destination must be a member of the sender (its SCAMP partial view);
// otherwise it is dropped.
#include "psim_internal.h"
#include <cstdio>
#include "../../include/psim.h"

namespace psim {

namespace {

enum { PD_BROADCAST = 1, PD_PRUNE, PD_IHAVE, PD_IGNORED, PD_GRAFT };
enum { S_MEM = 0, S_CE, S_CL, S_EAG, S_LAZ, S_NSET };
static_assert(S_NSET == kPdSets, "mask layout");
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kPdStrideBlocks = 2048;

struct Ctx {
    const PdArgs* a;
    uint32_t v;
    PdHead h;
    uint32_t* tab;                 // row in HBM
    PdBits m[S_NSET];              // masks over the row
    PdRow* rows;                   // outstanding rows in HBM
    const uint32_t* pv;            // SCAMP partial view row
    uint32_t npv;
    unsigned long long sent;       // 12 bits per message kind 1..5 (kind k at bit 12 (k - 1): 60 bits)
    uint32_t dropped, deliv, err;
    WaveQ<PdMsg> q;                // this wave's send buffer (LDS)
};

__device__ __forceinline__ bool connected(const Ctx& c, uint32_t t) { return t != c.v && row_has(c.pv, c.npv, t); }

__device__ __forceinline__ void send_conn(Ctx& c, uint32_t t, uint32_t type, uint32_t mono, uint32_t round) {
    const PdArgs& a = *c.a;
    const uint32_t sh = 12u * (type - 1u);
    if (((c.sent >> sh) & 0xFFFull) == 0xFFFull) c.err |= 16u;   // a 13th bit would carry into the next kind
    else c.sent += 1ull << sh;
    wq_send(c.q, a.nout, a.out, a.out_cap, c.err, PdMsg{type, c.v, t, c.h.seq++, round, mono});
}
__device__ __forceinline__ void send(Ctx& c, uint32_t t, uint32_t type, uint32_t mono, uint32_t round) {
    if (!connected(c, t)) { c.dropped++; return; }
    send_conn(c, t, type, mono, round);
}

static_assert(kPdTab % 8 == 0, "row_find reads the peer table as quad pairs");
__device__ __forceinline__ int tab_find(const Ctx& c, uint32_t x) { return row_find(c.tab, c.h.ntab, x); }

// drop ids no set refers to (keeps the masks aligned with the row)
__device__ __forceinline__ void tab_compact(Ctx& c) {
    PdBits any = PdBits::none();
    #pragma unroll
    for (int k = 0; k < S_NSET; k++) any |= c.m[k];
    uint32_t w = 0;
    PdBits nm[S_NSET];
    #pragma unroll
    for (int k = 0; k < S_NSET; k++) nm[k] = PdBits::none();
    for (uint32_t i = 0; i < c.h.ntab; i++) {
        if (!any.test(i)) continue;
        c.tab[w] = c.tab[i];
        #pragma unroll
        for (int k = 0; k < S_NSET; k++)
            if (c.m[k].test(i)) nm[k] |= PdBits::one((int)w);
        w++;
    }
    c.h.ntab = w;
    #pragma unroll
    for (int k = 0; k < S_NSET; k++) c.m[k] = nm[k];
}

__device__ __forceinline__ int tab_insert(Ctx& c, uint32_t x) {
    const int f = tab_find(c, x);
    if (f >= 0) return f;
    if (c.h.ntab >= kPdTab) tab_compact(c);
    if (c.h.ntab >= kPdTab) { c.err |= 2u; return -1; }
    c.tab[c.h.ntab] = x;
    return (int)c.h.ntab++;
}

__device__ __forceinline__ PdBits bit(int i) { return PdBits::one(i); }
// pop the lowest member of b (b non-empty)
__device__ __forceinline__ int pop_low(PdBits& b) {
    if (b.w[0]) { const int i = __ffsll(b.w[0]) - 1; b.w[0] &= b.w[0] - 1; return i; }
    const int i = __ffsll(b.w[1]) - 1; b.w[1] &= b.w[1] - 1; return 64 + i;
}

// all_peers/3 materialised: set_peers/4 creates the root's map entries
__device__ __forceinline__ void ensure_root_sets(Ctx& c) {
    if (c.h.flags & 1u) return;
    c.m[S_EAG] = c.m[S_CE];
    c.m[S_LAZ] = c.m[S_CL];
    c.h.flags |= 1u;
}
__device__ __forceinline__ void add_eager(Ctx& c, const PdBits& b) {
    ensure_root_sets(c);
    c.m[S_EAG] |= b;
    c.m[S_LAZ] &= ~b;
}
__device__ __forceinline__ void add_lazy(Ctx& c, const PdBits& b) {
    ensure_root_sets(c);
    c.m[S_EAG] &= ~b;
    c.m[S_LAZ] |= b;
}
// x if f else y, blended by value: a select between two members' addresses
// would keep the whole context in scratch memory
__device__ __forceinline__ PdBits blend(bool f, const PdBits& x, const PdBits& y) {
    const unsigned long long k = f ? ~0ull : 0ull;
    return PdBits{{(x.w[0] & k) | (y.w[0] & ~k), (x.w[1] & k) | (y.w[1] & ~k)}};
}
__device__ __forceinline__ PdBits eager_now(const Ctx& c) { return blend(c.h.flags & 1u, c.m[S_EAG], c.m[S_CE]); }
__device__ __forceinline__ PdBits lazy_now(const Ctx& c) { return blend(c.h.flags & 1u, c.m[S_LAZ], c.m[S_CL]); }

// the backend's timestamp ISet for the root (partisan_plumtree_backend.erl
// is_stale/1 :229-244, add_timestamp): heartbeat serials dbase-63..dbase
__device__ __forceinline__ bool delivered(Ctx& c, uint32_t mono) {
    const uint32_t k = c.h.dbase - mono;
    if (mono > c.h.dbase || mono == 0) return false;
    if (k >= 64) { c.err |= 8u; return true; }
    return (c.h.dmask >> k) & 1ull;
}
__device__ __forceinline__ void mark_delivered(Ctx& c, uint32_t mono) {
    const uint32_t k = c.h.dbase - mono;
    if (k >= 64) { c.err |= 8u; return; }
    c.h.dmask |= 1ull << k;
}

// add_all_outstanding/5 (:1215-1219)
__device__ __forceinline__ void add_row(Ctx& c, uint32_t peer, uint32_t mono, uint32_t round) {
    if (c.h.nrow >= kPdRows) { c.err |= 4u; return; }
    c.rows[c.h.nrow++] = PdRow{peer, mono, round};
}
// ack_outstanding/5 (:1207-1211): ets:delete_object removes every identical row
__device__ __forceinline__ void ack_rows(Ctx& c, uint32_t peer, uint32_t mono, uint32_t round) {
    uint32_t w = 0;
    for (uint32_t i = 0; i < c.h.nrow; i++) {
        const PdRow r = c.rows[i];
        if (r.peer == peer && r.mono == mono && r.round == round) continue;
        if (w != i) c.rows[w] = r;
        w++;
    }
    c.h.nrow = w;
}

// eager_push/7 (:962-970) to eager peers -- From, schedule_lazy_push/6 (:974-988)
// The eager pushes test the connection rule on the member mask instead of
// scanning the partial view: after this round's {update, Members} casts are
// applied (pd_process step 1; pd_origin runs between rounds, after them),
// S_MEM holds exactly the manager's members -- the partial view the send
// rule reads (oracle/c3.c connected) -- so tab[i] is connected iff it is not
// this vertex and bit i of S_MEM is set.  -DPD_CONN_CHECK builds compare the
// two on every push and raise error bit 64 (PSIM_ESTATE) on a difference.
#ifndef PD_CONN_MASK
#define PD_CONN_MASK 1
#endif
__device__ __forceinline__ void push(Ctx& c, const PdBits& from_bit, uint32_t mono, uint32_t round) {
    PdBits e = eager_now(c) & ~from_bit;
#if PD_CONN_MASK
    while (e.any()) {
        const int i = pop_low(e);
        const uint32_t t = c.tab[i];
        const bool conn = t != c.v && c.m[S_MEM].test((uint32_t)i);
#ifdef PD_CONN_CHECK
        if (conn != connected(c, t)) c.err |= 64u;
#endif
        if (!conn) c.dropped++;
        else send_conn(c, t, PD_BROADCAST, mono, round);
    }
#else
    while (e.any()) send(c, c.tab[pop_low(e)], PD_BROADCAST, mono, round);
#endif
    PdBits l = lazy_now(c) & ~from_bit;
    while (l.any()) add_row(c, c.tab[pop_low(l)], mono, round);
}

__device__ __forceinline__ void handle(Ctx& c, const PdMsg& m) {
    const PdArgs& a = *c.a;
    switch (m.type) {
    case PD_BROADCAST: {                           // :571-578 -> handle_broadcast/8 :843-857
        const PdBits b = bit(tab_insert(c, m.src));
        if (!delivered(c, m.mono)) {               // merge/2: not stale -> add_timestamp
            mark_delivered(c, m.mono);
            if (m.mono == a.mono) c.h.myround = m.round + 1;
            c.deliv++;
            add_eager(c, b);
            push(c, b, m.mono, m.round + 1);
        } else {
            add_lazy(c, b);
            send(c, m.src, PD_PRUNE, 0, 0);
        }
        break;
    }
    case PD_PRUNE:                                 // :580-584
        add_lazy(c, bit(tab_insert(c, m.src)));
        break;
    case PD_IHAVE:                                 // :586-590 -> handle_ihave/7 :861-876
        if (delivered(c, m.mono)) {
            send(c, m.src, PD_IGNORED, m.mono, m.round);
        } else {
            send(c, m.src, PD_GRAFT, m.mono, m.round);
            add_eager(c, bit(tab_insert(c, m.src)));
        }
        break;
    case PD_IGNORED:                               // :592-598 ack_outstanding/5
        ack_rows(c, m.src, m.mono, m.round);
        break;
    case PD_GRAFT:                                 // :600-605 -> handle_graft/7 :880-906
        if (delivered(c, m.mono)) {                // Mod:graft -> {ok, M} (one epoch: never stale)
            add_eager(c, bit(tab_insert(c, m.src)));
            send(c, m.src, PD_BROADCAST, m.mono, m.round);
        }                                          // {error, not_found}: logged only
        break;
    default:
        break;
    }
}

// {update, Members} as a set delta (:607-639)
__device__ __forceinline__ void apply_update(Ctx& c, uint32_t added, uint32_t removed) {
    if (added != kNone) {
        const PdBits b = bit(tab_insert(c, added));
        c.m[S_MEM] |= b;
        if (added != c.v) c.m[S_CE] |= b;          // common_eagers U New, minus self (reset_peers)
        c.m[S_EAG] = PdBits::none();                 // reset_peers: the per-root maps are dropped
        c.m[S_LAZ] = PdBits::none();
        c.h.flags &= ~1u;
    }
    if (removed != kNone) {                        // neighbors_down/2
        const int i = tab_find(c, removed);
        if (i >= 0)
            #pragma unroll
            for (int k = 0; k < S_NSET; k++) c.m[k] &= ~bit(i);
        uint32_t w = 0;                            // ... and deletes the outstanding rows to it
        for (uint32_t j = 0; j < c.h.nrow; j++) {
            const PdRow r = c.rows[j];
            if (r.peer == removed) continue;
            if (w != j) c.rows[w] = r;
            w++;
        }
        c.h.nrow = w;
    }
}

__device__ __forceinline__ bool msg_less(const PdMsg& x, const PdMsg& y) {
    return x.src < y.src || (x.src == y.src && x.seq < y.seq);
}
__device__ __forceinline__ uint32_t n_in(const PdArgs& a) { return *a.nin < a.out_cap ? *a.nin : a.out_cap; }

__global__ __launch_bounds__(kBlock) void pd_count(PdArgs a) {
    const uint32_t k = n_in(a);
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < k; i += kPdStrideBlocks * kBlock) {
        const uint32_t d = a.in[i].dst - a.v_lo;
        if (d < a.n) atomicAdd(&a.cnt[d], 1u);
        else if (a.stats) atomicOr(&a.stats[9], 32ull);   // a record off this range: reported, never indexed
    }
}
__global__ __launch_bounds__(kBlock) void pd_scan_blocks(PdArgs a) {
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
__global__ __launch_bounds__(1024) void pd_scan_sums(PdArgs a, uint32_t nb) {
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x, per = (nb + 1023) / 1024;
    const uint32_t lo = t * per, hi = min(nb, lo + per);
    uint32_t s = 0;
    for (uint32_t b = lo; b < hi; b++) s += a.bsum[b];
    part[t] = s;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
        const uint32_t y = t >= o ? part[t - o] : 0u;
        __syncthreads();
        part[t] += y;
        __syncthreads();
    }
    uint32_t run = part[t] - s;
    for (uint32_t b = lo; b < hi; b++) { const uint32_t x = a.bsum[b]; a.bsum[b] = run; run += x; }
    if (t == 1023) a.off[a.n] = part[1023];
}
__global__ __launch_bounds__(kBlock) void pd_scan_add(PdArgs a) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < a.n) a.off[i] += a.bsum[blockIdx.x];
}
__global__ __launch_bounds__(kBlock) void pd_scatter(PdArgs a) {
    const uint32_t k = n_in(a);
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < k; i += kPdStrideBlocks * kBlock) {
        const uint32_t d = a.in[i].dst - a.v_lo;
        if (d < a.n) a.idx[a.off[d] + atomicAdd(&a.cur[d], 1u)] = i;
    }
}

__device__ __forceinline__ void load(Ctx& c, const PdArgs& a, uint32_t v) {
    c.a = &a;
    c.v = v;
    c.h = a.head[v];
    c.tab = a.tab + (size_t)v * kPdTab;
    #pragma unroll
    for (int k = 0; k < S_NSET; k++) c.m[k] = a.mask[(size_t)v * S_NSET + k];
    c.rows = a.rows + (size_t)v * kPdRows;
    if (a.mono > c.h.dbase) {                      // slide the delivered window to the newest serial
        const uint32_t d = a.mono - c.h.dbase;
        c.h.dmask = d >= 64 ? 0ull : c.h.dmask << d;
        c.h.dbase = a.mono;
    }
    c.pv = a.pv + (size_t)v * kScPv;
    c.npv = a.sch[v].npv;
    c.sent = 0;
    c.dropped = c.deliv = c.err = 0;
}
__device__ __forceinline__ void store(const Ctx& c) {
    const PdArgs& a = *c.a;
    a.head[c.v] = c.h;
    #pragma unroll
    for (int k = 0; k < S_NSET; k++) a.mask[(size_t)c.v * S_NSET + k] = c.m[k];
}

__device__ __forceinline__ void reduce_stats(const PdArgs& a, const unsigned long long* vals) {
#pragma unroll
    for (int i = 1; i < kPdNStat; i++) {
        unsigned long long x = vals[i];
        if (i == 9) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o, 64);
            if ((threadIdx.x & 63) == 0 && x) atomicOr(&a.stats[(blockIdx.x % kRoundStatShards) * kPdNStat + i], x);
            continue;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
        if ((threadIdx.x & 63) == 0 && x) atomicAdd(&a.stats[(blockIdx.x % kRoundStatShards) * kPdNStat + i], x);
    }
}

// stats: [1..5] sent by kind, 6 dropped, 7 delivered_new, 8 active, 9 error bits,
// 10 updates applied, 11 delivered_live, 12 live, 13 outstanding rows to connected live peers
#ifdef C3_PROF
// [0..5) cycles of load+updates / sort / inbox / lazy tick / store (per wave),
// [5..11) messages handled by kind, [11] i_have rows walked, [12] waves,
// [13] load cycles alone, [14] update events
__device__ unsigned long long g_pd_prof[kProfSlots];
#endif

__global__ __launch_bounds__(kBlock) void pd_process(PdArgs a) {
    __shared__ PdMsg qbuf[kBlock / 64][kWq];
    __shared__ uint32_t qn[kBlock / 64];
    const uint32_t v = blockIdx.x * kBlock + threadIdx.x;
    const WaveQ<PdMsg> q{qbuf[threadIdx.x >> 6], &qn[threadIdx.x >> 6]};
    wq_init(q.n);
    uint32_t qerr = 0;
    unsigned long long vals[kPdNStat];
#pragma unroll
    for (int i = 0; i < kPdNStat; i++) vals[i] = 0;
    if (v < a.n && a.alive[v]) {
#ifdef C3_PROF
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        unsigned long long kinds = 0;
#endif
        Ctx c;
        load(c, a, v);
        c.q = q;
#ifdef C3_PROF
        const unsigned long long tl = __builtin_amdgcn_s_memtime();
#endif
        const bool fresh = (c.h.flags & 2u) != 0;
        c.h.flags &= ~2u;
        // 1. the manager's update casts of this round, in order
        const uint32_t ne = a.ev_cnt ? a.ev_cnt[v] : 0u;
        for (uint32_t i = 0; i < ne; i++) {
            const uint2 e = a.ev[(size_t)v * kScEv + i];
            apply_update(c, e.x, e.y);
        }
        vals[10] = ne;
#ifdef C3_PROF
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
#endif
        // 2. the inbox in (src, seq) order (a restarted vertex drops it)
        const uint32_t lo = a.off[v], hi = a.off[v + 1];
        if (!fresh && hi > lo) {
            for (uint32_t i = lo + 1; i < hi; i++) {
                const uint32_t x = a.idx[i];
                const PdMsg mx = a.in[x];
                uint32_t j = i;
                while (j > lo && msg_less(mx, a.in[a.idx[j - 1]])) { a.idx[j] = a.idx[j - 1]; j--; }
                a.idx[j] = x;
            }
        }
#ifdef C3_PROF
        const unsigned long long t2 = __builtin_amdgcn_s_memtime();
#endif
        if (!fresh && hi > lo) {
            for (uint32_t i = lo; i < hi; i++) {
#ifdef C3_PROF
                kinds += 1ull << (10 * (a.in[a.idx[i]].type % 6));
#endif
                handle(c, a.in[a.idx[i]]);
            }
            vals[8] = 1;
        }
#ifdef C3_PROF
        const unsigned long long t3 = __builtin_amdgcn_s_memtime();
#endif
        // 3. handle_info(lazy_tick): send_lazy/0, rows persist
        unsigned long long live_rows = 0;
        const uint32_t nr = c.h.nrow;
        for (uint32_t i = 0; i < nr; i++) {
            const PdRow r = c.rows[i];
            if (!a.alive[r.peer] || !connected(c, r.peer)) continue;
            live_rows++;
            if (a.tick) send(c, r.peer, PD_IHAVE, r.mono, r.round);
        }
#ifdef C3_PROF
        const unsigned long long t4 = __builtin_amdgcn_s_memtime();
#endif
        if (c.h.ntab > kPdTab - 8) tab_compact(c);
        store(c);
#ifdef C3_PROF
        const unsigned long long t5 = __builtin_amdgcn_s_memtime();
        prof_add(g_pd_prof, 0, t1 - t0);
        prof_add(g_pd_prof, 1, t2 - t1);
        prof_add(g_pd_prof, 2, t3 - t2);
        prof_add(g_pd_prof, 3, t4 - t3);
        prof_add(g_pd_prof, 4, t5 - t4);
        prof_add(g_pd_prof, 12, 1);
        prof_add(g_pd_prof, 13, tl - t0);
        atomicAdd(&g_pd_prof[11], (unsigned long long)nr);
        atomicAdd(&g_pd_prof[14], (unsigned long long)ne);
        for (int k = 0; k < 6; k++)
            if ((kinds >> (10 * k)) & 1023ull) atomicAdd(&g_pd_prof[5 + k], (kinds >> (10 * k)) & 1023ull);
#endif
#pragma unroll
        for (int i = 1; i <= 5; i++) vals[i] = (c.sent >> (12 * (i - 1))) & 0xFFFull;
        vals[6] = c.dropped;
        vals[7] = c.deliv;
        vals[9] = c.err;
        vals[11] = delivered(c, a.mono);
        vals[12] = 1;
        vals[13] = live_rows;
    }
    wq_flush(q, a.nout, a.out, a.out_cap, qerr);          // every lane of the wave: what is still staged
    vals[9] |= qerr;
    if (v < a.n) {          // zero for the next round's bucket pass (instead of host fills)
        a.cnt[v] = 0;
        a.cur[v] = 0;
    }
    reduce_stats(a, vals);
}

// heartbeat at the root: the backend's add_timestamp + the plumtree cast
// {broadcast, Id, Payload, Mod} (:565-569) -> eager_push/4, schedule_lazy_push/3
__global__ void pd_origin(PdArgs a, uint32_t root) {
    // one thread sends; the wave's 64 lanes move its buffer (wq_flush)
    __shared__ PdMsg qbuf[kWq];
    __shared__ uint32_t qn;
    if (blockIdx.x != 0 || threadIdx.x >= 64) return;
    wq_init(&qn);
    const WaveQ<PdMsg> q{qbuf, &qn};
    uint32_t err = 0;
    if (threadIdx.x == 0) {
        Ctx c;
        load(c, a, root);
        c.q = q;
        mark_delivered(c, a.mono);
        c.h.myround = 0;
        push(c, PdBits::none(), a.mono, 0u);
        store(c);
        err = c.err;
        atomicAdd(&a.stats[6], (unsigned long long)c.dropped);
    }
    wq_flush(q, a.nout, a.out, a.out_cap, err);
    if (threadIdx.x == 0 && err) atomicOr(&a.stats[9], (unsigned long long)err);   // lane 0 holds every bit
}

// start_link/0 with members = {self}: fresh state (every vertex, or a crash list)
__global__ __launch_bounds__(kBlock) void pd_init(PdArgs a, const uint32_t* __restrict__ list, uint32_t k) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= (list ? k : a.n)) return;
    const uint32_t v = list ? list[i] : i;
    PdHead h = list ? a.head[v] : PdHead{};
    h.ntab = 1;
    h.flags = list ? 2u : 0u;        // restarted: its inbox holds messages for the old incarnation
    h.myround = 0;
    h.dbase = a.mono;
    h.dmask = 0;
    h.nrow = 0;
    if (!list) h.seq = 0;
    a.head[v] = h;
    a.tab[(size_t)v * kPdTab] = v;
    a.mask[(size_t)v * S_NSET + S_MEM] = PdBits::one(0);   // all_members = {self}
    for (int m = 1; m < S_NSET; m++) a.mask[(size_t)v * S_NSET + m] = PdBits::none();
}

inline uint32_t nblk(uint32_t n) { return (n + kBlock - 1) / kBlock; }

}  // namespace

hipError_t launch_pd_init(const PdArgs& a, const uint32_t* list, uint32_t k, hipStream_t s) {
    const uint32_t m = list ? k : a.n;
    if (m) hipLaunchKernelGGL(pd_init, dim3(nblk(m)), dim3(kBlock), 0, s, a, list, k);
    return hipGetLastError();
}

hipError_t launch_pd_origin(const PdArgs& a, uint32_t root, hipStream_t s) {
    hipLaunchKernelGGL(pd_origin, dim3(1), dim3(64), 0, s, a, root);
    return hipGetLastError();
}

// zeroed: cnt / cur are known zero (pd_process leaves them so for the next round)
hipError_t launch_pd_bucket(const PdArgs& a, hipStream_t s, bool zeroed) {
    hipError_t e;
    if (!zeroed && (e = hipMemsetAsync(a.cnt, 0, size_t(a.n) * 4, s)) != hipSuccess) return e;
    if (!zeroed && (e = hipMemsetAsync(a.cur, 0, size_t(a.n) * 4, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(pd_count, dim3(kPdStrideBlocks), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(pd_scan_blocks, dim3(nblk(a.n)), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(pd_scan_sums, dim3(1), dim3(1024), 0, s, a, nblk(a.n));
    hipLaunchKernelGGL(pd_scan_add, dim3(nblk(a.n)), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(pd_scatter, dim3(kPdStrideBlocks), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

// the round's stats rows and outgoing count zeroed: one launch instead of two fills
__global__ __launch_bounds__(kBlock) void pd_prep(PdArgs a) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < kRoundStatShards * kPdNStat) a.stats[i] = 0ull;
    if (i == 0) *a.nout = 0u;
}

hipError_t launch_pd_round(const PdArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(pd_prep, dim3(nblk(kRoundStatShards * kPdNStat)), dim3(kBlock), 0, s, a);
    const hipError_t e = launch_pd_bucket(a, s, true);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(pd_process, dim3(nblk(a.n)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace psim

// ---------------------------------------------------------------------------
// host side: the psim_c3_* entry points of include/psim.h
// ---------------------------------------------------------------------------
#include <algorithm>
#include <cstring>
#include <vector>

using namespace psim;

namespace {

struct PdState : ModuleState {
    uint32_t n = 0, cap = 0, mono = 0, root = 0;
    PdHead* head = nullptr;
    uint32_t* tab = nullptr;
    PdBits* mask = nullptr;
    unsigned long long* stats = nullptr;
    PdRow* rows = nullptr;
    PdMsg* msg[2] = {nullptr, nullptr};
    uint32_t* nmsg = nullptr;
    uint32_t *cnt = nullptr, *cur = nullptr, *off = nullptr, *idx = nullptr, *bsum = nullptr;
    uint32_t par = 0;
    uint64_t round = 0;
    unsigned long long* h_stats = nullptr;   // pinned: a round's stats rows
    // psim_c3_run: the stats rows of every round of one call (heartbeat,
    // SCAMP, Plumtree) on the device and their pinned mirror, the call's
    // crash lists and sorted calls (pinned staging, one upload to d_in), and
    // four timing events per round
    unsigned long long *h_run = nullptr, *d_run = nullptr;
    size_t run_rounds = 0;
    uint32_t *h_in = nullptr, *d_in = nullptr;
    size_t in_cap = 0;
    bool run_pending = false;                // a run returned early: its copies may still be queued
    std::vector<hipEvent_t> run_ev;
    ~PdState() override {
        void* p[] = {head, tab, mask, rows, stats, msg[0], msg[1], nmsg, cnt, cur, off, idx, bsum, d_run, d_in};
        for (void* x : p)
            if (x) (void)hipFree(x);
        if (h_stats) (void)hipHostFree(h_stats);
        if (h_run) (void)hipHostFree(h_run);
        if (h_in) (void)hipHostFree(h_in);
        for (hipEvent_t e : run_ev) (void)hipEventDestroy(e);
    }
};

PdState* pd_of(psim_handle* h) { return static_cast<PdState*>(handle_module(h, MOD_PTDYN)); }

#define PDCHK(h, x)                                                                         \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess)                                                               \
            return handle_fail((h), PSIM_EHIP, "%s failed: %s", #x, hipGetErrorString(e_)); \
    } while (0)

bool pd_alloc(void** p, size_t bytes) {
    return alloc_zero(p, bytes);
}

int pd_args(psim_handle* h, const PdState& s, PdArgs& a) {
    ScView sv;
    const int rc = scamp_view(h, &sv, true);
    if (rc) return rc;
    a = PdArgs{};
    a.n = s.n; a.mono = s.mono; a.tick = 1;
    a.alive = sv.alive; a.pv = sv.pv; a.sch = sv.head; a.ev_cnt = sv.ev_cnt; a.ev = sv.ev;
    a.head = s.head; a.tab = s.tab; a.mask = s.mask; a.rows = s.rows;
    a.in = s.msg[s.par]; a.nin = s.nmsg + s.par;
    a.out = s.msg[s.par ^ 1]; a.nout = s.nmsg + (s.par ^ 1);
    a.out_cap = s.cap;
    a.cnt = s.cnt; a.cur = s.cur; a.off = s.off; a.idx = s.idx; a.bsum = s.bsum;
    a.stats = s.stats;
    return PSIM_OK;
}

int pd_check(psim_handle* h, unsigned long long err, uint64_t round) {
    if (err & 1ull) return handle_fail(h, PSIM_EOVERFLOW, "c3 round %llu: plumtree message queue full", (unsigned long long)round);
    if (err & 2ull) return handle_fail(h, PSIM_EOVERFLOW, "c3 round %llu: a peer table exceeded %u ids",
                                       (unsigned long long)round, kPdTab);
    if (err & 4ull) return handle_fail(h, PSIM_EOVERFLOW, "c3 round %llu: a vertex exceeded %u outstanding rows",
                                       (unsigned long long)round, kPdRows);
    if (err & 8ull) return handle_fail(h, PSIM_EOVERFLOW, "c3 round %llu: a heartbeat older than 64 serials is still in flight",
                                       (unsigned long long)round);
    if (err & 16ull) return handle_fail(h, PSIM_EOVERFLOW, "c3 round %llu: a vertex sent more than 4095 messages of one kind",
                                        (unsigned long long)round);
    if (err & 32ull) return handle_fail(h, PSIM_EHIP, "c3 round %llu: a message record addressed off the cluster",
                                        (unsigned long long)round);
    if (err & 64ull) return handle_fail(h, PSIM_ESTATE, "c3 round %llu: member mask and partial view disagree "
                                        "(PD_CONN_CHECK)", (unsigned long long)round);
    return PSIM_OK;
}

}  // namespace

extern "C" {

int psim_c3_setup(psim_handle* h, uint32_t n, uint32_t c, uint32_t periodic_rounds) {
    if (!h) return PSIM_EINVAL;
    int rc = psim_scamp_setup(h, n, 2, c, periodic_rounds);
    if (rc) return rc;
    ScView sv;
    rc = scamp_view(h, &sv, true);
    if (rc) return rc;
    ModuleState*& slot = handle_module(h, MOD_PTDYN);
    delete slot;
    slot = nullptr;
    PdState* s = new PdState();
    s->n = n;
    s->cap = (uint32_t)std::min<uint64_t>(16ull * n + 4096, 0xFFFFFFF0ull);
    const size_t N = n;
    const uint32_t nb = (n + kBlock - 1) / kBlock;
    const bool ok = pd_alloc((void**)&s->head, N * sizeof(PdHead)) && pd_alloc((void**)&s->tab, N * kPdTab * 4) &&
                    pd_alloc((void**)&s->mask, N * kPdSets * sizeof(PdBits)) &&
                    pd_alloc((void**)&s->rows, N * kPdRows * sizeof(PdRow)) && pd_alloc((void**)&s->stats, kRoundStatShards * kPdNStat * 8) &&
                    pd_alloc((void**)&s->msg[0], size_t(s->cap) * sizeof(PdMsg)) &&
                    pd_alloc((void**)&s->msg[1], size_t(s->cap) * sizeof(PdMsg)) && pd_alloc((void**)&s->nmsg, 16) &&
                    pd_alloc((void**)&s->cnt, N * 4) && pd_alloc((void**)&s->cur, N * 4) &&
                    pd_alloc((void**)&s->off, (N + 1) * 4) && pd_alloc((void**)&s->idx, size_t(s->cap) * 4) &&
                    pd_alloc((void**)&s->bsum, size_t(nb) * 4);
    if (!ok) {
        delete s;
        return handle_fail(h, PSIM_ENOMEM, "c3 plumtree state for n=%u", n);
    }
    slot = s;
    PdArgs a;
    rc = pd_args(h, *s, a);
    if (rc) return rc;
    PDCHK(h, launch_pd_init(a, nullptr, 0, handle_stream(h)));
    PDCHK(h, hipStreamSynchronize(handle_stream(h)));
    return PSIM_OK;
}

int psim_c3_join(psim_handle* h, const uint32_t* v, const uint32_t* contact, size_t k) {
    return psim_scamp_join(h, v, contact, k);
}

int psim_c3_crash(psim_handle* h, const uint32_t* v, size_t k) {
    if (!h || (k && !v)) return PSIM_EINVAL;
    PdState* s = pd_of(h);
    if (!s) return handle_fail(h, PSIM_ESTATE, "psim_c3_setup not called");
    int rc = scamp_crash_list(h, v, k);     // validates the list, uploads it, restarts the SCAMP side
    if (rc || !k) return rc;
    ScView sv;
    rc = scamp_view(h, &sv, true);
    if (rc) return rc;
    PdArgs a;
    rc = pd_args(h, *s, a);
    if (rc) return rc;
    // the same device list, on the same stream: nothing is copied twice and nothing waits
    PDCHK(h, launch_pd_init(a, sv.list, (uint32_t)k, handle_stream(h)));
    return PSIM_OK;
}

int psim_c3_heartbeat(psim_handle* h, uint32_t root, uint32_t* mono_out) {
    if (!h) return PSIM_EINVAL;
    PdState* s = pd_of(h);
    if (!s) return handle_fail(h, PSIM_ESTATE, "psim_c3_setup not called");
    if (root >= s->n) return PSIM_EINVAL;
    s->mono++;
    s->root = root;
    PdArgs a;
    int rc = pd_args(h, *s, a);
    if (rc) return rc;
    a.out = s->msg[s->par];          // the origin's pushes are read by the next round
    a.nout = s->nmsg + s->par;
    PDCHK(h, hipMemsetAsync(s->stats, 0, kRoundStatShards * kPdNStat * 8, handle_stream(h)));
    PDCHK(h, launch_pd_origin(a, root, handle_stream(h)));
    unsigned long long raw[kRoundStatShards * kPdNStat], r[kPdNStat];
    PDCHK(h, hipMemcpyAsync(raw, s->stats, sizeof raw, hipMemcpyDeviceToHost, handle_stream(h)));
    PDCHK(h, hipStreamSynchronize(handle_stream(h)));
    fold_stat_shards(raw, r, kPdNStat, 9);
    if (mono_out) *mono_out = s->mono;
    return pd_check(h, r[9], s->round);
}

// psim_c3_run: the per-round counters of a Plumtree round from its stats rows
static void pd_fill(const PdState& s, const unsigned long long* r, float ms, psim_c3_stats* o) {
    for (int k = 1; k <= 5; k++) o->pt_sent[k] = r[k];
    o->pt_sent[0] = 0;
    o->pt_dropped = r[6];
    o->delivered_new = r[7];
    o->active = r[8];
    o->updates = r[10];
    o->delivered_live = r[11];
    o->live = r[12];
    o->outstanding_live = r[13];
    uint64_t msgs = 0;
    for (int k = 1; k <= 5; k++) msgs += r[k];
    o->pt_algo_bytes = 48ull * msgs + 24ull * msgs + 12ull * s.n + 64ull * r[12];
    o->pt_kernel_ms = ms;
}

int psim_c3_step(psim_handle* h, uint32_t rounds, psim_c3_stats* out, size_t cap) {
    if (!h) return PSIM_EINVAL;
    PdState* s = pd_of(h);
    if (!s) return handle_fail(h, PSIM_ESTATE, "psim_c3_setup not called");
    const hipStream_t st = handle_stream(h);
    if (!s->h_stats && hipHostMalloc((void**)&s->h_stats, kRoundStatShards * kPdNStat * 8) != hipSuccess) {
        s->h_stats = nullptr;
        return handle_fail(h, PSIM_ENOMEM, "c3: pinned stats rows");
    }
    for (uint32_t i = 0; i < rounds; i++) {
        psim_c3_stats* o = out && i < cap ? &out[i] : nullptr;
        // the SCAMP round and the Plumtree round that reads its updates are
        // enqueued back to back and the host waits once for both; a SCAMP
        // error is still reported first (the handle's C3 state is then spent)
        int rc = scamp_round_launch(h);
        if (rc) return rc;
        PdArgs a;
        rc = pd_args(h, *s, a);
        if (rc) return rc;
        PDCHK(h, hipEventRecord(handle_event(h, 2), st));
        PDCHK(h, launch_pd_round(a, st));
        PDCHK(h, hipEventRecord(handle_event(h, 3), st));
        unsigned long long r[kPdNStat];
        PDCHK(h, hipMemcpyAsync(s->h_stats, s->stats, kRoundStatShards * kPdNStat * 8, hipMemcpyDeviceToHost, st));
        PDCHK(h, handle_wait(h));
        rc = scamp_round_finish(h, o ? &o->scamp : nullptr);
        if (rc) return rc;
        fold_stat_shards(s->h_stats, r, kPdNStat, 9);
#ifdef C3_PROF
        {
            static unsigned long long tot[kProfSlots];
            unsigned long long x[kProfSlots];
            PDCHK(h, hipMemcpyFromSymbol(x, HIP_SYMBOL(g_pd_prof), sizeof x));
            const unsigned long long z[kProfSlots] = {};
            PDCHK(h, hipMemcpyToSymbol(HIP_SYMBOL(g_pd_prof), z, sizeof z));
            fprintf(stderr, "pd_prof");
            for (int i = 0; i < kProfSlots; i++) fprintf(stderr, " %llu", tot[i] += x[i]);
            fprintf(stderr, "\n");
        }
#endif
        float ms = 0.f;
        PDCHK(h, hipEventElapsedTime(&ms, handle_event(h, 2), handle_event(h, 3)));
        s->par ^= 1u;
        s->round++;
        rc = pd_check(h, r[9], s->round);
        if (rc) return rc;
        if (o) pd_fill(*s, r, ms, o);
    }
    return PSIM_OK;
}

// Rounds of churn in one call (include/psim.h): round i is, in this order,
// the heartbeat at hb_root when hb_every && i % hb_every == 0, the crash list
// crash_v[crash_off[i], crash_off[i+1]), the joins join_v / join_c over
// [join_off[i], join_off[i+1]), then one psim_c3_step round -- exactly the
// calls psim_c3_heartbeat / crash / join / step would make, enqueued on the
// handle's stream with no wait between rounds.  The crash lists and sorted
// calls of every kC3Block rounds travel in one upload, each round's stats
// rows stay in a device row of their own, and the rows come back in one copy
// after the last round: the per-round work on the stream is the kernels
// alone.  A bad list fails the call at its round (the rounds before it were
// run); the first failing round's error is returned, as the per-round calls
// would have (the handle's C3 state is then spent).
int psim_c3_run(psim_handle* h, uint32_t rounds, const uint32_t* crash_off, const uint32_t* crash_v,
                const uint32_t* join_off, const uint32_t* join_v, const uint32_t* join_c, uint32_t hb_every,
                uint32_t hb_root, psim_c3_stats* out, size_t cap) {
    if (!h || (rounds && (!crash_off || !join_off))) return PSIM_EINVAL;
    PdState* s = pd_of(h);
    if (!s) return handle_fail(h, PSIM_ESTATE, "psim_c3_setup not called");
    if (hb_every && hb_root >= s->n) return handle_fail(h, PSIM_EINVAL, "heartbeat root %u >= n %u", hb_root, s->n);
    if (scamp_calls_pending(h))
        return handle_fail(h, PSIM_ESTATE, "c3 run: %zu joins made since the last round (step first, or pass them "
                           "in round 0's lists)", scamp_calls_pending(h));
    if (!rounds) return PSIM_OK;
    size_t words = 0;
    for (uint32_t i = 0; i < rounds; i++) {
        if (crash_off[i + 1] < crash_off[i] || join_off[i + 1] < join_off[i])
            return handle_fail(h, PSIM_EINVAL, "round %u: decreasing list offsets", i);
        if ((crash_off[i + 1] > crash_off[i] && !crash_v) || (join_off[i + 1] > join_off[i] && (!join_v || !join_c)))
            return PSIM_EINVAL;
    }
    words = size_t(crash_off[rounds] - crash_off[0]) + 2ull * (join_off[rounds] - join_off[0]);
    const hipStream_t st = handle_stream(h);
    if (s->run_pending) {                         // the staging below may be refilled or freed
        PDCHK(h, hipStreamSynchronize(st));
        s->run_pending = false;
    }
    constexpr size_t kSc = kRoundStatShards * 16, kPd = kRoundStatShards * kPdNStat;   // u64 per stats row
    constexpr size_t kRow = 2 * kPd + kSc;                                               // heartbeat, SCAMP, Plumtree
    if (rounds > s->run_rounds) {
        if (s->h_run) (void)hipHostFree(s->h_run);
        if (s->d_run) (void)hipFree(s->d_run);
        s->h_run = s->d_run = nullptr;
        s->run_rounds = 0;
        if (hipHostMalloc((void**)&s->h_run, size_t(rounds) * kRow * 8) != hipSuccess) {
            s->h_run = nullptr;
            return handle_fail(h, PSIM_ENOMEM, "c3: pinned stats rows for %u rounds", rounds);
        }
        if (!pd_alloc((void**)&s->d_run, size_t(rounds) * kRow * 8))
            return handle_fail(h, PSIM_ENOMEM, "c3: device stats rows for %u rounds", rounds);
        s->run_rounds = rounds;
    }
    if (words > s->in_cap) {
        if (s->h_in) (void)hipHostFree(s->h_in);
        if (s->d_in) (void)hipFree(s->d_in);
        s->h_in = s->d_in = nullptr;
        s->in_cap = 0;
        if (hipHostMalloc((void**)&s->h_in, words * 4) != hipSuccess) {
            s->h_in = nullptr;
            return handle_fail(h, PSIM_ENOMEM, "c3: pinned staging for %zu list words", words);
        }
        if (!pd_alloc((void**)&s->d_in, words * 4)) return handle_fail(h, PSIM_ENOMEM, "c3: %zu list words", words);
        s->in_cap = words;
    }
    while (s->run_ev.size() < 4ull * rounds) {
        hipEvent_t e;
        PDCHK(h, hipEventCreate(&e));
        s->run_ev.push_back(e);
    }
    // rounds go out in blocks of kC3Block: a block's lists are checked and
    // staged (round i's crash list at cpos[i], its sorted calls -- vertices,
    // then targets -- at jpos[i]) and uploaded in one copy, then its rounds
    // are enqueued; the host stages the next block while the device runs
    // this one.  Segments never overlap, so no upload waits for another.
    constexpr uint32_t kC3Block = 4;
    std::vector<size_t> cpos(rounds), jpos(rounds);
    std::vector<uint64_t> sc_round(rounds);
    std::vector<uint8_t> beat(rounds, 0);
    size_t w = 0;
    s->run_pending = true;
    PDCHK(h, hipMemsetAsync(s->d_run, 0, size_t(rounds) * kRow * 8, st));
    for (uint32_t b0 = 0; b0 < rounds; b0 += kC3Block) {
        const uint32_t b1 = std::min(rounds, b0 + kC3Block);
        const size_t w0 = w;
        for (uint32_t i = b0; i < b1; i++) {
            const size_t kc = crash_off[i + 1] - crash_off[i], kj = join_off[i + 1] - join_off[i];
            cpos[i] = w;
            if (kc) {
                int rc = scamp_check_crash(h, crash_v + crash_off[i], kc);
                if (rc) return rc;
                memcpy(s->h_in + w, crash_v + crash_off[i], kc * 4);
                w += kc;
            }
            jpos[i] = w;
            if (kj) {
                int rc = scamp_check_calls(h, join_v + join_off[i], join_c + join_off[i], kj, s->h_in + w);
                if (rc) return rc;
                w += 2 * kj;
            }
        }
        if (w > w0) PDCHK(h, hipMemcpyAsync(s->d_in + w0, s->h_in + w0, (w - w0) * 4, hipMemcpyHostToDevice, st));
        for (uint32_t i = b0; i < b1; i++) {
            unsigned long long* row = s->d_run + size_t(i) * kRow;
            PdArgs a;
            int rc;
            if (hb_every && i % hb_every == 0) {      // psim_c3_heartbeat (its stats row was zeroed above)
                s->mono++;
                s->root = hb_root;
                rc = pd_args(h, *s, a);
                if (rc) return rc;
                a.out = s->msg[s->par];
                a.nout = s->nmsg + s->par;
                a.stats = row;
                PDCHK(h, launch_pd_origin(a, hb_root, st));
                beat[i] = 1;
            }
            const size_t kc = crash_off[i + 1] - crash_off[i], kj = join_off[i + 1] - join_off[i];
            if (kc) {                                 // psim_c3_crash: both processes restart
                rc = scamp_crash_dev(h, s->d_in + cpos[i], kc);
                if (rc) return rc;
                rc = pd_args(h, *s, a);
                if (rc) return rc;
                PDCHK(h, launch_pd_init(a, s->d_in + cpos[i], (uint32_t)kc, st));
            }
            hipEvent_t* ev = s->run_ev.data() + 4ull * i;
            ScLaunch o;
            o.e0 = ev[0];
            o.e1 = ev[1];
            o.d_stats = row + kPd;
            o.d_calls = kj ? s->d_in + jpos[i] : nullptr;
            o.d_ncalls = (uint32_t)kj;
            rc = scamp_round_launch_to(h, o, &sc_round[i]);
            if (rc) return rc;
            rc = pd_args(h, *s, a);
            if (rc) return rc;
            a.stats = row + kPd + kSc;
            PDCHK(h, hipEventRecord(ev[2], st));
            PDCHK(h, launch_pd_round(a, st));
            PDCHK(h, hipEventRecord(ev[3], st));
            s->par ^= 1u;
            s->round++;
        }
    }
    PDCHK(h, hipMemcpyAsync(s->h_run, s->d_run, size_t(rounds) * kRow * 8, hipMemcpyDeviceToHost, st));
    PDCHK(h, handle_wait(h));
    s->run_pending = false;
    const uint64_t round0 = s->round - rounds;
    for (uint32_t i = 0; i < rounds; i++) {
        const unsigned long long* row = s->h_run + size_t(i) * kRow;
        const hipEvent_t* ev = s->run_ev.data() + 4ull * i;
        psim_c3_stats* o = out && i < cap ? &out[i] : nullptr;
        unsigned long long r[kPdNStat];
        int rc;
        if (beat[i]) {
            fold_stat_shards(row, r, kPdNStat, 9);
            rc = pd_check(h, r[9], round0 + i);
            if (rc) return rc;
        }
        float ms = 0.f;
        PDCHK(h, hipEventElapsedTime(&ms, ev[0], ev[1]));
        rc = scamp_round_report(h, row + kPd, ms, sc_round[i], o ? &o->scamp : nullptr);
        if (rc) return rc;
        fold_stat_shards(row + kPd + kSc, r, kPdNStat, 9);
        PDCHK(h, hipEventElapsedTime(&ms, ev[2], ev[3]));
        rc = pd_check(h, r[9], round0 + i + 1);
        if (rc) return rc;
        if (o) pd_fill(*s, r, ms, o);
    }
    return PSIM_OK;
}

int psim_c3_get_plumtree(const psim_handle* h, uint32_t v, uint32_t* eager, size_t* ne, uint32_t* lazy, size_t* nl,
                         uint32_t* outstanding, size_t* no, size_t cap, uint32_t* delivered_mono,
                         uint32_t* recv_round) {
    if (!h) return PSIM_EINVAL;
    psim_handle* hh = const_cast<psim_handle*>(h);
    PdState* s = pd_of(hh);
    if (!s) return PSIM_ESTATE;
    if (v >= s->n) return PSIM_EINVAL;
    PDCHK(hh, hipStreamSynchronize(handle_stream(h)));
    PdHead hd;
    uint32_t tab[kPdTab];
    PdBits m[kPdSets];
    PdRow rows[kPdRows];
    PDCHK(hh, hipMemcpy(&hd, s->head + v, sizeof hd, hipMemcpyDeviceToHost));
    PDCHK(hh, hipMemcpy(tab, s->tab + size_t(v) * kPdTab, sizeof tab, hipMemcpyDeviceToHost));
    PDCHK(hh, hipMemcpy(m, s->mask + size_t(v) * kPdSets, sizeof m, hipMemcpyDeviceToHost));
    PDCHK(hh, hipMemcpy(rows, s->rows + size_t(v) * kPdRows, sizeof rows, hipMemcpyDeviceToHost));
    const bool sets = hd.flags & 1u;
    const PdBits E = sets ? m[3] : m[1], L = sets ? m[4] : m[2];
    auto emit = [&](std::vector<uint32_t>& ids, uint32_t* dst, size_t* n) {
        std::sort(ids.begin(), ids.end());
        ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
        if (dst)
            for (size_t i = 0; i < ids.size() && i < cap; i++) dst[i] = ids[i];
        if (n) *n = ids.size();
    };
    auto out = [&](const PdBits& mk, uint32_t* dst, size_t* n) {
        std::vector<uint32_t> ids;
        for (uint32_t i = 0; i < hd.ntab && i < kPdTab; i++)
            if (mk.test(i)) ids.push_back(tab[i]);
        emit(ids, dst, n);
    };
    out(E, eager, ne);
    out(L, lazy, nl);
    std::vector<uint32_t> peers;
    for (uint32_t i = 0; i < hd.nrow && i < kPdRows; i++) peers.push_back(rows[i].peer);
    emit(peers, outstanding, no);
    const bool cur = s->mono && hd.dbase == s->mono && (hd.dmask & 1ull);   // a lagging window top: not seen
    if (delivered_mono) *delivered_mono = cur ? s->mono : 0;
    if (recv_round) *recv_round = cur ? hd.myround : 0;
    return PSIM_OK;
}

}  // extern "C"
