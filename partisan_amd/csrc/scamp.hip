// scamp.hip -- SCAMP v1 / v2 membership strategies
// (src/partisan_scamp_v{1,2}_membership_strategy.erl) as run by the
// pluggable peer service manager, one gfx950 thread per vertex and round.
//
// Same round shape as the HyParView engine: fixed 24-byte message records
// in an HBM queue, bucketed by destination (count, 3-phase scan, scatter),
// then one thread per vertex sorts its bucket by (src, emission seq) -- the
// schedule's order, so the atomicAdd slot a message landed in never
// matters -- and runs, in order: the leave and join calls made since the
// last round, the handle_message/2 clauses with the manager's stop check,
// and periodic/1.  Views live in HBM as fixed-capacity rows (partial view
// kScPv ids, in-view kScIv ids) in the reference's list order (v2: prepend;
// v1: sets in id order, Q28) and are edited in place.
//
// The connection rule of DESIGN.md "SCAMP" (a handler at u reaches t iff
// t != u, t was up at the start of the round and t is a member before or
// after the handler) is evaluated against the live row: every handler's
// membership change is a single add (join, keep), a map (replace) or a
// single removal (v1 leave, v2 remove -- `extra` re-admits the removed
// node), and bootstrap_remove sends before it clears the row.
#include "psim_internal.h"
#include "philox.h"
#include <cstdio>
#include "../../include/psim.h"

namespace psim {

namespace {

enum { SC_FWD = 1, SC_KEEP, SC_PING, SC_REMOVE, SC_REPLACE, SC_BOOT };
constexpr uint32_t kScStrideBlocks = 2048;
constexpr uint32_t kScMaxSel = 16;   // select_random_sublist sizes (c, c - 1)

struct Ctx {
    const ScArgs* a;
    uint32_t v;
    ScHead h;
    uint32_t* pv;      // row in HBM
    uint32_t* iv;
    uint32_t sent[7];
    uint32_t dropped, ndraw, err, resub;
    uint32_t nev;      // update events recorded this round
    WaveQ<ScMsg> q;    // this wave's send buffer (LDS)
};

// partisan_peer_service_events:update(Members) after a handler that changed
// the members' set: {added, removed} (each handler adds or removes at most one)
__device__ void record_update(Ctx& c, uint32_t added, uint32_t removed) {
    if (!c.a->ev_cnt || (added == 0xFFFFFFFFu && removed == 0xFFFFFFFFu)) return;
    if (c.nev >= kScEv) { c.err |= 16u; return; }
    c.a->ev[(size_t)c.v * kScEv + c.nev] = make_uint2(added, removed);
    c.nev++;
}

__device__ uint64_t draw64(Ctx& c) {
    const uint4 r = philox4x32_10(make_uint4(c.v, c.h.draws, KIND_SCAMP, c.h.inc), c.a->key);
    c.h.draws++;
    c.ndraw++;
    return (uint64_t)r.x | ((uint64_t)r.y << 32);
}

__device__ __forceinline__ bool in_pv(const Ctx& c, uint32_t t) { return row_has(c.pv, c.h.npv, t); }

// select_random_sublist(L, K) = lists:sublist(shuffle(L), K): one uniform()
// per element in list order, then the K smallest (r >> 11, N) in order.
// The top-k list is kept by a carry pass over compile-time slots (registers;
// a run-time-indexed array would live in scratch).
template <uint32_t K>
__device__ uint32_t select_top(Ctx& c, uint32_t k, uint32_t* out) {
    const uint32_t m = c.h.npv;
    unsigned long long key[K];
    uint32_t val[K];
#pragma unroll
    for (uint32_t j = 0; j < K; j++) { key[j] = ~0ull; val[j] = 0xFFFFFFFFu; }
    for (uint32_t i = 0; i < m; i++) {
        unsigned long long r = draw64(c) >> 11;     // < 2^53: never the empty-slot key
        uint32_t e = c.pv[i];
#pragma unroll
        for (uint32_t j = 0; j < K; j++) {
            const bool lt = r < key[j] || (r == key[j] && e < val[j]);
            const unsigned long long kr = lt ? key[j] : r;
            const uint32_t ke = lt ? val[j] : e;
            if (lt) { key[j] = r; val[j] = e; }
            r = kr;
            e = ke;
        }
    }
    const uint32_t got = m < k ? m : k;
#pragma unroll
    for (uint32_t j = 0; j < K; j++)
        if (j < got) out[j] = val[j];
    return got;
}
__device__ uint32_t select_sublist(Ctx& c, uint32_t k, uint32_t* out) {
    return k <= 4 ? select_top<4>(c, k, out) : select_top<kScMaxSel>(c, k, out);
}

// select_random_sublist(L, 1): the same draws, the smallest (r >> 11, N) kept
// in registers (the top-k arrays above are indexed at run time: scratch)
__device__ uint32_t select_one(Ctx& c, uint32_t* out) {
    const uint32_t m = c.h.npv;
    unsigned long long best = ~0ull;
    uint32_t bv = 0;
    for (uint32_t i = 0; i < m; i++) {
        const unsigned long long r = draw64(c) >> 11;
        const uint32_t e = c.pv[i];
        if (i == 0 || r < best || (r == best && e < bv)) { best = r; bv = e; }
    }
    out[0] = bv;
    return m ? 1u : 0u;
}

// `member`: the caller took t from the live partial view (a member now), so
// the connection rule needs no scan of the row -- every send but
// bootstrap_remove's, whose targets come from the in-view
__device__ void emit(Ctx& c, uint32_t t, uint32_t type, uint32_t x, uint32_t y, uint32_t extra, bool member = false) {
    const ScArgs& a = *c.a;
    const bool conn = t != c.v && a.alive0[t] && (member || t == extra || in_pv(c, t));
    if (!conn) { c.dropped++; return; }
#pragma unroll
    for (uint32_t k = 1; k < 7; k++) c.sent[k] += type == k ? 1u : 0u;   // compile-time slots: registers
    wq_send(c.q, a.nout, a.out, a.out_cap, c.err, ScMsg{type, c.v, t, c.h.seq++, x, y});
}

__device__ void pv_push_front(Ctx& c, uint32_t x) {
    if (c.h.npv >= kScPv) { c.err |= 2u; return; }
    for (uint32_t i = c.h.npv; i > 0; i--) c.pv[i] = c.pv[i - 1];
    c.pv[0] = x;
    c.h.npv++;
}
__device__ void pv_set_add(Ctx& c, uint32_t x) {     // v1: sets, id order
    if (in_pv(c, x)) return;
    if (c.h.npv >= kScPv) { c.err |= 2u; return; }
    uint32_t i = c.h.npv;
    while (i > 0 && c.pv[i - 1] > x) { c.pv[i] = c.pv[i - 1]; i--; }
    c.pv[i] = x;
    c.h.npv++;
}
// deletes the first x; returns its index (npv before the call if absent)
__device__ uint32_t pv_del_first(Ctx& c, uint32_t x) {
    for (uint32_t i = 0; i < c.h.npv; i++)
        if (c.pv[i] == x) {
            for (uint32_t j = i + 1; j < c.h.npv; j++) c.pv[j - 1] = c.pv[j];
            c.h.npv--;
            return i;
        }
    return c.h.npv;
}
// entry i of the row as it was before pv_del_first(x) returned `at`
__device__ __forceinline__ uint32_t pv_before(const Ctx& c, uint32_t i, uint32_t at, uint32_t x) {
    return i < at ? c.pv[i] : (i == at ? x : c.pv[i - 1]);
}

// join/3 (v2 :89-137, v1 :69-119)
__device__ void do_join(Ctx& c, uint32_t node) {
    const uint32_t k = c.a->ver == 2 ? c.a->c - 1 : c.a->c;   // Q15
    uint32_t sel[kScMaxSel];
    const uint32_t ns = select_sublist(c, k, sel);            // over the members before the add
    const uint32_t n0 = c.h.npv;
    const bool had = in_pv(c, node);
    if (c.a->ver == 2) pv_push_front(c, node);
    else pv_set_add(c, node);
    if (!had) record_update(c, node, 0xFFFFFFFFu);
    emit(c, node, SC_FWD, c.v, 0, node);                      // forward_subscription(Myself)
    // to each member known before (v2: list order; v1: sets:fold = id order):
    // v2 prepended one element, v1 inserted `node` unless present
    for (uint32_t i = 0; i < c.h.npv; i++) {
        const uint32_t t = c.pv[i];
        if (c.a->ver == 2) { if (i == 0) continue; }
        else if (t == node && c.h.npv != n0) continue;
        emit(c, t, SC_FWD, node, 0, node, true);
    }
#pragma unroll
    for (uint32_t i = 0; i < kScMaxSel; i++)         // drawn from the row, which only grew
        if (i < ns) emit(c, sel[i], SC_FWD, node, 0, node, true);
}

// leave/2 (v2 :140-146, v1 :122-142)
__device__ void do_leave(Ctx& c, uint32_t node) {
    if (c.a->ver == 2) {
        for (uint32_t i = 0; i < c.h.npv; i++) emit(c, c.pv[i], SC_BOOT, node, 0, 0xFFFFFFFFu, true);
        return;
    }
    // members(State0) in id order, `node` deleted from the set first
    const bool had = in_pv(c, node);
    const uint32_t n0 = c.h.npv;
    const uint32_t at = had ? pv_del_first(c, node) : n0;
    if (had) record_update(c, 0xFFFFFFFFu, node);
    for (uint32_t i = 0; i < n0; i++) {   // the old row minus node is still in the row; node itself is `extra`
        const uint32_t t = pv_before(c, i, at, node);
        emit(c, t, SC_REMOVE, node, 0, had ? node : 0xFFFFFFFFu, t != node);
    }
}

// periodic/1 (v2 :180-221, v1 :174-216); isolation per Q19
__device__ void do_periodic(Ctx& c) {
    const bool isolated = c.h.last_ping >= 0 && (uint32_t)c.h.last_ping < c.a->round;
    if (isolated) {
        uint32_t sel;
        const uint32_t ns = select_one(c, &sel);
        c.resub++;
        if (ns) emit(c, sel, SC_FWD, c.v, 0, 0xFFFFFFFFu, true);
    }
    // the pings (one per live member but self, in list order): one wave
    // reservation for all of them instead of one per emit
    const ScArgs& a = *c.a;
    uint32_t k = 0;
    for (uint32_t i = 0; i < c.h.npv; i++) {
        const uint32_t t = c.pv[i];
        if (t != c.v && a.alive0[t]) k++;
        else c.dropped++;
    }
    uint32_t pos = wave_reserve_n(a.nout, k);                // k <= kScPv < 2^10
    c.sent[SC_PING] += k;
    for (uint32_t i = 0; i < c.h.npv && k; i++) {
        const uint32_t t = c.pv[i];
        if (t == c.v || !a.alive0[t]) continue;
        if (pos >= a.out_cap) { c.err |= 1u; break; }
        ScMsg m;
        m.type = SC_PING; m.src = c.v; m.dst = t; m.seq = c.h.seq++; m.a = c.v; m.b = 0;
        a.out[pos++] = m;
    }
}

// handle_message/2; returns false when the manager stops (:1791-1803)
__device__ bool do_message(Ctx& c, const ScMsg& m) {
    const ScArgs& a = *c.a;
    switch (m.type) {
    case SC_PING:                                             // v2 :224-229, v1 :219-227
        c.h.last_ping = (int32_t)a.round;
        break;
    case SC_FWD: {                                            // v2 :313-341, v1 :264-297
        const uint32_t node = m.a;
        const uint32_t r10 = 1u + (uint32_t)__umul64hi(draw64(c), 10ull);   // random_0_or_1: uniform(10) >= 5
        const bool keep = r10 < 5 && !in_pv(c, node);
        if (keep) {
            if (a.ver == 2) {
                pv_push_front(c, node);
                record_update(c, node, 0xFFFFFFFFu);
                emit(c, node, SC_KEEP, c.v, 0, node);
            } else {
                pv_set_add(c, node);
                record_update(c, node, 0xFFFFFFFFu);
            }
        } else {
            uint32_t sel;
            const uint32_t ns = select_one(c, &sel);
            if (ns) emit(c, sel, SC_FWD, node, 0, 0xFFFFFFFFu, true);
        }
        break;
    }
    case SC_KEEP:                                             // v2 :342-347
        if (c.h.niv >= kScIv) { c.err |= 2u; break; }
        for (uint32_t i = c.h.niv; i > 0; i--) c.iv[i] = c.iv[i - 1];
        c.iv[0] = m.a;
        c.h.niv++;
        break;
    case SC_REMOVE: {                                         // v2 :295-312, v1 :230-262
        const uint32_t node = m.a;
        if (!in_pv(c, node)) break;
        if (a.ver == 1) { c.err |= 8u; return false; }       // Q17: the manager stops
        const uint32_t n0 = c.h.npv;
        const uint32_t at = pv_del_first(c, node);
        if (!in_pv(c, node)) record_update(c, 0xFFFFFFFFu, node);   // a duplicate keeps it a member
        for (uint32_t i = 0; i < n0; i++) {
            const uint32_t t = pv_before(c, i, at, node);
            emit(c, t, SC_REMOVE, node, 0, node, t != node);
        }
        break;
    }
    case SC_REPLACE: {                                        // v2 :275-294
        if (m.a == m.b || !in_pv(c, m.a)) break;
        const bool had_b = in_pv(c, m.b);
        for (uint32_t i = 0; i < c.h.npv; i++)
            if (c.pv[i] == m.a) c.pv[i] = m.b;
        record_update(c, had_b ? 0xFFFFFFFFu : m.b, m.a);
        break;
    }
    case SC_BOOT: {                                           // v2 :230-274
        if (m.a != c.v) break;
        const int32_t L = (int32_t)c.h.niv, P = (int32_t)c.h.npv;
        const int32_t num = L - (int32_t)(a.c - 1), rem = L - num;
        bool crash = false;                                   // lists:nth/2 out of range (Q18)
        if (num > 0)
            for (int32_t N = 1; N <= num && !crash; N++)
                if (P == 0 || N / P < 1 || N / P > P) crash = true;
        if (!crash && rem > L) crash = true;
        if (crash) { c.err |= 4u; return false; }
        if (num > 0)
            for (int32_t N = 1; N <= num; N++) emit(c, c.iv[N - 1], SC_REPLACE, c.v, c.pv[N / P - 1], 0xFFFFFFFFu);
        if (rem > 0)
            for (int32_t N = 1; N <= rem; N++) emit(c, c.iv[N - 1], SC_REMOVE, c.v, 0, 0xFFFFFFFFu);
        c.h.npv = 0;
        c.h.niv = 0;
        break;
    }
    default:
        break;
    }
    return in_pv(c, c.v);
}

__device__ __forceinline__ bool msg_less(const ScMsg& x, const ScMsg& y) {
    return x.src < y.src || (x.src == y.src && x.seq < y.seq);
}

__device__ __forceinline__ uint32_t n_in(const ScArgs& a) { return *a.nin < a.out_cap ? *a.nin : a.out_cap; }

__global__ __launch_bounds__(kBlock) void sc_count(ScArgs a) {
    const uint32_t k = n_in(a);
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < k; i += kScStrideBlocks * kBlock) {
        const uint32_t d = a.in[i].dst;
        if (d < a.n) atomicAdd(&a.cnt[d], 1u);
        else atomicOr(&a.stats[11], 32ull);           // a record off the cluster: reported, never indexed
    }
}
__global__ __launch_bounds__(kBlock) void sc_scan_blocks(ScArgs a) {
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
__global__ __launch_bounds__(1024) void sc_scan_sums(ScArgs a, uint32_t nb) {
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
__global__ __launch_bounds__(kBlock) void sc_scan_add(ScArgs a) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < a.n) a.off[i] += a.bsum[blockIdx.x];
}
__global__ __launch_bounds__(kBlock) void sc_scatter(ScArgs a) {
    const uint32_t k = n_in(a);
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < k; i += kScStrideBlocks * kBlock) {
        const uint32_t d = a.in[i].dst;
        if (d < a.n) a.idx[a.off[d] + atomicAdd(&a.cur[d], 1u)] = i;
    }
}

// Before a round's passes, in one launch: the stats rows and the outgoing
// queue's count zeroed, alive copied to alive0 (up at the start of the
// round), and each vertex's first call indexed (call_start).
__global__ __launch_bounds__(kBlock) void sc_prep(ScArgs a) {
    const uint32_t i0 = blockIdx.x * kBlock + threadIdx.x, st = gridDim.x * kBlock;
    for (uint32_t i = i0; i < kRoundStatShards * 16; i += st) a.stats[i] = 0ull;
    if (i0 == 0) *a.nout = 0u;
    uint8_t* a0 = const_cast<uint8_t*>(a.alive0);
    const uint32_t n16 = a.n / 16;
    for (uint32_t q = i0; q < n16; q += st)
        reinterpret_cast<uint4*>(a0)[q] = reinterpret_cast<const uint4*>(a.alive_now)[q];
    for (uint32_t j = n16 * 16 + i0; j < a.n; j += st) a0[j] = a.alive_now[j];
    for (uint32_t c = i0; c < a.ncalls; c += st)
        if (c == 0 || a.call_v[c] != a.call_v[c - 1]) a.call_start[a.call_v[c]] = c + 1;
}

#ifdef C3_PROF
// [0..4) cycles of the phases calls / sort / inbox / periodic (per wave),
// [4..11) messages handled by kind, [11] draws in calls, [12] draws in the
// inbox, [13] draws in periodic, [14] waves, [15] vertices with calls
__device__ unsigned long long g_sc_prof[kProfSlots];
#endif

__global__ __launch_bounds__(kBlock) void sc_process(ScArgs a) {
    __shared__ ScMsg qbuf[kBlock / 64][kWq];
    __shared__ uint32_t qn[kBlock / 64];
    const uint32_t v = blockIdx.x * kBlock + threadIdx.x;
    const WaveQ<ScMsg> q{qbuf[threadIdx.x >> 6], &qn[threadIdx.x >> 6]};
    wq_init(q.n);
    uint32_t sent[7] = {0, 0, 0, 0, 0, 0, 0};
    uint32_t dropped = 0, ndraw = 0, err = 0, resub = 0, nproc = 0, stopped = 0, npv = 0, niv = 0, nev = 0;
    const uint32_t j0 = v < a.n ? a.call_start[v] : 0u;
    if (v < a.n && !a.alive0[v] && a.head[v].fresh) a.head[v].fresh = 0;
    if (v < a.n && a.alive0[v]) {
        Ctx c;
        c.a = &a;
        c.v = v;
        c.h = a.head[v];
        c.pv = a.pv + (size_t)v * kScPv;
        c.iv = a.iv + (size_t)v * kScIv;
        for (int i = 0; i < 7; i++) c.sent[i] = 0;
        c.dropped = c.ndraw = c.err = c.resub = 0;
        c.nev = 0;
        c.q = q;
        const bool fresh = c.h.fresh != 0;
        c.h.fresh = 0;
        bool up = true;
#ifdef C3_PROF
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        const uint32_t d0 = c.ndraw;
        unsigned long long kinds = 0;
#endif
        // leave calls, then join calls (made since the last round, in call order)
        for (uint32_t i = j0 ? j0 - 1 : a.ncalls; i < a.ncalls && a.call_v[i] == v; i++) {
            const uint32_t x = a.calls[i];
            if (x >> 31) do_leave(c, x & 0x7FFFFFFFu);
            else if (x != v && a.alive0[x]) do_join(c, x);   // connect/1 succeeds iff the peer is up
        }
#ifdef C3_PROF
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        const uint32_t d1 = c.ndraw;
#endif
        // inbox in (src, seq) order; a restarted vertex drops what was sent to its old incarnation
        const uint32_t lo = a.off[v], hi = a.off[v + 1];
        if (!fresh && hi > lo) {
            for (uint32_t i = lo + 1; i < hi; i++) {
                const uint32_t x = a.idx[i];
                const ScMsg mx = a.in[x];
                uint32_t j = i;
                while (j > lo && msg_less(mx, a.in[a.idx[j - 1]])) { a.idx[j] = a.idx[j - 1]; j--; }
                a.idx[j] = x;
            }
        }
#ifdef C3_PROF
        const unsigned long long t2 = __builtin_amdgcn_s_memtime();
#endif
        if (!fresh && hi > lo) {
            for (uint32_t i = lo; i < hi && up; i++) {
                nproc++;
#ifdef C3_PROF
                kinds += 1ull << (9 * (a.in[a.idx[i]].type % 7));       // 9-bit fields by kind
#endif
                if (!do_message(c, a.in[a.idx[i]])) up = false;
            }
        }
#ifdef C3_PROF
        const unsigned long long t3 = __builtin_amdgcn_s_memtime();
        const uint32_t d3 = c.ndraw;
#endif
        if (up && a.periodic) do_periodic(c);
#ifdef C3_PROF
        const unsigned long long t4 = __builtin_amdgcn_s_memtime();
        prof_add(g_sc_prof, 0, t1 - t0);
        prof_add(g_sc_prof, 1, t2 - t1);
        prof_add(g_sc_prof, 2, t3 - t2);
        prof_add(g_sc_prof, 3, t4 - t3);
        atomicAdd(&g_sc_prof[11], (unsigned long long)(d1 - d0));
        atomicAdd(&g_sc_prof[12], (unsigned long long)(d3 - d1));
        atomicAdd(&g_sc_prof[13], (unsigned long long)(c.ndraw - d3));
        prof_add(g_sc_prof, 14, 1);
        if (j0) atomicAdd(&g_sc_prof[15], 1ull);
        for (int k = 0; k < 7; k++)
            if ((kinds >> (9 * k)) & 511ull) atomicAdd(&g_sc_prof[4 + k], (kinds >> (9 * k)) & 511ull);
#endif
        if (!up) {
            a.alive[v] = 0;
            stopped = 1;
        } else {
            npv = c.h.npv;
            niv = c.h.niv;
        }
        a.head[v] = c.h;
        nev = c.nev;
        for (int i = 0; i < 7; i++) sent[i] = c.sent[i];
        dropped = c.dropped; ndraw = c.ndraw; err = c.err; resub = c.resub;
    }
    wq_flush(q, a.nout, a.out, a.out_cap, err);           // every lane of the wave: what is still staged
    if (v < a.n) {          // what the next round expects zero (instead of host fills before it)
        if (j0) a.call_start[v] = 0;
        a.cnt[v] = 0;
        a.cur[v] = 0;
        if (a.ev_cnt) a.ev_cnt[v] = nev;
    }
    // counters: [1..6] sent by kind, 7 dropped, 8 processed, 9 draws, 10 stopped,
    // 11 error bits (OR), 12 pv_sum, 13 inview_sum, 14 resub
    unsigned long long vals[15];
    for (int i = 1; i < 7; i++) vals[i] = sent[i];
    vals[7] = dropped; vals[8] = nproc; vals[9] = ndraw; vals[10] = stopped; vals[11] = 0;
    vals[12] = npv; vals[13] = niv; vals[14] = resub;
    for (int i = 1; i <= 14; i++) {
        if (i == 11) continue;
        unsigned long long x = vals[i];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
        if ((threadIdx.x & 63) == 0 && x) atomicAdd(&a.stats[(blockIdx.x % kRoundStatShards) * 16 + i], x);
    }
    unsigned long long e = err;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) e |= __shfl_xor(e, o, 64);
    if ((threadIdx.x & 63) == 0 && e) atomicOr(&a.stats[(blockIdx.x % kRoundStatShards) * 16 + 11], e);
}

// init/1 (v2 :75-85, v1 :56-66) for every vertex, or crash-restart of a list
__global__ __launch_bounds__(kBlock) void sc_init(ScArgs a, const uint32_t* __restrict__ list, uint32_t k) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= (list ? k : a.n)) return;
    const uint32_t v = list ? list[i] : i;
    ScHead h = list ? a.head[v] : ScHead{};
    h.npv = 1;
    h.niv = 0;
    h.draws = 0;
    h.last_ping = -1;
    if (list) {
        h.inc++;
        h.fresh = 1;
        a.alive[v] = 1;
    } else {
        h.inc = 0;
        h.seq = 0;
        h.fresh = 0;
    }
    a.head[v] = h;
    a.pv[(size_t)v * kScPv] = v;
}

inline uint32_t nblk(uint32_t n) { return (n + kBlock - 1) / kBlock; }

}  // namespace

hipError_t launch_sc_init(const ScArgs& a, const uint32_t* list, uint32_t k, hipStream_t s) {
    const uint32_t m = list ? k : a.n;
    if (m) hipLaunchKernelGGL(sc_init, dim3(nblk(m)), dim3(kBlock), 0, s, a, list, k);
    return hipGetLastError();
}

hipError_t launch_sc_round(const ScArgs& a, hipStream_t s) {
    // cnt / cur / call_start / ev_cnt were left zero by the last sc_process
    uint32_t w = a.n / 16 > a.ncalls ? a.n / 16 : a.ncalls;
    if (w < kRoundStatShards * 16) w = kRoundStatShards * 16;
    hipLaunchKernelGGL(sc_prep, dim3(nblk(w) < 2048u ? nblk(w) : 2048u), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(sc_count, dim3(kScStrideBlocks), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(sc_scan_blocks, dim3(nblk(a.n)), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(sc_scan_sums, dim3(1), dim3(1024), 0, s, a, nblk(a.n));
    hipLaunchKernelGGL(sc_scan_add, dim3(nblk(a.n)), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(sc_scatter, dim3(kScStrideBlocks), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(sc_process, dim3(nblk(a.n)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace psim

// ---------------------------------------------------------------------------
// host side: the psim_scamp_* entry points of include/psim.h
// ---------------------------------------------------------------------------
#include <algorithm>
#include <cstring>
#include <vector>

using namespace psim;

namespace {

struct ScState : ModuleState {
    uint32_t n = 0, ver = 2, c = 5, periodic = 0, cap = 0;
    ScHead* head = nullptr;
    uint32_t *pv = nullptr, *iv = nullptr;
    uint8_t *alive = nullptr, *alive0 = nullptr;
    ScMsg* msg[2] = {nullptr, nullptr};
    uint32_t* nmsg = nullptr;
    uint32_t *cnt = nullptr, *cur = nullptr, *off = nullptr, *idx = nullptr, *bsum = nullptr;
    uint32_t *call_start = nullptr, *call_v = nullptr, *calls = nullptr, *list = nullptr;
    size_t calls_cap = 0, list_cap = 0;
    unsigned long long* stats = nullptr;
    uint32_t* ev_cnt = nullptr;     // update events (C3), allocated on demand
    uint2* ev = nullptr;
    uint32_t par = 0;
    uint64_t round = 0;
    std::vector<uint32_t> cv, cx;   // calls since the last round: vertex, (bit31 = leave) | target
    std::vector<uint32_t> stamp;    // psim_scamp_crash's duplicate test
    uint32_t stamp_gen = 0;
    // host -> device uploads (crash lists, a round's calls) go through pinned
    // staging, so the copies are asynchronous and no call waits for the
    // device; `up_ev` marks the last upload, awaited before the buffer is reused
    uint32_t* h_up = nullptr;
    size_t h_up_cap = 0;
    hipEvent_t up_ev = nullptr;
    bool up_pending = false;
    unsigned long long* h_stats = nullptr;   // pinned: a round's stats rows
    ~ScState() override {
        void* p[] = {head, pv, iv, alive, alive0, msg[0], msg[1], nmsg, cnt, cur, off, idx, bsum, call_start, call_v,
                     calls, list, stats, ev_cnt, ev};
        for (void* x : p)
            if (x) (void)hipFree(x);
        if (h_up) (void)hipHostFree(h_up);
        if (h_stats) (void)hipHostFree(h_stats);
        if (up_ev) (void)hipEventDestroy(up_ev);
    }
};

ScState* sc_of(psim_handle* h) { return static_cast<ScState*>(handle_module(h, MOD_SCAMP)); }
const ScState* sc_of(const psim_handle* h) { return static_cast<const ScState*>(handle_module(h, MOD_SCAMP)); }

#define SCCHK(h, x)                                                                         \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess)                                                               \
            return handle_fail((h), PSIM_EHIP, "%s failed: %s", #x, hipGetErrorString(e_)); \
    } while (0)

bool sc_alloc(void** p, size_t bytes) {
    return alloc_zero(p, bytes);
}

ScArgs sc_args(const psim_handle* h, const ScState& s) {
    ScArgs a{};
    a.n = s.n; a.ver = s.ver; a.c = s.c;
    a.round = (uint32_t)(s.round + 1);
    a.periodic = s.periodic && ((s.round + 1) % s.periodic) == 0;
    const uint64_t seed = handle_seed(h);
    a.key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
    a.alive0 = s.alive0; a.alive = s.alive;
    a.head = s.head; a.pv = s.pv; a.iv = s.iv;
    a.in = s.msg[s.par]; a.nin = s.nmsg + s.par;
    a.out = s.msg[s.par ^ 1]; a.nout = s.nmsg + (s.par ^ 1);
    a.out_cap = s.cap;
    a.cnt = s.cnt; a.cur = s.cur; a.off = s.off; a.idx = s.idx; a.bsum = s.bsum;
    a.call_start = s.call_start; a.call_v = s.call_v; a.calls = s.calls;
    a.ncalls = 0;
    a.alive_now = s.alive;
    a.stats = s.stats;
    a.ev_cnt = s.ev_cnt;
    a.ev = s.ev;
    return a;
}

// A pinned staging area of `words` u32 for the next upload (waits for the
// previous upload out of it, long finished in practice)
uint32_t* sc_stage(psim_handle* h, ScState& s, size_t words) {
    if (s.up_pending) {
        if (hipEventSynchronize(s.up_ev) != hipSuccess) return nullptr;
        s.up_pending = false;
    }
    if (!s.up_ev && hipEventCreateWithFlags(&s.up_ev, hipEventDisableTiming) != hipSuccess) return nullptr;
    if (words > s.h_up_cap) {
        if (s.h_up) (void)hipHostFree(s.h_up);
        s.h_up = nullptr;
        s.h_up_cap = std::max<size_t>(words, 2 * s.h_up_cap);
        if (hipHostMalloc((void**)&s.h_up, s.h_up_cap * 4) != hipSuccess) {
            s.h_up_cap = 0;
            return nullptr;
        }
    }
    (void)h;
    return s.h_up;
}

// Calls sorted by vertex: leaves first, then joins, each in call order
// (sc_prep indexes each vertex's first one on the device), written to `up`
// as k vertices then k targets.  An LSD radix sort of key 2 v + join, stable:
// O(k) per 11-bit digit, where a comparison sort of 50k calls took
// milliseconds of host time; calls already in key order -- a churn batch's
// joins -- are copied as they are.
void sc_sort_calls(uint32_t n, const uint32_t* cv, const uint32_t* cx, size_t k, uint32_t* up) {
    auto key = [&](size_t i) -> uint64_t { return 2ull * cv[i] + ((cx[i] >> 31) ^ 1u); };   // leave first
    bool sorted = true;
    for (size_t i = 1; i < k && sorted; i++) sorted = key(i - 1) <= key(i);
    if (sorted) {
        memcpy(up, cv, k * 4);
        memcpy(up + k, cx, k * 4);
        return;
    }
    std::vector<uint32_t> ord(k), tmp(k);
    for (size_t i = 0; i < k; i++) ord[i] = uint32_t(i);
    for (uint32_t shift = 0; shift < 64 && (2ull * n) >> shift; shift += 11) {
        uint32_t cnt[2049] = {0};
        for (size_t i = 0; i < k; i++) cnt[((key(ord[i]) >> shift) & 2047u) + 1]++;
        for (int d = 0; d < 2048; d++) cnt[d + 1] += cnt[d];
        for (size_t i = 0; i < k; i++) tmp[cnt[(key(ord[i]) >> shift) & 2047u]++] = ord[i];
        ord.swap(tmp);
    }
    for (size_t i = 0; i < k; i++) { up[i] = cv[ord[i]]; up[k + i] = cx[ord[i]]; }
}

// A round's first half: the calls made since the last round sorted and
// uploaded, the round launched, its stats rows copied to the pinned mirror --
// nothing waits; sc_round_finish reads them once the stream got there.
// `o` (psim_c3_run; null: the handle's own buffers and events 0 / 1): the
// events around the round's kernels, and either a pinned row the stats are
// copied to or a device row they stay in (d_stats), and the round's calls
// already sorted and on the device (d_calls: d_ncalls vertices then targets)
int sc_round_launch(psim_handle* h, ScState& s, const ScLaunch* o = nullptr) {
    const hipStream_t st = handle_stream(h);
    const uint32_t* d_calls = o ? o->d_calls : nullptr;
    const size_t k = d_calls ? o->d_ncalls : s.cv.size();
    if (d_calls && !s.cv.empty()) return handle_fail(h, PSIM_ESTATE, "scamp: calls pending beside a run's call list");
    uint32_t* up = k && !d_calls ? sc_stage(h, s, 2 * k) : nullptr;
    if (k && !d_calls && !up) return handle_fail(h, PSIM_ENOMEM, "scamp: pinned staging for %zu calls", k);
    if (k && !d_calls) sc_sort_calls(s.n, s.cv.data(), s.cx.data(), k, up);
    if (k > s.calls_cap && !d_calls) {
        if (s.calls) (void)hipFree(s.calls);
        if (s.call_v) (void)hipFree(s.call_v);
        s.calls = s.call_v = nullptr;
        s.calls_cap = std::max<size_t>(k, 2 * s.calls_cap);
        if (!sc_alloc((void**)&s.calls, s.calls_cap * 4) || !sc_alloc((void**)&s.call_v, s.calls_cap * 4))
            return handle_fail(h, PSIM_ENOMEM, "scamp: call list");
    }
    if (k && !d_calls) {
        SCCHK(h, hipMemcpyAsync(s.call_v, up, k * 4, hipMemcpyHostToDevice, st));
        SCCHK(h, hipMemcpyAsync(s.calls, up + k, k * 4, hipMemcpyHostToDevice, st));
        SCCHK(h, hipEventRecord(s.up_ev, st));
        s.up_pending = true;
    }
    s.cv.clear();
    s.cx.clear();
    unsigned long long* dst = o ? o->h_dst : nullptr;
    unsigned long long* d_stats = o ? o->d_stats : nullptr;
    if (!dst && !d_stats && !s.h_stats && hipHostMalloc((void**)&s.h_stats, kRoundStatShards * 16 * 8) != hipSuccess) {
        s.h_stats = nullptr;
        return handle_fail(h, PSIM_ENOMEM, "scamp: pinned stats rows");
    }
    if (!dst) dst = s.h_stats;
    const hipEvent_t e0 = o && o->e0 ? o->e0 : handle_event(h, 0);
    const hipEvent_t e1 = o && o->e1 ? o->e1 : handle_event(h, 1);
    ScArgs a = sc_args(h, s);
    a.ncalls = uint32_t(k);
    if (d_calls) {
        a.call_v = d_calls;
        a.calls = d_calls + k;
    }
    if (d_stats) a.stats = d_stats;
    SCCHK(h, hipEventRecord(e0, st));
    SCCHK(h, launch_sc_round(a, st));
    SCCHK(h, hipEventRecord(e1, st));
    if (!d_stats) SCCHK(h, hipMemcpyAsync(dst, s.stats, kRoundStatShards * 16 * 8, hipMemcpyDeviceToHost, st));
    return PSIM_OK;
}

// A round's report from its stats rows (`round` = its 1-based number): the
// kernel time into the handle's totals, the error bits as PSIM codes, the
// counters into `out`
int sc_round_report(psim_handle* h, const ScState& s, const unsigned long long* rows, float ms, uint64_t round,
                    psim_scamp_stats* out) {
    unsigned long long r[16];
    fold_stat_shards(rows, r, 16, 11);
    handle_add_round(h, ms);
    if (r[11] & 1ull) return handle_fail(h, PSIM_EOVERFLOW, "scamp round %llu: message queue over %u records",
                                         (unsigned long long)round, s.cap);
    if (r[11] & 2ull) return handle_fail(h, PSIM_EOVERFLOW, "scamp round %llu: a view exceeded %u / %u entries",
                                         (unsigned long long)round, kScPv, kScIv);
    if (r[11] & 16ull) return handle_fail(h, PSIM_EOVERFLOW, "scamp round %llu: > %u membership updates at a vertex",
                                          (unsigned long long)round, kScEv);
    if (r[11] & 32ull) return handle_fail(h, PSIM_EHIP, "scamp round %llu: a message record addressed off the cluster",
                                          (unsigned long long)round);
    if (out) {
        memset(out, 0, sizeof *out);
        uint64_t emitted = 0;
        for (int k = 1; k < 7; k++) { out->sent[k] = r[k]; emitted += r[k]; }
        out->dropped = r[7]; out->processed = r[8]; out->draws = r[9]; out->stopped = r[10];
        out->error = r[11]; out->pv_sum = r[12]; out->inview_sum = r[13]; out->resub = r[14];
        // records read (bucket + handler) and written, bucket counts/offsets, and
        // one pass over each live vertex's head and partial-view row
        out->algo_bytes = 48ull * r[8] + 28ull * emitted + 12ull * s.n + 64ull * s.n + 4ull * r[12];
        out->kernel_ms = ms;
    }
    return PSIM_OK;
}

// A round's second half, after the stream passed sc_round_launch's copy
int sc_round_finish(psim_handle* h, ScState& s, psim_scamp_stats* out) {
#ifdef C3_PROF
    {
        static unsigned long long tot[kProfSlots];
        unsigned long long x[kProfSlots];
        SCCHK(h, hipMemcpyFromSymbol(x, HIP_SYMBOL(g_sc_prof), sizeof x));
        const unsigned long long z[kProfSlots] = {};
        SCCHK(h, hipMemcpyToSymbol(HIP_SYMBOL(g_sc_prof), z, sizeof z));
        fprintf(stderr, "sc_prof");
        for (int i = 0; i < kProfSlots; i++) fprintf(stderr, " %llu", tot[i] += x[i]);
        fprintf(stderr, "\n");
    }
#endif
    float ms = 0.f;
    SCCHK(h, hipEventElapsedTime(&ms, handle_event(h, 0), handle_event(h, 1)));
    s.round++;
    s.par ^= 1u;
    return sc_round_report(h, s, s.h_stats, ms, s.round, out);
}

int sc_round(psim_handle* h, ScState& s, psim_scamp_stats* out) {
    int rc = sc_round_launch(h, s);
    if (rc) return rc;
    SCCHK(h, handle_wait(h));
    return sc_round_finish(h, s, out);
}

int sc_upload_list(psim_handle* h, ScState& s, const uint32_t* v, size_t k) {
    if (k > s.list_cap) {
        if (s.list) (void)hipFree(s.list);
        s.list = nullptr;
        s.list_cap = std::max<size_t>(k, 2 * s.list_cap);
        if (!sc_alloc((void**)&s.list, s.list_cap * 4)) return handle_fail(h, PSIM_ENOMEM, "scamp: vertex list");
    }
    uint32_t* up = sc_stage(h, s, k);
    if (!up) return handle_fail(h, PSIM_ENOMEM, "scamp: pinned staging for %zu vertices", k);
    memcpy(up, v, k * 4);
    SCCHK(h, hipMemcpyAsync(s.list, up, k * 4, hipMemcpyHostToDevice, handle_stream(h)));
    SCCHK(h, hipEventRecord(s.up_ev, handle_stream(h)));
    s.up_pending = true;
    return PSIM_OK;
}

}  // namespace

namespace psim {

int scamp_view(psim_handle* h, ScView* out, bool want_events) {
    ScState* s = sc_of(h);
    if (!s) return PSIM_ESTATE;
    if (want_events && !s->ev_cnt) {
        if (!sc_alloc((void**)&s->ev_cnt, size_t(s->n) * 4) || !sc_alloc((void**)&s->ev, size_t(s->n) * kScEv * 8))
            return handle_fail(h, PSIM_ENOMEM, "scamp: update event arrays");
    }
    out->n = s->n;
    out->list = s->list;
    out->pv = s->pv;
    out->head = s->head;
    out->alive = s->alive;
    out->ev_cnt = s->ev_cnt;
    out->ev = s->ev;
    return PSIM_OK;
}

int scamp_round(psim_handle* h, psim_scamp_stats* out) {
    ScState* s = sc_of(h);
    if (!s) return handle_fail(h, PSIM_ESTATE, "psim_scamp_setup not called");
    return sc_round(h, *s, out);
}

int scamp_round_launch(psim_handle* h) {
    ScState* s = sc_of(h);
    if (!s) return handle_fail(h, PSIM_ESTATE, "psim_scamp_setup not called");
    return sc_round_launch(h, *s);
}

int scamp_round_finish(psim_handle* h, psim_scamp_stats* out) {
    ScState* s = sc_of(h);
    if (!s) return handle_fail(h, PSIM_ESTATE, "psim_scamp_setup not called");
    return sc_round_finish(h, *s, out);
}

int scamp_round_launch_to(psim_handle* h, const ScLaunch& o, uint64_t* round) {
    ScState* s = sc_of(h);
    if (!s) return handle_fail(h, PSIM_ESTATE, "psim_scamp_setup not called");
    const int rc = sc_round_launch(h, *s, &o);
    if (rc) return rc;
    s->round++;                                       // the next launch's arguments (sc_args) follow this round
    s->par ^= 1u;
    if (round) *round = s->round;
    return PSIM_OK;
}

int scamp_round_report(psim_handle* h, const unsigned long long* rows, float ms, uint64_t round, psim_scamp_stats* out) {
    ScState* s = sc_of(h);
    if (!s) return handle_fail(h, PSIM_ESTATE, "psim_scamp_setup not called");
    return sc_round_report(h, *s, rows, ms, round, out);
}

int scamp_crash_list(psim_handle* h, const uint32_t* v, size_t k) { return psim_scamp_crash(h, v, k); }

int scamp_check_calls(psim_handle* h, const uint32_t* v, const uint32_t* x, size_t k, uint32_t* sorted) {
    ScState* s = sc_of(h);
    if (!s) return handle_fail(h, PSIM_ESTATE, "psim_scamp_setup not called");
    for (size_t i = 0; i < k; i++)
        if (v[i] >= s->n || x[i] >= s->n) return handle_fail(h, PSIM_EINVAL, "call %zu: vertex out of range", i);
    sc_sort_calls(s->n, v, x, k, sorted);
    return PSIM_OK;
}

size_t scamp_calls_pending(psim_handle* h) {
    ScState* s = sc_of(h);
    return s ? s->cv.size() : 0;
}

int scamp_check_crash(psim_handle* h, const uint32_t* v, size_t k) {
    ScState* s = sc_of(h);
    if (k && !v) return PSIM_EINVAL;
    if (!s) return handle_fail(h, PSIM_ESTATE, "psim_scamp_setup not called");
    if (s->stamp.size() != s->n || ++s->stamp_gen == 0) {
        s->stamp.assign(s->n, 0u);
        s->stamp_gen = 1;
    }
    for (size_t i = 0; i < k; i++) {
        if (v[i] >= s->n) return handle_fail(h, PSIM_EINVAL, "crash %zu: vertex out of range", i);
        if (s->stamp[v[i]] == s->stamp_gen) return handle_fail(h, PSIM_EINVAL, "crash %zu: vertex %u listed twice", i, v[i]);
        s->stamp[v[i]] = s->stamp_gen;
    }
    return PSIM_OK;
}

int scamp_crash_dev(psim_handle* h, const uint32_t* dv, size_t k) {
    ScState* s = sc_of(h);
    if (!s) return handle_fail(h, PSIM_ESTATE, "psim_scamp_setup not called");
    if (!k) return PSIM_OK;
    SCCHK(h, launch_sc_init(sc_args(h, *s), dv, (uint32_t)k, handle_stream(h)));
    return PSIM_OK;
}

}  // namespace psim

extern "C" {

int psim_scamp_setup(psim_handle* h, uint32_t n, uint32_t version, uint32_t c, uint32_t periodic_rounds) {
    if (!h) return PSIM_EINVAL;
    if (n < 1 || n >= 0x7FFFFFFFu || (version != 1 && version != 2) || c < 1 || c > kScMaxSel)
        return handle_fail(h, PSIM_EINVAL, "scamp: need n >= 1, version 1 or 2, 1 <= c <= %u", kScMaxSel);
    SCCHK(h, hipSetDevice(handle_device(h)));
    SCCHK(h, hipStreamSynchronize(handle_stream(h)));
    ModuleState*& slot = handle_module(h, MOD_SCAMP);
    delete slot;
    slot = nullptr;
    ScState* s = new ScState();
    s->n = n; s->ver = version; s->c = c; s->periodic = periodic_rounds;
    s->cap = (uint32_t)std::min<uint64_t>(8ull * n + 4096, 0xFFFFFFF0ull);
    const size_t N = n;
    const uint32_t nb = (n + kBlock - 1) / kBlock;
    const bool ok = sc_alloc((void**)&s->head, N * sizeof(ScHead)) && sc_alloc((void**)&s->pv, N * kScPv * 4) &&
                    sc_alloc((void**)&s->iv, N * kScIv * 4) && sc_alloc((void**)&s->alive, N) &&
                    sc_alloc((void**)&s->alive0, N) && sc_alloc((void**)&s->msg[0], size_t(s->cap) * sizeof(ScMsg)) &&
                    sc_alloc((void**)&s->msg[1], size_t(s->cap) * sizeof(ScMsg)) && sc_alloc((void**)&s->nmsg, 16) &&
                    sc_alloc((void**)&s->cnt, N * 4) && sc_alloc((void**)&s->cur, N * 4) &&
                    sc_alloc((void**)&s->off, (N + 1) * 4) && sc_alloc((void**)&s->idx, size_t(s->cap) * 4) &&
                    sc_alloc((void**)&s->bsum, size_t(nb) * 4) && sc_alloc((void**)&s->call_start, N * 4) &&
                    sc_alloc((void**)&s->stats, kRoundStatShards * 16 * 8);
    if (!ok) {
        delete s;
        return handle_fail(h, PSIM_ENOMEM, "scamp state for n=%u", n);
    }
    slot = s;
    SCCHK(h, hipMemsetAsync(s->alive, 1, N, handle_stream(h)));
    SCCHK(h, launch_sc_init(sc_args(h, *s), nullptr, 0, handle_stream(h)));
    SCCHK(h, hipStreamSynchronize(handle_stream(h)));
    return PSIM_OK;
}

int psim_scamp_set_alive(psim_handle* h, const uint8_t* alive, size_t n) {
    if (!h || !alive) return PSIM_EINVAL;
    ScState* s = sc_of(h);
    if (!s) return handle_fail(h, PSIM_ESTATE, "psim_scamp_setup not called");
    if (n != s->n) return handle_fail(h, PSIM_EINVAL, "alive has %zu entries, cluster has %u", n, s->n);
    std::vector<uint8_t> a(n);
    for (size_t i = 0; i < n; i++) a[i] = alive[i] ? 1 : 0;
    SCCHK(h, hipSetDevice(handle_device(h)));
    SCCHK(h, hipMemcpy(s->alive, a.data(), n, hipMemcpyHostToDevice));
    return PSIM_OK;
}

static int sc_calls(psim_handle* h, const uint32_t* v, const uint32_t* x, size_t k, uint32_t leave_bit) {
    if (!h || (k && (!v || !x))) return PSIM_EINVAL;
    ScState* s = sc_of(h);
    if (!s) return handle_fail(h, PSIM_ESTATE, "psim_scamp_setup not called");
    for (size_t i = 0; i < k; i++)
        if (v[i] >= s->n || x[i] >= s->n) return handle_fail(h, PSIM_EINVAL, "call %zu: vertex out of range", i);
    for (size_t i = 0; i < k; i++) {
        s->cv.push_back(v[i]);
        s->cx.push_back(x[i] | leave_bit);
    }
    return PSIM_OK;
}

int psim_scamp_join(psim_handle* h, const uint32_t* v, const uint32_t* contact, size_t k) {
    return sc_calls(h, v, contact, k, 0u);
}

int psim_scamp_leave(psim_handle* h, const uint32_t* v, const uint32_t* node, size_t k) {
    return sc_calls(h, v, node, k, 0x80000000u);
}

int psim_scamp_crash(psim_handle* h, const uint32_t* v, size_t k) {
    if (!h || (k && !v)) return PSIM_EINVAL;
    ScState* s = sc_of(h);
    if (!s) return handle_fail(h, PSIM_ESTATE, "psim_scamp_setup not called");
    const int crc = scamp_check_crash(h, v, k);   // range, duplicates (generation stamps: no O(n) clear per call)
    if (crc || !k) return crc;
    SCCHK(h, hipSetDevice(handle_device(h)));
    int rc = sc_upload_list(h, *s, v, k);
    if (rc) return rc;
    // no wait: the restart is ordered before every later round and read-back on the stream
    SCCHK(h, launch_sc_init(sc_args(h, *s), s->list, (uint32_t)k, handle_stream(h)));
    return PSIM_OK;
}

int psim_scamp_step(psim_handle* h, uint32_t rounds, psim_scamp_stats* stats, size_t cap) {
    if (!h) return PSIM_EINVAL;
    ScState* s = sc_of(h);
    if (!s) return handle_fail(h, PSIM_ESTATE, "psim_scamp_setup not called");
    SCCHK(h, hipSetDevice(handle_device(h)));
    for (uint32_t i = 0; i < rounds; i++) {
        const int rc = sc_round(h, *s, stats && i < cap ? &stats[i] : nullptr);
        if (rc) return rc;
    }
    return PSIM_OK;
}

int psim_scamp_get_views(const psim_handle* h, uint32_t* pv, uint32_t* npv, uint32_t* iv, uint32_t* niv, size_t n) {
    if (!h) return PSIM_EINVAL;
    const ScState* s = sc_of(h);
    if (!s) return PSIM_ESTATE;
    psim_handle* hh = const_cast<psim_handle*>(h);
    if (n != s->n) return handle_fail(hh, PSIM_EINVAL, "want n=%u", s->n);
    SCCHK(hh, hipSetDevice(handle_device(h)));
    SCCHK(hh, hipStreamSynchronize(handle_stream(h)));
    if (pv) SCCHK(hh, hipMemcpy(pv, s->pv, n * kScPv * 4, hipMemcpyDeviceToHost));
    if (iv) SCCHK(hh, hipMemcpy(iv, s->iv, n * kScIv * 4, hipMemcpyDeviceToHost));
    if (npv || niv) {
        std::vector<ScHead> hd(n);
        SCCHK(hh, hipMemcpy(hd.data(), s->head, n * sizeof(ScHead), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n; i++) {
            if (npv) npv[i] = hd[i].npv;
            if (niv) niv[i] = hd[i].niv;
        }
    }
    return PSIM_OK;
}

int psim_scamp_get_nodes(const psim_handle* h, uint64_t* draws, int32_t* last_ping, uint8_t* alive, size_t n) {
    if (!h) return PSIM_EINVAL;
    const ScState* s = sc_of(h);
    if (!s) return PSIM_ESTATE;
    psim_handle* hh = const_cast<psim_handle*>(h);
    if (n != s->n) return handle_fail(hh, PSIM_EINVAL, "want n=%u", s->n);
    SCCHK(hh, hipSetDevice(handle_device(h)));
    SCCHK(hh, hipStreamSynchronize(handle_stream(h)));
    std::vector<ScHead> hd(n);
    SCCHK(hh, hipMemcpy(hd.data(), s->head, n * sizeof(ScHead), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n; i++) {
        if (draws) draws[i] = hd[i].draws;
        if (last_ping) last_ping[i] = hd[i].last_ping;
    }
    if (alive) SCCHK(hh, hipMemcpy(alive, s->alive, n, hipMemcpyDeviceToHost));
    return PSIM_OK;
}

int psim_scamp_inflight(const psim_handle* h, uint64_t* messages) {
    if (!h || !messages) return PSIM_EINVAL;
    const ScState* s = sc_of(h);
    if (!s) return PSIM_ESTATE;
    psim_handle* hh = const_cast<psim_handle*>(h);
    SCCHK(hh, hipSetDevice(handle_device(h)));
    SCCHK(hh, hipStreamSynchronize(handle_stream(h)));
    uint32_t c = 0;
    SCCHK(hh, hipMemcpy(&c, s->nmsg + s->par, 4, hipMemcpyDeviceToHost));
    *messages = c;
    return PSIM_OK;
}

}  // extern "C"

namespace {
// The queue the next round reads, copied down (record order is the
// atomics' order: meaningless; callers sort).
int sc_queue(psim_handle* h, const ScState& s, std::vector<ScMsg>& q) {
    SCCHK(h, hipSetDevice(handle_device(h)));
    SCCHK(h, hipStreamSynchronize(handle_stream(h)));
    uint32_t c = 0;
    SCCHK(h, hipMemcpy(&c, s.nmsg + s.par, 4, hipMemcpyDeviceToHost));
    q.resize(std::min(c, s.cap));
    if (!q.empty()) SCCHK(h, hipMemcpy(q.data(), s.msg[s.par], q.size() * sizeof(ScMsg), hipMemcpyDeviceToHost));
    return PSIM_OK;
}
bool handling_less(const ScMsg& x, const ScMsg& y) {
    return x.dst != y.dst ? x.dst < y.dst : (x.src != y.src ? x.src < y.src : x.seq < y.seq);
}
psim_scamp_msg to_abi(const ScMsg& m) { return psim_scamp_msg{m.type, m.src, m.dst, m.seq, m.a, m.b}; }
}  // namespace

extern "C" {

int psim_scamp_messages(const psim_handle* h, psim_scamp_msg* out, size_t cap, size_t* count) {
    if (!h || !count || (cap && !out)) return PSIM_EINVAL;
    const ScState* s = sc_of(h);
    if (!s) return PSIM_ESTATE;
    psim_handle* hh = const_cast<psim_handle*>(h);
    std::vector<ScMsg> q;
    if (int rc = sc_queue(hh, *s, q)) return rc;
    std::sort(q.begin(), q.end(), handling_less);
    *count = q.size();
    for (size_t i = 0; i < q.size() && i < cap; i++) out[i] = to_abi(q[i]);
    return PSIM_OK;
}

int psim_scamp_take(psim_handle* h, uint32_t dst, psim_scamp_msg* out, size_t cap, size_t* count) {
    if (!h || !count || (cap && !out)) return PSIM_EINVAL;
    ScState* s = sc_of(h);
    if (!s) return PSIM_ESTATE;
    if (dst >= s->n) return handle_fail(h, PSIM_EINVAL, "scamp_take: vertex %u of %u", dst, s->n);
    std::vector<ScMsg> q, keep, took;
    if (int rc = sc_queue(h, *s, q)) return rc;
    for (const ScMsg& m : q) (m.dst == dst ? took : keep).push_back(m);
    *count = took.size();
    if (took.size() > cap) return handle_fail(h, PSIM_EINVAL, "scamp_take: %zu messages for %u, room for %zu",
                                              took.size(), dst, cap);
    std::sort(took.begin(), took.end(), handling_less);
    for (size_t i = 0; i < took.size(); i++) out[i] = to_abi(took[i]);
    if (took.empty()) return PSIM_OK;
    const hipStream_t st = handle_stream(h);
    const uint32_t k = uint32_t(keep.size());
    if (k) SCCHK(h, hipMemcpyAsync(s->msg[s->par], keep.data(), keep.size() * sizeof(ScMsg), hipMemcpyHostToDevice, st));
    SCCHK(h, hipMemcpyAsync(s->nmsg + s->par, &k, 4, hipMemcpyHostToDevice, st));
    SCCHK(h, hipStreamSynchronize(st));
    return PSIM_OK;
}

int psim_scamp_put(psim_handle* h, const psim_scamp_msg* msgs, size_t k) {
    if (!h || (k && !msgs)) return PSIM_EINVAL;
    ScState* s = sc_of(h);
    if (!s) return PSIM_ESTATE;
    std::vector<ScMsg> add(k);
    for (size_t i = 0; i < k; i++) {
        const psim_scamp_msg& m = msgs[i];
        if (m.type < PSIM_SC_FORWARD || m.type > PSIM_SC_BOOTSTRAP_REMOVE || m.dst >= s->n || m.a >= s->n ||
            (m.type == PSIM_SC_REPLACE && m.b >= s->n))
            return handle_fail(h, PSIM_EINVAL, "scamp_put: message %zu (type %u, dst %u, a %u, b %u)", i, m.type, m.dst,
                               m.a, m.b);
        add[i] = ScMsg{m.type, m.src, m.dst, m.seq, m.a, m.b};
    }
    if (!k) return PSIM_OK;
    SCCHK(h, hipSetDevice(handle_device(h)));
    const hipStream_t st = handle_stream(h);
    SCCHK(h, hipStreamSynchronize(st));
    uint32_t c = 0;
    SCCHK(h, hipMemcpy(&c, s->nmsg + s->par, 4, hipMemcpyDeviceToHost));
    if (uint64_t(c) + k > s->cap)
        return handle_fail(h, PSIM_EOVERFLOW, "scamp_put: %u + %zu messages > queue of %u", c, k, s->cap);
    SCCHK(h, hipMemcpyAsync(s->msg[s->par] + c, add.data(), k * sizeof(ScMsg), hipMemcpyHostToDevice, st));
    const uint32_t nc = c + uint32_t(k);
    SCCHK(h, hipMemcpyAsync(s->nmsg + s->par, &nc, 4, hipMemcpyHostToDevice, st));
    SCCHK(h, hipStreamSynchronize(st));
    return PSIM_OK;
}

}  // extern "C"
