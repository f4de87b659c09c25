// ptwin.hip -- window lanes of the static-overlay Plumtree engine: a root
// heartbeats again while its previous heartbeat is still in flight
// (partisan_plumtree_backend.erl:341-368 fires every heartbeat interval,
// whatever the state of the last flood).  The messages of the heartbeats in
// flight share the root's eager / lazy sets (partisan_plumtree_broadcast.erl
// all_peers/3 :1278-1282) and differ in their id {Root, Epoch, Monotonic},
// so a lane keeps per vertex:
//   * the slot-mask eager / lazy sets, tree epoch, and Round / serial tag of
//     the newest heartbeat, exactly as the static engine (vs records);
//   * the backend's timestamp set for the root (add_timestamp/1 :400-417,
//     is_stale/1 :229-244): a partisan_interval_sets value of <= kWinIs
//     disjoint, non-adjacent intervals [lo, hi] of Monotonics;
//   * the outstanding ETS rows {Peer, {Id, Mod, Round, Root}} as
//     {peer, Monotonic, Round} in insertion order (add_all_outstanding/5
//     :1215-1219 appends, ack_outstanding/5 :1207-1211 deletes every match);
//   * an emission counter, so the messages of one sender are handled in the
//     order it sent them.
// Messages are PdMsg records; a round buckets them by receiver (the C3
// engine's counting sort) and each vertex handles its bucket in (src, seq)
// order -- the schedule of DESIGN.md 3 -- then fires its lazy tick.  One
// thread per vertex; a window lane is a fault / overlap mode, the static
// engine's words stay the hot path.
#include "psim_internal.h"
#include "../../include/psim.h"

namespace psim {

namespace {

__device__ __forceinline__ bool alive_bit(const uint32_t* __restrict__ a, uint32_t v) {
    return (a[v >> 5] >> (v & 31)) & 1u;
}

// ---- the timestamp interval set (partisan_interval_sets on one origin) ----
struct ISet {
    uint32_t lo[kWinIs], hi[kWinIs];
};
__device__ __forceinline__ ISet is_load(const WinArgs& a, uint32_t v) {
    const uint4 x = a.iset[2 * size_t(v)], y = a.iset[2 * size_t(v) + 1];
    return ISet{{x.x, x.y, x.z, x.w}, {y.x, y.y, y.z, y.w}};
}
__device__ __forceinline__ void is_store(const WinArgs& a, uint32_t v, const ISet& s) {
    a.iset[2 * size_t(v)] = make_uint4(s.lo[0], s.lo[1], s.lo[2], s.lo[3]);
    a.iset[2 * size_t(v) + 1] = make_uint4(s.hi[0], s.hi[1], s.hi[2], s.hi[3]);
}
// is_element/2
__device__ __forceinline__ bool is_member(const ISet& s, uint32_t x) {
    bool r = false;
#pragma unroll
    for (uint32_t i = 0; i < kWinIs; i++) r |= s.lo[i] && s.lo[i] <= x && x <= s.hi[i];
    return r;
}
// add_element/2: intervals stay sorted, disjoint and non-adjacent; false
// when a fifth interval would be needed
__device__ bool is_add(ISet& s, uint32_t x) {
    if (is_member(s, x)) return true;
    uint32_t k = 0;
    while (k < kWinIs && s.lo[k] && s.hi[k] < x) k++;      // first interval above x (or a free one)
    const bool left = k > 0 && s.hi[k - 1] + 1 == x;
    const bool right = k < kWinIs && s.lo[k] && s.lo[k] == x + 1;
    if (left && right) {                                  // x bridges k-1 and k
        s.hi[k - 1] = s.hi[k];
        for (uint32_t i = k; i + 1 < kWinIs; i++) { s.lo[i] = s.lo[i + 1]; s.hi[i] = s.hi[i + 1]; }
        s.lo[kWinIs - 1] = s.hi[kWinIs - 1] = 0;
        return true;
    }
    if (left) { s.hi[k - 1] = x; return true; }
    if (right) { s.lo[k] = x; return true; }
    if (s.lo[kWinIs - 1]) return false;                   // full
    for (uint32_t i = kWinIs - 1; i > k; i--) { s.lo[i] = s.lo[i - 1]; s.hi[i] = s.hi[i - 1]; }
    s.lo[k] = s.hi[k] = x;
    return true;
}

// ---- the backend's table row for the root: {Root, Epoch, ISet} ----------
// A heartbeat id is epoch << 24 | Monotonic (psim_plumtree_restart_backend:
// the root's backend restarted that many times); every interval of a set
// holds ids of one epoch, so the set's epoch is that of its first interval.
__device__ __forceinline__ uint32_t id_epoch(uint32_t id) { return id >> 24; }
__device__ __forceinline__ bool is_empty(const ISet& s) { return s.lo[0] == 0u; }
// is_stale/1 (backend :229-244): same epoch -> is_element; else Epoch0 > Epoch
__device__ __forceinline__ bool ts_stale(const ISet& s, uint32_t id) {
    if (is_empty(s)) return false;
    const uint32_t e = id_epoch(s.lo[0]);
    return e == id_epoch(id) ? is_member(s, id) : e > id_epoch(id);
}
// add_timestamp/1 (:400-417): a newer epoch replaces the set, an older one is ignored
__device__ bool ts_add(ISet& s, uint32_t id) {
    if (!is_empty(s)) {
        const uint32_t e = id_epoch(s.lo[0]);
        if (e > id_epoch(id)) return true;
        if (e < id_epoch(id)) s = ISet{};
    }
    return is_add(s, id);
}
// graft/1 (:254-280): 0 {ok, M}, 1 stale, 2 {error, not_found}
__device__ __forceinline__ int ts_graft(const ISet& s, uint32_t id) {
    if (is_empty(s)) return 2;
    const uint32_t e = id_epoch(s.lo[0]);
    if (e == id_epoch(id)) return is_member(s, id) ? 0 : 2;
    return e > id_epoch(id) ? 1 : 2;
}

// ---- one vertex of a window lane for one round ----
struct Ctr {
    uint32_t sent[6], deliv, active, senders, degsum, overflow;
    int32_t ost_delta, live_delta;
};

struct V {
    uint32_t v, rs, deg;
    uint32_t eager, lazy, rmask, myround, rseq, ep;
    uint32_t nrow, seq;
    ISet is;
    bool sent;
};

__device__ __forceinline__ uint32_t peer(const WinArgs& a, const V& x, uint32_t s) { return a.col[x.rs + s]; }

// the slot of peer p in v's row (rows are sorted; ELL padding sorts last)
__device__ __forceinline__ int find_slot(const WinArgs& a, const V& x, uint32_t p) {
    uint32_t lo = 0, hi = x.deg;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (a.col[x.rs + m] < p) lo = m + 1; else hi = m;
    }
    return lo < x.deg && a.col[x.rs + lo] == p ? (int)lo : -1;
}

// partisan:cast_message over slot s (omission faults: sent, counted, lost)
__device__ void emit(const WinArgs& a, V& x, Ctr& c, uint32_t s, uint32_t type, uint32_t mono, uint32_t round) {
    const uint32_t seq = x.seq++;
    c.sent[type]++;
    x.sent = true;
    const uint32_t e = x.rs + s;
    if (a.omit && ((a.omit[e >> 5] >> (e & 31)) & 1u)) return;
    const uint32_t pos = wave_reserve(a.nout);
    if (pos >= a.cap) { c.overflow |= 16u; return; }
    PdMsg m;
    m.type = type; m.src = a.v_lo + x.v; m.dst = a.col[e]; m.seq = seq; m.round = round; m.mono = mono;
    a.out[pos] = m;
}

__device__ __forceinline__ void add_row(const WinArgs& a, V& x, Ctr& c, uint32_t s, uint32_t mono, uint32_t round) {
    if (x.nrow >= kWinRows) { c.overflow |= 32u; return; }
    a.rows[size_t(x.v) * kWinRows + x.nrow++] = PdRow{peer(a, x, s), mono, round};
    x.rmask |= 1u << s;
}

// ets:delete_object: every row {peer, mono, round} goes
__device__ void ack_rows(const WinArgs& a, V& x, uint32_t s, uint32_t mono, uint32_t round) {
    PdRow* r = a.rows + size_t(x.v) * kWinRows;
    const uint32_t p = peer(a, x, s);
    uint32_t w = 0;
    bool still = false;
    for (uint32_t i = 0; i < x.nrow; i++) {
        const PdRow q = r[i];
        if (q.peer == p && q.mono == mono && q.round == round) continue;
        still |= q.peer == p;
        if (w != i) r[w] = q;
        w++;
    }
    x.nrow = w;
    if (!still) x.rmask &= ~(1u << s);
}

// eager_push/7 (:962-970) and schedule_lazy_push/6 (:974-988), From = slot
// `from` (kNoPeer: the origin), Round = `round`
__device__ void push(const WinArgs& a, V& x, Ctr& c, uint32_t from, uint32_t mono, uint32_t round) {
    const uint32_t fb = from < 32 ? 1u << from : 0u;
    uint32_t e = x.eager & ~fb;
    while (e) {
        const uint32_t s = __ffs(e) - 1;
        e &= e - 1;
        emit(a, x, c, s, PSIM_MSG_BROADCAST, mono, round);
    }
    uint32_t l = x.lazy & ~fb;
    while (l) {
        const uint32_t s = __ffs(l) - 1;
        l &= l - 1;
        add_row(a, x, c, s, mono, round);
    }
}

__device__ __forceinline__ void to_eager(V& x, uint32_t s) { x.eager |= 1u << s; x.lazy &= ~(1u << s); }
__device__ __forceinline__ void to_lazy(V& x, uint32_t s) { x.lazy |= 1u << s; x.eager &= ~(1u << s); }

// handle_cast clauses (:571-605) for a message over slot s
__device__ void handle(const WinArgs& a, V& x, Ctr& c, uint32_t s, const PdMsg& m) {
    switch (m.type) {
    case PSIM_MSG_BROADCAST:                          // handle_broadcast/8 :843-857
        if (!ts_stale(x.is, m.mono)) {                // merge/2: not stale -> add_timestamp, true
            if (!ts_add(x.is, m.mono)) c.overflow |= 64u;
            c.deliv++;
            if (m.mono == a.mono) {                   // the newest heartbeat's Round / serial tag
                x.myround = m.round + 1;
                if (x.myround > 0xFFFFu) { c.overflow |= 2u; x.myround = 0xFFFFu; }
                x.rseq = a.mono8;
            }
            to_eager(x, s);                           // add_eager(From, Root)
            push(a, x, c, s, m.mono, m.round + 1);
        } else {
            to_lazy(x, s);                            // add_lazy(From, Root)
            emit(a, x, c, s, PSIM_MSG_PRUNE, 0, 0);
        }
        break;
    case PSIM_MSG_PRUNE:                              // :580-584
        to_lazy(x, s);
        break;
    case PSIM_MSG_IHAVE:                              // handle_ihave/7 :861-876
        if (ts_stale(x.is, m.mono)) {
            emit(a, x, c, s, PSIM_MSG_IGNORED, m.mono, m.round);
        } else {
            emit(a, x, c, s, PSIM_MSG_GRAFT, m.mono, m.round);
            to_eager(x, s);
        }
        break;
    case PSIM_MSG_IGNORED:                            // ack_outstanding/5
        ack_rows(a, x, s, m.mono, m.round);
        break;
    case PSIM_MSG_GRAFT: {                            // handle_graft/7 :880-906
        const int g = ts_graft(x.is, m.mono);
        if (g == 0) {                                 // {ok, M}
            to_eager(x, s);
            emit(a, x, c, s, PSIM_MSG_BROADCAST, m.mono, m.round);
        } else if (g == 1) {                          // stale: ack_outstanding
            ack_rows(a, x, s, m.mono, m.round);
        }                                             // {error, not_found}: logged only
        break;
    }
    default:
        break;
    }
}

__device__ __forceinline__ uint32_t live_slots(const WinArgs& a, const V& x) {
    uint32_t m = x.rmask, k = 0;
    while (m) {
        const uint32_t s = __ffs(m) - 1;
        m &= m - 1;
        k += alive_bit(a.alive, peer(a, x, s));
    }
    return k;
}

__device__ __forceinline__ void v_load(const WinArgs& a, uint32_t v, V& x) {
    x.v = v;
    x.rs = a.ell ? v * a.ell : a.rowp[v];
    x.deg = a.ell ? a.ell : a.rowp[v + 1] - x.rs;
    const uint4 st = a.vs[v];
    x.eager = st.x; x.lazy = st.y; x.rmask = st.z;
    x.myround = st.w & 0xFFFFu; x.rseq = (st.w >> 16) & 0xFFu; x.ep = st.w >> 24;
    if (x.ep != a.epoch8) {                           // no map entry for the root: the common sets
        x.eager = a.memb[v];
        x.lazy = 0;
        x.ep = a.epoch8;
    }
    const uint2 h = a.head[v];
    x.nrow = h.x; x.seq = h.y;
    x.is = is_load(a, v);
    x.sent = false;
}
__device__ __forceinline__ void v_store(const WinArgs& a, const V& x) {
    a.vs[x.v] = make_uint4(x.eager, x.lazy, x.rmask, x.myround | (x.rseq << 16) | (x.ep << 24));
    a.head[x.v] = make_uint2(x.nrow, x.seq);
    is_store(a, x.v, x.is);
}

__device__ void flush(const WinArgs& a, const Ctr& c) {
    unsigned long long v[kNStat] = {};
    for (int t = 1; t <= 5; t++) v[t] = c.sent[t];
    v[S_DELIV] = c.deliv; v[S_ACTIVE] = c.active; v[S_SENDERS] = c.senders; v[S_DEGSUM] = c.degsum;
    v[S_OST_DELTA] = (unsigned long long)(long long)c.ost_delta;
    v[S_LIVE_DELTA] = (unsigned long long)(long long)c.live_delta;
    v[S_OVERFLOW] = c.overflow;
    unsigned long long* row = a.stats + (blockIdx.x & (kStatShards - 1)) * kNStat;
    for (int i = 1; i < kNStat; i++) {
        unsigned long long x = v[i];
        if (i == S_OVERFLOW) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o, 64);
            if ((threadIdx.x & 63) == 0 && x) atomicOr(&row[i], x);
        } else {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
            if ((threadIdx.x & 63) == 0 && x) atomicAdd(&row[i], x);
        }
    }
}

__device__ __forceinline__ bool msg_less(const PdMsg& x, const PdMsg& y) {
    return x.src < y.src || (x.src == y.src && x.seq < y.seq);
}

__global__ __launch_bounds__(kBlock) void win_round_kernel(WinArgs a) {
    const uint32_t v = blockIdx.x * kBlock + threadIdx.x;
    Ctr c{};
    if (v < a.n && alive_bit(a.alive, a.v_lo + v)) {
        const uint32_t lo = a.off[v], hi = a.off[v + 1];
        const uint32_t nrow = a.head[v].x;
        if (hi > lo || (a.tick && nrow)) {
            V x;
            v_load(a, v, x);
            const uint32_t live0 = live_slots(a, x);
            const bool rows0 = x.nrow != 0;
            // the inbox in (src, seq) order
            for (uint32_t i = lo + 1; i < hi; i++) {
                const uint32_t q = a.idx[i];
                const PdMsg mq = a.in[q];
                uint32_t j = i;
                while (j > lo && msg_less(mq, a.in[a.idx[j - 1]])) { a.idx[j] = a.idx[j - 1]; j--; }
                a.idx[j] = q;
            }
            for (uint32_t i = lo; i < hi; i++) {
                const PdMsg m = a.in[a.idx[i]];
                const int s = find_slot(a, x, m.src);
                if (s < 0) { c.overflow |= 128u; continue; }   // not an overlay edge: cannot happen
                handle(a, x, c, (uint32_t)s, m);
            }
            // handle_info(lazy_tick): send_lazy/0, connected peers only, rows persist
            if (a.tick) {
                const PdRow* r = a.rows + size_t(v) * kWinRows;
                for (uint32_t i = 0; i < x.nrow; i++) {
                    const PdRow q = r[i];
                    if (!alive_bit(a.alive, q.peer)) continue;
                    const int s = find_slot(a, x, q.peer);
                    if (s >= 0) emit(a, x, c, (uint32_t)s, PSIM_MSG_IHAVE, q.mono, q.round);
                }
            }
            c.active = 1;
            if (x.sent) {
                c.senders = 1;
                uint32_t d = 0;
                for (uint32_t s = 0; s < x.deg; s++) d += a.col[x.rs + s] != kNoPeer;
                c.degsum = d;
            }
            c.live_delta = (int32_t)live_slots(a, x) - (int32_t)live0;
            c.ost_delta = (int32_t)(x.nrow != 0) - (int32_t)rows0;
            if (c.ost_delta) a.ost[v] = x.nrow != 0;
            v_store(a, x);
        }
    }
    flush(a, c);
}

// The origin's {broadcast, Id, Payload, Mod} cast (:565-569) after the
// backend's add_timestamp: eager_push/4, schedule_lazy_push/3, Round 0.
__global__ void win_origin_kernel(WinArgs a, uint32_t root) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    Ctr c{};
    V x;
    v_load(a, root, x);
    const uint32_t live0 = live_slots(a, x);
    const bool rows0 = x.nrow != 0;
    if (!ts_add(x.is, a.mono)) c.overflow |= 64u;
    x.myround = 0;
    x.rseq = a.mono8;
    push(a, x, c, kNoPeer, a.mono, 0);
    if ((x.nrow != 0) != rows0) a.ost[root] = x.nrow != 0;
    v_store(a, x);
    unsigned long long* row = a.stats;
    atomicAdd(&row[PSIM_MSG_BROADCAST], (unsigned long long)c.sent[PSIM_MSG_BROADCAST]);
    atomicAdd(&row[S_LIVE_DELTA], (unsigned long long)(long long)((int32_t)live_slots(a, x) - (int32_t)live0));
    atomicAdd(&row[S_OST_DELTA], (unsigned long long)(long long)((int32_t)(x.nrow != 0) - (int32_t)rows0));
    if (c.overflow) atomicOr(&row[S_OVERFLOW], (unsigned long long)c.overflow);
}

// Static lane -> window lane.  The static engine holds one heartbeat per
// root: its outstanding mask becomes rows of the current Monotonic (in slot
// = insertion order: schedule_lazy_push adds a delivery's rows in ordset
// order), a delivered vertex's timestamp set is {mono}, and each live word
// of the next round becomes records in FIFO order (seq 0..3; every vertex's
// counter then starts at 4, after them).  Round of a graft / ignored_i_have
// = the receiver's own pushed Round (that of the i_have it answers).
__global__ __launch_bounds__(kBlock) void win_convert_kernel(WinArgs a, PtArgs pa) {
    const uint32_t v = blockIdx.x * kBlock + threadIdx.x;
    if (v >= a.n) return;
    const uint4 st = a.vs[v];
    const uint32_t rs = a.ell ? v * a.ell : a.rowp[v];
    const uint32_t deg = a.ell ? a.ell : a.rowp[v + 1] - rs;
    const bool got = ((st.w >> 16) & 0xFFu) == a.mono8;
    ISet is{};
    if (got) { is.lo[0] = is.hi[0] = a.mono; }
    is_store(a, v, is);
    const uint32_t myround = st.w & 0xFFFFu;
    uint32_t nrow = 0, m = st.z;
    while (m && nrow < kWinRows) {
        const uint32_t s = __ffs(m) - 1;
        m &= m - 1;
        a.rows[size_t(v) * kWinRows + nrow++] = PdRow{a.col[rs + s], a.mono, myround};
    }
    a.head[v] = make_uint2(nrow, 4u);
    for (uint32_t s = 0; s < deg; s++) {
        const uint32_t w = pa.in_cur[rs + s];
        if (!live_word(w, pa.ctag)) continue;
        uint32_t f = w & kFifoMask, k = 0;
        while (f) {
            const uint32_t t = f & 7u;
            f >>= kKindBits;
            PdMsg r;
            r.type = t; r.src = a.col[rs + s]; r.dst = a.v_lo + v; r.seq = k++;
            r.mono = t == PSIM_MSG_PRUNE ? 0u : a.mono;              // a prune carries no id
            r.round = (t == PSIM_MSG_BROADCAST || t == PSIM_MSG_IHAVE) ? (w >> kRoundShift)
                    : (t == PSIM_MSG_PRUNE ? 0u : myround);
            const uint32_t pos = wave_reserve(a.nout);
            if (pos < a.cap) a.out[pos] = r;
        }
    }
}

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// sum over in-flight records of mix(mix(dst << 32 | src) ^ (mono << 32 | Round << 8 | kind))
__global__ __launch_bounds__(kBlock) void win_hash_kernel(WinArgs a, unsigned long long* out) {
    unsigned long long sum = 0;
    const uint32_t k = min(*a.nin, a.cap);
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < k; i += gridDim.x * kBlock) {
        const PdMsg m = a.in[i];
        const unsigned long long r = m.type == PSIM_MSG_PRUNE ? 0ull : (unsigned long long)(m.round & 0xFFFFFFu);
        sum += mix64(mix64(((unsigned long long)m.dst << 32) | m.src) ^
                     (((unsigned long long)m.mono << 32) | (r << 8) | m.type));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if ((threadIdx.x & 63) == 0 && sum) atomicAdd(&out[1], sum);
}

__global__ __launch_bounds__(kBlock) void win_delivered_kernel(WinArgs a, uint32_t mono, uint8_t* out) {
    const uint32_t v = blockIdx.x * kBlock + threadIdx.x;
    if (v < a.n) out[v] = ts_stale(is_load(a, v), mono) ? 1 : 0;
}

// Sharded window lanes: the records a round emitted are split by the shard
// owning their receiver (contiguous ranges lo(r) = n r / W, psim_load_csr).
__device__ __forceinline__ uint32_t owner(uint32_t v, uint32_t n, uint32_t W) {
    uint32_t r = uint32_t((uint64_t(v) * W) / n);
    while (r + 1 < W && uint32_t((uint64_t(n) * (r + 1)) / W) <= v) r++;
    while (r > 0 && uint32_t((uint64_t(n) * r) / W) > v) r--;
    return r;
}

__global__ __launch_bounds__(kBlock) void win_split_count_kernel(const PdMsg* __restrict__ m, const uint32_t* nm,
                                                                 uint32_t cap, uint32_t n, uint32_t W,
                                                                 uint32_t* __restrict__ counts) {
    __shared__ uint32_t hist[kWinMaxWorld];
    for (uint32_t i = threadIdx.x; i < W; i += kBlock) hist[i] = 0;
    __syncthreads();
    const uint32_t k = min(*nm, cap);
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < k; i += gridDim.x * kBlock)
        atomicAdd(&hist[owner(m[i].dst, n, W)], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < W; i += kBlock)
        if (hist[i]) atomicAdd(&counts[i], hist[i]);
}

__global__ __launch_bounds__(kBlock) void win_split_scatter_kernel(const PdMsg* __restrict__ m, const uint32_t* nm,
                                                                   uint32_t cap, uint32_t n, uint32_t W,
                                                                   const uint32_t* __restrict__ base,
                                                                   uint32_t* __restrict__ cursor,
                                                                   PdMsg* __restrict__ out) {
    const uint32_t k = min(*nm, cap);
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < k; i += gridDim.x * kBlock) {
        const PdMsg x = m[i];
        const uint32_t r = owner(x.dst, n, W);
        out[base[r] + atomicAdd(&cursor[r], 1u)] = x;
    }
}

inline uint32_t blocks(uint32_t n) { return n ? (n + kBlock - 1) / kBlock : 1u; }

}  // namespace

hipError_t launch_win_round(const WinArgs& a, uint32_t* cnt, uint32_t* cur, uint32_t* bsum, hipStream_t s) {
    PdArgs b{};
    b.n = a.n;
    b.v_lo = a.v_lo;
    b.in = a.in;
    b.nin = a.nin;
    b.out_cap = a.cap;
    b.cnt = cnt;
    b.cur = cur;
    b.off = const_cast<uint32_t*>(a.off);
    b.idx = a.idx;
    b.bsum = bsum;
    hipError_t e = launch_pd_bucket(b, s, false);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(win_round_kernel, dim3(blocks(a.n)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_win_split(const PdMsg* m, const uint32_t* nm, uint32_t cap, uint32_t n_global, uint32_t world,
                            uint32_t* counts, hipStream_t s) {
    if (world > kWinMaxWorld) return hipErrorInvalidValue;
    hipLaunchKernelGGL(win_split_count_kernel, dim3(256), dim3(kBlock), 0, s, m, nm, cap, n_global, world, counts);
    return hipGetLastError();
}

hipError_t launch_win_scatter(const PdMsg* m, const uint32_t* nm, uint32_t cap, uint32_t n_global, uint32_t world,
                              const uint32_t* base, uint32_t* cursor, PdMsg* out, hipStream_t s) {
    hipLaunchKernelGGL(win_split_scatter_kernel, dim3(256), dim3(kBlock), 0, s, m, nm, cap, n_global, world, base,
                       cursor, out);
    return hipGetLastError();
}

hipError_t launch_win_origin(const WinArgs& a, uint32_t root_local, hipStream_t s) {
    hipLaunchKernelGGL(win_origin_kernel, dim3(1), dim3(64), 0, s, a, root_local);
    return hipGetLastError();
}

hipError_t launch_win_convert(const WinArgs& a, const PtArgs& pa, hipStream_t s) {
    hipLaunchKernelGGL(win_convert_kernel, dim3(blocks(a.n)), dim3(kBlock), 0, s, a, pa);
    return hipGetLastError();
}

hipError_t launch_win_hash(const WinArgs& a, unsigned long long* out, hipStream_t s) {
    hipLaunchKernelGGL(win_hash_kernel, dim3(1024), dim3(kBlock), 0, s, a, out);
    return hipGetLastError();
}

// psim_plumtree_restart_backend at local vertex v of one lane: the backend's
// new ETS table has no row for the lane's root -- the static record's
// delivered tag stops matching (bad = a tag no heartbeat of the lane uses)
// and a window lane's timestamp set empties
__global__ void pt_forget_kernel(uint4* vs, uint4* iset, uint32_t v, uint32_t bad) {
    if (threadIdx.x != 0) return;
    uint4 st = vs[v];
    st.w = (st.w & 0xFF00FFFFu) | ((bad & 0xFFu) << 16);
    vs[v] = st;
    if (iset) {
        iset[2 * size_t(v)] = make_uint4(0u, 0u, 0u, 0u);
        iset[2 * size_t(v) + 1] = make_uint4(0u, 0u, 0u, 0u);
    }
}

hipError_t launch_pt_forget(uint4* vs, uint4* iset, uint32_t v, uint32_t bad, hipStream_t s) {
    hipLaunchKernelGGL(pt_forget_kernel, dim3(1), dim3(64), 0, s, vs, iset, v, bad);
    return hipGetLastError();
}

hipError_t launch_win_delivered(const WinArgs& a, uint32_t mono, uint8_t* out, hipStream_t s) {
    hipLaunchKernelGGL(win_delivered_kernel, dim3(blocks(a.n)), dim3(kBlock), 0, s, a, mono, out);
    return hipGetLastError();
}

}  // namespace psim
