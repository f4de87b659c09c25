// plumtree.hip -- CDNA4 (gfx950) kernels for one round of Partisan's Plumtree
// (src/partisan_plumtree_broadcast.erl) with the heartbeat handler
// (src/partisan_plumtree_backend.erl) as Mod.
//
// Formulation (DESIGN.md "Plumtree kernel"):
//   * one thread per vertex, grid-stride; a vertex is visited when its inbox
//     flag is set or when the lazy tick fires and it holds outstanding rows;
//   * the inbox of v is one 32-bit word per peer slot of v: a FIFO of up to
//     four 4-bit message kinds plus the 16-bit Round carried by broadcast /
//     i_have.  Each word is written by exactly one sender per round, so there
//     are no atomics on the data path and the result never depends on
//     arrival order;
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
#include "../../include/psim.h"

namespace psim {

namespace {

__device__ __forceinline__ bool bit_alive(const uint32_t* __restrict__ alive, uint32_t v) {
    return (alive[v >> 5] >> (v & 31)) & 1u;
}

// Per-thread counters.  Message kinds are packed 12 bits each into one
// 64-bit word (a thread emits < 4096 messages per round) so that no counter
// is indexed at run time (that would spill the array to scratch).
struct Ctr {
    unsigned long long kinds;   // field t (t = 1..5) at bits [12t, 12t+12)
    uint32_t deliv, active, senders, degsum, ost_delta, live_delta, overflow;
    __device__ __forceinline__ void zero() {
        kinds = 0; deliv = active = senders = degsum = ost_delta = live_delta = overflow = 0;
    }
    __device__ __forceinline__ void kind(uint32_t t) { kinds += 1ull << (12 * t); }
    __device__ __forceinline__ unsigned long long get(int i) const {
        switch (i) {
        case 1: case 2: case 3: case 4: case 5: return (kinds >> (12 * i)) & 0xFFFull;
        case S_DELIV: return deliv;
        case S_ACTIVE: return active;
        case S_SENDERS: return senders;
        case S_DEGSUM: return degsum;
        case S_OST_DELTA: return (unsigned long long)(long long)(int32_t)ost_delta;
        case S_LIVE_DELTA: return (unsigned long long)(long long)(int32_t)live_delta;
        case S_OVERFLOW: return overflow;
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
                                               int* ost_total) {
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
    if (threadIdx.x < kNStat && threadIdx.x >= 1) {
        const int i = threadIdx.x;
        unsigned long long s = 0;
        if (i == S_OVERFLOW) {
            for (int w = 0; w < kBlock / 64; w++) s |= red[w][i];
            if (s) atomicOr(&stats[(blockIdx.x & (kStatShards - 1)) * kNStat + i], s);
        } else {
            for (int w = 0; w < kBlock / 64; w++) s += red[w][i];
            if (s) atomicAdd(&stats[(blockIdx.x & (kStatShards - 1)) * kNStat + i], s);
            if (s && i == S_OST_DELTA && ost_total) atomicAdd(ost_total, (int)(long long)s);
        }
    }
}

// Append the nibble FIFO `f` holding `k` messages to (fifo, n); count kinds.
__device__ __forceinline__ void fifo_append(uint32_t& fifo, uint32_t& n, uint32_t f, Ctr& c) {
    while (f) {
        const uint32_t t = f & 0xFu;
        f >>= 4;
        if (n < 4) fifo |= t << (4 * n);
        else c.overflow |= 1u;
        n++;
        c.kind(t);
    }
}

// Hand the word for sender slot e to its receiver: a local receiver slot
// (rev[e] is a global slot id) plus its group flag, or -- receiver on another
// shard -- the staging word of the sender slot, packed by pt_compact_kernel.
__device__ __forceinline__ void deliver_word(const PtArgs& a, uint32_t e, uint32_t w) {
    const uint32_t u = a.col[e] - a.v_lo;
    if (u < a.n) {
        a.in_nxt[a.rev[e] - a.slot_base] = w;
        a.pend_nxt[u >> kGroupShift] = 1;
    } else {
        a.stage[e] = w;
    }
}

// One vertex, one round.  `rep` is this thread's LDS column (stride kBlock)
// for the reply FIFOs of its slots.  `pend`: the vertex's 16-vertex group
// was flagged (it may have words); `due`: the lazy tick fires and it holds
// outstanding rows.
__device__ __forceinline__ void pt_vertex(const PtArgs& a, uint32_t v, bool pend, bool due, uint16_t* rep,
                                          Ctr& c) {
    const uint32_t rs = a.rowp[v];
    const uint32_t deg = a.rowp[v + 1] - rs;
    if (pend) {
        uint32_t any = 0;
        for (uint32_t s = 0; s < deg; s++) any |= a.in_cur[rs + s];
        pend = any != 0;
    }
    if (!pend && !due) return;
    if (!bit_alive(a.alive, a.v_lo + v)) {
        // a dead vertex receives nothing: the words are dropped (cleared)
        if (pend)
            for (uint32_t s = 0; s < deg; s++)
                if (a.in_cur[rs + s]) a.in_cur[rs + s] = 0;
        return;
    }
    c.active++;
    const uint4 st = a.vs[v];
    uint32_t eager = st.x, lazy = st.y, outst = st.z;
    uint32_t myround = st.w & 0xFFFFu;
    uint32_t rseq = (st.w >> 16) & 0xFFu;
    uint32_t ep = st.w >> 24;
    if (ep != a.epoch8) {       // all_peers/3 (:1278-1282): no map entry -> common sets
        eager = a.memb[v];      // common_eagers = Members -- self
        lazy = 0;               // common_lazys = [] (start_link/0 :253-254)
        ep = a.epoch8;
    }
    bool rcv = rseq == a.mono8;
    const uint32_t outst0 = outst;
    uint32_t push_mask = 0, push_pos = 0xFFFFFFFFu;
    int32_t live_delta = 0;

    if (pend) {
        for (uint32_t s = 0; s < deg; s++) {
            const uint32_t w = a.in_cur[rs + s];
            uint32_t r = 0, rn = 0;
            if (w) {
                a.in_cur[rs + s] = 0;
                const uint32_t b = 1u << s;
                uint32_t f = w & 0xFFFFu;
                const uint32_t rnd = w >> 16;
                while (f) {
                    const uint32_t t = f & 0xFu;
                    f >>= 4;
                    uint32_t reply = 0;
                    switch (t) {
                    case PSIM_MSG_BROADCAST:           // handle_cast :571-578
                        if (!rcv) {                    // merge/2 -> true; handle_broadcast(true) :852-857
                            rcv = true;
                            rseq = a.mono8;
                            myround = rnd + 1;
                            if (myround > 0xFFFFu) { c.overflow |= 2u; myround = 0xFFFFu; }
                            c.deliv++;
                            eager |= b;                // add_eager(From, Root)
                            lazy &= ~b;
                            push_mask = eager & ~b;    // eager_push(.., Round+1, Root, From)
                            push_pos = s;
                            if (outst) c.overflow |= 4u;
                            {                          // schedule_lazy_push(.., Round+1, Root, From)
                                uint32_t add = lazy & ~b & ~outst;
                                outst |= lazy & ~b;
                                while (add) {
                                    const uint32_t q = __ffs(add) - 1;
                                    add &= add - 1;
                                    live_delta += bit_alive(a.alive, a.col[rs + q]);
                                }
                            }
                        } else {                       // handle_broadcast(false) :843-850
                            eager &= ~b;               // add_lazy(From, Root)
                            lazy |= b;
                            reply = PSIM_MSG_PRUNE;
                        }
                        break;
                    case PSIM_MSG_PRUNE:               // :580-584
                        eager &= ~b;
                        lazy |= b;
                        break;
                    case PSIM_MSG_IHAVE:               // :586-590 -> handle_ihave/7 :861-876
                        if (rcv) {
                            reply = PSIM_MSG_IGNORED;
                        } else {
                            reply = PSIM_MSG_GRAFT;
                            eager |= b;
                            lazy &= ~b;
                        }
                        break;
                    case PSIM_MSG_IGNORED:             // :592-598 ack_outstanding/5
                        if (outst & b) {
                            outst &= ~b;
                            live_delta -= bit_alive(a.alive, a.col[rs + s]);
                        }
                        break;
                    case PSIM_MSG_GRAFT:               // :600-605 -> handle_graft/7 :880-906
                        if (rcv) {                     // Mod:graft -> {ok, M}
                            eager |= b;
                            lazy &= ~b;
                            reply = PSIM_MSG_BROADCAST;  // same Round (Q3)
                        }                              // {error, not_found}: logged only
                        break;
                    default:
                        break;
                    }
                    if (reply) {
                        if (rn < 4) r |= reply << (4 * rn);
                        else c.overflow |= 1u;
                        rn++;
                    }
                }
            }
            rep[s * kBlock] = (uint16_t)r;
        }
    }

    // lazy tick: send_lazy/0 (:992-1019), connected peers only, rows persist
    uint32_t ihave = 0;
    if (a.tick && outst) {
        uint32_t m = outst;
        while (m) {
            const uint32_t q = __ffs(m) - 1;
            m &= m - 1;
            if (bit_alive(a.alive, a.col[rs + q])) ihave |= 1u << q;
        }
    }

    // compose and scatter the outgoing words
    const uint32_t any = push_mask | ihave;
    bool sent = false;
    for (uint32_t s = 0; s < deg; s++) {
        const uint32_t r = pend ? rep[s * kBlock] : 0u;
        const uint32_t b = 1u << s;
        if (!r && !(any & b)) continue;
        uint32_t fifo = 0, n = 0;
        const bool p = (push_mask & b) != 0;
        if (p && s > push_pos) fifo_append(fifo, n, PSIM_MSG_BROADCAST, c);
        fifo_append(fifo, n, r, c);
        if (p && s < push_pos) fifo_append(fifo, n, PSIM_MSG_BROADCAST, c);
        if (ihave & b) fifo_append(fifo, n, PSIM_MSG_IHAVE, c);
        const uint32_t e = rs + s;
        deliver_word(a, e, fifo | (myround << 16));
        sent = true;
    }
    if (sent) {
        c.senders++;
        c.degsum += deg;
    }

    const uint32_t nw = myround | (rseq << 16) | (ep << 24);
    if (eager != st.x || lazy != st.y || outst != st.z || nw != st.w)
        a.vs[v] = make_uint4(eager, lazy, outst, nw);
    if ((outst0 != 0) != (outst != 0)) {
        a.ost[v] = outst != 0;
        c.ost_delta += outst != 0 ? 1u : 0xFFFFFFFFu;
    }
    c.live_delta += (uint32_t)live_delta;
}

// A workgroup owns kChunkV consecutive vertices.  Each thread looks at 4 of
// them: their group flag (set by any sender to the group) and, on a tick
// round while some vertex holds outstanding rows, their outstanding byte.
// Candidates are compacted into an LDS list and spread over the threads.
__global__ __launch_bounds__(kBlock) void pt_round_kernel(PtArgs a) {
    __shared__ uint16_t rep[kMaxDeg * kBlock];
    __shared__ uint32_t cand[kChunkV];
    __shared__ uint32_t ncand;
    const uint32_t t = threadIdx.x;
    const uint32_t base = blockIdx.x * kChunkV;
    if (t == 0) ncand = 0;
    __syncthreads();
    const uint32_t v0 = base + 4 * t;
    uint32_t pmask = 0, dmask = 0;
    if (v0 < a.n) {
        const uint32_t g = v0 >> kGroupShift;
        if (a.pend_cur[g]) {
            pmask = 0xFu;
            if ((t & 3) == 0) a.pend_cur[g] = 0;   // the 4 threads of a group share the byte
        }
        if (a.tick && *a.ost_total > 0) {
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
            if (m & (1u << i)) cand[k++] = ((v0 + i) << 2) | (((pmask >> i) & 1u) << 1) | ((dmask >> i) & 1u);
    }
    __syncthreads();
    const uint32_t nc = ncand;
    if (nc == 0) return;                          // uniform: idle chunk
    Ctr c;
    c.zero();
    for (uint32_t i = t; i < nc; i += kBlock) {
        const uint32_t x = cand[i];
        pt_vertex(a, x >> 2, (x >> 1) & 1u, x & 1u, &rep[t], c);
    }
    flush_counters(c, a.stats, a.ost_total);
}

// The origin's {broadcast, Id, Payload, Mod} cast (:565-569): eager_push/4
// and schedule_lazy_push/3 with Round 0, Root = From = the origin; the
// backend already did add_timestamp (backend :341-368).
__global__ void pt_origin_kernel(PtArgs a) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint32_t v = a.root;   // local index of the origin (only its owner launches this)
    const uint32_t rs = a.rowp[v];
    const uint32_t deg = a.rowp[v + 1] - rs;
    const uint4 st = a.vs[v];
    uint32_t eager = st.x, lazy = st.y, outst = st.z;
    uint32_t ep = st.w >> 24;
    if (ep != a.epoch8) { eager = a.memb[v]; lazy = 0; ep = a.epoch8; }
    unsigned long long add_live = 0, flags = 0;
    if (outst) flags |= 4u;
    const uint32_t outst0 = outst;
    uint32_t nmsg = 0;
    for (uint32_t s = 0; s < deg; s++) {
        const uint32_t b = 1u << s;
        const uint32_t e = rs + s;
        if (eager & b) {
            deliver_word(a, e, PSIM_MSG_BROADCAST);  // Round 0
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
        atomicAdd(&a.stats[S_OST_DELTA], 1ull);
        atomicAdd(a.ost_total, 1);
    }
    if (add_live) atomicAdd(&a.stats[S_LIVE_DELTA], add_live);
    if (nmsg) atomicAdd(&a.stats[PSIM_MSG_BROADCAST], (unsigned long long)nmsg);
    if (flags) atomicOr(&a.stats[S_OVERFLOW], flags);
}

// Outstanding rows to live peers, counted densely (after psim_set_alive).
__global__ __launch_bounds__(kBlock) void pt_count_live_kernel(PtArgs a, unsigned long long* out) {
    unsigned long long cnt = 0;
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t v = blockIdx.x * kBlock + threadIdx.x; v < a.n; v += stride) {
        if (!a.ost[v] || !bit_alive(a.alive, a.v_lo + v)) continue;
        uint32_t m = a.vs[v].z;
        const uint32_t rs = a.rowp[v];
        while (m) {
            const uint32_t q = __ffs(m) - 1;
            m &= m - 1;
            cnt += bit_alive(a.alive, a.col[rs + q]);
        }
    }
    cnt = wave_sum(cnt);
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(out, cnt);
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

// Pack the staged cross-shard words into (global receiver slot, word)
// records, one region per destination shard.  A workgroup owns <= 1024
// entries of ONE destination's remote-slot list (blk = {rank, start, len}),
// so it reserves its run with a single atomicAdd.  Record order inside a
// region is irrelevant: every receiver slot has one writer per round.
__global__ __launch_bounds__(kBlock) void pt_compact_kernel(PtArgs a, const uint32_t* __restrict__ rem,
                                                            const uint4* __restrict__ blk,
                                                            const uint32_t* __restrict__ send_base,
                                                            uint32_t* __restrict__ cursor, uint2* __restrict__ out) {
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
    if (t == 0) base = tot ? atomicAdd(&cursor[b.x], tot) : 0u;
    __syncthreads();
    uint32_t pos = send_base[b.x] + base + pre + x - cnt;
#pragma unroll
    for (int i = 0; i < 4; i++)
        if (w[i]) out[pos++] = make_uint2(a.rev[e[i]], w[i]);
}

// Scatter records received from other shards into the local receiver slots.
__global__ __launch_bounds__(kBlock) void pt_ingest_kernel(PtArgs a, const uint2* __restrict__ rec, uint32_t nrec,
                                                           const uint32_t* __restrict__ slot2v) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nrec) return;
    const uint2 r = rec[i];
    const uint32_t ls = r.x - a.slot_base;
    a.in_nxt[ls] = r.y;
    a.pend_nxt[slot2v[ls] >> kGroupShift] = 1;
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
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < nrecv; i += stride) {
        const uint32_t w = recv[i];
        if (!w) continue;
        const uint32_t ls = recv_map[i];
        a.in_nxt[ls] = w;
        a.pend_nxt[slot2v[ls] >> kGroupShift] = 1;
    }
}

uint32_t grid_chunks(uint32_t n) { return (n + kChunkV - 1) / kChunkV; }

uint32_t grid_for(uint32_t n) {
    uint32_t g = (n + kBlock - 1) / kBlock;
    if (g > 8192) g = 8192;     // grid-stride beyond 32 blocks per CU
    return g ? g : 1;
}

}  // namespace

hipError_t launch_pt_round(const PtArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(pt_round_kernel, dim3(grid_chunks(a.n)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_pt_origin(const PtArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(pt_origin_kernel, dim3(1), dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_pt_count_live(const PtArgs& a, unsigned long long* out, hipStream_t s) {
    hipLaunchKernelGGL(pt_count_live_kernel, dim3(grid_for(a.n)), dim3(kBlock), 0, s, a, out);
    return hipGetLastError();
}

hipError_t launch_pt_compact(const PtArgs& a, const uint32_t* rem, const uint4* blk, uint32_t nblk,
                             const uint32_t* send_base, uint32_t* cursor, uint2* out, hipStream_t s) {
    if (nblk == 0) return hipSuccess;
    hipLaunchKernelGGL(pt_compact_kernel, dim3(nblk), dim3(kBlock), 0, s, a, rem, blk, send_base, cursor, out);
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

hipError_t launch_pt_ingest_dense(const PtArgs& a, const uint32_t* recv, const uint32_t* recv_map, uint32_t nrecv,
                                  const uint32_t* slot2v, hipStream_t s) {
    if (nrecv == 0) return hipSuccess;
    hipLaunchKernelGGL(pt_ingest_dense_kernel, dim3(grid_for(nrecv)), dim3(kBlock), 0, s, a, recv, recv_map, nrecv,
                       slot2v);
    return hipGetLastError();
}

hipError_t launch_pt_renorm(const PtArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(pt_renorm_kernel, dim3(grid_for(a.n)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace psim
