// demers.hip -- Demers rumor mongering + anti-entropy
// (protocols/demers_rumor_mongering.erl :92-186, protocols/demers_anti_entropy.erl
// :95-227) as one gfx950 kernel per round; the store of each vertex is a
// 64-bit seen-set (one bit per rumor id).  Host side: demers_host.hip.
//
// Round formulation, one thread per vertex:
//  * every process draws from its own sequential Philox stream (philox.h
//    draw64 / select2): a vertex's RM process calls select_random_sublist once
//    per rumor it accepts (and once per rumor it originates), in the order it
//    handles them; its AE process once per tick;
//  * RM inbox = three 64-bit planes per vertex -- rumors received this round
//    from >= 1, >= 2, >= 3 senders -- raised by the senders with atomicOr
//    cascades.  The schedule handles RM messages by (rumor, class, sender),
//    class 0 = senders that are not among the receiver's own two targets for
//    the rumor, so the FromNode that `-- [MyNode, FromNode]` drops is a
//    non-target (no effect) whenever the senders outnumber the targets that
//    sent it, else the smallest target that sent it.  Whether target T sent it:
//    T called select for the rumor last round (rmnew_prev) and drew the
//    receiver -- recomputed from T's call count (ncall_prev) and T's stream;
//  * AE pushes: the sender appends its id to the receiver's list (atomicAdd
//    slot); the receiver sorts its list (schedule: by sender), merges each
//    pusher's snapshot and answers with its prefix union into the pusher's
//    pull slot k (k = the receiver's index in the pusher's target pair: the
//    pusher's tick-th AE call, a pure function of (pusher, tick));
//  * AE tick (end of the round): snapshot + push to the tick's select -- [v].
#include "psim_internal.h"
#include "philox.h"
#include "../../include/psim.h"

namespace psim {

namespace {

struct DmCtr {
    uint32_t rm, push, pull, deliv, complete, overflow;
};

__device__ __forceinline__ unsigned long long wsum(unsigned long long x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

__device__ __forceinline__ void dm_flush(const DmCtr& c, unsigned long long* __restrict__ stats) {
    __shared__ unsigned long long red[kBlock / 64][8];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned long long v[6] = {c.rm, c.push, c.pull, c.deliv, c.complete, 0};
    unsigned long long ov = c.overflow;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ov |= __shfl_xor(ov, off, 64);
#pragma unroll
    for (int i = 0; i < 5; i++) {
        const unsigned long long s = wsum(v[i]);
        if (lane == 0) red[wv][i + 1] = s;
    }
    if (lane == 0) red[wv][6] = ov;
    __syncthreads();
    if (threadIdx.x >= 1 && threadIdx.x <= 6) {
        const int i = threadIdx.x;
        unsigned long long s = 0;
        for (int w = 0; w < kBlock / 64; w++) s = (i == 6) ? (s | red[w][i]) : (s + red[w][i]);
        if (s) {
            unsigned long long* p = &stats[(blockIdx.x & (kStatShards - 1)) * kNStat + i];
            if (i == 6) atomicOr(p, s);
            else atomicAdd(p, s);
        }
    }
}

// send RM(m) to t: raise the first count plane of t's rumor-m bit that was clear
// (>= 1, >= 2, >= 3 senders); the planes saturate at 3
__device__ __forceinline__ void rm_send(const DmArgs& a, uint32_t t, uint32_t m, DmCtr& c) {
    const unsigned long long b = 1ull << m;
    if (atomicOr(&a.rm_nxt_any[t], b) & b)
        if (atomicOr(&a.rm_nxt_multi[t], b) & b) atomicOr(&a.rm_nxt_tri[t], b);
    c.rm++;
}

// Did target T send rumor m to v last round?  T called select_random_sublist
// for m last round (its call index: the calls before that round plus its
// earlier rumors of that round, handled in rumor order) and drew v.  The
// FromNode T excluded cannot be v: v did not hold m.
__device__ __forceinline__ bool rm_sent_by(const DmArgs& a, uint32_t T, uint32_t v, uint32_t m) {
    const unsigned long long rn = a.rmnew_prev[T];
    if (T == v || !((rn >> m) & 1ull)) return false;
    const uint64_t calls = a.ncall_prev[T] + (uint32_t)__popcll(rn & ((1ull << m) - 1ull));
    const uint2 u = select2(a.key, T, KIND_RM, a.n_global, a.dpc * calls);
    return u.x == v || u.y == v;
}

__global__ __launch_bounds__(kBlock) void dm_round_kernel(DmArgs a) {
    DmCtr c = {0, 0, 0, 0, 0, 0};
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < a.n; i += stride) {
        const uint32_t v = a.v_lo + i;   // global id; i indexes this shard's arrays
        unsigned long long s = a.seen[i];
        const unsigned long long s0 = s;
        // ---- direct mail: handle_info({broadcast, Id, ...}) stores only
        // (demers_direct_mail.erl:127-143); the origins sent to every other member
        s |= a.dm_mail;

        // ---- rumor mongering: handle_info({broadcast, Id, ..., FromNode}) :127-158
        if (a.rm_on) {
            const unsigned long long rn_prev = a.rmnew_prev[v];
            const uint32_t calls0 = a.ncall_prev[v] + (uint32_t)__popcll(rn_prev);   // calls before this round
            unsigned long long rn = 0;
            // the inbox planes are read once (then cleared): non-temporal, ~1-3 % per C4 round
            const unsigned long long any = __builtin_nontemporal_load(a.rm_cur_any + i);
            if (any) {
                const unsigned long long multi = a.rm_cur_multi[i], tri = a.rm_cur_tri[i];
                a.rm_cur_any[i] = 0;
                if (multi) a.rm_cur_multi[i] = 0;
                if (tri) a.rm_cur_tri[i] = 0;
                unsigned long long nw = any & ~s;
                while (nw) {
                    const uint32_t m = __ffsll(nw) - 1;
                    nw &= nw - 1;
                    s |= 1ull << m;                                  // deliver + ets:insert
                    const uint2 tp = select2(a.key, v, KIND_RM, a.n_global,
                                             a.dpc * (calls0 + (uint32_t)__popcll(rn)));
                    rn |= 1ull << m;
                    // FromNode: a non-target sender comes first in the schedule; only when every
                    // sender is one of the two targets is it the smaller target that sent
                    uint32_t from = 0xFFFFFFFFu;
                    const uint32_t senders = 1u + (uint32_t)((multi >> m) & 1ull) + (uint32_t)((tri >> m) & 1ull);
                    if (senders <= 2) {
                        const bool s0 = rm_sent_by(a, tp.x, v, m), s1 = rm_sent_by(a, tp.y, v, m);
                        if (senders == (s0 ? 1u : 0u) + (s1 ? 1u : 0u))
                            from = s0 && s1 ? min(tp.x, tp.y) : (s0 ? tp.x : tp.y);
                    }
                    if (tp.x != v && tp.x != from) rm_send(a, tp.x, m, c);
                    if (tp.y != v && tp.y != from) rm_send(a, tp.y, m, c);
                }
            }
            a.rmnew_cur[v] = rn;            // every vertex, every round: the next round's rmnew_prev
            a.ncall_cur[v] = calls0;
        }

        // ---- anti-entropy push: handle_info({push, FromNode, TheirMessages}) :143-176
        const uint32_t np = a.pushcnt_cur[i];
        if (np) {
            a.pushcnt_cur[i] = 0;
            const uint32_t cnt = np < kDmPushCap ? np : kDmPushCap;
            if (np > a.push_cap) c.overflow |= 1u;
            const uint32_t* lst = a.pushlist_cur + (size_t)i * kDmPushCap;
            if (cnt <= kDmFastPush) {
                // the usual case (Poisson(2) in-degree): the list in registers,
                // sorted there, and every pusher's snapshot requested at once --
                // one dependent round trip instead of one per pusher
                uint32_t x[kDmFastPush];
#pragma unroll
                for (uint32_t j = 0; j < kDmFastPush; j++) x[j] = j < cnt ? lst[j] : 0xFFFFFFFFu;
#pragma unroll
                for (uint32_t j = 1; j < kDmFastPush; j++)          // sorting network over 8 lanes
#pragma unroll
                    for (uint32_t q = j; q > 0; q--) {
                        const uint32_t lo = x[q - 1] < x[q] ? x[q - 1] : x[q];
                        const uint32_t hi = x[q - 1] < x[q] ? x[q] : x[q - 1];
                        x[q - 1] = lo;
                        x[q] = hi;
                    }
                unsigned long long P[kDmFastPush];
#pragma unroll
                for (uint32_t j = 0; j < kDmFastPush; j++) P[j] = j < cnt ? a.snap[x[j]] : 0ull;
#pragma unroll
                for (uint32_t j = 0; j < kDmFastPush; j++) {
                    if (j >= cnt) break;
                    s |= P[j];
                    const uint2 sp = select2(a.key, x[j], KIND_AE, a.n_global, a.dpc * (a.prev_tick - 1u));
                    a.pull_nxt[2 * (size_t)x[j] + (sp.x == v ? 0u : 1u)] = s;   // {pull, MyNode, OurMessages}
                    c.pull++;
                }
            } else {
            uint32_t last = 0;
            bool first = true;
            for (uint32_t k = 0; k < cnt; k++) {                     // senders in id order
                uint32_t best = 0xFFFFFFFFu;
                for (uint32_t j = 0; j < cnt; j++) {
                    const uint32_t x = lst[j];
                    if ((first || x > last) && x < best) best = x;
                }
                first = false;
                last = best;
                const unsigned long long P = a.snap[best];
                s |= P;
                const uint2 sp = select2(a.key, best, KIND_AE, a.n_global, a.dpc * (a.prev_tick - 1u));
                const uint32_t slot = sp.x == v ? 0u : 1u;
                a.pull_nxt[2 * (size_t)best + slot] = s;             // {pull, MyNode, OurMessages}
                c.pull++;
            }
            }
        }

        // ---- anti-entropy pull: handle_info({pull, _, Messages}) :178-195
        // the inbox sets are read once (then cleared): non-temporal, ~1-3 % per C4 round
        const unsigned long long p0 = __builtin_nontemporal_load(a.pull_cur + 2 * (size_t)i),
                                 p1 = __builtin_nontemporal_load(a.pull_cur + 2 * (size_t)i + 1);
        if (p0 | p1) {
            s |= p0 | p1;
            if (p0) a.pull_cur[2 * (size_t)i] = 0;
            if (p1) a.pull_cur[2 * (size_t)i + 1] = 0;
        }

        if (s != s0) {
            a.seen[i] = s;
            c.deliv += __popcll(s & ~s0);
        }

        // ---- anti-entropy tick: handle_info(antientropy) :118-141
        if (a.tick) {
            a.snap[v] = s;
            const uint2 tp = select2(a.key, v, KIND_AE, a.n_global, a.dpc * (a.tick_idx - 1u));   // the tick-th call
            const uint32_t tg[2] = {tp.x, tp.y};
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const uint32_t t = tg[j];
                if (t == v) continue;
                c.push++;
                if (a.sharded) continue;                            // listed by dm_pushscan_kernel
                const uint32_t pos = atomicAdd(&a.pushcnt_nxt[t], 1u);
                if (pos < kDmPushCap) a.pushlist_nxt[(size_t)t * kDmPushCap + pos] = v;
            }
        }
        c.complete += (s & a.full) == a.full;
    }
    dm_flush(c, a.stats);
}

// handle_cast({broadcast, ServerRef, Message}) at every origin (RM :92-115,
// AE :95-106), one thread per rumor; the origins come from the workload stream.
// An origin's RM process makes one select call per rumor it originates, in
// rumor order; the calls are "round 0" for the next round's sender checks
// (rmnew_cur: the buffer round 1 reads as rmnew_prev, zeroed with ncall_cur).
__global__ void dm_broadcast_kernel(DmArgs a, const uint32_t* __restrict__ origin, const uint32_t* __restrict__ idbit) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    DmCtr c = {0, 0, 0, 0, 0, 0};
    if (i < a.m && origin[i] - a.v_lo < a.n) {      // only the origin's shard
        const uint32_t o = origin[i];
        atomicOr(&a.seen[o - a.v_lo], 1ull << idbit[i]);
        if (a.rm_on) {
            uint32_t rank = 0;                       // the origin's earlier rumors
            for (uint32_t j = 0; j < i; j++) rank += origin[j] == o ? 1u : 0u;
            atomicOr(&a.rmnew_cur[o], 1ull << i);
            const uint2 tp = select2(a.key, o, KIND_RM, a.n_global, a.dpc * rank);
            if (tp.x != o) rm_send(a, tp.x, i, c);
            if (tp.y != o) rm_send(a, tp.y, i, c);
        }
    }
    if (c.rm) atomicAdd(&a.stats[1], (unsigned long long)c.rm);
}

// Sharded AE tick: every shard recomputes each global pusher's two targets
// (the Philox stream (u, tick, AE) is a pure function) and lists the pushers
// whose target it owns; the receiver sorts its list by pusher id, so the
// atomicAdd slot order does not matter.
__global__ __launch_bounds__(kBlock) void dm_pushscan_kernel(DmArgs a, uint32_t tick_idx) {
    const uint32_t stride = gridDim.x * kBlock;
    unsigned long long ov = 0;
    for (uint32_t u = blockIdx.x * kBlock + threadIdx.x; u < a.n_global; u += stride) {
        const uint2 tp = select2(a.key, u, KIND_AE, a.n_global, a.dpc * (tick_idx - 1u));
        const uint32_t tg[2] = {tp.x, tp.y};
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const uint32_t t = tg[j];
            if (t == u) continue;
            const uint32_t lt = t - a.v_lo;
            if (lt >= a.n) continue;
            const uint32_t pos = atomicAdd(&a.pushcnt_nxt[lt], 1u);
            if (pos < kDmPushCap) a.pushlist_nxt[(size_t)lt * kDmPushCap + pos] = u;
        }
    }
    (void)ov;
}

// Sharded ingest: this shard's RM count planes = the saturating sum of the
// slices every shard wrote for its range (world slices of `chunk`); its pull
// slots = the reduce-scattered slice (one writer per slot).
__global__ __launch_bounds__(kBlock) void dm_ingest_kernel(DmArgs a, const unsigned long long* __restrict__ rm_recv,
                                                           const unsigned long long* __restrict__ pull_recv,
                                                           uint32_t world, uint32_t chunk) {
    const uint32_t stride = gridDim.x * kBlock;
    const size_t plane = (size_t)world * chunk;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < a.n; i += stride) {
        unsigned long long A = 0, M = 0, T = 0;      // >= 1, >= 2, >= 3 senders so far
        for (uint32_t g = 0; g < world; g++) {
            const size_t o = (size_t)g * chunk + i;
            const unsigned long long x1 = rm_recv[o], x2 = rm_recv[plane + o], x3 = rm_recv[2 * plane + o];
            T |= x3 | (M & x1) | (A & x2);
            M |= x2 | (A & x1);
            A |= x1;
        }
        a.rm_nxt_any[i] = A;
        a.rm_nxt_multi[i] = M;
        a.rm_nxt_tri[i] = T;
        a.pull_nxt[2 * (size_t)i] = pull_recv[2 * (size_t)i];
        a.pull_nxt[2 * (size_t)i + 1] = pull_recv[2 * (size_t)i + 1];
    }
}

// the pull slots of this shard as every source shard wrote them: slice g of
// `in` came from shard g (one writer per slot, so the sum is the one value)
__global__ __launch_bounds__(kBlock) void dm_sum_slices_kernel(const unsigned long long* __restrict__ in,
                                                               uint32_t world, size_t len,
                                                               unsigned long long* __restrict__ out) {
    for (size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x; i < len; i += size_t(gridDim.x) * kBlock) {
        unsigned long long x = 0;
        for (uint32_t g = 0; g < world; g++) x += in[size_t(g) * len + i];
        out[i] = x;
    }
}

// ---- sparse exchange records (psim.h "vertex-sharded Demers") -------------
// A round whose RM messages reach few slots sends {slot, any, multi, tri}
// records (7 words) instead of the three dense 8 B x C slices per peer, and
// its RM call records as {vertex, rumors called, calls before} (4 words)
// instead of the all-gathered 12 B x C planes.

// per destination shard g != rank: slots of slice g with an RM bit (any is
// the superset plane); cnt[world]: this shard's vertices that called select
__global__ __launch_bounds__(kBlock) void dm_xcount_kernel(const unsigned long long* __restrict__ any, uint32_t world,
                                                           uint32_t rank, uint32_t chunk,
                                                           const unsigned long long* __restrict__ rn_own,
                                                           uint32_t n_own, uint32_t* __restrict__ cnt) {
    const size_t total = size_t(world) * chunk;
    const size_t stride = size_t(gridDim.x) * kBlock;
    for (size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x; i < total + n_own; i += stride) {
        bool hit;
        uint32_t g;
        if (i < total) {
            g = (uint32_t)(i / chunk);
            hit = g != rank && any[i] != 0ull;
        } else {
            g = world;
            hit = rn_own[i - total] != 0ull;
        }
        // one atomic per wave and destination: the lanes of a wave share g
        // except where a slice boundary falls inside the wave (lane 0, the
        // lowest index, is active whenever any lane is)
        const uint32_t g0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)g);
        const unsigned long long same = __ballot(hit && g == g0);
        if ((threadIdx.x & 63) == 0 && same) atomicAdd(&cnt[g0], (uint32_t)__popcll(same));
        if (hit && g != g0) atomicAdd(&cnt[g], 1u);
    }
}

// records of the RM slots for shard g at rec + 7 (off[g] + k), k from cursor[g]
__global__ __launch_bounds__(kBlock) void dm_xpack_rm_kernel(const unsigned long long* __restrict__ rm, size_t plane,
                                                             uint32_t world, uint32_t rank, uint32_t chunk,
                                                             const uint32_t* __restrict__ off,
                                                             uint32_t* __restrict__ cursor, uint32_t* __restrict__ rec) {
    const size_t stride = size_t(gridDim.x) * kBlock;
    for (size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x; i < plane; i += stride) {
        const uint32_t g = (uint32_t)(i / chunk);
        const unsigned long long a = rm[i];
        if (g == rank || a == 0ull) continue;
        const unsigned long long m = rm[plane + i], t = rm[2 * plane + i];
        uint32_t* o = rec + 7 * (size_t)(off[g] + atomicAdd(&cursor[g], 1u));
        o[0] = (uint32_t)(i - size_t(g) * chunk);
        o[1] = (uint32_t)a;
        o[2] = (uint32_t)(a >> 32);
        o[3] = (uint32_t)m;
        o[4] = (uint32_t)(m >> 32);
        o[5] = (uint32_t)t;
        o[6] = (uint32_t)(t >> 32);
    }
}

// received RM records into the dense receive planes (slice s = records from
// shard s, off[s] .. off[s+1]; the slices were zeroed)
__global__ __launch_bounds__(kBlock) void dm_xunpack_rm_kernel(const uint32_t* __restrict__ rec,
                                                               const uint32_t* __restrict__ off, uint32_t world,
                                                               uint32_t chunk, size_t plane,
                                                               unsigned long long* __restrict__ rm) {
    const uint32_t total = off[world];
    for (uint32_t j = blockIdx.x * kBlock + threadIdx.x; j < total; j += gridDim.x * kBlock) {
        uint32_t s = 0;
        while (off[s + 1] <= j) s++;
        const uint32_t* x = rec + 7 * (size_t)j;
        const size_t i = size_t(s) * chunk + x[0];
        rm[i] = (unsigned long long)x[1] | ((unsigned long long)x[2] << 32);
        rm[plane + i] = (unsigned long long)x[3] | ((unsigned long long)x[4] << 32);
        rm[2 * plane + i] = (unsigned long long)x[5] | ((unsigned long long)x[6] << 32);
    }
}

// this shard's RM call records {global vertex, rumors called, calls before},
// written once per other shard (regions of `per` records, own region skipped)
__global__ __launch_bounds__(kBlock) void dm_xpack_rmx_kernel(const unsigned long long* __restrict__ rn,
                                                              const uint32_t* __restrict__ ncall, uint32_t v_lo,
                                                              uint32_t n_own, uint32_t world, uint32_t rank,
                                                              uint32_t per, uint32_t* __restrict__ cursor,
                                                              uint32_t* __restrict__ rec) {
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n_own; i += gridDim.x * kBlock) {
        const unsigned long long x = rn[v_lo + i];
        if (x == 0ull) continue;
        const uint32_t k = atomicAdd(cursor, 1u);
        for (uint32_t g = 0, q = 0; g < world; g++) {
            if (g == rank) continue;
            uint32_t* o = rec + 4 * ((size_t)q * per + k);
            o[0] = v_lo + i;
            o[1] = (uint32_t)x;
            o[2] = (uint32_t)(x >> 32);
            o[3] = ncall[v_lo + i];
            q++;
        }
    }
}

__global__ __launch_bounds__(kBlock) void dm_xunpack_rmx_kernel(const uint32_t* __restrict__ rec, uint32_t nrec,
                                                                unsigned long long* __restrict__ rn,
                                                                uint32_t* __restrict__ ncall) {
    for (uint32_t j = blockIdx.x * kBlock + threadIdx.x; j < nrec; j += gridDim.x * kBlock) {
        const uint32_t* x = rec + 4 * (size_t)j;
        rn[x[0]] = (unsigned long long)x[1] | ((unsigned long long)x[2] << 32);
        ncall[x[0]] = x[3];
    }
}

__global__ void dm_origin_kernel(uint2 key, uint32_t n, uint32_t m, uint32_t* __restrict__ origin) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint4 r = philox4x32_10(make_uint4(i, 0u, KIND_WORKLOAD, 0u), key);
    origin[i] = (uint32_t)__umul64hi((uint64_t)r.x | ((uint64_t)r.y << 32), (uint64_t)n);
}

}  // namespace

hipError_t launch_dm_origins(uint2 key, uint32_t n, uint32_t m, uint32_t* origin, hipStream_t s) {
    hipLaunchKernelGGL(dm_origin_kernel, dim3(1), dim3(64), 0, s, key, n, m, origin);
    return hipGetLastError();
}

hipError_t launch_dm_broadcast(const DmArgs& a, const uint32_t* origin, const uint32_t* idbit, hipStream_t s) {
    hipLaunchKernelGGL(dm_broadcast_kernel, dim3(1), dim3(64), 0, s, a, origin, idbit);
    return hipGetLastError();
}

hipError_t launch_dm_pushscan(const DmArgs& a, uint32_t tick_idx, hipStream_t s) {
    uint32_t g = (a.n_global + kBlock - 1) / kBlock;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(dm_pushscan_kernel, dim3(g), dim3(kBlock), 0, s, a, tick_idx);
    return hipGetLastError();
}

hipError_t launch_dm_sum_slices(const unsigned long long* in, uint32_t world, size_t len, unsigned long long* out,
                                hipStream_t s) {
    size_t g = (len + kBlock - 1) / kBlock;
    if (g > 8192) g = 8192;
    if (g == 0) return hipSuccess;
    hipLaunchKernelGGL(dm_sum_slices_kernel, dim3((uint32_t)g), dim3(kBlock), 0, s, in, world, len, out);
    return hipGetLastError();
}

hipError_t launch_dm_ingest_rm(const DmArgs& a, const unsigned long long* rm_recv, const unsigned long long* pull_recv,
                               uint32_t world, uint32_t chunk, hipStream_t s) {
    uint32_t g = (a.n + kBlock - 1) / kBlock;
    if (g > 8192) g = 8192;
    if (g == 0) return hipSuccess;
    hipLaunchKernelGGL(dm_ingest_kernel, dim3(g), dim3(kBlock), 0, s, a, rm_recv, pull_recv, world, chunk);
    return hipGetLastError();
}

static uint32_t dm_grid(size_t n) {
    size_t g = (n + kBlock - 1) / kBlock;
    return (uint32_t)(g > 8192 ? 8192 : (g ? g : 1));
}

hipError_t launch_dm_xcount(const unsigned long long* any, uint32_t world, uint32_t rank, uint32_t chunk,
                            const unsigned long long* rn_own, uint32_t n_own, uint32_t* cnt, hipStream_t s) {
    hipLaunchKernelGGL(dm_xcount_kernel, dim3(dm_grid(size_t(world) * chunk + n_own)), dim3(kBlock), 0, s, any, world,
                       rank, chunk, rn_own, n_own, cnt);
    return hipGetLastError();
}

hipError_t launch_dm_xpack_rm(const unsigned long long* rm, uint32_t world, uint32_t rank, uint32_t chunk,
                              const uint32_t* off, uint32_t* cursor, uint32_t* rec, hipStream_t s) {
    const size_t plane = size_t(world) * chunk;
    hipLaunchKernelGGL(dm_xpack_rm_kernel, dim3(dm_grid(plane)), dim3(kBlock), 0, s, rm, plane, world, rank, chunk, off,
                       cursor, rec);
    return hipGetLastError();
}

hipError_t launch_dm_xunpack_rm(const uint32_t* rec, const uint32_t* off, uint32_t world, uint32_t chunk,
                                uint32_t nrec, unsigned long long* rm, hipStream_t s) {
    if (nrec == 0) return hipSuccess;
    hipLaunchKernelGGL(dm_xunpack_rm_kernel, dim3(dm_grid(nrec)), dim3(kBlock), 0, s, rec, off, world, chunk,
                       size_t(world) * chunk, rm);
    return hipGetLastError();
}

hipError_t launch_dm_xpack_rmx(const unsigned long long* rn, const uint32_t* ncall, uint32_t v_lo, uint32_t n_own,
                               uint32_t world, uint32_t rank, uint32_t per, uint32_t* cursor, uint32_t* rec,
                               hipStream_t s) {
    if (n_own == 0) return hipSuccess;
    hipLaunchKernelGGL(dm_xpack_rmx_kernel, dim3(dm_grid(n_own)), dim3(kBlock), 0, s, rn, ncall, v_lo, n_own, world,
                       rank, per, cursor, rec);
    return hipGetLastError();
}

hipError_t launch_dm_xunpack_rmx(const uint32_t* rec, uint32_t nrec, unsigned long long* rn, uint32_t* ncall,
                                 hipStream_t s) {
    if (nrec == 0) return hipSuccess;
    hipLaunchKernelGGL(dm_xunpack_rmx_kernel, dim3(dm_grid(nrec)), dim3(kBlock), 0, s, rec, nrec, rn, ncall);
    return hipGetLastError();
}

hipError_t launch_dm_round(const DmArgs& a, hipStream_t s) {
    uint32_t g = (a.n + kBlock - 1) / kBlock;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(dm_round_kernel, dim3(g), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace psim
