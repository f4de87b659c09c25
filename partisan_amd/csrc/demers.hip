// demers.hip -- Demers rumor mongering + anti-entropy
// (protocols/demers_rumor_mongering.erl :92-186, protocols/demers_anti_entropy.erl
// :95-227) as one gfx950 kernel per round; the store of each vertex is a
// 64-bit seen-set (one bit per rumor id).
//
// Round formulation (DESIGN.md "Demers"), one thread per vertex:
//  * RM inbox = three 64-bit sets per vertex, written by senders with atomicOr:
//    `reg` (sender is not one of the receiver's own forward targets for the
//    rumor), `t0`/`t1` (sender is the receiver's first/second target).  The
//    schedule processes RM messages by (rumor, class, sender), so for a new
//    rumor the FromNode excluded by `-- [MyNode, FromNode]` is a regular
//    sender (never a target: no effect) unless only targets sent it, in
//    which case it is the smaller of them -- computable from the three sets
//    alone.  Forward draws are the Philox stream (v, rumor, RM), so every
//    vertex can recompute any other vertex's targets: no sorting needed.
//  * AE pushes: the sender appends its id to the receiver's list (atomicAdd
//    slot); the receiver sorts its list (schedule: by sender), merges each
//    pusher's snapshot and answers with its prefix union into the pusher's
//    pull slot k (k = the receiver's index in the pusher's target pair).
//  * AE tick (end of the round): snapshot + push to sample2(v, tick, AE) -- [v].
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

// send RM(m) from v to t: the class is decided by t's own targets for m
__device__ __forceinline__ void rm_send(const DmArgs& a, uint32_t v, uint32_t t, uint32_t m, DmCtr& c) {
    const uint2 tp = sample2(a.key, t, m, KIND_RM, a.n);
    const unsigned long long b = 1ull << m;
    unsigned long long* dst = v == tp.x ? a.rm_nxt_t0 : (v == tp.y ? a.rm_nxt_t1 : a.rm_nxt_reg);
    atomicOr(&dst[t], b);
    c.rm++;
}

__global__ __launch_bounds__(kBlock) void dm_round_kernel(DmArgs a) {
    DmCtr c = {0, 0, 0, 0, 0, 0};
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t v = blockIdx.x * kBlock + threadIdx.x; v < a.n; v += stride) {
        unsigned long long s = a.seen[v];
        const unsigned long long s0 = s;

        // ---- rumor mongering: handle_info({broadcast, Id, ..., FromNode}) :127-158
        if (a.rm_on) {
            const unsigned long long reg = a.rm_cur_reg[v], t0 = a.rm_cur_t0[v], t1 = a.rm_cur_t1[v];
            if (reg | t0 | t1) {
                if (reg) a.rm_cur_reg[v] = 0;
                if (t0) a.rm_cur_t0[v] = 0;
                if (t1) a.rm_cur_t1[v] = 0;
                unsigned long long nw = (reg | t0 | t1) & ~s;
                while (nw) {
                    const uint32_t m = __ffsll(nw) - 1;
                    nw &= nw - 1;
                    s |= 1ull << m;                                  // deliver + ets:insert
                    const uint2 tp = sample2(a.key, v, m, KIND_RM, a.n);
                    uint32_t from = 0xFFFFFFFFu;                     // a regular sender: not a target
                    if (!((reg >> m) & 1ull)) {
                        const bool f0 = (t0 >> m) & 1ull, f1 = (t1 >> m) & 1ull;
                        if (f0 && f1) from = tp.x < tp.y ? tp.x : tp.y;
                        else from = f0 ? tp.x : tp.y;
                    }
                    if (tp.x != v && tp.x != from) rm_send(a, v, tp.x, m, c);
                    if (a.n > 1 && tp.y != v && tp.y != from) rm_send(a, v, tp.y, m, c);
                }
            }
        }

        // ---- anti-entropy push: handle_info({push, FromNode, TheirMessages}) :143-176
        const uint32_t np = a.pushcnt_cur[v];
        if (np) {
            a.pushcnt_cur[v] = 0;
            const uint32_t cnt = np < kDmPushCap ? np : kDmPushCap;
            if (np > kDmPushCap) c.overflow |= 1u;
            const uint32_t* lst = a.pushlist_cur + (size_t)v * kDmPushCap;
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
                const uint2 sp = sample2(a.key, best, a.prev_tick, KIND_AE, a.n);
                const uint32_t slot = sp.x == v ? 0u : 1u;
                a.pull_nxt[2 * (size_t)best + slot] = s;             // {pull, MyNode, OurMessages}
                c.pull++;
            }
        }

        // ---- anti-entropy pull: handle_info({pull, _, Messages}) :178-195
        const unsigned long long p0 = a.pull_cur[2 * (size_t)v], p1 = a.pull_cur[2 * (size_t)v + 1];
        if (p0 | p1) {
            s |= p0 | p1;
            if (p0) a.pull_cur[2 * (size_t)v] = 0;
            if (p1) a.pull_cur[2 * (size_t)v + 1] = 0;
        }

        if (s != s0) {
            a.seen[v] = s;
            c.deliv += __popcll(s & ~s0);
        }

        // ---- anti-entropy tick: handle_info(antientropy) :118-141
        if (a.tick) {
            a.snap[v] = s;
            const uint2 tp = sample2(a.key, v, a.tick_idx, KIND_AE, a.n);
            const uint32_t tg[2] = {tp.x, tp.y};
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const uint32_t t = tg[j];
                if (t == v || (j == 1 && a.n < 2)) continue;
                const uint32_t pos = atomicAdd(&a.pushcnt_nxt[t], 1u);
                if (pos < kDmPushCap) a.pushlist_nxt[(size_t)t * kDmPushCap + pos] = v;
                c.push++;
            }
        }
        c.complete += (s & a.full) == a.full;
    }
    dm_flush(c, a.stats);
}

// handle_cast({broadcast, ServerRef, Message}) at every origin (RM :92-115,
// AE :95-106), one thread per rumor; the origins come from the workload stream.
__global__ void dm_broadcast_kernel(DmArgs a, const uint32_t* __restrict__ origin, const uint32_t* __restrict__ idbit) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    DmCtr c = {0, 0, 0, 0, 0, 0};
    if (i < a.m) {
        const uint32_t o = origin[i];
        atomicOr(&a.seen[o], 1ull << idbit[i]);
        if (a.rm_on) {
            const uint2 tp = sample2(a.key, o, i, KIND_RM, a.n);
            if (tp.x != o) rm_send(a, o, tp.x, i, c);
            if (a.n > 1 && tp.y != o) rm_send(a, o, tp.y, i, c);
        }
    }
    if (c.rm) atomicAdd(&a.stats[1], (unsigned long long)c.rm);
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

hipError_t launch_dm_round(const DmArgs& a, hipStream_t s) {
    uint32_t g = (a.n + kBlock - 1) / kBlock;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(dm_round_kernel, dim3(g), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace psim
