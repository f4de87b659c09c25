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
    const uint2 tp = sample2(a.key, t, m, KIND_RM, a.n_global);
    const unsigned long long b = 1ull << m;
    unsigned long long* dst = v == tp.x ? a.rm_nxt_t0 : (v == tp.y ? a.rm_nxt_t1 : a.rm_nxt_reg);
    atomicOr(&dst[t], b);
    c.rm++;
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
#ifndef DM_TEMPORAL_INBOX   // the inbox sets are read once (then cleared): non-temporal, ~1-3 % per C4 round
            const unsigned long long reg = __builtin_nontemporal_load(a.rm_cur_reg + i),
                                     t0 = __builtin_nontemporal_load(a.rm_cur_t0 + i),
                                     t1 = __builtin_nontemporal_load(a.rm_cur_t1 + i);
#else
            const unsigned long long reg = a.rm_cur_reg[i], t0 = a.rm_cur_t0[i], t1 = a.rm_cur_t1[i];
#endif
            if (reg | t0 | t1) {
                if (reg) a.rm_cur_reg[i] = 0;
                if (t0) a.rm_cur_t0[i] = 0;
                if (t1) a.rm_cur_t1[i] = 0;
                unsigned long long nw = (reg | t0 | t1) & ~s;
                while (nw) {
                    const uint32_t m = __ffsll(nw) - 1;
                    nw &= nw - 1;
                    s |= 1ull << m;                                  // deliver + ets:insert
                    const uint2 tp = sample2(a.key, v, m, KIND_RM, a.n_global);
                    uint32_t from = 0xFFFFFFFFu;                     // a regular sender: not a target
                    if (!((reg >> m) & 1ull)) {
                        const bool f0 = (t0 >> m) & 1ull, f1 = (t1 >> m) & 1ull;
                        if (f0 && f1) from = tp.x < tp.y ? tp.x : tp.y;
                        else from = f0 ? tp.x : tp.y;
                    }
                    if (tp.x != v && tp.x != from) rm_send(a, v, tp.x, m, c);
                    if (a.n_global > 1 && tp.y != v && tp.y != from) rm_send(a, v, tp.y, m, c);
                }
            }
        }

        // ---- anti-entropy push: handle_info({push, FromNode, TheirMessages}) :143-176
        const uint32_t np = a.pushcnt_cur[i];
        if (np) {
            a.pushcnt_cur[i] = 0;
            const uint32_t cnt = np < kDmPushCap ? np : kDmPushCap;
            if (np > kDmPushCap) c.overflow |= 1u;
            const uint32_t* lst = a.pushlist_cur + (size_t)i * kDmPushCap;
#ifndef DM_NO_FAST_AE
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
                    const uint2 sp = sample2(a.key, x[j], a.prev_tick, KIND_AE, a.n_global);
                    a.pull_nxt[2 * (size_t)x[j] + (sp.x == v ? 0u : 1u)] = s;   // {pull, MyNode, OurMessages}
                    c.pull++;
                }
            } else
#endif
            {
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
                const uint2 sp = sample2(a.key, best, a.prev_tick, KIND_AE, a.n_global);
                const uint32_t slot = sp.x == v ? 0u : 1u;
                a.pull_nxt[2 * (size_t)best + slot] = s;             // {pull, MyNode, OurMessages}
                c.pull++;
            }
            }
        }

        // ---- anti-entropy pull: handle_info({pull, _, Messages}) :178-195
#ifndef DM_TEMPORAL_INBOX   // the inbox sets are read once (then cleared): non-temporal, ~1-3 % per C4 round
        const unsigned long long p0 = __builtin_nontemporal_load(a.pull_cur + 2 * (size_t)i),
                                 p1 = __builtin_nontemporal_load(a.pull_cur + 2 * (size_t)i + 1);
#else
        const unsigned long long p0 = a.pull_cur[2 * (size_t)i], p1 = a.pull_cur[2 * (size_t)i + 1];
#endif
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
            const uint2 tp = sample2(a.key, v, a.tick_idx, KIND_AE, a.n_global);
            const uint32_t tg[2] = {tp.x, tp.y};
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const uint32_t t = tg[j];
                if (t == v || (j == 1 && a.n_global < 2)) continue;
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
__global__ void dm_broadcast_kernel(DmArgs a, const uint32_t* __restrict__ origin, const uint32_t* __restrict__ idbit) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    DmCtr c = {0, 0, 0, 0, 0, 0};
    if (i < a.m && origin[i] - a.v_lo < a.n) {      // only the origin's shard
        const uint32_t o = origin[i];
        atomicOr(&a.seen[o - a.v_lo], 1ull << idbit[i]);
        if (a.rm_on) {
            const uint2 tp = sample2(a.key, o, i, KIND_RM, a.n_global);
            if (tp.x != o) rm_send(a, o, tp.x, i, c);
            if (a.n_global > 1 && tp.y != o) rm_send(a, o, tp.y, i, c);
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
        const uint2 tp = sample2(a.key, u, tick_idx, KIND_AE, a.n_global);
        const uint32_t tg[2] = {tp.x, tp.y};
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const uint32_t t = tg[j];
            if (t == u || (j == 1 && a.n_global < 2)) continue;
            const uint32_t lt = t - a.v_lo;
            if (lt >= a.n) continue;
            const uint32_t pos = atomicAdd(&a.pushcnt_nxt[lt], 1u);
            if (pos < kDmPushCap) a.pushlist_nxt[(size_t)lt * kDmPushCap + pos] = u;
        }
    }
    (void)ov;
}

// Sharded ingest: this shard's RM inboxes = OR of the slices every shard
// wrote for its range (world slices of `chunk`); its pull slots = the
// reduce-scattered slice (one writer per slot).
__global__ __launch_bounds__(kBlock) void dm_ingest_kernel(DmArgs a, const unsigned long long* __restrict__ rm_recv,
                                                           const unsigned long long* __restrict__ pull_recv,
                                                           uint32_t world, uint32_t chunk) {
    const uint32_t stride = gridDim.x * kBlock;
    const size_t plane = (size_t)world * chunk;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < a.n; i += stride) {
        unsigned long long r0 = 0, r1 = 0, r2 = 0;
        for (uint32_t g = 0; g < world; g++) {
            const size_t o = (size_t)g * chunk + i;
            r0 |= rm_recv[o];
            r1 |= rm_recv[plane + o];
            r2 |= rm_recv[2 * plane + o];
        }
        a.rm_nxt_reg[i] = r0;
        a.rm_nxt_t0[i] = r1;
        a.rm_nxt_t1[i] = r2;
        a.pull_nxt[2 * (size_t)i] = pull_recv[2 * (size_t)i];
        a.pull_nxt[2 * (size_t)i + 1] = pull_recv[2 * (size_t)i + 1];
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

hipError_t launch_dm_ingest(const DmArgs& a, const unsigned long long* rm_recv, const unsigned long long* pull_recv,
                            uint32_t world, uint32_t chunk, hipStream_t s) {
    uint32_t g = (a.n + kBlock - 1) / kBlock;
    if (g > 8192) g = 8192;
    if (g == 0) return hipSuccess;
    hipLaunchKernelGGL(dm_ingest_kernel, dim3(g), dim3(kBlock), 0, s, a, rm_recv, pull_recv, world, chunk);
    return hipGetLastError();
}

hipError_t launch_dm_round(const DmArgs& a, hipStream_t s) {
    uint32_t g = (a.n + kBlock - 1) / kBlock;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(dm_round_kernel, dim3(g), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace psim

// ---------------------------------------------------------------------------
// host side of the vertex-sharded Demers epidemic (psim_demers_shard_*):
// shard r owns global ids [r C, min((r+1) C, n)), C = ceil(n / world).  A
// round is split-phase so that the transport stays the caller's:
//   psim_demers_shard_round  -- the local round; RM messages to any vertex
//       land in the caller's rm_shadow [3][world C] (OR), pull replies in
//       pull_shadow [world C][2] (one writer per slot), the tick's snapshot
//       in snap_all[v];
//   caller: all_to_all of rm_shadow (slice d -> shard d), reduce_scatter(sum)
//       of pull_shadow, all_gather of snap_all after a tick (RCCL on a node);
//   psim_demers_shard_ingest -- OR the received RM slices into the inboxes,
//       take the pull slice, list the tick's pushers per local receiver.
// ---------------------------------------------------------------------------
#include <algorithm>
#include <cstring>
#include <vector>

using namespace psim;

namespace {

struct DmShard : ModuleState {
    uint32_t n_global = 0, m = 0, ae_period = 0, rm_on = 0, world = 1, rank = 0, chunk = 0, v_lo = 0, n = 0;
    unsigned long long full = 0;
    unsigned long long *seen = nullptr, *rm[3] = {}, *pull = nullptr, *stats = nullptr;
    uint32_t *pushcnt[2] = {}, *pushlist[2] = {}, *origin = nullptr, *idbit = nullptr;
    std::vector<uint32_t> h_origin;
    uint32_t par = 0;
    uint64_t round = 0;
    ~DmShard() override {
        void* p[] = {seen, rm[0], rm[1], rm[2], pull, stats, pushcnt[0], pushcnt[1], pushlist[0], pushlist[1], origin,
                     idbit};
        for (void* x : p)
            if (x) (void)hipFree(x);
    }
};

DmShard* dms_of(psim_handle* h) { return static_cast<DmShard*>(handle_module(h, MOD_DMSHARD)); }
const DmShard* dms_of(const psim_handle* h) { return static_cast<const DmShard*>(handle_module(h, MOD_DMSHARD)); }

#define DMCHK(h, x)                                                                         \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess)                                                               \
            return handle_fail((h), PSIM_EHIP, "%s failed: %s", #x, hipGetErrorString(e_)); \
    } while (0)

DmArgs dms_args(const psim_handle* h, const DmShard& d, void* rm_shadow, void* pull_shadow, void* snap_all) {
    DmArgs a{};
    a.n = d.n;
    a.m = d.m;
    a.v_lo = d.v_lo;
    a.n_global = d.n_global;
    a.sharded = 1;
    const uint64_t seed = handle_seed(h);
    a.key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
    a.rm_on = d.rm_on;
    a.full = d.full;
    a.seen = d.seen;
    a.snap = (unsigned long long*)snap_all;
    a.rm_cur_reg = d.rm[0];
    a.rm_cur_t0 = d.rm[1];
    a.rm_cur_t1 = d.rm[2];
    const size_t plane = (size_t)d.world * d.chunk;
    unsigned long long* rs = (unsigned long long*)rm_shadow;
    a.rm_nxt_reg = rs;
    a.rm_nxt_t0 = rs ? rs + plane : nullptr;
    a.rm_nxt_t1 = rs ? rs + 2 * plane : nullptr;
    a.pushcnt_cur = d.pushcnt[d.par];
    a.pushcnt_nxt = d.pushcnt[d.par ^ 1];
    a.pushlist_cur = d.pushlist[d.par];
    a.pushlist_nxt = d.pushlist[d.par ^ 1];
    a.pull_cur = d.pull;
    a.pull_nxt = (unsigned long long*)pull_shadow;
    a.stats = d.stats;
    return a;
}

}  // namespace

extern "C" {

int psim_demers_shard_setup(psim_handle* h, uint32_t n, uint32_t m, uint32_t ae_period, uint32_t rm_on, int rank,
                            int world, uint64_t* chunk_out) {
    if (!h || n < 2 || m == 0 || m > 64 || ae_period == 1 || rm_on > 1 || world < 1 || rank < 0 || rank >= world)
        return PSIM_EINVAL;
    DMCHK(h, hipSetDevice(handle_device(h)));
    DMCHK(h, hipStreamSynchronize(handle_stream(h)));
    ModuleState*& slot = handle_module(h, MOD_DMSHARD);
    delete slot;
    slot = nullptr;
    DmShard* d = new DmShard();
    d->n_global = n;
    d->m = m;
    d->ae_period = ae_period;
    d->rm_on = rm_on ? 1u : 0u;
    d->world = (uint32_t)world;
    d->rank = (uint32_t)rank;
    d->chunk = (uint32_t)((uint64_t(n) + world - 1) / world);
    d->v_lo = std::min<uint32_t>(n, d->chunk * (uint32_t)rank);
    d->n = std::min<uint32_t>(n, d->v_lo + d->chunk) - d->v_lo;
    const size_t N = std::max<uint32_t>(d->n, 1);
    auto A = [&](void** p, size_t bytes) { return alloc_zero(p, bytes); };
    bool ok = A((void**)&d->seen, N * 8) && A((void**)&d->pull, N * 16) && A((void**)&d->stats, kStatShards * kNStat * 8) &&
              A((void**)&d->origin, 64 * 4) && A((void**)&d->idbit, 64 * 4);
    for (int k = 0; k < 3 && ok; k++) ok = A((void**)&d->rm[k], N * 8);
    for (int p = 0; p < 2 && ok; p++)
        ok = A((void**)&d->pushcnt[p], N * 4) && A((void**)&d->pushlist[p], N * kDmPushCap * 4);
    if (!ok) {
        const uint32_t nl = d->n;
        delete d;
        return handle_fail(h, PSIM_ENOMEM, "demers shard state for %u vertices", nl);
    }
    slot = d;
    const uint64_t seed = handle_seed(h);
    const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
    DMCHK(h, launch_dm_origins(key, n, m, d->origin, handle_stream(h)));
    d->h_origin.assign(m, 0);
    DMCHK(h, hipMemcpyAsync(d->h_origin.data(), d->origin, m * 4, hipMemcpyDeviceToHost, handle_stream(h)));
    DMCHK(h, hipStreamSynchronize(handle_stream(h)));
    std::vector<uint32_t> idbit(m);
    for (uint32_t i = 0; i < m; i++) {
        idbit[i] = i;
        if (!d->rm_on)   // anti-entropy alone: ids {Node, 0} (Q20)
            for (uint32_t j = 0; j < i; j++)
                if (d->h_origin[j] == d->h_origin[i]) { idbit[i] = idbit[j]; break; }
        d->full |= 1ull << idbit[i];
    }
    DMCHK(h, hipMemcpy(d->idbit, idbit.data(), m * 4, hipMemcpyHostToDevice));
    if (chunk_out) *chunk_out = d->chunk;
    return PSIM_OK;
}

int psim_demers_shard_info(const psim_handle* h, uint32_t* v_lo, uint32_t* n_local, uint64_t* chunk) {
    if (!h) return PSIM_EINVAL;
    const DmShard* d = dms_of(h);
    if (!d) return PSIM_ESTATE;
    if (v_lo) *v_lo = d->v_lo;
    if (n_local) *n_local = d->n;
    if (chunk) *chunk = d->chunk;
    return PSIM_OK;
}

int psim_demers_shard_broadcast_all(psim_handle* h, void* rm_shadow) {
    if (!h || !rm_shadow) return PSIM_EINVAL;
    DmShard* d = dms_of(h);
    if (!d) return handle_fail(h, PSIM_ESTATE, "psim_demers_shard_setup not called");
    DMCHK(h, hipSetDevice(handle_device(h)));
    DMCHK(h, hipMemsetAsync(d->stats, 0, kStatShards * kNStat * 8, handle_stream(h)));
    DmArgs a = dms_args(h, *d, rm_shadow, nullptr, nullptr);
    DMCHK(h, launch_dm_broadcast(a, d->origin, d->idbit, handle_stream(h)));
    DMCHK(h, hipStreamSynchronize(handle_stream(h)));
    return PSIM_OK;
}

int psim_demers_shard_round(psim_handle* h, void* rm_shadow, void* pull_shadow, void* snap_all,
                            psim_demers_stats* st, uint32_t* tick) {
    if (!h || !rm_shadow || !pull_shadow || !snap_all) return PSIM_EINVAL;
    DmShard* d = dms_of(h);
    if (!d) return handle_fail(h, PSIM_ESTATE, "psim_demers_shard_setup not called");
    const hipStream_t s = handle_stream(h);
    DMCHK(h, hipSetDevice(handle_device(h)));
    DMCHK(h, hipMemsetAsync(d->stats, 0, kStatShards * kNStat * 8, s));
    DmArgs a = dms_args(h, *d, rm_shadow, pull_shadow, snap_all);
    const uint64_t t = d->round + 1;
    a.tick = d->ae_period && (t % d->ae_period) == 0;
    a.tick_idx = d->ae_period ? (uint32_t)(t / d->ae_period) : 0;
    a.prev_tick = d->ae_period ? (uint32_t)(d->round / d->ae_period) : 0;
    DMCHK(h, hipEventRecord(handle_event(h, 0), s));
    DMCHK(h, launch_dm_round(a, s));
    DMCHK(h, hipEventRecord(handle_event(h, 1), s));
    std::vector<unsigned long long> hs(size_t(kStatShards) * kNStat);
    DMCHK(h, hipMemcpyAsync(hs.data(), d->stats, hs.size() * 8, hipMemcpyDeviceToHost, s));
    DMCHK(h, hipStreamSynchronize(s));
    unsigned long long r[kNStat] = {0};
    for (int sh = 0; sh < kStatShards; sh++)
        for (int i = 0; i < kNStat; i++) {
            if (i == 6) r[i] |= hs[sh * kNStat + i];
            else r[i] += hs[sh * kNStat + i];
        }
    float ms = 0.f;
    DMCHK(h, hipEventElapsedTime(&ms, handle_event(h, 0), handle_event(h, 1)));
    handle_add_round(h, ms);
    d->round = t;
    if (tick) *tick = a.tick;
    if (r[6]) return handle_fail(h, PSIM_EOVERFLOW, "demers shard round %llu: > %u anti-entropy pushes to one vertex",
                                 (unsigned long long)t, kDmPushCap);
    if (st) {
        memset(st, 0, sizeof *st);
        st->rm_sent = r[1];
        st->push_sent = r[2];
        st->pull_sent = r[3];
        st->delivered_new = r[4];
        st->complete = r[5];
        const uint64_t msgs = r[1] + r[2] + r[3];
        st->algo_bytes = 2ull * d->n * d->m / 8 + r[2] * 6ull * d->m / 8 + 32ull * msgs;
        st->kernel_ms = ms;
    }
    return PSIM_OK;
}

int psim_demers_shard_ingest(psim_handle* h, const void* rm_recv, const void* pull_recv, uint32_t tick) {
    if (!h || !rm_recv || !pull_recv) return PSIM_EINVAL;
    DmShard* d = dms_of(h);
    if (!d) return handle_fail(h, PSIM_ESTATE, "psim_demers_shard_setup not called");
    const hipStream_t s = handle_stream(h);
    DMCHK(h, hipSetDevice(handle_device(h)));
    DmArgs a = dms_args(h, *d, nullptr, nullptr, nullptr);
    a.rm_nxt_reg = d->rm[0];          // the inboxes the next round reads
    a.rm_nxt_t0 = d->rm[1];
    a.rm_nxt_t1 = d->rm[2];
    a.pull_nxt = d->pull;
    DMCHK(h, launch_dm_ingest(a, (const unsigned long long*)rm_recv, (const unsigned long long*)pull_recv, d->world,
                              d->chunk, s));
    if (tick) DMCHK(h, launch_dm_pushscan(a, (uint32_t)(d->round / d->ae_period), s));
    DMCHK(h, hipStreamSynchronize(s));
    d->par ^= 1u;
    return PSIM_OK;
}

int psim_demers_shard_get_seen(const psim_handle* h, uint64_t* seen, size_t n) {
    if (!h || !seen) return PSIM_EINVAL;
    const DmShard* d = dms_of(h);
    if (!d) return PSIM_ESTATE;
    psim_handle* hh = const_cast<psim_handle*>(h);
    if (n != d->n) return handle_fail(hh, PSIM_EINVAL, "shard holds %u vertices", d->n);
    DMCHK(hh, hipSetDevice(handle_device(h)));
    DMCHK(hh, hipStreamSynchronize(handle_stream(h)));
    if (n) DMCHK(hh, hipMemcpy(seen, d->seen, n * 8, hipMemcpyDeviceToHost));
    return PSIM_OK;
}

}  // extern "C"
