// relay.hip -- transitive relay over Plumtree out-links for gfx950 (SURVEY
// 8(f) row 2): do_send_message/3 with `transitive => true`
// (src/partisan_hyparview_peer_service_manager.erl:2220-2290), do_tree_forward/4
// (:2796-2842) and handle_message({relay_message, Node, Message, TTL})
// (:1800-1832), for a batch of sends over millions of virtual peers.
//
// The reference keeps no relay state and no dedup: every copy is handled on
// its own, so a round is a queue of copies and the only outputs are counts
// (copies that reached each destination, the first arrival round, per-round
// totals) -- all independent of the order copies are handled in.  That makes
// the device formulation plain and exact:
//   * one thread per copy; a copy is an 8-byte record {at, k<<8 | kind<<7 | ttl}
//     (kind 0 = relay_message to `at`, 1 = Message arriving at dst[k]);
//   * a thread decides its copy's fate (member scans of two short CSR rows),
//     keeps the surviving out-links as a bit mask, and the wave appends all
//     of its emissions with ONE atomicAdd on the next queue's counter
//     (inclusive scan over the 64 lanes with shuffles) -- contiguous runs;
//   * counters are reduced per workgroup in LDS and added to one of 64
//     shards of this round's stats row.
// Bound: HBM latency/bandwidth of the random row reads (no MFMA: no
// contraction).  Per copy: 8 B record read, 8 B per emitted record written,
// the copy vertex's two row offsets and row ids.
#include "psim_internal.h"
#include "../../include/psim.h"

#include <algorithm>
#include <vector>

namespace psim {

namespace {

constexpr int kRlNStat = 5;               // direct, relay, dropped, lost, arrived
constexpr uint32_t kRlMaxOl = 64;         // out-links per vertex (u64 mask)

struct RlArgs {
    const uint32_t *act_ptr, *act, *peer_ptr, *peer, *ol_ptr, *ol;
    const uint8_t* alive;
    const unsigned long long* olmask;     // [n] out-links that are connected (bit j = ol[ol_ptr[v] + j])
    const uint8_t* nlost;                 // [n] out-links (minus self) that are not
    const uint32_t *src, *dst;
    unsigned long long* delivered;
    uint32_t* first_round;
    const uint2* cur;
    uint32_t ncur;
    uint2* nxt;
    uint32_t* nnxt;                        // next queue's append counter
    uint32_t* ovf;                         // set when a round exceeds cap
    uint32_t cap;
    unsigned long long* stats;             // this round: [kStatShards][kRlNStat]
    uint32_t round, relay_ttl;
};

__device__ __forceinline__ bool member(const uint32_t* __restrict__ ptr, const uint32_t* __restrict__ ids,
                                       uint32_t v, uint32_t x) {
    const uint32_t e = ptr[v + 1];
    for (uint32_t i = ptr[v]; i < e; i++)
        if (ids[i] == x) return true;
    return false;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    return x;
}

// kOrigin: round 0, thread i handles send i at its origin (do_send_message:
// connected -> send, else do_tree_forward with relay_ttl).  Otherwise thread
// i handles copy i of the current queue.
template <bool kOrigin>
__global__ __launch_bounds__(kBlock) void rl_round_kernel(RlArgs a) {
    __shared__ unsigned long long red[kBlock / 64][kRlNStat];
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t c_direct = 0, c_relay = 0, c_drop = 0, c_lost = 0, c_arr = 0;
    // what this thread emits: a direct copy, or relays over the out-links in mask
    uint32_t v = 0, k = 0, ttl = 0, nemit = 0;
    bool emit_direct = false;
    unsigned long long mask = 0;
    if (i < a.ncur) {
        bool live = true, origin = kOrigin;
        if (kOrigin) {
            v = a.src[i];
            k = i;
            ttl = a.relay_ttl;
            live = a.alive[v] != 0;             // a dead origin sends nothing
        } else {
            const uint2 r = a.cur[i];
            v = r.x;
            k = r.y >> 8;
            ttl = r.y & 0x7Fu;
            if ((r.y >> 7) & 1u) {              // Message reached Node
                atomicAdd(&a.delivered[k], 1ull);
                atomicMin(&a.first_round[k], a.round);
                c_arr = 1;
                live = false;
            }
        }
        if (live) {
            const uint32_t d = a.dst[k];
            // origin: connected (a peer) -- relay: lists:member(Node, ActiveMembers)
            const bool direct = a.alive[d] &&
                                (origin ? member(a.peer_ptr, a.peer, v, d) : member(a.act_ptr, a.act, v, d));
            if (direct) {
                emit_direct = true;
                nemit = 1;
                c_direct = 1;
            } else if (!origin && ttl == 0) {
                c_drop = 1;                     // TTL expired: dropped
            } else {                            // do_tree_forward: OutLinks -- [MyNode]
                mask = a.olmask[v];             // connectivity is fixed during a run (rl_prep_kernel)
                nemit = __popcll(mask);
                c_lost = a.nlost[v];            // not connected: the send fails, no retry
                c_relay = nemit;
            }
        }
    }
    // wave-aggregated append: one atomic per wave on the next queue's counter
    const uint32_t incl = wave_incl_scan(nemit);
    uint32_t base = 0;
    if (lane == 63 && incl) base = atomicAdd(a.nnxt, incl);
    base = __shfl(base, 63, 64);
    const uint32_t total = __shfl(incl, 63, 64);
    if (total) {
        uint32_t pos = base + incl - nemit;
        if (base + total > a.cap) *a.ovf = 1u;
        if (emit_direct) {
            if (pos < a.cap) a.nxt[pos] = make_uint2(a.dst[k], (k << 8) | (1u << 7));
        } else if (mask) {
            const uint32_t b = a.ol_ptr[v];
            const uint32_t nt = ttl - 1;        // {relay_message, Node, Message, TTL - 1}
            while (mask) {
                const uint32_t j = __ffsll(mask) - 1;
                mask &= mask - 1;
                if (pos < a.cap) a.nxt[pos] = make_uint2(a.ol[b + j], (k << 8) | nt);
                pos++;
            }
        }
    }
    // per-workgroup counters -> one of 64 shards
    const uint32_t cs[kRlNStat] = {c_direct, c_relay, c_drop, c_lost, c_arr};
#pragma unroll
    for (int s = 0; s < kRlNStat; s++) {
        unsigned long long x = cs[s];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
        if (lane == 0) red[wv][s] = x;
    }
    __syncthreads();
    if (threadIdx.x < kRlNStat) {
        unsigned long long x = 0;
        for (int w = 0; w < kBlock / 64; w++) x += red[w][threadIdx.x];
        if (x) atomicAdd(&a.stats[(blockIdx.x & (kStatShards - 1)) * kRlNStat + threadIdx.x], x);
    }
}

// Per vertex, once per run: which out-links are connected (live and a peer)
// -- views and liveness do not change while a batch is relayed, so every copy
// at v reuses the mask instead of rescanning v's peer row per out-link.
__global__ __launch_bounds__(kBlock) void rl_prep_kernel(RlArgs a, uint32_t n, unsigned long long* olmask,
                                                         uint8_t* nlost) {
    const uint32_t v = blockIdx.x * kBlock + threadIdx.x;
    if (v >= n) return;
    const uint32_t b = a.ol_ptr[v], e = a.ol_ptr[v + 1];
    unsigned long long m = 0;
    uint32_t lost = 0;
    for (uint32_t j = b; j < e; j++) {
        const uint32_t p = a.ol[j];
        if (p == v) continue;
        if (a.alive[p] && member(a.peer_ptr, a.peer, v, p)) m |= 1ull << (j - b);
        else lost++;
    }
    olmask[v] = m;
    nlost[v] = (uint8_t)lost;
}

// Device buffers kept on the handle between runs (grown on demand).
struct RelayState : ModuleState {
    void* buf[18] = {};
    size_t cap[18] = {};
    ~RelayState() override {
        for (void* p : buf)
            if (p) (void)hipFree(p);
    }
    // buffer slot i with at least `bytes` bytes (contents undefined)
    void* get(int i, size_t bytes) {
        if (bytes == 0) bytes = 8;
        if (cap[i] < bytes) {
            if (buf[i]) (void)hipFree(buf[i]);
            buf[i] = nullptr;
            cap[i] = 0;
            if (hipMalloc(&buf[i], bytes) != hipSuccess) return nullptr;
            cap[i] = bytes;
        }
        return buf[i];
    }
};

// u64 CSR offsets -> u32 device offsets (checked)
bool narrow(const uint64_t* p, uint32_t n, std::vector<uint32_t>& out) {
    out.resize((size_t)n + 1);
    for (size_t i = 0; i <= n; i++) {
        if (p[i] > 0xFFFFFFFFull || (i && p[i] < p[i - 1])) return false;
        out[i] = (uint32_t)p[i];
    }
    return true;
}

}  // namespace

}  // namespace psim

#define RL_HIP(h, x)                                                                                    \
    do {                                                                                                \
        hipError_t e_ = (x);                                                                            \
        if (e_ != hipSuccess) return psim::handle_fail((h), PSIM_EHIP, "%s failed: %s", #x, hipGetErrorString(e_)); \
    } while (0)

extern "C" int64_t psim_relay_run(psim_handle* h, uint32_t n, const uint64_t* act_ptr, const uint32_t* act,
                                  uint64_t act_len, const uint64_t* ol_ptr, const uint32_t* ol, uint64_t ol_len,
                                  const uint8_t* alive, uint32_t k,
                                  const uint32_t* src, const uint32_t* dst, uint32_t relay_ttl,
                                  uint64_t* delivered, uint32_t* first_round, psim_relay_stats* stats,
                                  size_t cap, size_t max_copies) {
    using namespace psim;
    if (!h) return PSIM_EINVAL;
    if (!act_ptr || !ol_ptr || !alive || n == 0 || (k && (!src || !dst || !delivered || !first_round)))
        return handle_fail(h, PSIM_EINVAL, "psim_relay_run: null argument");
    if (relay_ttl == 0 || relay_ttl > 127) return handle_fail(h, PSIM_EINVAL, "relay_ttl %u not in 1..127", relay_ttl);
    if (k >= (1u << 24)) return handle_fail(h, PSIM_EINVAL, "k = %u sends (max 2^24 - 1)", k);
    if (max_copies == 0 || max_copies > 0x7FFFFFFFull) return handle_fail(h, PSIM_EINVAL, "max_copies %zu", max_copies);
    for (uint32_t i = 0; i < k; i++)
        if (src[i] >= n || dst[i] >= n || src[i] == dst[i])
            return handle_fail(h, PSIM_EINVAL, "send %u: %u -> %u (n = %u)", i, src[i], dst[i], n);
    std::vector<uint32_t> ap, op;
    if (!narrow(act_ptr, n, ap) || !narrow(ol_ptr, n, op))
        return handle_fail(h, PSIM_EINVAL, "CSR offsets not monotone or >= 2^32");
    if (ap[0] != 0 || ap[n] != act_len || op[0] != 0 || op[n] != ol_len || (act_len && !act) || (ol_len && !ol))
        return handle_fail(h, PSIM_EINVAL, "CSR rows do not cover act[%llu] / ol[%llu] exactly",
                           (unsigned long long)act_len, (unsigned long long)ol_len);
    const uint64_t na = ap[n], no = op[n];
    for (uint64_t i = 0; i < na; i++)
        if (act[i] >= n) return handle_fail(h, PSIM_EINVAL, "act[%llu] = %u >= n", (unsigned long long)i, act[i]);
    for (uint32_t v = 0; v < n; v++) {
        if (op[v + 1] - op[v] > kRlMaxOl)
            return handle_fail(h, PSIM_EINVAL, "vertex %u has %u out-links (max %u)", v, op[v + 1] - op[v], kRlMaxOl);
        for (uint32_t j = op[v]; j < op[v + 1]; j++)
            if (ol[j] >= n) return handle_fail(h, PSIM_EINVAL, "ol[%u] = %u >= n", j, ol[j]);
    }
    if (2 * na > 0xFFFFFFFFull) return handle_fail(h, PSIM_EINVAL, "too many view entries");
    // peers = view members plus the vertices whose view lists v (connections are symmetric)
    std::vector<uint32_t> pp((size_t)n + 1, 0), pe(2 * na), fill(n, 0);
    for (uint32_t v = 0; v < n; v++)
        for (uint32_t i = ap[v]; i < ap[v + 1]; i++) {
            pp[v + 1]++;
            pp[act[i] + 1]++;
        }
    for (uint32_t v = 0; v < n; v++) pp[v + 1] += pp[v];
    for (uint32_t v = 0; v < n; v++)
        for (uint32_t i = ap[v]; i < ap[v + 1]; i++) {
            pe[pp[v] + fill[v]++] = act[i];
            pe[pp[act[i]] + fill[act[i]]++] = v;
        }
    {   // a symmetric pair lists each peer twice: sort + unique every row (shorter member scans)
        uint32_t out = 0;
        for (uint32_t v = 0; v < n; v++) {
            const uint32_t b = pp[v], e = pp[v + 1];
            std::sort(pe.begin() + b, pe.begin() + e);
            const uint32_t start = out;
            for (uint32_t i = b; i < e; i++)
                if (i == b || pe[i] != pe[i - 1]) pe[out++] = pe[i];
            pp[v] = start;
        }
        pp[n] = out;
        pe.resize(out ? out : 1);
    }

    ModuleState*& slot = handle_module(h, MOD_RELAY);
    if (!slot) slot = new RelayState();
    RelayState* st = static_cast<RelayState*>(slot);
    const hipStream_t s = handle_stream(h);
    RL_HIP(h, hipSetDevice(handle_device(h)));
    const size_t nrounds_max = (size_t)relay_ttl + 3;
    const size_t stat_row = (size_t)kStatShards * kRlNStat;
    RlArgs a{};
    uint32_t *d_ap = (uint32_t*)st->get(0, ap.size() * 4), *d_act = (uint32_t*)st->get(1, na * 4),
             *d_pp = (uint32_t*)st->get(2, pp.size() * 4), *d_pe = (uint32_t*)st->get(3, pe.size() * 4),
             *d_op = (uint32_t*)st->get(4, op.size() * 4), *d_ol = (uint32_t*)st->get(5, no * 4),
             *d_src = (uint32_t*)st->get(7, (size_t)k * 4), *d_dst = (uint32_t*)st->get(8, (size_t)k * 4),
             *d_first = (uint32_t*)st->get(10, (size_t)k * 4), *d_cnt = (uint32_t*)st->get(13, 64);
    uint8_t* d_alive = (uint8_t*)st->get(6, n);
    unsigned long long* d_deliv = (unsigned long long*)st->get(9, (size_t)k * 8);
    uint2 *d_q0 = (uint2*)st->get(11, max_copies * 8), *d_q1 = (uint2*)st->get(12, max_copies * 8);
    unsigned long long* d_stats = (unsigned long long*)st->get(14, nrounds_max * stat_row * 8);
    unsigned long long* d_olmask = (unsigned long long*)st->get(15, (size_t)n * 8);
    uint8_t* d_nlost = (uint8_t*)st->get(16, n);
    if (!d_ap || !d_act || !d_pp || !d_pe || !d_op || !d_ol || !d_src || !d_dst || !d_first || !d_cnt || !d_alive ||
        !d_deliv || !d_q0 || !d_q1 || !d_stats || !d_olmask || !d_nlost)
        return handle_fail(h, PSIM_ENOMEM, "relay buffers (%zu copies per round)", max_copies);
    RL_HIP(h, hipMemcpyAsync(d_ap, ap.data(), ap.size() * 4, hipMemcpyHostToDevice, s));
    if (na) RL_HIP(h, hipMemcpyAsync(d_act, act, na * 4, hipMemcpyHostToDevice, s));
    RL_HIP(h, hipMemcpyAsync(d_pp, pp.data(), pp.size() * 4, hipMemcpyHostToDevice, s));
    if (pp[n]) RL_HIP(h, hipMemcpyAsync(d_pe, pe.data(), (size_t)pp[n] * 4, hipMemcpyHostToDevice, s));
    RL_HIP(h, hipMemcpyAsync(d_op, op.data(), op.size() * 4, hipMemcpyHostToDevice, s));
    if (no) RL_HIP(h, hipMemcpyAsync(d_ol, ol, no * 4, hipMemcpyHostToDevice, s));
    RL_HIP(h, hipMemcpyAsync(d_alive, alive, n, hipMemcpyHostToDevice, s));
    if (k) {
        RL_HIP(h, hipMemcpyAsync(d_src, src, (size_t)k * 4, hipMemcpyHostToDevice, s));
        RL_HIP(h, hipMemcpyAsync(d_dst, dst, (size_t)k * 4, hipMemcpyHostToDevice, s));
        RL_HIP(h, hipMemsetAsync(d_deliv, 0, (size_t)k * 8, s));
        RL_HIP(h, hipMemsetAsync(d_first, 0xFF, (size_t)k * 4, s));
    }
    RL_HIP(h, hipMemsetAsync(d_cnt, 0, 64, s));
    RL_HIP(h, hipMemsetAsync(d_stats, 0, nrounds_max * stat_row * 8, s));
    a.act_ptr = d_ap; a.act = d_act; a.peer_ptr = d_pp; a.peer = d_pe; a.ol_ptr = d_op; a.ol = d_ol;
    a.alive = d_alive; a.src = d_src; a.dst = d_dst; a.delivered = d_deliv; a.first_round = d_first;
    a.ovf = d_cnt + 8;
    a.cap = (uint32_t)max_copies;
    a.relay_ttl = relay_ttl;
    hipLaunchKernelGGL(rl_prep_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, a, n, d_olmask, d_nlost);
    RL_HIP(h, hipGetLastError());
    a.olmask = d_olmask;
    a.nlost = d_nlost;

    hipEvent_t e0 = handle_event(h, 0), e1 = handle_event(h, 1);
    uint2* q[2] = {d_q0, d_q1};
    uint32_t ncur = k, hc[16];
    int64_t rounds = 0;
    double ms_total = 0;
    int err = PSIM_OK;
    for (;;) {
        // round `rounds`: origins (0) or the copies sent last round
        if (rounds >= (int64_t)nrounds_max) { err = handle_fail(h, PSIM_EINVAL, "relay did not quiesce"); break; }
        a.round = (uint32_t)rounds;
        a.cur = q[rounds & 1];
        a.nxt = q[(rounds + 1) & 1];
        a.ncur = ncur;
        a.nnxt = d_cnt + ((rounds + 1) & 1);
        a.stats = d_stats + (size_t)rounds * stat_row;
        RL_HIP(h, hipMemsetAsync(a.nnxt, 0, 4, s));
        RL_HIP(h, hipEventRecord(e0, s));
        if (ncur) {
            const dim3 grid((ncur + kBlock - 1) / kBlock);
            if (rounds == 0) hipLaunchKernelGGL(rl_round_kernel<true>, grid, dim3(kBlock), 0, s, a);
            else hipLaunchKernelGGL(rl_round_kernel<false>, grid, dim3(kBlock), 0, s, a);
            RL_HIP(h, hipGetLastError());
        }
        RL_HIP(h, hipEventRecord(e1, s));
        RL_HIP(h, hipMemcpyAsync(hc, d_cnt, 64, hipMemcpyDeviceToHost, s));
        RL_HIP(h, hipStreamSynchronize(s));
        float ms = 0;
        RL_HIP(h, hipEventElapsedTime(&ms, e0, e1));
        ms_total += ms;
        rounds++;
        if (hc[8]) { err = handle_fail(h, PSIM_EOVERFLOW, "a round holds more than %zu copies", max_copies); break; }
        ncur = hc[rounds & 1];
        if (ncur == 0) break;
    }
    handle_add_round(h, ms_total);
    if (err) return err;
    if (k) {
        RL_HIP(h, hipMemcpyAsync(delivered, d_deliv, (size_t)k * 8, hipMemcpyDeviceToHost, s));
        RL_HIP(h, hipMemcpyAsync(first_round, d_first, (size_t)k * 4, hipMemcpyDeviceToHost, s));
    }
    std::vector<unsigned long long> hs((size_t)rounds * stat_row);
    RL_HIP(h, hipMemcpyAsync(hs.data(), d_stats, hs.size() * 8, hipMemcpyDeviceToHost, s));
    RL_HIP(h, hipStreamSynchronize(s));
    for (int64_t r = 0; r < rounds && (size_t)r < cap && stats; r++) {
        unsigned long long t[kRlNStat] = {};
        for (int sh = 0; sh < kStatShards; sh++)
            for (int c = 0; c < kRlNStat; c++) t[c] += hs[(size_t)r * stat_row + sh * kRlNStat + c];
        stats[r].direct = t[0];
        stats[r].relay = t[1];
        stats[r].dropped = t[2];
        stats[r].lost = t[3];
        stats[r].arrived = t[4];
    }
    return rounds;
}
