// fullmem.hip -- the full-membership strategy
// (src/partisan_full_membership_strategy.erl:70-268) over the OR-set behind
// src/partisan_membership_set.erl (state_orset, types 0.1.8), one gfx950
// wavefront per node and round.
//
// State layout (DESIGN.md "Full membership"): the token universe of the
// cluster is indexed (token v = node v's init/1 add; self-leaves allocate
// fresh tokens n, n+1, ...), and a node's #full_v1{} payload is two bitmaps
// over it: K = tokens present, R = tokens present and inactive.  Then
//   state_orset:merge = K|K', R|R'   (a token on both sides is active iff
//                                      active on both; one side: its flag)
//   state_orset:equal = K == K' and R == R'
//   query / to_list   = elements of the tokens in K & ~R
// so each handler is a handful of wave-wide bitwise ops: lane l < W holds K
// word l, lane W + l holds R word l.
//
// A message is a snapshot of the sender's state plus its recipient bitmap
// (to_peer_list of the state it gossips about, minus self, masked by the
// nodes alive at the start of the round -- a send to a dead node is lost).
// Snapshots are stored in (src, emission seq) order: every node emits
// into its own range [base[v], base[v+1]), computed by a counting pass, so
// the receive order of the schedule is the storage order and nothing
// depends on atomic arrival order.
#include "psim_internal.h"
#include "../../include/psim.h"

namespace psim {

namespace {

struct FmCtx {
    uint32_t count;                 // emissions so far (all lanes agree)
    unsigned long long st[6];       // 0 sent, 1 processed, 2 merges, 3 updates, 4 inflight, 5 member_sum
};

// members of state x (this lane's word) -> pm (node bitmap, LDS)
__device__ void members_of(const FmArgs& a, unsigned long long x, unsigned long long* pm) {
    const uint32_t lane = threadIdx.x;
    if (lane < a.NW) pm[lane] = 0;
    __syncthreads();
    const unsigned long long r = __shfl(x, (int)((lane + a.W) & 63), 64);
    if (lane < a.W) {
        unsigned long long act = x & ~r;
        while (act) {
            const uint32_t b = __ffsll(act) - 1;
            act &= act - 1;
            const uint32_t e = a.elem[lane * 64 + b];
            atomicOr(&pm[e >> 6], 1ull << (e & 63));
        }
    }
    __syncthreads();
}

__device__ bool members_differ(const FmArgs& a, const unsigned long long* p, const unsigned long long* q) {
    const uint32_t lane = threadIdx.x;
    const bool d = lane < a.NW && p[lane] != q[lane];
    return __ballot(d) != 0;
}

// gossip_messages/2 (:247-268): state x to the members in `to` except self
__device__ void emit(const FmArgs& a, uint32_t v, unsigned long long x, const unsigned long long* to, FmCtx& c) {
    const uint32_t lane = threadIdx.x;
    unsigned long long peers = 0, live = 0;
    if (lane < a.NW) {
        peers = to[lane];
        if (lane == (v >> 6)) peers &= ~(1ull << (v & 63));
        live = peers & a.alive0_bm[lane];
    }
    if (a.pass == 1) {
        const size_t k = (size_t)a.base[v] + c.count;
        if (lane < 2 * a.W) a.out_st[k * (2 * a.W) + lane] = x;
        if (lane < a.NW) a.out_p[k * a.NW + lane] = live;
        if (lane == 0) a.out_src[k] = v;
        unsigned long long np = __popcll(peers), nl = __popcll(live);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            np += __shfl_xor(np, off, 64);
            nl += __shfl_xor(nl, off, 64);
        }
        c.st[0] += np;
        c.st[4] += nl;
    }
    c.count++;
}

__device__ void save_members(const FmArgs& a, const unsigned long long* pm, unsigned long long* pm0) {
    for (uint32_t j = threadIdx.x; j < a.NW; j += 64) pm0[j] = pm[j];
    __syncthreads();
}

// one node, one round (pass 0: count emissions; pass 1: emit and store)
__global__ __launch_bounds__(64) void fm_round_kernel(FmArgs a) {
    __shared__ unsigned long long pm[kFmMaxNW], pm0[kFmMaxNW];
    const uint32_t v = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    const uint32_t L = 2 * a.W;
    FmCtx c;
    c.count = 0;
    for (int i = 0; i < 6; i++) c.st[i] = 0;
    unsigned long long x = lane < L ? a.st_cur[(size_t)v * L + lane] : 0ull;
    bool alive = a.alive0[v] != 0;
    if (alive) {
        members_of(a, x, pm);
        // ---- leave calls (internal_leave -> leave/2 :177-214)
        for (uint32_t i = a.lo[v]; i < a.lo[v + 1]; i++) {
            const uint32_t who = a.lw[i];
            // remove every token of `who`: R |= K & tokens(who)
            unsigned long long m = 0;
            if (lane < a.W) {
                unsigned long long k = x;
                while (k) {
                    const uint32_t b = __ffsll(k) - 1;
                    k &= k - 1;
                    if (a.elem[lane * 64 + b] == who) m |= 1ull << b;
                }
            }
            const unsigned long long mr = __shfl(m, (int)((lane + 64 - a.W) & 63), 64);
            const unsigned long long g = (lane >= a.W && lane < L) ? (x | mr) : x;
            emit(a, v, g, pm, c);                      // to the peers of State0 (:212)
            save_members(a, pm, pm0);
            if (who == v) {                            // new_state(Actor) (:288-294)
                const uint32_t t = a.lt[i];
                x = (lane == (t >> 6)) ? (1ull << (t & 63)) : 0ull;
            } else {
                x = g;
            }
            members_of(a, x, pm);
            if (members_differ(a, pm, pm0)) c.st[3]++;
        }
        // ---- {connected, Peer, _, _, RemoteState} -> join/3 (:85-96)
        for (uint32_t i = a.jo[v]; i < a.jo[v + 1]; i++) {
            const uint32_t p = a.jp[i];
            if (p == v || !a.alive0[p]) continue;      // never connects to a dead peer
            const unsigned long long y = lane < L ? a.st_cur[(size_t)p * L + lane] : 0ull;
            save_members(a, pm, pm0);
            x |= y;                                    // partisan_membership_set:merge/2
            c.st[2]++;
            members_of(a, x, pm);
            if (members_differ(a, pm, pm0)) c.st[3]++;
            emit(a, v, x, pm, c);
        }
        // ---- inbox in (src, seq) order: handle_message/2 (:135-167)
        for (uint32_t k = 0; k < a.S && alive; k++) {
            const unsigned long long w = a.snap_p[(size_t)k * a.NW + (v >> 6)];
            if (!((w >> (v & 63)) & 1ull)) continue;
            c.st[1]++;
            const unsigned long long y = lane < L ? a.snap_st[(size_t)k * L + lane] : 0ull;
            if (__ballot(y != x) == 0) continue;       // equal/2: converged here
            save_members(a, pm, pm0);
            x |= y;
            c.st[2]++;
            members_of(a, x, pm);
            if (members_differ(a, pm, pm0)) c.st[3]++;
            emit(a, v, x, pm, c);
            if (!((pm[v >> 6] >> (v & 63)) & 1ull)) alive = false;   // {stop, normal} (:1791-1803)
        }
        // ---- handle_info(periodic) -> periodic/1 (:106-111)
        if (alive && a.periodic) emit(a, v, x, pm, c);
        if (alive && lane < a.NW) c.st[5] = __popcll(pm[lane]);
    }
    if (a.pass == 0) {
        if (lane == 0) a.cnt[v] = c.count;
        return;
    }
    if (lane < L) a.st_nxt[(size_t)v * L + lane] = x;
    if (lane == 0) a.alive_nxt[v] = alive ? 1 : 0;
    unsigned long long ms = c.st[5];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ms += __shfl_xor(ms, off, 64);
    c.st[5] = ms;
    if (lane == 0)
        for (int i = 0; i < 6; i++)
            if (c.st[i]) atomicAdd(&a.stats[i], c.st[i]);
}

// exclusive scan of the emission counts (n <= 2048): one workgroup
__global__ __launch_bounds__(256) void fm_scan_kernel(const uint32_t* __restrict__ cnt, uint32_t* __restrict__ base,
                                                      uint32_t n) {
    __shared__ uint32_t part[256];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (n + 255) / 256;
    uint32_t s = 0;
    for (uint32_t i = t * per; i < (t + 1) * per && i < n; i++) s += cnt[i];
    part[t] = s;
    __syncthreads();
    if (t == 0) {
        uint32_t acc = 0;
        for (int i = 0; i < 256; i++) {
            const uint32_t y = part[i];
            part[i] = acc;
            acc += y;
        }
        base[n] = acc;
    }
    __syncthreads();
    uint32_t acc = part[t];
    for (uint32_t i = t * per; i < (t + 1) * per && i < n; i++) {
        base[i] = acc;
        acc += cnt[i];
    }
}

// alive bytes -> bitmap
__global__ __launch_bounds__(64) void fm_alive_bm_kernel(const uint8_t* __restrict__ alive, uint32_t n,
                                                         unsigned long long* __restrict__ bm, uint32_t nw) {
    for (uint32_t w = threadIdx.x; w < nw; w += 64) {
        unsigned long long b = 0;
        for (uint32_t j = 0; j < 64 && w * 64 + j < n; j++)
            if (alive[w * 64 + j]) b |= 1ull << j;
        bm[w] = b;
    }
}

}  // namespace

hipError_t launch_fm_round(const FmArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(fm_round_kernel, dim3(a.n), dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_fm_scan(const uint32_t* cnt, uint32_t* base, uint32_t n, hipStream_t s) {
    hipLaunchKernelGGL(fm_scan_kernel, dim3(1), dim3(256), 0, s, cnt, base, n);
    return hipGetLastError();
}

hipError_t launch_fm_alive_bm(const uint8_t* alive, uint32_t n, unsigned long long* bm, uint32_t nw, hipStream_t s) {
    hipLaunchKernelGGL(fm_alive_bm_kernel, dim3(1), dim3(64), 0, s, alive, n, bm, nw);
    return hipGetLastError();
}

}  // namespace psim

// ---------------------------------------------------------------------------
// host side: the psim_fm_* entry points of include/psim.h
// ---------------------------------------------------------------------------
#include <algorithm>
#include <cstring>
#include <vector>

using namespace psim;

namespace {

struct FmState : ModuleState {
    uint32_t n = 0, W = 0, NW = 0, T = 0, periodic = 0, next_tok = 0;
    std::vector<uint32_t> h_elem;
    unsigned long long *st[2] = {}, *snap_st[2] = {}, *snap_p[2] = {}, *alive_bm = nullptr, *stats = nullptr;
    uint8_t* alive[2] = {};
    uint32_t *snap_src[2] = {}, *cnt = nullptr, *base = nullptr, *elem = nullptr;
    uint32_t *jo = nullptr, *lo = nullptr, *lists = nullptr;   // lists: [jp | lw | lt], capacity list_cap each
    size_t snap_cap[2] = {0, 0}, list_cap = 0;
    uint32_t S = 0, par = 0;
    uint64_t round = 0;
    // seq of each in-flight snapshot when psim_fm_put placed some (empty: the
    // sender's emission index, i.e. the position inside its run of snapshots)
    std::vector<uint32_t> hseq;
    std::vector<uint32_t> jv, jpeer, lv, lwho, ltok;   // calls made since the last round
    ~FmState() override {
        void* p[] = {st[0], st[1], snap_st[0], snap_st[1], snap_p[0], snap_p[1], alive_bm, stats, alive[0], alive[1],
                     snap_src[0], snap_src[1], cnt, base, elem, jo, lo, lists};
        for (void* x : p)
            if (x) (void)hipFree(x);
    }
};

FmState* fm_of(psim_handle* h) { return static_cast<FmState*>(handle_module(h, MOD_FULLMEM)); }
const FmState* fm_of(const psim_handle* h) { return static_cast<const FmState*>(handle_module(h, MOD_FULLMEM)); }

#define FMCHK(h, x)                                                                         \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess)                                                               \
            return handle_fail((h), PSIM_EHIP, "%s failed: %s", #x, hipGetErrorString(e_)); \
    } while (0)

bool fm_alloc(void** p, size_t bytes) {
    return alloc_zero(p, bytes);
}

// grow the snapshot buffer `which` to hold k records
int fm_reserve(psim_handle* h, FmState& f, int which, size_t k) {
    if (k <= f.snap_cap[which]) return PSIM_OK;
    size_t cap = std::max<size_t>(k, 2 * f.snap_cap[which]);
    if (f.snap_st[which]) (void)hipFree(f.snap_st[which]);
    if (f.snap_p[which]) (void)hipFree(f.snap_p[which]);
    if (f.snap_src[which]) (void)hipFree(f.snap_src[which]);
    f.snap_st[which] = f.snap_p[which] = nullptr;
    f.snap_src[which] = nullptr;
    f.snap_cap[which] = 0;
    if (!fm_alloc((void**)&f.snap_st[which], cap * 2 * f.W * 8) || !fm_alloc((void**)&f.snap_p[which], cap * f.NW * 8) ||
        !fm_alloc((void**)&f.snap_src[which], cap * 4))
        return handle_fail(h, PSIM_ENOMEM, "full membership: %zu message snapshots", cap);
    f.snap_cap[which] = cap;
    return PSIM_OK;
}

// calls grouped by the calling vertex, call order kept (stable)
void group_calls(uint32_t n, const std::vector<uint32_t>& who, std::vector<uint32_t>& off, std::vector<uint32_t>& order) {
    off.assign(n + 1, 0);
    for (uint32_t v : who) off[v + 1]++;
    for (uint32_t v = 0; v < n; v++) off[v + 1] += off[v];
    order.assign(who.size(), 0);
    std::vector<uint32_t> fill(off.begin(), off.end() - 1);
    for (size_t i = 0; i < who.size(); i++) order[fill[who[i]]++] = (uint32_t)i;
}

int fm_round(psim_handle* h, FmState& f, psim_fm_stats* out) {
    const hipStream_t s = handle_stream(h);
    // this round's leave / join calls, CSR by caller
    std::vector<uint32_t> joff, jord, loff, lord;
    group_calls(f.n, f.jv, joff, jord);
    group_calls(f.n, f.lv, loff, lord);
    const size_t nj = jord.size(), nl = lord.size();
    if (std::max(nj, nl) > f.list_cap) {
        if (f.lists) (void)hipFree(f.lists);
        f.lists = nullptr;
        f.list_cap = std::max<size_t>(std::max(nj, nl), 2 * f.list_cap);
        if (!fm_alloc((void**)&f.lists, 3 * f.list_cap * 4))
            return handle_fail(h, PSIM_ENOMEM, "full membership: %zu calls", f.list_cap);
    }
    std::vector<uint32_t> lst(3 * f.list_cap, 0);
    for (size_t i = 0; i < nj; i++) lst[i] = f.jpeer[jord[i]];
    for (size_t i = 0; i < nl; i++) {
        lst[f.list_cap + i] = f.lwho[lord[i]];
        lst[2 * f.list_cap + i] = f.ltok[lord[i]];
    }
    FMCHK(h, hipMemcpyAsync(f.jo, joff.data(), (f.n + 1) * 4, hipMemcpyHostToDevice, s));
    FMCHK(h, hipMemcpyAsync(f.lo, loff.data(), (f.n + 1) * 4, hipMemcpyHostToDevice, s));
    FMCHK(h, hipMemcpyAsync(f.lists, lst.data(), lst.size() * 4, hipMemcpyHostToDevice, s));
    f.jv.clear(); f.jpeer.clear(); f.lv.clear(); f.lwho.clear(); f.ltok.clear();

    const uint64_t t = f.round + 1;
    FmArgs a{};
    a.n = f.n; a.W = f.W; a.NW = f.NW; a.S = f.S;
    a.periodic = f.periodic && (t % f.periodic) == 0;
    a.elem = f.elem;
    a.st_cur = f.st[f.par]; a.st_nxt = f.st[f.par ^ 1];
    a.alive0 = f.alive[f.par]; a.alive_nxt = f.alive[f.par ^ 1];
    a.alive0_bm = f.alive_bm;
    a.snap_st = f.snap_st[f.par]; a.snap_p = f.snap_p[f.par];
    a.cnt = f.cnt; a.base = f.base;
    a.jo = f.jo; a.jp = f.lists; a.lo = f.lo; a.lw = f.lists + f.list_cap; a.lt = f.lists + 2 * f.list_cap;
    a.stats = f.stats;
    FMCHK(h, hipMemsetAsync(f.stats, 0, 8 * 8, s));
    FMCHK(h, hipEventRecord(handle_event(h, 0), s));
    FMCHK(h, launch_fm_alive_bm(a.alive0, f.n, f.alive_bm, f.NW, s));
    a.pass = 0;
    FMCHK(h, launch_fm_round(a, s));
    FMCHK(h, launch_fm_scan(f.cnt, f.base, f.n, s));
    uint32_t total = 0;
    FMCHK(h, hipMemcpyAsync(&total, f.base + f.n, 4, hipMemcpyDeviceToHost, s));
    FMCHK(h, hipStreamSynchronize(s));
    const int rc = fm_reserve(h, f, f.par ^ 1, total);
    if (rc) return rc;
    a.out_st = f.snap_st[f.par ^ 1]; a.out_p = f.snap_p[f.par ^ 1]; a.out_src = f.snap_src[f.par ^ 1];
    a.pass = 1;
    FMCHK(h, launch_fm_round(a, s));
    FMCHK(h, hipEventRecord(handle_event(h, 1), s));
    unsigned long long r[8];
    FMCHK(h, hipMemcpyAsync(r, f.stats, sizeof r, hipMemcpyDeviceToHost, s));
    FMCHK(h, hipStreamSynchronize(s));
    float ms = 0.f;
    FMCHK(h, hipEventElapsedTime(&ms, handle_event(h, 0), handle_event(h, 1)));
    handle_add_round(h, ms);
    if (out) {
        memset(out, 0, sizeof *out);
        out->sent = r[0]; out->processed = r[1]; out->merges = r[2]; out->updates = r[3];
        out->inflight = r[4]; out->member_sum = r[5];
        // recipient-word scan + handled states + emitted records + state read/write
        out->algo_bytes = 8ull * f.S * f.n + 16ull * f.W * r[1] + (16ull * f.W + 8ull * f.NW) * total +
                          32ull * f.W * f.n;
        out->kernel_ms = ms;
    }
    f.S = total;
    f.par ^= 1u;
    f.round = t;
    f.hseq.clear();
    return PSIM_OK;
}

// The in-flight snapshots on the host: states [S][2W], recipients [S][NW], src, seq.
struct FmWire {
    std::vector<unsigned long long> st, p;
    std::vector<uint32_t> src, seq;
};

int fm_download(psim_handle* h, const FmState& f, FmWire& w) {
    const size_t S = f.S, L = 2 * f.W;
    w.st.resize(S * L);
    w.p.resize(S * f.NW);
    w.src.resize(S);
    if (S) {
        FMCHK(h, hipMemcpy(w.st.data(), f.snap_st[f.par], w.st.size() * 8, hipMemcpyDeviceToHost));
        FMCHK(h, hipMemcpy(w.p.data(), f.snap_p[f.par], w.p.size() * 8, hipMemcpyDeviceToHost));
        FMCHK(h, hipMemcpy(w.src.data(), f.snap_src[f.par], S * 4, hipMemcpyDeviceToHost));
    }
    if (f.hseq.size() == S) {
        w.seq = f.hseq;
    } else {                      // emission index: position inside the sender's run (storage is (src, seq) order)
        w.seq.resize(S);
        for (size_t k = 0; k < S; k++) w.seq[k] = (k && w.src[k - 1] == w.src[k]) ? w.seq[k - 1] + 1 : 0;
    }
    return PSIM_OK;
}

// the messages of the snapshots to `dst` (or every recipient: dst = ~0u) in
// handling order (dst, src, seq); take: clear the recipients' bits
size_t fm_collect(const FmState& f, FmWire& w, uint32_t dst, bool take, psim_fm_msg* out, uint64_t* known,
                  uint64_t* removed, size_t cap) {
    const size_t L = 2 * f.W;
    size_t c = 0;
    const uint32_t lo = dst == ~0u ? 0 : dst, hi = dst == ~0u ? f.n : dst + 1;
    for (uint32_t d = lo; d < hi; d++)
        for (size_t k = 0; k < f.S; k++) {
            unsigned long long& b = w.p[k * f.NW + (d >> 6)];
            if (!((b >> (d & 63)) & 1ull)) continue;
            if (c < cap) {
                if (out) out[c] = psim_fm_msg{w.src[k], d, w.seq[k], 0u};
                for (uint32_t j = 0; j < f.W; j++) {
                    if (known) known[c * f.W + j] = w.st[k * L + j];
                    if (removed) removed[c * f.W + j] = w.st[k * L + f.W + j];
                }
            }
            if (take) b &= ~(1ull << (d & 63));
            c++;
        }
    return c;
}

}  // namespace

extern "C" {

int psim_fm_setup(psim_handle* h, uint32_t n, uint32_t periodic_rounds, uint32_t max_tokens) {
    if (!h) return PSIM_EINVAL;
    if (n < 1 || n > 64 * kFmMaxNW || max_tokens < n || max_tokens > 64 * kFmMaxW)
        return handle_fail(h, PSIM_EINVAL, "full membership: need 1 <= n <= %u and n <= max_tokens <= %u",
                           64 * kFmMaxNW, 64 * kFmMaxW);
    FMCHK(h, hipSetDevice(handle_device(h)));
    FMCHK(h, hipStreamSynchronize(handle_stream(h)));
    ModuleState*& slot = handle_module(h, MOD_FULLMEM);
    delete slot;
    slot = nullptr;
    FmState* f = new FmState();
    f->n = n;
    f->W = (max_tokens + 63) / 64;
    f->T = 64 * f->W;
    f->NW = (n + 63) / 64;
    f->periodic = periodic_rounds;
    f->next_tok = n;
    const size_t L = 2 * f->W;
    bool ok = fm_alloc((void**)&f->st[0], size_t(n) * L * 8) && fm_alloc((void**)&f->st[1], size_t(n) * L * 8) &&
              fm_alloc((void**)&f->alive[0], n) && fm_alloc((void**)&f->alive[1], n) &&
              fm_alloc((void**)&f->alive_bm, f->NW * 8) && fm_alloc((void**)&f->stats, 64) &&
              fm_alloc((void**)&f->cnt, size_t(n) * 4) && fm_alloc((void**)&f->base, (size_t(n) + 1) * 4) &&
              fm_alloc((void**)&f->elem, size_t(f->T) * 4) && fm_alloc((void**)&f->jo, (size_t(n) + 1) * 4) &&
              fm_alloc((void**)&f->lo, (size_t(n) + 1) * 4);
    if (!ok) {
        delete f;
        return handle_fail(h, PSIM_ENOMEM, "full membership state for n=%u", n);
    }
    slot = f;
    // init/1 -> new_state/1 (:288-294): node v holds {v: {token v: active}}
    std::vector<unsigned long long> st(size_t(n) * L, 0ull);
    for (uint32_t v = 0; v < n; v++) st[size_t(v) * L + (v >> 6)] = 1ull << (v & 63);
    f->h_elem.assign(f->T, 0xFFFFFFFFu);
    for (uint32_t v = 0; v < n; v++) f->h_elem[v] = v;
    std::vector<uint8_t> al(n, 1);
    FMCHK(h, hipMemcpy(f->st[0], st.data(), st.size() * 8, hipMemcpyHostToDevice));
    FMCHK(h, hipMemcpy(f->elem, f->h_elem.data(), size_t(f->T) * 4, hipMemcpyHostToDevice));
    FMCHK(h, hipMemcpy(f->alive[0], al.data(), n, hipMemcpyHostToDevice));
    return PSIM_OK;
}

int psim_fm_set_alive(psim_handle* h, const uint8_t* alive, size_t n) {
    if (!h || !alive) return PSIM_EINVAL;
    FmState* f = fm_of(h);
    if (!f) return handle_fail(h, PSIM_ESTATE, "psim_fm_setup not called");
    if (n != f->n) return handle_fail(h, PSIM_EINVAL, "alive has %zu entries, cluster has %u", n, f->n);
    std::vector<uint8_t> a(n);
    for (size_t i = 0; i < n; i++) a[i] = alive[i] ? 1 : 0;
    FMCHK(h, hipSetDevice(handle_device(h)));
    FMCHK(h, hipMemcpy(f->alive[f->par], a.data(), n, hipMemcpyHostToDevice));
    return PSIM_OK;
}

int psim_fm_join(psim_handle* h, const uint32_t* v, const uint32_t* peer, size_t k) {
    if (!h || (k && (!v || !peer))) return PSIM_EINVAL;
    FmState* f = fm_of(h);
    if (!f) return handle_fail(h, PSIM_ESTATE, "psim_fm_setup not called");
    for (size_t i = 0; i < k; i++)
        if (v[i] >= f->n || peer[i] >= f->n) return handle_fail(h, PSIM_EINVAL, "join %zu: vertex out of range", i);
    f->jv.insert(f->jv.end(), v, v + k);
    f->jpeer.insert(f->jpeer.end(), peer, peer + k);
    return PSIM_OK;
}

int psim_fm_leave(psim_handle* h, const uint32_t* v, const uint32_t* leaving, size_t k) {
    if (!h || (k && (!v || !leaving))) return PSIM_EINVAL;
    FmState* f = fm_of(h);
    if (!f) return handle_fail(h, PSIM_ESTATE, "psim_fm_setup not called");
    for (size_t i = 0; i < k; i++) {
        if (v[i] >= f->n || leaving[i] >= f->n) return handle_fail(h, PSIM_EINVAL, "leave %zu: vertex out of range", i);
        if (v[i] == leaving[i] && f->next_tok >= f->T)
            return handle_fail(h, PSIM_EOVERFLOW, "full membership: token universe of %u exhausted", f->T);
    }
    for (size_t i = 0; i < k; i++) {
        uint32_t tok = 0;
        if (v[i] == leaving[i]) {           // new_state(Actor) gets a fresh token, numbered in call order
            tok = f->next_tok++;
            f->h_elem[tok] = v[i];
            FMCHK(h, hipMemcpy(f->elem + tok, &f->h_elem[tok], 4, hipMemcpyHostToDevice));
        }
        f->lv.push_back(v[i]);
        f->lwho.push_back(leaving[i]);
        f->ltok.push_back(tok);
    }
    return PSIM_OK;
}

int psim_fm_step(psim_handle* h, uint32_t rounds, psim_fm_stats* stats, size_t cap) {
    if (!h) return PSIM_EINVAL;
    FmState* f = fm_of(h);
    if (!f) return handle_fail(h, PSIM_ESTATE, "psim_fm_setup not called");
    FMCHK(h, hipSetDevice(handle_device(h)));
    for (uint32_t i = 0; i < rounds; i++) {
        const int rc = fm_round(h, *f, stats && i < cap ? &stats[i] : nullptr);
        if (rc) return rc;
    }
    return PSIM_OK;
}

int psim_fm_get_state(const psim_handle* h, uint64_t* known, uint64_t* removed, uint8_t* alive, size_t n,
                      size_t words) {
    if (!h) return PSIM_EINVAL;
    const FmState* f = fm_of(h);
    if (!f) return PSIM_ESTATE;
    psim_handle* hh = const_cast<psim_handle*>(h);
    if (n != f->n || words != f->W) return handle_fail(hh, PSIM_EINVAL, "want n=%u, words=%u", f->n, f->W);
    FMCHK(hh, hipSetDevice(handle_device(h)));
    FMCHK(hh, hipStreamSynchronize(handle_stream(h)));
    const size_t L = 2 * f->W;
    std::vector<unsigned long long> st(n * L);
    FMCHK(hh, hipMemcpy(st.data(), f->st[f->par], st.size() * 8, hipMemcpyDeviceToHost));
    for (size_t v = 0; v < n; v++)
        for (size_t w = 0; w < words; w++) {
            if (known) known[v * words + w] = st[v * L + w];
            if (removed) removed[v * words + w] = st[v * L + f->W + w];
        }
    if (alive) FMCHK(hh, hipMemcpy(alive, f->alive[f->par], n, hipMemcpyDeviceToHost));
    return PSIM_OK;
}

int psim_fm_tokens(const psim_handle* h, uint32_t* token_node, size_t ntok, uint32_t* used) {
    if (!h) return PSIM_EINVAL;
    const FmState* f = fm_of(h);
    if (!f) return PSIM_ESTATE;
    if (token_node)
        for (size_t t = 0; t < ntok && t < f->T; t++) token_node[t] = f->h_elem[t];
    if (used) *used = f->next_tok;
    return PSIM_OK;
}

int psim_fm_messages(const psim_handle* h, psim_fm_msg* out, uint64_t* known, uint64_t* removed, size_t cap,
                     size_t words, size_t* count) {
    if (!h || !count || (cap && (!out || !known || !removed))) return PSIM_EINVAL;
    const FmState* f = fm_of(h);
    if (!f) return PSIM_ESTATE;
    psim_handle* hh = const_cast<psim_handle*>(h);
    if (cap && words != f->W) return handle_fail(hh, PSIM_EINVAL, "want words=%u", f->W);
    FMCHK(hh, hipSetDevice(handle_device(h)));
    FMCHK(hh, hipStreamSynchronize(handle_stream(h)));
    FmWire w;
    const int rc = fm_download(hh, *f, w);
    if (rc) return rc;
    *count = fm_collect(*f, w, ~0u, false, out, known, removed, cap);
    return PSIM_OK;
}

int psim_fm_take(psim_handle* h, uint32_t dst, psim_fm_msg* out, uint64_t* known, uint64_t* removed, size_t cap,
                 size_t words, size_t* count) {
    if (!h || !count || (cap && (!out || !known || !removed))) return PSIM_EINVAL;
    FmState* f = fm_of(h);
    if (!f) return PSIM_ESTATE;
    if (dst >= f->n) return handle_fail(h, PSIM_EINVAL, "take: node %u of %u", dst, f->n);
    if (cap && words != f->W) return handle_fail(h, PSIM_EINVAL, "want words=%u", f->W);
    FMCHK(h, hipSetDevice(handle_device(h)));
    FMCHK(h, hipStreamSynchronize(handle_stream(h)));
    FmWire w;
    int rc = fm_download(h, *f, w);
    if (rc) return rc;
    const size_t need = fm_collect(*f, w, dst, false, nullptr, nullptr, nullptr, 0);
    *count = need;
    if (need > cap) return handle_fail(h, PSIM_EINVAL, "take: %zu messages for node %u, room for %zu", need, dst, cap);
    fm_collect(*f, w, dst, true, out, known, removed, cap);
    if (f->S) FMCHK(h, hipMemcpy(f->snap_p[f->par], w.p.data(), w.p.size() * 8, hipMemcpyHostToDevice));
    return PSIM_OK;
}

int psim_fm_put(psim_handle* h, const psim_fm_msg* msgs, const uint64_t* known, const uint64_t* removed, size_t k,
                size_t words) {
    if (!h || (k && (!msgs || !known || !removed))) return PSIM_EINVAL;
    FmState* f = fm_of(h);
    if (!f) return PSIM_ESTATE;
    if (!k) return PSIM_OK;
    if (words != f->W) return handle_fail(h, PSIM_EINVAL, "want words=%u", f->W);
    for (size_t i = 0; i < k; i++) {
        if (msgs[i].dst >= f->n) return handle_fail(h, PSIM_EINVAL, "put %zu: node %u of %u", i, msgs[i].dst, f->n);
        for (uint32_t j = 0; j < f->W; j++) {
            const unsigned long long K = known[i * f->W + j], R = removed[i * f->W + j];
            // a state over the tokens allocated so far; removed tokens are present ones (state_orset)
            const uint32_t t0 = 64 * j;
            const unsigned long long alloc = f->next_tok <= t0 ? 0ull
                                           : f->next_tok >= t0 + 64 ? ~0ull : (1ull << (f->next_tok - t0)) - 1ull;
            if ((K & ~alloc) || (R & ~K))
                return handle_fail(h, PSIM_EINVAL, "put %zu: a token outside the cluster's universe", i);
        }
    }
    FMCHK(h, hipSetDevice(handle_device(h)));
    FMCHK(h, hipStreamSynchronize(handle_stream(h)));
    FmWire w;
    int rc = fm_download(h, *f, w);
    if (rc) return rc;
    // merge: storage (= handling) order is (src, seq), a put after existing ties
    const size_t S0 = f->S, S1 = S0 + k, L = 2 * f->W;
    std::vector<size_t> add(k);
    for (size_t i = 0; i < k; i++) add[i] = i;
    std::stable_sort(add.begin(), add.end(), [&](size_t x, size_t y) {
        return msgs[x].src != msgs[y].src ? msgs[x].src < msgs[y].src : msgs[x].seq < msgs[y].seq;
    });
    FmWire m;
    m.st.resize(S1 * L);
    m.p.assign(S1 * f->NW, 0ull);
    m.src.resize(S1);
    m.seq.resize(S1);
    size_t a = 0, b = 0;
    for (size_t o = 0; o < S1; o++) {
        const bool old = b == k || (a < S0 && (w.src[a] != msgs[add[b]].src ? w.src[a] < msgs[add[b]].src
                                                                           : w.seq[a] <= msgs[add[b]].seq));
        if (old) {
            std::copy(w.st.begin() + a * L, w.st.begin() + (a + 1) * L, m.st.begin() + o * L);
            std::copy(w.p.begin() + a * f->NW, w.p.begin() + (a + 1) * f->NW, m.p.begin() + o * f->NW);
            m.src[o] = w.src[a];
            m.seq[o] = w.seq[a];
            a++;
        } else {
            const psim_fm_msg& x = msgs[add[b]];
            for (uint32_t j = 0; j < f->W; j++) {
                m.st[o * L + j] = known[add[b] * f->W + j];
                m.st[o * L + f->W + j] = removed[add[b] * f->W + j];
            }
            m.p[o * f->NW + (x.dst >> 6)] = 1ull << (x.dst & 63);
            m.src[o] = x.src;
            m.seq[o] = x.seq;
            b++;
        }
    }
    rc = fm_reserve(h, *f, f->par, S1);
    if (rc) return rc;
    FMCHK(h, hipMemcpy(f->snap_st[f->par], m.st.data(), m.st.size() * 8, hipMemcpyHostToDevice));
    FMCHK(h, hipMemcpy(f->snap_p[f->par], m.p.data(), m.p.size() * 8, hipMemcpyHostToDevice));
    FMCHK(h, hipMemcpy(f->snap_src[f->par], m.src.data(), S1 * 4, hipMemcpyHostToDevice));
    f->S = (uint32_t)S1;
    f->hseq = m.seq;
    return PSIM_OK;
}

int psim_fm_inflight(const psim_handle* h, uint64_t* messages) {
    if (!h || !messages) return PSIM_EINVAL;
    const FmState* f = fm_of(h);
    if (!f) return PSIM_ESTATE;
    psim_handle* hh = const_cast<psim_handle*>(h);
    FMCHK(hh, hipSetDevice(handle_device(h)));
    FMCHK(hh, hipStreamSynchronize(handle_stream(h)));
    std::vector<unsigned long long> p(size_t(f->S) * f->NW);
    if (!p.empty()) FMCHK(hh, hipMemcpy(p.data(), f->snap_p[f->par], p.size() * 8, hipMemcpyDeviceToHost));
    uint64_t c = 0;
    for (unsigned long long x : p) c += __builtin_popcountll(x);
    *messages = c;
    return PSIM_OK;
}

}  // extern "C"
