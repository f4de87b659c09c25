// causal_host.hip -- host side of the causal delivery engine (kernels:
// causal.hip): psim_causal_* on one GPU and vertex-sharded.
// The engine's device state is a module of the handle (ModuleState).
#include "psim_internal.h"
#include "../../include/psim.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace psim;

namespace {

#define HIPCHK(h, x)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess)                                                               \
            return handle_fail((h), PSIM_EHIP, "%s failed: %s", #x, hipGetErrorString(e_)); \
    } while (0)

struct CsState : ModuleState {
    uint32_t n = 0, m = 0, period = 1, dmax = 1, redeliver = 1;
    uint32_t n_global = 0, v_lo = 0, rank = 0, world = 1;   // vertex shard [v_lo, v_lo + n) of n_global
    uint32_t *clk = nullptr, *self = nullptr, *buf = nullptr, *nbuf = nullptr, *base = nullptr, *dring = nullptr;
    unsigned long long *delivered = nullptr, *stats = nullptr, *h_stats = nullptr;
    uint32_t* x_slab = nullptr;        // the in-library exchange's slab (psim_causal_shard_step)
    uint64_t round = 0;
    ~CsState() override {
        void* ptrs[] = {clk, self, buf, nbuf, base, delivered, stats, x_slab, dring};
        for (void* p : ptrs)
            if (p) (void)hipFree(p);
        if (h_stats) (void)hipHostFree(h_stats);
    }
};

CsState& cs_ref(psim_handle* h) {
    ModuleState*& m = handle_module(h, MOD_CAUSAL);
    if (!m) m = new CsState();
    return *static_cast<CsState*>(m);
}
const CsState& cs_ref(const psim_handle* h) {
    static const CsState none;
    const ModuleState* m = handle_module(h, MOD_CAUSAL);
    return m ? *static_cast<const CsState*>(m) : none;
}
CsState& cs_reset(psim_handle* h) {
    ModuleState*& m = handle_module(h, MOD_CAUSAL);
    delete m;
    m = new CsState();
    return *static_cast<CsState*>(m);
}

}  // namespace

namespace {

CsArgs make_cs_args(const psim_handle* h, uint32_t t) {
    const auto& c = cs_ref(h);
    CsArgs a{};
    a.n = c.n;
    a.m = c.m;
    a.period = c.period;
    a.dmax = c.dmax;
    a.redeliver = c.redeliver;
    a.v_lo = c.v_lo;
    a.n_global = c.n_global;
    a.key = make_uint2((uint32_t)handle_seed(h), (uint32_t)(handle_seed(h) >> 32));
    a.t = t;
    a.clk = c.clk;
    a.self = c.self;
    a.buf = c.buf;
    a.nbuf = c.nbuf;
    a.delivered = c.delivered;
    a.base = c.base;
    a.stats = c.stats;
    a.dring = c.dring;
    a.bufcap = env_cap("PSIM_CS_BUFCAP", kCsBufCap);
    return a;
}

}  // namespace

extern "C" {

int psim_causal_setup(psim_handle* h, uint32_t n, uint32_t m, uint32_t period, uint32_t dmax, uint32_t redeliver) {
    return psim_causal_shard_setup(h, n, m, period, dmax, redeliver, 0, 1);
}

int psim_causal_shard_setup(psim_handle* h, uint32_t n, uint32_t m, uint32_t period, uint32_t dmax,
                            uint32_t redeliver, int rank, int world) {
    if (!h || world < 1 || rank < 0 || rank >= world) return PSIM_EINVAL;
    if (n < 2 || m < 1 || m > kCsLanes || m > n || period < 1 || dmax < 1 || dmax > 30 ||
        dmax + 2 * redeliver + period + 2 >= kCsWindow)
        return handle_fail(h, PSIM_EINVAL, "causal: need 2 <= n, 1 <= m <= min(64, n), period >= 1, 1 <= dmax <= 30, "
                                    "dmax + 2 redeliver + period + 2 < %u", kCsWindow);
    HIPCHK(h, hipSetDevice(handle_device(h)));
    HIPCHK(h, hipStreamSynchronize(handle_stream(h)));
    auto& c = cs_reset(h);
    const uint32_t lo = uint32_t((uint64_t(n) * rank) / world), hi = uint32_t((uint64_t(n) * (rank + 1)) / world);
    const size_t N = std::max<uint32_t>(hi - lo, 1);
    auto A = [&](void** p, size_t bytes) { return alloc_zero(p, bytes); };
    const bool ok = A((void**)&c.clk, N * kCsLanes * 4) && A((void**)&c.self, N * 4) &&
                    A((void**)&c.buf, N * kCsBufCap * 4) && A((void**)&c.nbuf, N * 4) &&
                    A((void**)&c.base, size_t(kCsWindow) * kCsLanes * kCsLanes * 4) &&
                    A((void**)&c.delivered, N * 8) && A((void**)&c.stats, kStatShards * kCsNStat * 8) &&
                    hipHostMalloc((void**)&c.h_stats, kStatShards * kCsNStat * 8, 0) == hipSuccess;
    // each message's delay drawn once, in the round after its broadcast, and
    // kept until it lands, instead of redrawn in each round of its window
    const bool ring_ok = !ok || dmax > kCsRingMax || A((void**)&c.dring, N * kCsLanes * 4);
    if (!ok || !ring_ok) {
        cs_reset(h);
        return handle_fail(h, PSIM_ENOMEM, "causal state for n=%u", n);
    }
    c.n = hi - lo;
    c.n_global = n;
    c.v_lo = lo;
    c.rank = (uint32_t)rank;
    c.world = (uint32_t)world;
    c.m = m;
    c.period = period;
    c.dmax = dmax;
    c.redeliver = redeliver;
    return PSIM_OK;
}

int psim_causal_step(psim_handle* h, uint32_t rounds, psim_causal_stats* out, size_t cap) {
    if (!h) return PSIM_EINVAL;
    auto& c = cs_ref(h);
    if (!c.n_global) return handle_fail(h, PSIM_ESTATE, "psim_causal_setup not called");
    if (c.world > 1) return handle_fail(h, PSIM_ESTATE, "sharded causal handle: use psim_causal_shard_round");
    HIPCHK(h, hipSetDevice(handle_device(h)));
    for (uint32_t i = 0; i < rounds; i++) {
        const uint64_t t = c.round + 1;
        if (t >= (1u << 24)) return handle_fail(h, PSIM_EOVERFLOW, "causal: round %llu exceeds 2^24", (unsigned long long)t);
        CsArgs a = make_cs_args(h, (uint32_t)t);
        HIPCHK(h, hipMemsetAsync(c.stats, 0, kStatShards * kCsNStat * 8, handle_stream(h)));
        HIPCHK(h, hipEventRecord(handle_event(h, 0), handle_stream(h)));
        HIPCHK(h, launch_cs_round(a, handle_stream(h)));
        HIPCHK(h, launch_cs_broadcast(a, handle_stream(h)));
        HIPCHK(h, hipEventRecord(handle_event(h, 1), handle_stream(h)));
        HIPCHK(h, hipMemcpyAsync(c.h_stats, c.stats, kStatShards * kCsNStat * 8, hipMemcpyDeviceToHost, handle_stream(h)));
        HIPCHK(h, handle_wait(h));
        c.round = t;
        unsigned long long r[kCsNStat] = {0};
        unsigned long long err = 0;
        for (int sh = 0; sh < kStatShards; sh++)
            for (int q = 0; q < kCsNStat; q++) {
                if (q == 5) err |= c.h_stats[sh * kCsNStat + q];
                else r[q] += c.h_stats[sh * kCsNStat + q];
            }
#ifdef CS_PROF
        fprintf(stderr, "cs_prof round %llu received %llu fast %llu general-fold checks %llu\n", (unsigned long long)t,
                r[1], r[0], r[7]);
#endif
        if (err & 1ull) return handle_fail(h, PSIM_EOVERFLOW, "causal round %llu: more than %u buffered messages at a vertex",
                                    (unsigned long long)t, kCsBufCap);
        if (err & 2ull) return handle_fail(h, PSIM_EOVERFLOW, "causal round %llu: a buffered message outlived the %u-round "
                                    "clock window", (unsigned long long)t, kCsWindow);
        if (err & 4ull) return handle_fail(h, PSIM_EOVERFLOW, "causal round %llu: a u32 clock entry overflowed",
                                    (unsigned long long)t);
        float ms = 0.f;
        HIPCHK(h, hipEventElapsedTime(&ms, handle_event(h, 0), handle_event(h, 1)));
        handle_add_round(h, ms);
        if (out && i < cap) {
            psim_causal_stats& o = out[i];
            memset(&o, 0, sizeof o);
            o.emitted = r[6];
            o.received = r[1];
            o.delivered = r[2];
            o.checks = r[3];
            o.buffered = r[4];
            o.algo_bytes = 1024ull * r[2] + 256ull * r[3] + 32ull * r[1];
            o.kernel_ms = ms;
        }
    }
    return PSIM_OK;
}

// Split-phase sharded round: the local round and the broadcasts of this
// shard's emitters; their base-clock rows go to the caller's `slab`
// (64 x 64 u32, zero elsewhere) to be sum-all-reduced, then
// psim_causal_shard_ingest installs the reduced slab for every receiver.
int psim_causal_shard_round(psim_handle* h, void* slab, psim_causal_stats* out) {
    if (!h || !slab) return PSIM_EINVAL;
    auto& c = cs_ref(h);
    if (!c.n_global) return handle_fail(h, PSIM_ESTATE, "psim_causal_shard_setup not called");
    HIPCHK(h, hipSetDevice(handle_device(h)));
    const uint64_t t = c.round + 1;
    if (t >= (1u << 24)) return handle_fail(h, PSIM_EOVERFLOW, "causal: round %llu exceeds 2^24", (unsigned long long)t);
    CsArgs a = make_cs_args(h, (uint32_t)t);
    uint32_t* sl = c.base + size_t(t % kCsWindow) * kCsLanes * kCsLanes;
    HIPCHK(h, hipMemsetAsync(c.stats, 0, kStatShards * kCsNStat * 8, handle_stream(h)));
    HIPCHK(h, hipEventRecord(handle_event(h, 0), handle_stream(h)));
    if (c.n) HIPCHK(h, launch_cs_round(a, handle_stream(h)));
    HIPCHK(h, hipMemsetAsync(sl, 0, kCsLanes * kCsLanes * 4, handle_stream(h)));
    HIPCHK(h, launch_cs_broadcast(a, handle_stream(h)));
    HIPCHK(h, hipEventRecord(handle_event(h, 1), handle_stream(h)));
    HIPCHK(h, hipMemcpyAsync(slab, sl, kCsLanes * kCsLanes * 4, hipMemcpyDeviceToDevice, handle_stream(h)));
    HIPCHK(h, hipMemcpyAsync(c.h_stats, c.stats, kStatShards * kCsNStat * 8, hipMemcpyDeviceToHost, handle_stream(h)));
    HIPCHK(h, handle_wait(h));
    c.round = t;
    unsigned long long r[kCsNStat] = {0};
    unsigned long long err = 0;
    for (int sh = 0; sh < kStatShards; sh++)
        for (int q = 0; q < kCsNStat; q++) {
            if (q == 5) err |= c.h_stats[sh * kCsNStat + q];
            else r[q] += c.h_stats[sh * kCsNStat + q];
        }
    if (err & 1ull) return handle_fail(h, PSIM_EOVERFLOW, "causal round %llu: more than %u buffered messages at a vertex",
                                (unsigned long long)t, a.bufcap);
    if (err & 2ull) return handle_fail(h, PSIM_EOVERFLOW, "causal round %llu: a buffered message outlived the %u-round "
                                "clock window", (unsigned long long)t, kCsWindow);
    if (err & 4ull) return handle_fail(h, PSIM_EOVERFLOW, "causal round %llu: a u32 clock entry overflowed",
                                (unsigned long long)t);
    float ms = 0.f;
    HIPCHK(h, hipEventElapsedTime(&ms, handle_event(h, 0), handle_event(h, 1)));
    handle_add_round(h, ms);
    if (out) {
        memset(out, 0, sizeof *out);
        out->emitted = r[6];
        out->received = r[1];
        out->delivered = r[2];
        out->checks = r[3];
        out->buffered = r[4];
        out->algo_bytes = 1024ull * r[2] + 256ull * r[3] + 32ull * r[1];
        out->kernel_ms = ms;
    }
    return PSIM_OK;
}

int psim_causal_shard_ingest(psim_handle* h, const void* slab) {
    if (!h || !slab) return PSIM_EINVAL;
    auto& c = cs_ref(h);
    if (!c.n_global) return handle_fail(h, PSIM_ESTATE, "psim_causal_shard_setup not called");
    HIPCHK(h, hipSetDevice(handle_device(h)));
    uint32_t* sl = c.base + size_t(c.round % kCsWindow) * kCsLanes * kCsLanes;
    HIPCHK(h, hipMemcpyAsync(sl, slab, kCsLanes * kCsLanes * 4, hipMemcpyDeviceToDevice, handle_stream(h)));
    HIPCHK(h, hipStreamSynchronize(handle_stream(h)));
    return PSIM_OK;
}

int psim_causal_shard_step(psim_handle* h, uint32_t rounds, psim_causal_stats* stats, size_t cap) {
    if (!h) return PSIM_EINVAL;
    auto& c = cs_ref(h);
    if (!c.n_global) return handle_fail(h, PSIM_ESTATE, "psim_causal_shard_setup not called");
    Transport* T = handle_transport(h);
    if (c.world > 1 && !T)
        return handle_fail(h, PSIM_ESTATE, "sharded causal without a transport (psim_shard_init_rccl / _set_transport)");
    HIPCHK(h, hipSetDevice(handle_device(h)));
    constexpr size_t kSlab = size_t(kCsLanes) * kCsLanes;
    if (!c.x_slab && !alloc_zero((void**)&c.x_slab, kSlab * 4)) return handle_fail(h, PSIM_ENOMEM, "causal slab");
    std::vector<uint32_t> hs(kSlab);
    std::vector<int64_t> v(kSlab + 6 + kNCodes);
    for (uint32_t i = 0; i < rounds; i++) {
        psim_causal_stats st;
        memset(&st, 0, sizeof st);
        int rc = psim_causal_shard_round(h, c.x_slab, &st);
        if (c.world == 1 && rc) return rc;
        if (c.world > 1) {
            // the broadcasting emitters' clocks: each row written by its owner,
            // zero elsewhere -- a sum all-reduce is the gather (16 KB), with the
            // round's counters and every shard's error flags in the same call: a
            // shard whose round failed (buffer cap, clock window, u32 overflow)
            // still joins it, so no peer waits forever, and all return alike
            std::fill(v.begin(), v.end(), 0);
            if (!rc && hipMemcpy(hs.data(), c.x_slab, kSlab * 4, hipMemcpyDeviceToHost) != hipSuccess)
                rc = handle_fail(h, PSIM_EHIP, "causal slab read-back");
            if (!rc) {
                for (size_t j = 0; j < kSlab; j++) v[j] = hs[j];
                const uint64_t loc[6] = {st.emitted, st.received, st.delivered, st.checks, st.buffered, st.algo_bytes};
                for (int j = 0; j < 6; j++) v[kSlab + j] = (int64_t)loc[j];
            }
            put_code(v.data() + kSlab + 6, rc);
            std::string err;
            const int trc = T->allreduce(v.data(), v.size(), handle_stream(h), &err);
            if (trc) return handle_fail(h, trc, "causal exchange: %s", err.c_str());
            rc = finish_code(h, v.data() + kSlab + 6, rc, "causal shard step");
            if (rc) return rc;
            for (size_t j = 0; j < kSlab; j++) hs[j] = (uint32_t)v[j];
            HIPCHK(h, hipMemcpy(c.x_slab, hs.data(), kSlab * 4, hipMemcpyHostToDevice));
            st.emitted = v[kSlab]; st.received = v[kSlab + 1]; st.delivered = v[kSlab + 2];
            st.checks = v[kSlab + 3]; st.buffered = v[kSlab + 4]; st.algo_bytes = v[kSlab + 5];
        }
        rc = psim_causal_shard_ingest(h, c.x_slab);
        if (rc) return rc;
        if (stats && i < cap) stats[i] = st;
    }
    return PSIM_OK;
}

int psim_causal_shard_info(const psim_handle* h, uint32_t* v_lo, uint32_t* n_local) {
    if (!h) return PSIM_EINVAL;
    if (v_lo) *v_lo = cs_ref(h).v_lo;
    if (n_local) *n_local = cs_ref(h).n;
    return PSIM_OK;
}

int psim_causal_get_clocks(const psim_handle* h, uint32_t* lanes, uint32_t* self, size_t n) {
    if (!h || n != cs_ref(h).n || !n) return PSIM_EINVAL;
    psim_handle* hh = const_cast<psim_handle*>(h);
    HIPCHK(hh, hipSetDevice(handle_device(h)));
    HIPCHK(hh, hipStreamSynchronize(handle_stream(h)));
    if (lanes) HIPCHK(hh, hipMemcpy(lanes, cs_ref(h).clk, n * kCsLanes * 4, hipMemcpyDeviceToHost));
    if (self) HIPCHK(hh, hipMemcpy(self, cs_ref(h).self, n * 4, hipMemcpyDeviceToHost));
    return PSIM_OK;
}

int psim_causal_get_buffered(const psim_handle* h, uint32_t v, uint32_t* k, uint32_t* round, size_t cap,
                             size_t* len) {
    if (!h || !len || v >= cs_ref(h).n) return PSIM_EINVAL;   // v: index in this shard's range
    psim_handle* hh = const_cast<psim_handle*>(h);
    HIPCHK(hh, hipSetDevice(handle_device(h)));
    HIPCHK(hh, hipStreamSynchronize(handle_stream(h)));
    uint32_t nb = 0;
    HIPCHK(hh, hipMemcpy(&nb, cs_ref(h).nbuf + v, 4, hipMemcpyDeviceToHost));
    std::vector<uint32_t> e(nb);
    if (nb) HIPCHK(hh, hipMemcpy(e.data(), cs_ref(h).buf + size_t(v) * kCsBufCap, nb * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < nb && i < cap; i++) {
        if (k) k[i] = e[i] >> 24;
        if (round) round[i] = e[i] & 0xFFFFFFu;
    }
    *len = nb;
    return PSIM_OK;
}

int psim_causal_get_delivered(const psim_handle* h, uint64_t* delivered, size_t n) {
    if (!h || !delivered || n != cs_ref(h).n || !n) return PSIM_EINVAL;
    psim_handle* hh = const_cast<psim_handle*>(h);
    HIPCHK(hh, hipSetDevice(handle_device(h)));
    HIPCHK(hh, hipStreamSynchronize(handle_stream(h)));
    HIPCHK(hh, hipMemcpy(delivered, cs_ref(h).delivered, n * 8, hipMemcpyDeviceToHost));
    return PSIM_OK;
}

int psim_causal_emitters(const psim_handle* h, uint32_t* emitters, size_t m) {
    if (!h || !emitters || m != cs_ref(h).m || !m) return PSIM_EINVAL;
    for (size_t k = 0; k < m; k++) emitters[k] = (uint32_t)((uint64_t(k) * cs_ref(h).n_global) / cs_ref(h).m);
    return PSIM_OK;
}

}  // extern "C"