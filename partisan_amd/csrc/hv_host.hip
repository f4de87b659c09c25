// hv_host.hip -- host side of the HyParView engine (kernels: hyparview.hip,
// DESIGN.md 5.2): psim_hv_*.  The engine's device state is a module of the
// handle (psim_internal.h ModuleState).
#include "psim_internal.h"
#include "../../include/psim.h"

#include <algorithm>
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

constexpr uint32_t kHvChunk = 16;   // HyParView rounds between host synchronisations

struct HvState : ModuleState {
    uint32_t n = 0, cap = 0;
    psim_hv_config cfg{};
    HvHead* head = nullptr;
    uint32_t *act = nullptr, *pas = nullptr, *alive = nullptr;
    unsigned long long *skey = nullptr, *rkey = nullptr;   // id-map hash tables
    uint2 *sval = nullptr, *rval = nullptr;
    uint32_t map_cap = 0;
    HvMsg* msg[2] = {nullptr, nullptr};
    uint32_t* nmsg = nullptr;                 // [2] device queue counts
    uint32_t *cnt = nullptr, *cur = nullptr, *off = nullptr, *idx = nullptr, *bsum = nullptr;
    uint32_t* idx2 = nullptr;                 // [cap] crowded buckets, sorted
    uint32_t* joinbuf = nullptr;              // [2][n] staged join pairs
    unsigned long long* stats = nullptr;      // [kHvChunk][kHvNStat]
    unsigned long long* h_stats = nullptr;    // pinned mirror
    hipEvent_t ev[2 * 16] = {};
    uint32_t par = 0;                         // queue the next round reads
    uint64_t round = 0;
    // psim_hv_join_seq: a chunk's join rows and round rows (device, pinned)
    unsigned long long* seq_stats = nullptr;
    unsigned long long* h_seq_stats = nullptr;
    ~HvState() override {
        void* ptrs[] = {head, act, pas, skey, sval, rkey, rval, alive, msg[0], msg[1], nmsg,
                        cnt, cur, off, idx, bsum, joinbuf, stats, idx2, seq_stats};
        for (void* p : ptrs)
            if (p) (void)hipFree(p);
        if (h_stats) (void)hipHostFree(h_stats);
        if (h_seq_stats) (void)hipHostFree(h_seq_stats);
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
    }
};

// the handle's HyParView state (an empty one before psim_hv_setup)
HvState& hv_ref(psim_handle* h) {
    ModuleState*& m = handle_module(h, MOD_HV);
    if (!m) m = new HvState();
    return *static_cast<HvState*>(m);
}
const HvState& hv_ref(const psim_handle* h) {
    static const HvState none;
    const ModuleState* m = handle_module(h, MOD_HV);
    return m ? *static_cast<const HvState*>(m) : none;
}
HvState& hv_reset(psim_handle* h) {
    ModuleState*& m = handle_module(h, MOD_HV);
    delete m;
    m = new HvState();
    return *static_cast<HvState*>(m);
}

}  // namespace

namespace {

HvArgs make_hv_args(const psim_handle* h, uint32_t par, unsigned long long* stats) {
    const auto& v = hv_ref(h);
    HvArgs a{};
    a.n = v.n;
    a.cfg = HvCfg{v.cfg.active_max_size, v.cfg.active_min_size, v.cfg.active_rwl, v.cfg.passive_max_size,
                  v.cfg.passive_rwl, v.cfg.shuffle_k_active, v.cfg.shuffle_k_passive};
    a.key = make_uint2((uint32_t)handle_seed(h), (uint32_t)(handle_seed(h) >> 32));
    a.alive = v.alive;
    a.head = v.head;
    a.act = v.act;
    a.pas = v.pas;
    a.skey = v.skey;
    a.sval = v.sval;
    a.rkey = v.rkey;
    a.rval = v.rval;
    a.map_mask = v.map_cap - 1;
    a.in = v.msg[par];
    a.nin = v.nmsg + par;
    a.out = v.msg[par ^ 1];
    a.nout = v.nmsg + (par ^ 1);
    a.out_cap = v.cap;
    a.cnt = v.cnt;
    a.cur = v.cur;
    a.off = v.off;
    a.idx = v.idx;
    a.idx2 = v.idx2;
    a.bsum = v.bsum;
    a.stats = stats;
    return a;
}

int hv_check_err(psim_handle* h, unsigned long long e, uint64_t round) {
    if (e & 1ull) return handle_fail(h, PSIM_EOVERFLOW, "hyparview round %llu: message queue over %u records",
                              (unsigned long long)round, hv_ref(h).cap);
    if (e & 2ull) return handle_fail(h, PSIM_EOVERFLOW, "hyparview round %llu: id-map table (%u slots) too full",
                              (unsigned long long)round, hv_ref(h).map_cap);
    if (e & 16ull) return handle_fail(h, PSIM_ESTATE, "hyparview round %llu: a view held a non-vertex id (engine bug)",
                               (unsigned long long)round);
    return PSIM_OK;
}

}  // namespace

extern "C" {

int psim_hv_setup(psim_handle* h, uint32_t n, const psim_hv_config* cfg) {
    if (!h || !cfg || n < 1) return PSIM_EINVAL;
    if (cfg->active_max_size < 2 || cfg->active_max_size > 8 || cfg->passive_max_size < 1 ||
        cfg->passive_max_size > 32 || cfg->active_rwl > 255 || cfg->passive_rwl > 255 ||
        cfg->shuffle_k_active + cfg->shuffle_k_passive > kHvX - 1)
        return handle_fail(h, PSIM_EINVAL, "hyparview config out of range (active <= 8, passive <= 32, k_a + k_p <= 7)");
    HIPCHK(h, hipSetDevice(handle_device(h)));
    HIPCHK(h, hipStreamSynchronize(handle_stream(h)));
    auto& v = hv_reset(h);
    const size_t N = n;
    const uint32_t cap = (uint32_t)std::min<uint64_t>(8ull * n + 4096, 0xFFFFFFF0ull);
    const uint32_t nb = (n + kBlock - 1) / kBlock;
    uint32_t mcap = 1u << 16;                  // id-map tables: >= 16 rows per vertex, power of two
    while (mcap < 16ull * n && mcap < (1u << 31)) mcap <<= 1;
    auto A = [&](void** p, size_t bytes) { return alloc_zero(p, bytes); };
    bool ok = A((void**)&v.head, N * sizeof(HvHead)) && A((void**)&v.act, N * 32) && A((void**)&v.pas, N * 128) &&
              A((void**)&v.skey, size_t(mcap) * 8) && A((void**)&v.sval, size_t(mcap) * 8) &&
              A((void**)&v.rkey, size_t(mcap) * 8) && A((void**)&v.rval, size_t(mcap) * 8) &&
              A((void**)&v.alive, ((N + 31) / 32) * 4) && A((void**)&v.msg[0], size_t(cap) * sizeof(HvMsg)) &&
              A((void**)&v.msg[1], size_t(cap) * sizeof(HvMsg)) && A((void**)&v.nmsg, 16) &&
              A((void**)&v.cnt, N * 4) && A((void**)&v.cur, N * 4) && A((void**)&v.off, (N + 1) * 4) &&
              A((void**)&v.idx, size_t(cap) * 4) && A((void**)&v.idx2, size_t(cap) * 4) &&
              A((void**)&v.bsum, size_t(nb) * 4) &&
              A((void**)&v.joinbuf, 2 * N * 4) && A((void**)&v.stats, kHvChunk * kHvNStat * 8) &&
              hipHostMalloc((void**)&v.h_stats, kHvChunk * kHvNStat * 8, 0) == hipSuccess;
    for (auto& e : v.ev) ok = ok && hipEventCreate(&e) == hipSuccess;
    if (!ok) {
        hv_reset(h);
        return handle_fail(h, PSIM_ENOMEM, "hyparview state for n=%u", n);
    }
    v.n = n;
    v.cap = cap;
    v.map_cap = mcap;
    v.cfg = *cfg;
    HIPCHK(h, hipMemsetAsync(v.skey, 0xFF, size_t(mcap) * 8, handle_stream(h)));
    HIPCHK(h, hipMemsetAsync(v.rkey, 0xFF, size_t(mcap) * 8, handle_stream(h)));
    HIPCHK(h, hipMemsetAsync(v.alive, 0xFF, ((N + 31) / 32) * 4, handle_stream(h)));
    HIPCHK(h, launch_hv_init(make_hv_args(h, 0, v.stats), handle_stream(h)));
    HIPCHK(h, hipStreamSynchronize(handle_stream(h)));
    return PSIM_OK;
}

int psim_hv_set_alive(psim_handle* h, const uint8_t* alive, size_t n) {
    if (!h || !alive) return PSIM_EINVAL;
    if (!hv_ref(h).n) return handle_fail(h, PSIM_ESTATE, "psim_hv_setup not called");
    if (n != hv_ref(h).n) return handle_fail(h, PSIM_EINVAL, "alive has %zu entries, cluster has %u", n, hv_ref(h).n);
    std::vector<uint32_t> bm((n + 31) / 32, 0);
    for (size_t i = 0; i < n; i++)
        if (alive[i]) bm[i >> 5] |= 1u << (i & 31);
    HIPCHK(h, hipSetDevice(handle_device(h)));
    HIPCHK(h, hipMemcpyAsync(hv_ref(h).alive, bm.data(), bm.size() * 4, hipMemcpyHostToDevice, handle_stream(h)));
    HIPCHK(h, hipStreamSynchronize(handle_stream(h)));
    return PSIM_OK;
}

int psim_hv_join(psim_handle* h, const uint32_t* v, const uint32_t* contact, size_t k) {
    if (!h || (k && (!v || !contact))) return PSIM_EINVAL;
    auto& hv = hv_ref(h);
    if (!hv.n) return handle_fail(h, PSIM_ESTATE, "psim_hv_setup not called");
    if (k > hv.n) return handle_fail(h, PSIM_EINVAL, "%zu joins for %u vertices", k, hv.n);
    std::vector<uint8_t> seen(hv.n, 0);
    for (size_t i = 0; i < k; i++) {
        if (v[i] >= hv.n || contact[i] >= hv.n) return handle_fail(h, PSIM_EINVAL, "join %zu: vertex out of range", i);
        if (seen[v[i]]) return handle_fail(h, PSIM_EINVAL, "join %zu: vertex %u joins twice in one batch", i, v[i]);
        seen[v[i]] = 1;
    }
    if (!k) return PSIM_OK;
    HIPCHK(h, hipSetDevice(handle_device(h)));
    HIPCHK(h, hipMemcpyAsync(hv.joinbuf, v, k * 4, hipMemcpyHostToDevice, handle_stream(h)));
    HIPCHK(h, hipMemcpyAsync(hv.joinbuf + hv.n, contact, k * 4, hipMemcpyHostToDevice, handle_stream(h)));
    HIPCHK(h, hipMemsetAsync(hv.stats, 0, kHvNStat * 8, handle_stream(h)));
    // the join messages go to the queue the next round reads
    HvArgs a = make_hv_args(h, hv.par ^ 1u, hv.stats);
    HIPCHK(h, launch_hv_join(a, hv.joinbuf, hv.joinbuf + hv.n, (uint32_t)k, handle_stream(h)));
    HIPCHK(h, hipMemcpyAsync(hv.h_stats, hv.stats, kHvNStat * 8, hipMemcpyDeviceToHost, handle_stream(h)));
    HIPCHK(h, hipStreamSynchronize(handle_stream(h)));
    return hv_check_err(h, hv.h_stats[11], hv.round);
}

int psim_hv_step(psim_handle* h, uint32_t rounds, psim_hv_stats* out, size_t cap) {
    if (!h) return PSIM_EINVAL;
    auto& v = hv_ref(h);
    if (!v.n) return handle_fail(h, PSIM_ESTATE, "psim_hv_setup not called");
    HIPCHK(h, hipSetDevice(handle_device(h)));
    uint32_t done = 0;
    while (done < rounds) {
        const uint32_t k = std::min(kHvChunk, rounds - done);
        HIPCHK(h, hipMemsetAsync(v.stats, 0, size_t(k) * kHvNStat * 8, handle_stream(h)));
        for (uint32_t i = 0; i < k; i++) {
            HvArgs a = make_hv_args(h, v.par, v.stats + size_t(i) * kHvNStat);
            const uint64_t t = v.round + i + 1;   // 1-based round; timers fire at its end
            a.timers = (v.cfg.promotion_rounds && t % v.cfg.promotion_rounds == 0 ? 1u : 0u) |
                       (v.cfg.shuffle_rounds && t % v.cfg.shuffle_rounds == 0 ? 2u : 0u);
            HIPCHK(h, hipMemsetAsync(v.nmsg + (v.par ^ 1u), 0, 4, handle_stream(h)));
            HIPCHK(h, hipEventRecord(v.ev[2 * i], handle_stream(h)));
            HIPCHK(h, launch_hv_round(a, handle_stream(h)));
            HIPCHK(h, hipEventRecord(v.ev[2 * i + 1], handle_stream(h)));
            v.par ^= 1u;
        }
        HIPCHK(h, hipMemcpyAsync(v.h_stats, v.stats, size_t(k) * kHvNStat * 8, hipMemcpyDeviceToHost, handle_stream(h)));
        HIPCHK(h, handle_wait(h));
        for (uint32_t i = 0; i < k; i++) {
            const unsigned long long* r = v.h_stats + size_t(i) * kHvNStat;
            const uint64_t t = v.round + i + 1;
            int rc = hv_check_err(h, r[11], t);
            if (rc != PSIM_OK) { v.round += k; return rc; }
            float ms = 0.f;
            HIPCHK(h, hipEventElapsedTime(&ms, v.ev[2 * i], v.ev[2 * i + 1]));
            handle_add_round(h, ms);
            const size_t j = done + i;
            if (out && j < cap) {
                psim_hv_stats& o = out[j];
                memset(&o, 0, sizeof o);
                uint64_t emitted = 0;
                for (int q = 1; q < 10; q++) { o.sent[q] = r[q]; emitted += r[q]; }
                o.draws = r[10];
                o.error = r[11];
                o.processed = r[12];
                o.active = r[13];
                o.algo_bytes = 64ull * (r[12] + emitted) + 2ull * 176ull * r[13] + 12ull * v.n;
                o.kernel_ms = ms;
            }
        }
        v.round += k;
        done += k;
    }
    return PSIM_OK;
}

int psim_hv_join_seq(psim_handle* h, const uint32_t* v, const uint32_t* contact, size_t k, uint32_t rounds,
                     psim_hv_stats* out, size_t cap) {
    if (!h || (k && (!v || !contact))) return PSIM_EINVAL;
    auto& hv = hv_ref(h);
    if (!hv.n) return handle_fail(h, PSIM_ESTATE, "psim_hv_setup not called");
    if (k > hv.n) return handle_fail(h, PSIM_EINVAL, "%zu joins for %u vertices", k, hv.n);
    for (size_t i = 0; i < k; i++)
        if (v[i] >= hv.n || contact[i] >= hv.n) return handle_fail(h, PSIM_EINVAL, "join %zu: vertex out of range", i);
    if (!k) return PSIM_OK;
    HIPCHK(h, hipSetDevice(handle_device(h)));
    const hipStream_t st = handle_stream(h);
    // every join pair uploaded once (join i reads entry i)
    HIPCHK(h, hipMemcpyAsync(hv.joinbuf, v, k * 4, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(hv.joinbuf + hv.n, contact, k * 4, hipMemcpyHostToDevice, st));
    // a chunk: J joins, each followed by `rounds` rounds, with an event pair per
    // round (the handle's 2 x 16 events) -- one host wait per chunk
    const uint32_t per = 1u + rounds;
    const uint32_t J = rounds ? std::max<uint32_t>(1u, kHvChunk / std::max<uint32_t>(1u, rounds)) : kHvChunk;
    if (rounds > kHvChunk) {
        // long waits between joins: one join at a time through the plain calls
        size_t used = 0;
        for (size_t i = 0; i < k; i++) {
            int rc = psim_hv_join(h, v + i, contact + i, 1);
            if (rc) return rc;
            std::vector<psim_hv_stats> tmp(rounds);
            rc = psim_hv_step(h, rounds, tmp.data(), rounds);
            if (rc) return rc;
            for (uint32_t r = 0; r < rounds && out && used < cap; r++) out[used++] = tmp[r];
        }
        return PSIM_OK;
    }
    // rows = J·(rounds+1) <= (kHvChunk/r)·(r+1) <= 2·kHvChunk for every rounds <= kHvChunk
    // (rounds = 1 is the worst, rounds = 0 needs kHvChunk): the buffers are sized once for
    // that bound, so a later call with another `rounds` on the same handle never outgrows them
    const size_t rows = size_t(J) * per;
    constexpr size_t kSeqRows = 2 * size_t(kHvChunk);
    if (rows > kSeqRows) return handle_fail(h, PSIM_ESTATE, "join sequence rows %zu > %zu", rows, kSeqRows);
    if (!hv.seq_stats) {
        if (!alloc_zero((void**)&hv.seq_stats, kSeqRows * kHvNStat * 8) ||
            hipHostMalloc((void**)&hv.h_seq_stats, kSeqRows * kHvNStat * 8, 0) != hipSuccess) {
            hv.h_seq_stats = nullptr;
            if (hv.seq_stats) (void)hipFree(hv.seq_stats);   // both or neither: the next call retries
            hv.seq_stats = nullptr;
            return handle_fail(h, PSIM_ENOMEM, "hyparview join sequence rows");
        }
    }
    size_t used = 0;
    for (size_t j0 = 0; j0 < k; j0 += J) {
        const uint32_t nj = (uint32_t)std::min<size_t>(J, k - j0);
        HIPCHK(h, hipMemsetAsync(hv.seq_stats, 0, size_t(nj) * per * kHvNStat * 8, st));
        for (uint32_t j = 0; j < nj; j++) {
            unsigned long long* jr = hv.seq_stats + size_t(j) * per * kHvNStat;
            // psim_hv_join: the join messages go to the queue the next round reads
            HvArgs a = make_hv_args(h, hv.par ^ 1u, jr);
            HIPCHK(h, launch_hv_join(a, hv.joinbuf + j0 + j, hv.joinbuf + hv.n + j0 + j, 1u, st));
            // psim_hv_step(rounds)
            for (uint32_t i = 0; i < rounds; i++) {
                HvArgs b = make_hv_args(h, hv.par, jr + size_t(1 + i) * kHvNStat);
                const uint64_t t = hv.round + uint64_t(j) * rounds + i + 1;
                b.timers = (hv.cfg.promotion_rounds && t % hv.cfg.promotion_rounds == 0 ? 1u : 0u) |
                           (hv.cfg.shuffle_rounds && t % hv.cfg.shuffle_rounds == 0 ? 2u : 0u);
                HIPCHK(h, hipMemsetAsync(hv.nmsg + (hv.par ^ 1u), 0, 4, st));
                HIPCHK(h, hipEventRecord(hv.ev[2 * (j * rounds + i)], st));
                HIPCHK(h, launch_hv_round(b, st));
                HIPCHK(h, hipEventRecord(hv.ev[2 * (j * rounds + i) + 1], st));
                hv.par ^= 1u;
            }
        }
        HIPCHK(h, hipMemcpyAsync(hv.h_seq_stats, hv.seq_stats, size_t(nj) * per * kHvNStat * 8, hipMemcpyDeviceToHost,
                                 st));
        HIPCHK(h, handle_wait(h));
        for (uint32_t j = 0; j < nj; j++) {
            const unsigned long long* jr = hv.h_seq_stats + size_t(j) * per * kHvNStat;
            int rc = hv_check_err(h, jr[11], hv.round);             // the join, as psim_hv_join reports it
            if (rc != PSIM_OK) { hv.round += uint64_t(nj - j) * rounds; return rc; }
            for (uint32_t i = 0; i < rounds; i++) {
                const unsigned long long* r = jr + size_t(1 + i) * kHvNStat;
                const uint64_t t = hv.round + 1;
                rc = hv_check_err(h, r[11], t);
                if (rc != PSIM_OK) { hv.round += uint64_t(nj - j) * rounds - i; return rc; }
                float ms = 0.f;
                HIPCHK(h, hipEventElapsedTime(&ms, hv.ev[2 * (j * rounds + i)], hv.ev[2 * (j * rounds + i) + 1]));
                handle_add_round(h, ms);
                if (out && used < cap) {
                    psim_hv_stats& o = out[used];
                    memset(&o, 0, sizeof o);
                    uint64_t emitted = 0;
                    for (int q = 1; q < 10; q++) { o.sent[q] = r[q]; emitted += r[q]; }
                    o.draws = r[10];
                    o.error = r[11];
                    o.processed = r[12];
                    o.active = r[13];
                    o.algo_bytes = 64ull * (r[12] + emitted) + 2ull * 176ull * r[13] + 12ull * hv.n;
                    o.kernel_ms = ms;
                }
                used++;
                hv.round++;
            }
        }
    }
    return PSIM_OK;
}

int psim_hv_get_views(const psim_handle* h, uint32_t* act, uint8_t* na, uint32_t* pas, uint8_t* np, size_t n) {
    if (!h || n != hv_ref(h).n || !n) return PSIM_EINVAL;
    psim_handle* hh = const_cast<psim_handle*>(h);
    const auto& v = hv_ref(h);
    HIPCHK(hh, hipSetDevice(handle_device(h)));
    HIPCHK(hh, hipStreamSynchronize(handle_stream(h)));
    if (act) HIPCHK(hh, hipMemcpy(act, v.act, n * 32, hipMemcpyDeviceToHost));
    if (pas) HIPCHK(hh, hipMemcpy(pas, v.pas, n * 128, hipMemcpyDeviceToHost));
    if (na || np) {
        std::vector<HvHead> hd(n);
        HIPCHK(hh, hipMemcpy(hd.data(), v.head, n * sizeof(HvHead), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n; i++) {
            if (na) na[i] = hd[i].na;
            if (np) np[i] = hd[i].np;
        }
    }
    return PSIM_OK;
}

int psim_hv_get_draws(const psim_handle* h, uint64_t* draws, size_t n) {
    if (!h || !draws || n != hv_ref(h).n || !n) return PSIM_EINVAL;
    psim_handle* hh = const_cast<psim_handle*>(h);
    HIPCHK(hh, hipSetDevice(handle_device(h)));
    HIPCHK(hh, hipStreamSynchronize(handle_stream(h)));
    std::vector<HvHead> hd(n);
    HIPCHK(hh, hipMemcpy(hd.data(), hv_ref(h).head, n * sizeof(HvHead), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n; i++) draws[i] = hd[i].draws;
    return PSIM_OK;
}

int psim_hv_get_idmap(const psim_handle* h, uint32_t v, int which, uint32_t* peer, uint32_t* epoch, uint32_t* cnt,
                      size_t cap, size_t* len) {
    if (!h || !len || v >= hv_ref(h).n || (which != 0 && which != 1)) return PSIM_EINVAL;
    psim_handle* hh = const_cast<psim_handle*>(h);
    HIPCHK(hh, hipSetDevice(handle_device(h)));
    HIPCHK(hh, hipStreamSynchronize(handle_stream(h)));
    HvHead hd;
    HIPCHK(hh, hipMemcpy(&hd, hv_ref(h).head + v, sizeof hd, hipMemcpyDeviceToHost));
    const uint32_t m = which ? hd.nrecv : hd.nsent;
    const size_t M = hv_ref(h).map_cap;
    std::vector<unsigned long long> keys(M);
    std::vector<uint2> vals(M);
    HIPCHK(hh, hipMemcpy(keys.data(), which ? hv_ref(h).rkey : hv_ref(h).skey, M * 8, hipMemcpyDeviceToHost));
    HIPCHK(hh, hipMemcpy(vals.data(), which ? hv_ref(h).rval : hv_ref(h).sval, M * 8, hipMemcpyDeviceToHost));
    size_t k = 0;
    for (size_t i = 0; i < M; i++) {
        if (keys[i] == ~0ull || (uint32_t)(keys[i] >> 32) != v) continue;
        if (k < cap) {
            if (peer) peer[k] = (uint32_t)keys[i];
            if (epoch) epoch[k] = vals[i].x;
            if (cnt) cnt[k] = vals[i].y;
        }
        k++;
    }
    if (k != m) return handle_fail(hh, PSIM_ESTATE, "id map of %u: %zu rows in the table, head says %u", v, k, m);
    *len = m;
    return PSIM_OK;
}

int psim_hv_inflight(const psim_handle* h, uint64_t* messages) {
    if (!h || !messages || !hv_ref(h).n) return PSIM_EINVAL;
    psim_handle* hh = const_cast<psim_handle*>(h);
    HIPCHK(hh, hipSetDevice(handle_device(h)));
    HIPCHK(hh, hipStreamSynchronize(handle_stream(h)));
    uint32_t c = 0;
    HIPCHK(hh, hipMemcpy(&c, hv_ref(h).nmsg + hv_ref(h).par, 4, hipMemcpyDeviceToHost));
    *messages = c;
    return PSIM_OK;
}

}  // extern "C"

