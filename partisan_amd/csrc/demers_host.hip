// demers_host.hip -- host side of the Demers epidemic (kernels: demers.hip).
//
// psim_demers_*: one GPU.  A round reads the RM count planes, pull slots and
// push lists of parity `par`, writes those of par ^ 1; the RM processes'
// per-round call records (rumors called this round, calls before it) are
// double-buffered the same way: round parity p reads rmx[p], writes rmx[p ^ 1].
//
// psim_demers_shard_*: the vertex-sharded form.  Shard r owns global ids
// [r C, min((r+1) C, n)), C = ceil(n / world).  A round is split-phase so that
// the transport stays the caller's:
//   psim_demers_shard_round  -- the local round; RM messages to any vertex
//       raise the count planes of the caller's rm_shadow [3][world C]
//       (>= 1 / >= 2 / >= 3 senders), pull replies land in pull_shadow
//       [world C][2] (one writer per slot), the tick's snapshot in snap_all[v],
//       this shard's RM call records in its slice of rmx_all;
//   caller: all_to_all of rm_shadow (slice d -> shard d), reduce_scatter(sum)
//       of pull_shadow, all_gather of rmx_all's two planes every round and of
//       snap_all after a tick (RCCL on a node);
//   psim_demers_shard_ingest -- the saturating sum of the received RM planes
//       into the inboxes, the pull slice, every shard's call records (a
//       receiver checks its own targets' sends from them), the tick's pushers
//       per local receiver.
#include "psim_internal.h"
#include "philox.h"
#include "../../include/psim.h"

#include <algorithm>
#include <cstring>
#include <vector>

using namespace psim;

namespace {

#define DMCHK(h, x)                                                                         \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess)                                                               \
            return handle_fail((h), PSIM_EHIP, "%s failed: %s", #x, hipGetErrorString(e_)); \
    } while (0)

uint2 key_of(const psim_handle* h) {
    const uint64_t seed = handle_seed(h);
    return make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
}

// rumor ids and the store bit of each (anti-entropy alone reuses {Node, 0}, Q20)
void id_bits(const std::vector<uint32_t>& origin, bool rm_on, std::vector<uint32_t>& idbit, unsigned long long& full) {
    const uint32_t m = (uint32_t)origin.size();
    idbit.assign(m, 0);
    full = 0;
    for (uint32_t i = 0; i < m; i++) {
        idbit[i] = i;
        if (!rm_on)   // anti-entropy alone: next_id never increments
            for (uint32_t j = 0; j < i; j++)
                if (origin[j] == origin[i]) { idbit[i] = idbit[j]; break; }
        full |= 1ull << idbit[i];
    }
}

void reduce_stats(const unsigned long long* hs, unsigned long long* r) {
    for (int i = 0; i < kNStat; i++) r[i] = 0;
    for (int sh = 0; sh < kStatShards; sh++)
        for (int i = 0; i < kNStat; i++) {
            if (i == 6) r[i] |= hs[sh * kNStat + i];
            else r[i] += hs[sh * kNStat + i];
        }
}

void fill_stats(psim_demers_stats& o, const unsigned long long* r, uint32_t n, uint32_t m, float ms) {
    memset(&o, 0, sizeof o);
    o.rm_sent = r[1];
    o.push_sent = r[2];
    o.pull_sent = r[3];
    o.delivered_new = r[4];
    o.complete = r[5];
    const uint64_t msgs = r[1] + r[2] + r[3];
    o.algo_bytes = 2ull * n * m / 8 + r[2] * 6ull * m / 8 + 32ull * msgs;
    o.kernel_ms = ms;
}

// ---- one GPU -----------------------------------------------------------------
struct DmState : ModuleState {
    uint32_t n = 0, m = 0, ae_period = 0, rm_on = 0;   // rm_on: 0 off, 1 rumor mongering, 2 direct mail
    unsigned long long full = 0;
    unsigned long long dm_pending = 0;                 // direct-mail ids the next round delivers
    unsigned long long *seen = nullptr, *snap = nullptr, *rm[2][3] = {}, *pull[2] = {}, *rmnew[2] = {};
    uint32_t *ncall[2] = {}, *pushcnt[2] = {}, *pushlist[2] = {}, *origin = nullptr, *idbit = nullptr;
    unsigned long long *stats = nullptr, *h_stats = nullptr;
    std::vector<uint32_t> h_origin;
    uint32_t par = 0;
    uint64_t round = 0, complete = 0;
    ~DmState() override {
        void* p[] = {seen, snap, rm[0][0], rm[0][1], rm[0][2], rm[1][0], rm[1][1], rm[1][2], pull[0], pull[1], rmnew[0],
                     rmnew[1], ncall[0], ncall[1], pushcnt[0], pushcnt[1], pushlist[0], pushlist[1], origin, idbit, stats};
        for (void* x : p)
            if (x) (void)hipFree(x);
        if (h_stats) (void)hipHostFree(h_stats);
    }
};

DmState* dm_of(psim_handle* h) { return static_cast<DmState*>(handle_module(h, MOD_DEMERS)); }
const DmState* dm_of(const psim_handle* h) { return static_cast<const DmState*>(handle_module(h, MOD_DEMERS)); }

DmArgs dm_args(const psim_handle* h, const DmState& d, uint32_t par) {
    DmArgs a{};
    a.n = d.n;
    a.m = d.m;
    a.v_lo = 0;
    a.n_global = d.n;
    a.sharded = 0;
    a.key = key_of(h);
    a.push_cap = env_cap("PSIM_DM_PUSHCAP", kDmPushCap);
    a.rm_on = d.rm_on == 1u;
    a.dpc = dm_draws_per_call(d.n);
    a.full = d.full;
    a.seen = d.seen;
    a.snap = d.snap;
    a.rm_cur_any = d.rm[par][0];
    a.rm_cur_multi = d.rm[par][1];
    a.rm_cur_tri = d.rm[par][2];
    a.rm_nxt_any = d.rm[par ^ 1][0];
    a.rm_nxt_multi = d.rm[par ^ 1][1];
    a.rm_nxt_tri = d.rm[par ^ 1][2];
    a.rmnew_prev = d.rmnew[par];
    a.ncall_prev = d.ncall[par];
    a.rmnew_cur = d.rmnew[par ^ 1];
    a.ncall_cur = d.ncall[par ^ 1];
    a.pushcnt_cur = d.pushcnt[par];
    a.pushcnt_nxt = d.pushcnt[par ^ 1];
    a.pushlist_cur = d.pushlist[par];
    a.pushlist_nxt = d.pushlist[par ^ 1];
    a.pull_cur = d.pull[par];
    a.pull_nxt = d.pull[par ^ 1];
    a.stats = d.stats;
    return a;
}

int dm_drive(psim_handle* h, uint32_t max_rounds, psim_demers_stats* out, size_t cap, bool stop, uint32_t* ran_out) {
    DmState* d = dm_of(h);
    if (!d) return handle_fail(h, PSIM_ESTATE, "psim_demers_setup not called");
    const hipStream_t s = handle_stream(h);
    uint32_t ran = 0;
    while (ran < max_rounds && !(stop && d->complete == d->n)) {
        DMCHK(h, hipMemsetAsync(d->stats, 0, kStatShards * kNStat * sizeof(unsigned long long), s));
        DmArgs a = dm_args(h, *d, d->par);
        const uint64_t t = d->round + 1;   // 1-based round being run
        a.tick = d->ae_period && (t % d->ae_period) == 0;
        a.tick_idx = d->ae_period ? (uint32_t)(t / d->ae_period) : 0;
        a.prev_tick = d->ae_period ? (uint32_t)(d->round / d->ae_period) : 0;
        a.dm_mail = d->dm_pending;
        d->dm_pending = 0;
        DMCHK(h, hipEventRecord(handle_event(h, 0), s));
        DMCHK(h, launch_dm_round(a, s));
        DMCHK(h, hipEventRecord(handle_event(h, 1), s));
        DMCHK(h, hipMemcpyAsync(d->h_stats, d->stats, kStatShards * kNStat * sizeof(unsigned long long),
                                hipMemcpyDeviceToHost, s));
        DMCHK(h, hipStreamSynchronize(s));
        d->par ^= 1u;
        d->round = t;
        unsigned long long r[kNStat];
        reduce_stats(d->h_stats, r);
        float ms = 0.f;
        DMCHK(h, hipEventElapsedTime(&ms, handle_event(h, 0), handle_event(h, 1)));
        if (r[6])
            return handle_fail(h, PSIM_EOVERFLOW, "demers round %llu: > %u anti-entropy pushes to one vertex",
                               (unsigned long long)t, kDmPushCap);
        d->complete = r[5];
        handle_add_round(h, ms);
        if (out && ran < cap) fill_stats(out[ran], r, d->n, d->m, ms);
        ran++;
    }
    if (ran_out) *ran_out = ran;
    return PSIM_OK;
}

// ---- sharded -------------------------------------------------------------------
struct DmShard : ModuleState {
    uint32_t n_global = 0, m = 0, ae_period = 0, rm_on = 0, world = 1, rank = 0, chunk = 0, v_lo = 0, n = 0;
    unsigned long long full = 0;
    unsigned long long *seen = nullptr, *rm[3] = {}, *pull = nullptr, *stats = nullptr;
    // every shard's RM call records of the last round (global ids): the
    // all-gathered rmx_all planes, copied by the ingest
    unsigned long long* rmnew_prev = nullptr;
    uint32_t* ncall_prev = nullptr;
    uint32_t *pushcnt[2] = {}, *pushlist[2] = {}, *origin = nullptr, *idbit = nullptr;
    std::vector<uint32_t> h_origin;
    uint32_t par = 0;
    uint64_t round = 0;
    // the in-library exchange (psim_demers_shard_step / _run): the caller-side
    // buffers of the split-phase entry points, owned here
    unsigned long long *x_rm_shadow = nullptr, *x_rm_recv = nullptr, *x_pull_shadow = nullptr, *x_pull_all = nullptr,
                       *x_pull_sum = nullptr, *x_snap_all = nullptr, *x_rmx_all = nullptr;
    uint64_t complete_g = 0;      // vertices holding every rumor, over all shards, after the last round
    // sparse records (dms_exchange): per-destination counts, record offsets
    // (device and pinned host: [cnt G+1][send G+1][recv G+1]), cursors, buffers
    int xmode = 0;                // 0 auto, 1 dense, 2 sparse (psim_demers_shard_set_exchange)
    uint32_t *x_cnt = nullptr, *x_off = nullptr, *x_cur = nullptr, *h_x = nullptr, *x_sp_send = nullptr,
             *x_sp_recv = nullptr;
    size_t x_cap_send = 0, x_cap_recv = 0;      // words
    uint64_t x_bytes = 0;                       // bytes this shard sent to other shards
    uint32_t x_rounds = 0, x_sparse_rm = 0, x_sparse_rmx = 0;
    ~DmShard() override {
        void* p[] = {seen, rm[0], rm[1], rm[2], pull, stats, rmnew_prev, ncall_prev, pushcnt[0], pushcnt[1],
                     pushlist[0], pushlist[1], origin, idbit, x_rm_shadow, x_rm_recv, x_pull_shadow, x_pull_all,
                     x_pull_sum, x_snap_all, x_rmx_all, x_cnt, x_off, x_cur, x_sp_send, x_sp_recv};
        for (void* x : p)
            if (x) (void)hipFree(x);
        if (h_x) (void)hipHostFree(h_x);
    }
};

DmShard* dms_of(psim_handle* h) { return static_cast<DmShard*>(handle_module(h, MOD_DMSHARD)); }
const DmShard* dms_of(const psim_handle* h) { return static_cast<const DmShard*>(handle_module(h, MOD_DMSHARD)); }

// rmx_all: [world C] u64 rumors called, then [world C] u32 calls before the round
DmArgs dms_args(const psim_handle* h, const DmShard& d, void* rm_shadow, void* pull_shadow, void* snap_all,
                void* rmx_all) {
    DmArgs a{};
    a.n = d.n;
    a.m = d.m;
    a.v_lo = d.v_lo;
    a.n_global = d.n_global;
    a.sharded = 1;
    a.key = key_of(h);
    a.push_cap = env_cap("PSIM_DM_PUSHCAP", kDmPushCap);
    a.rm_on = d.rm_on;
    a.dpc = dm_draws_per_call(d.n_global);
    a.full = d.full;
    a.seen = d.seen;
    a.snap = (unsigned long long*)snap_all;
    a.rm_cur_any = d.rm[0];
    a.rm_cur_multi = d.rm[1];
    a.rm_cur_tri = d.rm[2];
    const size_t plane = (size_t)d.world * d.chunk;
    unsigned long long* rs = (unsigned long long*)rm_shadow;
    a.rm_nxt_any = rs;
    a.rm_nxt_multi = rs ? rs + plane : nullptr;
    a.rm_nxt_tri = rs ? rs + 2 * plane : nullptr;
    a.rmnew_prev = d.rmnew_prev;
    a.ncall_prev = d.ncall_prev;
    a.rmnew_cur = (unsigned long long*)rmx_all;
    a.ncall_cur = rmx_all ? reinterpret_cast<uint32_t*>((unsigned long long*)rmx_all + plane) : nullptr;
    a.pushcnt_cur = d.pushcnt[d.par];
    a.pushcnt_nxt = d.pushcnt[d.par ^ 1];
    a.pushlist_cur = d.pushlist[d.par];
    a.pushlist_nxt = d.pushlist[d.par ^ 1];
    a.pull_cur = d.pull;
    a.pull_nxt = (unsigned long long*)pull_shadow;
    a.stats = d.stats;
    return a;
}

// ---- the exchange inside the library (the handle's transport) -----------------
int dms_x_buffers(psim_handle* h, DmShard& d) {
    if (d.world > 1 && !handle_transport(h))
        return handle_fail(h, PSIM_ESTATE, "sharded Demers without a transport (psim_shard_init_rccl / _set_transport)");
    if (d.x_rm_shadow) return PSIM_OK;
    const size_t NG = size_t(d.world) * d.chunk;
    auto A = [&](unsigned long long** p, size_t words) { return alloc_zero((void**)p, std::max<size_t>(words, 1) * 8); };
    const size_t G1 = size_t(d.world) + 1;
    if (!A(&d.x_rm_shadow, 3 * NG) || !A(&d.x_rm_recv, 3 * NG) || !A(&d.x_pull_shadow, 2 * NG) ||
        !A(&d.x_pull_all, 2 * NG) || !A(&d.x_pull_sum, 2 * size_t(d.chunk)) || !A(&d.x_snap_all, NG) ||
        !A(&d.x_rmx_all, NG + (NG + 1) / 2) || !alloc_zero((void**)&d.x_cnt, G1 * 4) ||
        !alloc_zero((void**)&d.x_off, 2 * G1 * 4) || !alloc_zero((void**)&d.x_cur, G1 * 4) ||
        hipHostMalloc((void**)&d.h_x, 3 * G1 * 4, 0) != hipSuccess) {
        // all or nothing: x_rm_shadow is the "present" test of every later call
        unsigned long long** dev64[] = {&d.x_rm_shadow, &d.x_rm_recv, &d.x_pull_shadow, &d.x_pull_all,
                                        &d.x_pull_sum, &d.x_snap_all, &d.x_rmx_all};
        for (auto** p : dev64) {
            if (*p) (void)hipFree(*p);
            *p = nullptr;
        }
        uint32_t** dev32[] = {&d.x_cnt, &d.x_off, &d.x_cur};
        for (auto** p : dev32) {
            if (*p) (void)hipFree(*p);
            *p = nullptr;
        }
        d.h_x = nullptr;      // hipHostMalloc is the last allocation: it is the one that failed, if any
        return handle_fail(h, PSIM_ENOMEM, "demers exchange buffers for %zu slots", NG);
    }
    return PSIM_OK;
}

// grow a record buffer to `words` u32 (contents not kept)
int dms_grow(psim_handle* h, uint32_t** p, size_t* cap, size_t words) {
    if (words <= *cap) return PSIM_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    const size_t w = std::max<size_t>(words + words / 4, 1024);
    if (hipMalloc((void**)p, w * 4) != hipSuccess) {
        *p = nullptr;
        return handle_fail(h, PSIM_ENOMEM, "demers sparse exchange buffer of %zu words", w);
    }
    *cap = w;
    return PSIM_OK;
}

// How the round's RM planes and call records travel: counts of this shard's
// RM slots per destination and of its vertices that called select, summed
// over the shards by the transport's host all-reduce (M[s G + g]: slots shard
// s sends shard g; M[G G + s]: shard s's call records).  Records when the
// round's traffic reaches fewer than n/8 slots (or always / never, xmode).
int dms_plan(psim_handle* h, DmShard& d, std::vector<int64_t>& M, bool& sp_rm, bool& sp_x, int lrc) {
    const hipStream_t s = handle_stream(h);
    const int G = (int)d.world, r = (int)d.rank;
    sp_rm = sp_x = false;
    // [G G] slot counts, [G] call records, [kNCodes] error flags: a shard whose
    // round failed still joins this all-reduce (its peers wait in it) and every
    // shard leaves with the same code
    M.assign(size_t(G) * G + G + kNCodes, 0);
    if (!lrc && d.xmode != 1) {
        if (hipMemsetAsync(d.x_cnt, 0, (G + 1) * 4, s) != hipSuccess ||
            launch_dm_xcount(d.x_rm_shadow, d.world, d.rank, d.chunk, d.x_rmx_all + d.v_lo, d.n, d.x_cnt, s) !=
                hipSuccess ||
            hipMemcpyAsync(d.h_x, d.x_cnt, (G + 1) * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            lrc = handle_fail(h, PSIM_EHIP, "demers exchange plan: counting kernel failed");
        } else {
            for (int g = 0; g < G; g++) M[size_t(r) * G + g] = d.h_x[g];
            M[size_t(G) * G + r] = d.h_x[G];
        }
    }
    put_code(M.data() + size_t(G) * G + G, lrc);
    std::string err;
    const int rc = handle_transport(h)->allreduce(M.data(), M.size(), s, &err);
    if (rc) return handle_fail(h, rc, "demers exchange plan all-reduce: %s", err.c_str());
    const int code = finish_code(h, M.data() + size_t(G) * G + G, lrc, "demers shard round");
    if (code) return code;
    if (d.xmode == 1) return PSIM_OK;
    int64_t rm = 0, x = 0;
    for (int i = 0; i < G * G; i++) rm += M[i];
    for (int i = 0; i < G; i++) x += M[size_t(G) * G + i];
    sp_rm = d.xmode == 2 || rm * 8 < int64_t(d.n_global);
    sp_x = d.xmode == 2 || x * 8 < int64_t(d.n_global);
    return PSIM_OK;
}

// Record regions of this round's sparse forms, grown before any of them is
// exchanged: a shard that cannot grow them tells the others in one more
// all-reduce instead of leaving them in an all-to-all-v.
int dms_sparse_grow(psim_handle* h, DmShard& d, const std::vector<int64_t>& M, bool sp_rm, bool sp_x) {
    const int G = (int)d.world, r = (int)d.rank;
    uint64_t rm_s = 0, rm_r = 0, x_s = 0, x_r = 0;
    for (int g = 0; g < G; g++) {
        if (g == r) continue;
        rm_s += 7 * uint64_t(M[size_t(r) * G + g]);
        rm_r += 7 * uint64_t(M[size_t(g) * G + r]);
        x_s += 4 * uint64_t(M[size_t(G) * G + r]);
        x_r += 4 * uint64_t(M[size_t(G) * G + g]);
    }
    const uint64_t snd = std::max(sp_rm ? rm_s : 0, sp_x ? x_s : 0);
    const uint64_t rcv = std::max(sp_rm ? rm_r : 0, sp_x ? x_r : 0);
    int lrc = dms_grow(h, &d.x_sp_send, &d.x_cap_send, snd);
    if (!lrc) lrc = dms_grow(h, &d.x_sp_recv, &d.x_cap_recv, rcv);
    return agree_rc(h, handle_transport(h), lrc, "demers sparse exchange buffers");
}

// RM slots as records: pack per destination, all-to-all-v, scatter into the
// zeroed receive slices (the own slice is copied by the caller)
int dms_sparse_rm(psim_handle* h, DmShard& d, const std::vector<int64_t>& M, std::string& err) {
    const hipStream_t s = handle_stream(h);
    const int G = (int)d.world, r = (int)d.rank;
    const size_t C = d.chunk, NG = size_t(G) * C;
    std::vector<uint64_t> so(G + 1, 0), ro(G + 1, 0);
    uint32_t* hs = d.h_x + (G + 1);
    uint32_t* hr = d.h_x + 2 * (G + 1);
    for (int g = 0; g < G; g++) {
        hs[g] = (uint32_t)(so[g] / 7);
        hr[g] = (uint32_t)(ro[g] / 7);
        so[g + 1] = so[g] + 7 * uint64_t(g == r ? 0 : M[size_t(r) * G + g]);
        ro[g + 1] = ro[g] + 7 * uint64_t(g == r ? 0 : M[size_t(g) * G + r]);
    }
    hs[G] = (uint32_t)(so[G] / 7);
    hr[G] = (uint32_t)(ro[G] / 7);
    int rc = dms_grow(h, &d.x_sp_send, &d.x_cap_send, so[G]);
    if (!rc) rc = dms_grow(h, &d.x_sp_recv, &d.x_cap_recv, ro[G]);
    if (rc) return rc;
    DMCHK(h, hipMemcpyAsync(d.x_off, hs, 2 * (G + 1) * 4, hipMemcpyHostToDevice, s));
    DMCHK(h, hipMemsetAsync(d.x_cur, 0, (G + 1) * 4, s));
    DMCHK(h, launch_dm_xpack_rm(d.x_rm_shadow, d.world, d.rank, d.chunk, d.x_off, d.x_cur, d.x_sp_send, s));
    rc = handle_transport(h)->alltoallv(d.x_sp_send, so.data(), d.x_sp_recv, ro.data(), r, G, s, &err);
    if (rc) return rc;
    DMCHK(h, hipMemsetAsync(d.x_rm_recv, 0, 3 * NG * 8, s));
    DMCHK(h, launch_dm_xunpack_rm(d.x_sp_recv, d.x_off + (G + 1), d.world, d.chunk, hr[G], d.x_rm_recv, s));
    d.x_bytes += so[G] * 4;
    d.x_sparse_rm++;
    return PSIM_OK;
}

// RM call records as {vertex, rumors called, calls before} to every other
// shard; their slices of the rumors-called plane are zeroed first (a call
// count is only read where a rumor bit is set; the own slice is intact)
int dms_sparse_rmx(psim_handle* h, DmShard& d, const std::vector<int64_t>& M, std::string& err) {
    const hipStream_t s = handle_stream(h);
    const int G = (int)d.world, r = (int)d.rank;
    const size_t C = d.chunk, NG = size_t(G) * C;
    const uint32_t per = (uint32_t)M[size_t(G) * G + r];
    std::vector<uint64_t> so(G + 1, 0), ro(G + 1, 0);
    for (int g = 0; g < G; g++) {
        so[g + 1] = so[g] + (g == r ? 0 : 4 * uint64_t(per));
        ro[g + 1] = ro[g] + (g == r ? 0 : 4 * uint64_t(M[size_t(G) * G + g]));
    }
    int rc = dms_grow(h, &d.x_sp_send, &d.x_cap_send, so[G]);
    if (!rc) rc = dms_grow(h, &d.x_sp_recv, &d.x_cap_recv, ro[G]);
    if (rc) return rc;
    unsigned long long* rn = d.x_rmx_all;
    uint32_t* nc = reinterpret_cast<uint32_t*>(d.x_rmx_all + NG);
    DMCHK(h, hipMemsetAsync(d.x_cur + G, 0, 4, s));
    DMCHK(h, launch_dm_xpack_rmx(rn, nc, d.v_lo, d.n, d.world, d.rank, per, d.x_cur + G, d.x_sp_send, s));
    rc = handle_transport(h)->alltoallv(d.x_sp_send, so.data(), d.x_sp_recv, ro.data(), r, G, s, &err);
    if (rc) return rc;
    if (r > 0) DMCHK(h, hipMemsetAsync(rn, 0, size_t(r) * C * 8, s));
    if (size_t(r + 1) * C < NG) DMCHK(h, hipMemsetAsync(rn + size_t(r + 1) * C, 0, (NG - size_t(r + 1) * C) * 8, s));
    DMCHK(h, launch_dm_xunpack_rmx(d.x_sp_recv, (uint32_t)(ro[G] / 4), rn, nc, s));
    d.x_bytes += so[G] * 4;
    d.x_sparse_rmx++;
    return PSIM_OK;
}

// The round's exchange (psim.h "vertex-sharded Demers"): all-to-all of the
// three RM count planes in slices of C (or their nonzero slots as records,
// dms_plan), the pull slots as an all-to-all whose slices the receiver sums
// (one writer per slot), all-gathers of both RM call record planes (or the
// callers' records) and, after an AE tick, of the snapshots -- RCCL on the
// handle's stream, or the caller's transport; the own slices are local copies.
// Without rumor mongering the RM planes and call records stay zero and do not
// travel.
// lrc: this shard's round result -- with several shards it is agreed on in the
// round's first collective (every shard fails with the same code, none waits).
int dms_exchange(psim_handle* h, DmShard& d, bool tick, int lrc = PSIM_OK) {
    const hipStream_t s = handle_stream(h);
    const size_t C = d.chunk, NG = size_t(d.world) * C;
    const int G = (int)d.world, r = (int)d.rank;
    Transport* T = handle_transport(h);
    std::string err;
    std::vector<uint64_t> off1(G + 1), off2(G + 1);
    for (int g = 0; g <= G; g++) {
        off1[g] = uint64_t(g) * 2 * C;     // C u64 per slice
        off2[g] = uint64_t(g) * 4 * C;     // 2C u64 per slice
    }
    const uint64_t peers = uint64_t(G - 1);
    std::vector<int64_t> M;
    bool sp_rm = false, sp_x = false;
    if (G > 1 && d.rm_on) {
        int rc = dms_plan(h, d, M, sp_rm, sp_x, lrc);
        if (!rc && (sp_rm || sp_x)) rc = dms_sparse_grow(h, d, M, sp_rm, sp_x);
        if (rc) return rc;
    } else if (G > 1) {
        const int rc = agree_rc(h, T, lrc, "demers shard round");
        if (rc) return rc;
    } else if (lrc) {
        return lrc;
    }
    if (d.rm_on) {
        if (G > 1 && sp_rm) {
            const int rc = dms_sparse_rm(h, d, M, err);
            if (rc) return handle_fail(h, rc, "demers RM records: %s", err.c_str());
        }
        for (int k = 0; k < 3; k++) {
            unsigned long long* snd = d.x_rm_shadow + k * NG;
            unsigned long long* rcv = d.x_rm_recv + k * NG;
            if (G > 1 && !sp_rm) {
                const int rc = T->alltoallv(reinterpret_cast<uint32_t*>(snd), off1.data(),
                                            reinterpret_cast<uint32_t*>(rcv), off1.data(), r, G, s, &err);
                if (rc) return handle_fail(h, rc, "demers RM exchange: %s", err.c_str());
                d.x_bytes += peers * C * 8;
            }
            DMCHK(h, hipMemcpyAsync(rcv + r * C, snd + r * C, C * 8, hipMemcpyDeviceToDevice, s));
        }
    }
    if (G > 1) {
        const int rc = T->alltoallv(reinterpret_cast<uint32_t*>(d.x_pull_shadow), off2.data(),
                                    reinterpret_cast<uint32_t*>(d.x_pull_all), off2.data(), r, G, s, &err);
        if (rc) return handle_fail(h, rc, "demers pull exchange: %s", err.c_str());
        d.x_bytes += peers * C * 16;
    }
    DMCHK(h, hipMemcpyAsync(d.x_pull_all + r * 2 * C, d.x_pull_shadow + r * 2 * C, 2 * C * 8, hipMemcpyDeviceToDevice, s));
    DMCHK(h, launch_dm_sum_slices(d.x_pull_all, d.world, 2 * C, d.x_pull_sum, s));
    if (G > 1) {
        uint32_t* rmx = reinterpret_cast<uint32_t*>(d.x_rmx_all);
        int rc = 0;
        if (d.rm_on && sp_x) {
            rc = dms_sparse_rmx(h, d, M, err);
        } else if (d.rm_on) {
            rc = T->allgather(rmx, 2 * C, r, G, s, &err);                             // rumors called (u64)
            if (!rc) rc = T->allgather(rmx + 2 * NG, C, r, G, s, &err);               // calls before the round (u32)
            d.x_bytes += peers * C * 12;
        }
        if (!rc && tick) {
            rc = T->allgather(reinterpret_cast<uint32_t*>(d.x_snap_all), 2 * C, r, G, s, &err);
            d.x_bytes += peers * C * 8;
        }
        if (rc) return handle_fail(h, rc, "demers all-gather: %s", err.c_str());
    }
    DMCHK(h, hipMemsetAsync(d.x_rm_shadow, 0, 3 * NG * 8, s));
    DMCHK(h, hipMemsetAsync(d.x_pull_shadow, 0, 2 * NG * 8, s));
    d.x_rounds++;
    return PSIM_OK;
}

// per-round stats over every shard (kernel_ms stays this shard's)
int dms_global(psim_handle* h, const DmShard& d, psim_demers_stats& st) {
    if (d.world == 1) return PSIM_OK;
    int64_t v[6] = {(int64_t)st.rm_sent, (int64_t)st.push_sent, (int64_t)st.pull_sent, (int64_t)st.delivered_new,
                    (int64_t)st.complete, (int64_t)st.algo_bytes};
    std::string err;
    const int rc = handle_transport(h)->allreduce(v, 6, handle_stream(h), &err);
    if (rc) return handle_fail(h, rc, "demers stats all-reduce: %s", err.c_str());
    st.rm_sent = v[0]; st.push_sent = v[1]; st.pull_sent = v[2]; st.delivered_new = v[3];
    st.complete = v[4]; st.algo_bytes = v[5];
    return PSIM_OK;
}

}  // namespace

extern "C" {

// ---- one GPU -----------------------------------------------------------------
int psim_demers_setup(psim_handle* h, uint32_t n, uint32_t m, uint32_t ae_period, uint32_t rm_on) {
    if (!h || n < 2 || m == 0 || m > 64 || ae_period == 1 || rm_on > 2) return PSIM_EINVAL;
    DMCHK(h, hipSetDevice(handle_device(h)));
    DMCHK(h, hipStreamSynchronize(handle_stream(h)));
    ModuleState*& slot = handle_module(h, MOD_DEMERS);
    delete slot;
    slot = nullptr;
    DmState* d = new DmState();
    const size_t N = n;
    auto A = [&](void** p, size_t bytes) { return alloc_zero(p, bytes); };
    bool ok = A((void**)&d->seen, N * 8) && A((void**)&d->snap, N * 8) && A((void**)&d->origin, 64 * 4) &&
              A((void**)&d->idbit, 64 * 4) && A((void**)&d->stats, kStatShards * kNStat * 8) &&
              hipHostMalloc((void**)&d->h_stats, kStatShards * kNStat * 8) == hipSuccess;
    for (int p = 0; p < 2 && ok; p++) {
        for (int k = 0; k < 3 && ok; k++) ok = A((void**)&d->rm[p][k], N * 8);
        ok = ok && A((void**)&d->pull[p], N * 16) && A((void**)&d->pushcnt[p], N * 4) &&
             A((void**)&d->pushlist[p], N * kDmPushCap * 4);
        if (rm_on == 1) ok = ok && A((void**)&d->rmnew[p], N * 8) && A((void**)&d->ncall[p], N * 4);
    }
    if (!ok) {
        delete d;
        return handle_fail(h, PSIM_ENOMEM, "demers state for n=%u", n);
    }
    slot = d;
    d->n = n;
    d->m = m;
    d->ae_period = ae_period;
    d->rm_on = rm_on;
    DMCHK(h, launch_dm_origins(key_of(h), n, m, d->origin, handle_stream(h)));
    d->h_origin.assign(m, 0);
    DMCHK(h, hipMemcpyAsync(d->h_origin.data(), d->origin, m * 4, hipMemcpyDeviceToHost, handle_stream(h)));
    DMCHK(h, hipStreamSynchronize(handle_stream(h)));
    std::vector<uint32_t> idbit;
    id_bits(d->h_origin, d->rm_on != 0, idbit, d->full);
    DMCHK(h, hipMemcpy(d->idbit, idbit.data(), m * 4, hipMemcpyHostToDevice));
    return PSIM_OK;
}

int psim_demers_broadcast_all(psim_handle* h) {
    DmState* d = h ? dm_of(h) : nullptr;
    if (!d) return PSIM_ESTATE;
    const hipStream_t s = handle_stream(h);
    DMCHK(h, hipSetDevice(handle_device(h)));
    DMCHK(h, hipMemsetAsync(d->stats, 0, kStatShards * kNStat * 8, s));
    DmArgs a = dm_args(h, *d, d->par ^ 1u);   // writes the inbox (and call records) the next round reads
    DMCHK(h, launch_dm_broadcast(a, d->origin, d->idbit, s));
    DMCHK(h, hipStreamSynchronize(s));
    if (d->rm_on == 2u) d->dm_pending |= d->full;   // every other member receives every rumor
    return PSIM_OK;
}

int psim_demers_step(psim_handle* h, uint32_t rounds, psim_demers_stats* stats, size_t cap) {
    if (!h) return PSIM_EINVAL;
    DMCHK(h, hipSetDevice(handle_device(h)));
    return dm_drive(h, rounds, stats, cap, false, nullptr);
}

int psim_demers_run(psim_handle* h, uint32_t max_rounds, psim_demers_stats* stats, size_t cap, uint32_t* rounds_run) {
    if (!h) return PSIM_EINVAL;
    DMCHK(h, hipSetDevice(handle_device(h)));
    return dm_drive(h, max_rounds, stats, cap, true, rounds_run);
}

int psim_demers_get_seen(const psim_handle* h, uint64_t* seen, size_t n) {
    const DmState* d = h ? dm_of(h) : nullptr;
    if (!d || !seen || n != d->n || !n) return PSIM_EINVAL;
    psim_handle* hh = const_cast<psim_handle*>(h);
    DMCHK(hh, hipSetDevice(handle_device(h)));
    DMCHK(hh, hipStreamSynchronize(handle_stream(h)));
    DMCHK(hh, hipMemcpy(seen, d->seen, n * 8, hipMemcpyDeviceToHost));
    return PSIM_OK;
}

int psim_demers_origins(const psim_handle* h, uint32_t* origins, size_t m) {
    const DmState* d = h ? dm_of(h) : nullptr;
    if (!d || !origins || m != d->m || !m) return PSIM_EINVAL;
    memcpy(origins, d->h_origin.data(), m * 4);
    return PSIM_OK;
}

// ---- sharded -------------------------------------------------------------------
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
    const size_t N = std::max<uint32_t>(d->n, 1), NG = size_t(d->world) * d->chunk;
    auto A = [&](void** p, size_t bytes) { return alloc_zero(p, bytes); };
    bool ok = A((void**)&d->seen, N * 8) && A((void**)&d->pull, N * 16) && A((void**)&d->stats, kStatShards * kNStat * 8) &&
              A((void**)&d->origin, 64 * 4) && A((void**)&d->idbit, 64 * 4);
    if (d->rm_on) ok = ok && A((void**)&d->rmnew_prev, NG * 8) && A((void**)&d->ncall_prev, NG * 4);
    for (int k = 0; k < 3 && ok; k++) ok = A((void**)&d->rm[k], N * 8);
    for (int p = 0; p < 2 && ok; p++)
        ok = A((void**)&d->pushcnt[p], N * 4) && A((void**)&d->pushlist[p], N * kDmPushCap * 4);
    if (!ok) {
        const uint32_t nl = d->n;
        delete d;
        return handle_fail(h, PSIM_ENOMEM, "demers shard state for %u vertices", nl);
    }
    slot = d;
    DMCHK(h, launch_dm_origins(key_of(h), n, m, d->origin, handle_stream(h)));
    d->h_origin.assign(m, 0);
    DMCHK(h, hipMemcpyAsync(d->h_origin.data(), d->origin, m * 4, hipMemcpyDeviceToHost, handle_stream(h)));
    DMCHK(h, hipStreamSynchronize(handle_stream(h)));
    std::vector<uint32_t> idbit;
    id_bits(d->h_origin, d->rm_on != 0, idbit, d->full);
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

int psim_demers_shard_broadcast_all(psim_handle* h, void* rm_shadow, void* rmx_all) {
    if (!h || !rm_shadow || !rmx_all) return PSIM_EINVAL;
    DmShard* d = dms_of(h);
    if (!d) return handle_fail(h, PSIM_ESTATE, "psim_demers_shard_setup not called");
    const hipStream_t s = handle_stream(h);
    DMCHK(h, hipSetDevice(handle_device(h)));
    DMCHK(h, hipMemsetAsync(d->stats, 0, kStatShards * kNStat * 8, s));
    // the origins' calls are round 0's records: the caller's planes start zeroed here
    DMCHK(h, hipMemsetAsync(rmx_all, 0, size_t(d->world) * d->chunk * 12, s));
    DmArgs a = dms_args(h, *d, rm_shadow, nullptr, nullptr, rmx_all);
    DMCHK(h, launch_dm_broadcast(a, d->origin, d->idbit, s));
    DMCHK(h, hipStreamSynchronize(s));
    return PSIM_OK;
}

int psim_demers_shard_round(psim_handle* h, void* rm_shadow, void* pull_shadow, void* snap_all, void* rmx_all,
                            psim_demers_stats* st, uint32_t* tick) {
    if (!h || !rm_shadow || !pull_shadow || !snap_all || !rmx_all) return PSIM_EINVAL;
    DmShard* d = dms_of(h);
    if (!d) return handle_fail(h, PSIM_ESTATE, "psim_demers_shard_setup not called");
    const hipStream_t s = handle_stream(h);
    DMCHK(h, hipSetDevice(handle_device(h)));
    DMCHK(h, hipMemsetAsync(d->stats, 0, kStatShards * kNStat * 8, s));
    DmArgs a = dms_args(h, *d, rm_shadow, pull_shadow, snap_all, rmx_all);
    const uint64_t t = d->round + 1;
    a.tick = d->ae_period && (t % d->ae_period) == 0;
    a.tick_idx = d->ae_period ? (uint32_t)(t / d->ae_period) : 0;
    a.prev_tick = d->ae_period ? (uint32_t)(d->round / d->ae_period) : 0;
    DMCHK(h, hipEventRecord(handle_event(h, 0), s));
    DMCHK(h, launch_dm_round(a, s));
    DMCHK(h, hipEventRecord(handle_event(h, 1), s));
    std::vector<unsigned long long> hs(size_t(kStatShards) * kNStat);
    DMCHK(h, hipMemcpyAsync(hs.data(), d->stats, hs.size() * 8, hipMemcpyDeviceToHost, s));
    DMCHK(h, handle_wait(h));
    unsigned long long r[kNStat];
    reduce_stats(hs.data(), r);
    float ms = 0.f;
    DMCHK(h, hipEventElapsedTime(&ms, handle_event(h, 0), handle_event(h, 1)));
    handle_add_round(h, ms);
    d->round = t;
    if (tick) *tick = a.tick;
    if (r[6]) return handle_fail(h, PSIM_EOVERFLOW, "demers shard round %llu: > %u anti-entropy pushes to one vertex",
                                 (unsigned long long)t, kDmPushCap);
    if (st) fill_stats(*st, r, d->n, d->m, ms);
    return PSIM_OK;
}

int psim_demers_shard_ingest(psim_handle* h, const void* rm_recv, const void* pull_recv, const void* rmx_all,
                             uint32_t tick) {
    if (!h || !rm_recv || !pull_recv || !rmx_all) return PSIM_EINVAL;
    DmShard* d = dms_of(h);
    if (!d) return handle_fail(h, PSIM_ESTATE, "psim_demers_shard_setup not called");
    const hipStream_t s = handle_stream(h);
    DMCHK(h, hipSetDevice(handle_device(h)));
    DmArgs a = dms_args(h, *d, nullptr, nullptr, nullptr, nullptr);
    a.rm_nxt_any = d->rm[0];          // the inboxes the next round reads
    a.rm_nxt_multi = d->rm[1];
    a.rm_nxt_tri = d->rm[2];
    a.pull_nxt = d->pull;
    DMCHK(h, launch_dm_ingest_rm(a, (const unsigned long long*)rm_recv, (const unsigned long long*)pull_recv, d->world,
                                 d->chunk, s));
    if (d->rm_on) {                   // every shard's call records of the round: the next round's senders checks
        const size_t NG = size_t(d->world) * d->chunk;
        DMCHK(h, hipMemcpyAsync(d->rmnew_prev, rmx_all, NG * 8, hipMemcpyDeviceToDevice, s));
        DMCHK(h, hipMemcpyAsync(d->ncall_prev, (const unsigned long long*)rmx_all + NG, NG * 4, hipMemcpyDeviceToDevice,
                                s));
    }
    if (tick) DMCHK(h, launch_dm_pushscan(a, (uint32_t)(d->round / d->ae_period), s));
    DMCHK(h, hipStreamSynchronize(s));
    d->par ^= 1u;
    return PSIM_OK;
}

int psim_demers_shard_broadcast_x(psim_handle* h) {
    if (!h) return PSIM_EINVAL;
    DmShard* d = dms_of(h);
    if (!d) return handle_fail(h, PSIM_ESTATE, "psim_demers_shard_setup not called");
    const bool fresh = !d->x_rm_shadow;
    int rc = dms_x_buffers(h, *d);
    // as in psim_demers_shard_step: a shard that cannot allocate must not leave the
    // others waiting in dms_exchange's collectives
    if (fresh && d->world > 1 && handle_transport(h)) rc = agree_rc(h, handle_transport(h), rc, "demers exchange buffers");
    if (rc) return rc;
    rc = dms_exchange(h, *d, false, psim_demers_shard_broadcast_all(h, d->x_rm_shadow, d->x_rmx_all));
    if (!rc) rc = psim_demers_shard_ingest(h, d->x_rm_recv, d->x_pull_sum, d->x_rmx_all, 0);
    return rc;
}

int psim_demers_shard_step(psim_handle* h, uint32_t rounds, psim_demers_stats* stats, size_t cap) {
    if (!h) return PSIM_EINVAL;
    DmShard* d = dms_of(h);
    if (!d) return handle_fail(h, PSIM_ESTATE, "psim_demers_shard_setup not called");
    const bool fresh = !d->x_rm_shadow;
    int rc = dms_x_buffers(h, *d);
    // the first call allocates the exchange buffers: a shard that cannot must
    // not leave the others in the round's collectives
    if (fresh && d->world > 1 && handle_transport(h)) rc = agree_rc(h, handle_transport(h), rc, "demers exchange buffers");
    for (uint32_t i = 0; i < rounds && !rc; i++) {
        psim_demers_stats st;
        uint32_t tick = 0;
        memset(&st, 0, sizeof st);
        const int lrc =
            psim_demers_shard_round(h, d->x_rm_shadow, d->x_pull_shadow, d->x_snap_all, d->x_rmx_all, &st, &tick);
        rc = dms_exchange(h, *d, tick != 0, lrc);
        if (!rc) rc = psim_demers_shard_ingest(h, d->x_rm_recv, d->x_pull_sum, d->x_rmx_all, tick);
        if (!rc) rc = dms_global(h, *d, st);
        if (!rc) {
            d->complete_g = st.complete;
            if (stats && i < cap) stats[i] = st;
        }
    }
    return rc;
}

int psim_demers_shard_run(psim_handle* h, uint32_t max_rounds, psim_demers_stats* stats, size_t cap,
                          uint32_t* rounds_run) {
    if (!h) return PSIM_EINVAL;
    DmShard* d = dms_of(h);
    if (!d) return handle_fail(h, PSIM_ESTATE, "psim_demers_shard_setup not called");
    uint32_t ran = 0;
    d->complete_g = 0;
    while (ran < max_rounds) {
        psim_demers_stats st;
        const int rc = psim_demers_shard_step(h, 1, &st, 1);
        if (rc) return rc;
        if (stats && ran < cap) stats[ran] = st;
        ran++;
        if (st.complete == d->n_global) break;      // every vertex holds every rumor (global count)
    }
    if (rounds_run) *rounds_run = ran;
    return PSIM_OK;
}

int psim_demers_shard_set_exchange(psim_handle* h, int mode) {
    if (!h || mode < 0 || mode > 2) return PSIM_EINVAL;
    DmShard* d = dms_of(h);
    if (!d) return handle_fail(h, PSIM_ESTATE, "psim_demers_shard_setup not called");
    d->xmode = mode;
    return PSIM_OK;
}

int psim_demers_shard_exchange_stats(const psim_handle* h, uint64_t* bytes_sent, uint32_t* rounds,
                                     uint32_t* sparse_rm_rounds, uint32_t* sparse_call_rounds) {
    if (!h) return PSIM_EINVAL;
    const DmShard* d = dms_of(h);
    if (!d) return PSIM_ESTATE;
    if (bytes_sent) *bytes_sent = d->x_bytes;
    if (rounds) *rounds = d->x_rounds;
    if (sparse_rm_rounds) *sparse_rm_rounds = d->x_sparse_rm;
    if (sparse_call_rounds) *sparse_call_rounds = d->x_sparse_rmx;
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
