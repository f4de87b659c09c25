// psim_host.hip -- the C ABI of libpsim.so (include/psim.h): handle
// lifecycle, overlay upload, the round driver and the getters.
// Device work is in plumtree.hip; nothing here computes protocol state on
// the CPU.  There is no fallback: without a usable gfx950 device every
// entry point that needs one returns PSIM_ENODEV / PSIM_EHIP.
#include "psim_internal.h"
#include "../../include/psim.h"

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <sched.h>
#include <string>
#include <unordered_map>
#include <vector>

using namespace psim;

namespace {
constexpr int kChunk = 16;  // rounds launched between host synchronisations (no-op rounds exit early)
constexpr int kMaxLanes = 16;   // concurrent heartbeat roots (single GPU, slot-scatter engine)
constexpr size_t kStatsRow = size_t(kStatShards) * kNStat + kDelayHist;   // shards, then messages per delay
}  // namespace

// A window lane's device state (ptwin.hip; psim_internal.h WinArgs)
struct Win {
    uint4* iset = nullptr;
    psim::PdRow* rows = nullptr;
    uint2* head = nullptr;
    psim::PdMsg* msg[2] = {nullptr, nullptr};   // records read / written by a round (lane parity)
    uint32_t* nmsg = nullptr;                   // [2] record counts
    uint32_t cap = 0;
    ~Win() {
        void* p[] = {iset, rows, head, msg[0], msg[1], nmsg};
        for (void* x : p)
            if (x) (void)hipFree(x);
    }
};

struct psim_handle {
    psim_config cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;

    uint32_t n = 0;
    uint64_t E = 0;                 // ABI (CSR) peer slots of this handle's vertices
    uint64_t Ed = 0;                // device slots: E (CSR) or n * ell (ELL rows)
    uint32_t ell = 0;               // ELL row width (single GPU, max degree <= kEllMax), 0 = CSR
    std::vector<uint64_t> h_rowp;   // slot layout
    std::vector<uint32_t> h_col;
    std::vector<uint32_t> h_memb;

    uint32_t* rowp = nullptr;
    uint32_t* col = nullptr;
    uint32_t* rev = nullptr;
    uint32_t* ecol = nullptr;       // ELL rows, n < 2^29: col << 3 | reverse slot (PtArgs::ecol)
    uint32_t* memb = nullptr;
    uint32_t* alive = nullptr;
    uint4* vs = nullptr;
    uint32_t* in[2] = {nullptr, nullptr};
    uint8_t* pend[2] = {nullptr, nullptr};
    uint8_t* ost = nullptr;
    uint32_t* omit = nullptr;       // omission faults: bitmap over local sender slots (psim_set_omissions)
    // delay faults (psim_set_delays): once installed, every lane's inbox is a
    // ring of kRing buffers (ring, pring: the focused lane's) instead of in/pend
    uint8_t* dly = nullptr;         // [Ed] extra rounds per device sender slot
    uint32_t* ring = nullptr;
    uint8_t* pring = nullptr;
    uint64_t due[kRing] = {};       // messages pending per arrival round mod kRing (focused lane)
    Win* win = nullptr;             // the focused lane's window state (null: a static lane)
    // window lanes' bucketing scratch (shared: lanes run one after another)
    uint32_t *w_cnt = nullptr, *w_cur = nullptr, *w_off = nullptr, *w_idx = nullptr, *w_bsum = nullptr;
    size_t w_idx_cap = 0;
    // sharded window lanes: records split by receiver shard (ptwin.hip)
    psim::PdMsg* w_send = nullptr;
    uint32_t *w_counts = nullptr, *w_rcnt = nullptr, *w_base = nullptr, *w_cursor = nullptr;
    uint32_t w_send_cap = 0;
    // binned engine (single GPU with PSIM_CFG_BINNED): DESIGN.md 5.1
    struct Bin {
        uint2 *rec_c = nullptr, *rec_f = nullptr;
        uint32_t *cnt_c[2] = {nullptr, nullptr}, *cnt_f = nullptr, *csub = nullptr, *fslot = nullptr, *obin = nullptr;
        uint32_t fv_shift = 0, cv_shift = 0, nf = 0, nc = 0, chunks = 0;
        std::vector<uint32_t> h_csub, h_fslot;
    } bin;
    unsigned long long* stats = nullptr;     // [kChunk * kMaxLanes + 1][kStatsRow] (+1: a deferred origin's row 0)
    unsigned long long* h_stats = nullptr;   // pinned mirror
    bool origin_pend = false;                // psim_plumtree_broadcast_run: the origin's row not read back yet
    psim::PtArgs* lane_args = nullptr;       // [kChunk][kMaxLanes] per-round lane arguments (device)
    psim::PtArgs* h_lane_args = nullptr;     // pinned staging
    unsigned long long* scratch = nullptr;   // 1 counter
    int* ost_total = nullptr;                // device mirror of ost_cnt (the focused lane's)
    int* ost_total_base = nullptr;           // [kMaxLanes] allocation
    uint32_t* mcnt_base = nullptr;           // [kMaxLanes][kMcntLane]: [4][64] per-round message counts
                                             // (PtArgs::mcnt), then [4][64] worklist counts (PtArgs::wlcnt)
    // group flags + worklist (ELL, one GPU): a pend buffer is the ng flag bytes, then at wl_off the
    // [64][wl_cap] worklist shards of the same round (PtArgs::wl_cur / wl_nxt)
    size_t pend_bytes = 0, wl_off = 0;
    uint32_t wl_cap = 0;
    uint32_t wl_thr = 0;                     // 0: ng / 8 (PSIM_WL_THR test knob: list mode up to that count)
    uint32_t dense_div = 4;                  // a round after >= n / dense_div messages is flag-free (PSIM_DENSE_DIV)
    uint32_t wl_gpc = 0;                     // listed groups per ELL chunk, 0: spread (PSIM_WL_GPC A/B knob)
    // list mode: the listed groups spread over at most wl_wgs workgroups (0:
    // the whole resident grid; PSIM_WL_WGS A/B knob).  A flood's rounds 5-7
    // (1-20k listed groups) take 19 / 20 / 26 us at 128-512 against 27 / 28 /
    // 31 us over all 1,280: the busy workgroups' fixed costs (counts, flag
    // claims, counter flushes) outweigh the spread (profiles/r05/experiments/ab_wl_wgs.txt)
    uint32_t wl_wgs = 256;
    uint32_t ell_grid = 0;                   // grid of the ELL round kernel (resident workgroups)
    hipEvent_t ev[2 * kChunk] = {};
    hipEvent_t ev_done = nullptr;            // end of a chunk's work, polled (chunk_wait)

    uint32_t par = 0;          // inbox buffer the next round reads
    uint64_t round = 0;        // rounds completed (lazy-tick schedule)
    uint64_t scrub = 0;        // round at which the focused lane's inbox held no word older than it
    uint32_t serial = 0;       // heartbeat serial (device tag, low 8 bits)
    uint32_t epoch = 1;        // tree epoch (device tag, low 8 bits)
    uint32_t root = 0;
    bool have_root = false;
    std::unordered_map<uint32_t, uint32_t> mono_of;  // backend #state per origin: epoch << 24 | monotonic
    std::unordered_map<uint32_t, uint32_t> next_epoch;  // origins whose backend restarted: the new epoch
    int64_t ost_cnt = 0;       // vertices with outstanding rows
    int64_t live_rows = 0;     // outstanding rows to live peers
    uint64_t inflight = 0;     // messages emitted by the last round / origin
    double kernel_ms_total = 0;
    uint64_t rounds_total = 0;

    // Multi-root heartbeat trees: on one
    // GPU with the slot-scatter engine each heartbeat root gets a lane --
    // its own vertex states, inbox and counters; the fields above (vs, in,
    // pend, ost, ost_total, par, serial, root, have_root, ost_cnt, live_rows,
    // inflight) are the focused lane's, the others wait in `lanes`.
    struct Lane {
        uint4* vs = nullptr;
        uint32_t* in[2] = {nullptr, nullptr};
        uint8_t* pend[2] = {nullptr, nullptr};
        uint8_t* ost = nullptr;
        int* ost_total = nullptr;
        uint32_t* ring = nullptr;
        uint8_t* pring = nullptr;
        uint32_t* srg = nullptr;          // sharded + delays: the lane's staging ring (Sh::srg while focused)
        uint64_t due[kRing] = {};
        Win* win = nullptr;
        // sharded handles: the lane's GLOBAL state after the last collective
        // (every rank decides busy / window / eviction on the same values)
        int64_t g_inflight = 0, g_live = 0, g_ost = 0;
        uint32_t par = 0, serial = 0, root = 0;
        bool have_root = false;
        int64_t ost_cnt = 0, live_rows = 0;
        uint64_t inflight = 0, scrub = 0;
    };
    std::vector<Lane> lanes;
    int cur_lane = 0;

    // The forest (psim_config.max_roots > kMaxLanes): every
    // root's arrays in one slab each (lane L = root L's slice), all lanes
    // launched together every round on the handle's round clock (par, round,
    // tags); the fields above (vs, in, pend, ost, ost_total, serial, root)
    // alias the focused lane's slices, and inflight / live_rows / ost_cnt
    // are the totals over every lane.
    struct Forest {
        bool on = false;
        uint32_t cap = 0, nl = 0;                // lanes the slabs hold / lanes holding a root
        uint4* vs = nullptr;
        uint32_t* in[2] = {nullptr, nullptr};
        uint8_t* pend[2] = {nullptr, nullptr};
        uint8_t* ost = nullptr;
        int* ost_total = nullptr;                // [cap][4]
        uint32_t* mcnt = nullptr;                // [cap][kMcntLane]
        uint2* info = nullptr;                   // [cap] {Monotonic tag, local root} (device)
        uint32_t* d_list = nullptr;              // [cap] lane lists for the origin / busy / renorm kernels
        uint32_t* d_busy = nullptr;              // [cap]
        uint64_t s_in = 0, s_pend = 0, s_ost = 0;
        // sharded forest (psim_shard_init, world > 1): each lane's staged remote
        // words, every lane's dense regions in one all-to-all-v per round
        uint32_t* stage = nullptr;               // [cap][s_stage]
        uint32_t* xsend = nullptr;               // [cap * send_base[W]] region d = lane after lane
        uint32_t* xrecv = nullptr;               // [cap * recv_base[W]]
        uint64_t* sb_d = nullptr;                // [W + 1] send / recv layout bases (device)
        uint64_t* rb_d = nullptr;
        uint64_t s_stage = 0;
        int64_t g_inflight = 0, g_live = 0;      // global totals after the last collective
        // delay faults (psim_set_delays, one GPU): each lane's inbox is a ring of
        // kRing word buffers (slot stride Ed) and flag buffers (stride ng), the
        // single-lane ring layout (set_round_ring) lane after lane
        uint32_t* ring = nullptr;                // [cap][s_ring]
        uint8_t* pring = nullptr;                // [cap][s_pring]
        uint64_t s_ring = 0, s_pring = 0;
        std::vector<uint2> h_info;               // slot -> {Monotonic tag, local root}
        std::vector<uint32_t> serial;            // slot -> heartbeats so far (the root's tag source)
        std::vector<uint32_t> root_of;           // lane -> root (kNoPeer: never used)
        std::unordered_map<uint32_t, uint32_t> lane_of;   // root -> lane, while it holds one
        // Parked roots (psim_forest_set_lanes, lanes < cap): a root's records
        // live in its state slot for good (vs: cap slots of 16 n bytes), while
        // the per-lane slabs (inbox, flags, rows, counts: ~40 n bytes) exist
        // for `lanes` roots at a time; a heartbeat takes a lane from a root
        // whose own heartbeat is done.  lanes == 0: one lane per root, slot =
        // lane (no indirection).  The extra lane `lanes` stays empty: the
        // getters' view of a parked root (nothing in flight, no rows).
        uint32_t lanes = 0;
        uint32_t ns = 0;                         // slots holding a root
        uint32_t* d_slot = nullptr;              // [lanes + 1] lane -> slot (device; parking only)
        std::vector<uint32_t> h_slot;            // lane -> slot
        std::vector<uint32_t> slot_root;         // slot -> root
        std::unordered_map<uint32_t, uint32_t> slot_of;   // root -> slot
        bool parking() const { return lanes != 0 && lanes < cap; }
        uint32_t nlanes() const { return parking() ? lanes : cap; }   // lanes that run roots
        uint32_t slabs() const { return parking() ? lanes + 1 : cap; }
        uint32_t slot(uint32_t lane) const { return parking() ? h_slot[lane] : lane; }
        int focus = -1;                          // focused lane; <= -2: parked slot -2 - focus
        uint32_t gx = 0;                         // workgroups per lane (PSIM_FOREST_GX A/B knob; 0: auto)
    } fo;
    void* scratch_buf = nullptr;   // growable device scratch for batched host-buffer ops
    size_t scratch_cap = 0;

    // vertex sharding over `world` GPUs (one process each)
    struct Sh {
        int rank = 0, world = 1;
        uint32_t n_global = 0, v_lo = 0;
        uint64_t slot_base = 0;         // ABI (CSR) global slot id of local slot 0
        uint64_t dev_slot_base = 0;     // the same in device slot ids (ELL: v_lo * W)
        uint32_t* stage = nullptr;       // [E_local] staged cross-shard words
        uint32_t* srg = nullptr;         // [kRing][E_local] staging ring once delay faults are installed
        std::vector<int64_t> pend_rows;  // delays: this shard's pending messages after each collected round
        uint32_t* rem = nullptr;         // local slots whose receiver is remote, grouped by shard
        uint4* blk = nullptr;            // compaction blocks {shard, start, len, 0}
        uint32_t nblk = 0;
        uint32_t* send_base_d = nullptr; // [world] region starts (records)
        uint32_t* cursor = nullptr;      // [world] records packed per region this round
        uint32_t* slot2v = nullptr;      // [E_local] receiver vertex of a local slot
        std::vector<uint64_t> send_base; // host copy, world + 1 entries (last = total)
        // dense exchange: word i of the receive buffer feeds local slot recv_map[i];
        // the region of source s is [recv_base[s], recv_base[s+1]) in that source's slot order
        uint32_t* recv_map = nullptr;
        std::vector<uint64_t> recv_base;
        // async rounds (psim_shard_round_async): per-round stats + events ring
        unsigned long long* ring = nullptr;   // [kRing][kStatShards][kNStat]
        hipEvent_t rev_[2 * 16] = {};
        uint32_t pending = 0;
        // the exchange inside the library (psim_shard_init_rccl / _set_transport, transport.hip)
        psim::Transport* xport = nullptr;
        uint32_t *xsend = nullptr, *xrecv = nullptr;   // dense word regions (psim_shard_layout / _recv_layout)
        // sparse rounds of the in-library exchange: fixed-size record regions
        // ({receiver slot, word}, rec_k per peer, rec_k <= rec_thr) sized from a bound
        // on the words the round can send (shard_drive_fast); plan_ok: the lane's
        // global counts g_inflight / g_ost are current, so the bound holds
        uint2 *xrs = nullptr, *xrr = nullptr;
        uint8_t* xrs_raw = nullptr;            // [256 B: per-peer cursors][records]: one memset clears both
        uint32_t* xcur = nullptr;
        uint64_t rec_thr = 0;
        // shard_drive_fast under PSIM_CFG_CHUNK_TIMING: no event markers and no stats
        // memset between a chunk's kernels; one event pair per chunk (rev_[0], rev_[1])
        bool chunk_mode = false;
        // shard_drive_fast: per-round message counts on (PtArgs::mcnt) -- the
        // round kernels' no-op exit and flag-free dense rounds, fed by the
        // ingests with the words received
        bool mcnt_on = false;
        uint32_t max_deg_g = 0;
        bool plan_ok = false;
        hipEvent_t xev[2 * 16] = {};                   // exchange start / end per pending round
    } sh;
    hipStream_t own_stream = nullptr;         // the handle's stream (psim_set_stream may override `stream`)
    hipStream_t cstream = nullptr;            // psim_plumtree_broadcast_run_n: read-back copies beside the rounds



    psim::ModuleState* mods[psim::MOD_COUNT] = {};   // fullmem / scamp host state

};

namespace {

thread_local std::string g_create_err;   // detail of the last failed psim_create on this thread

int fail(psim_handle* h, int code, const char* fmt, ...) {
    if (h) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        h->err = buf;
    }
    return code;
}

#define HIPCHK(h, x)                                                                     \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess)                                                            \
            return fail((h), PSIM_EHIP, "%s failed: %s", #x, hipGetErrorString(e_));     \
    } while (0)

void swap_lane(psim_handle* h, int j);
void save_lane(psim_handle* h);
void load_lane(psim_handle* h, int j);
int forest_renorm_all(psim_handle* h);
int forest_alloc(psim_handle* h);

void free_forest(psim_handle* h) {
    auto& f = h->fo;
    if (!f.on) return;
    // the handle's single-lane pointers alias the focused lane's slices
    h->vs = nullptr;
    h->in[0] = h->in[1] = nullptr;
    h->pend[0] = h->pend[1] = nullptr;
    h->ost = nullptr;
    h->ost_total = h->ost_total_base;
    void* fp[] = {f.vs, f.in[0], f.in[1], f.pend[0], f.pend[1], f.ost, f.ost_total, f.mcnt, f.info, f.d_list, f.d_busy,
                  f.stage, f.xsend, f.xrecv, f.sb_d, f.rb_d, f.ring, f.pring, f.d_slot};
    for (void* x : fp)
        if (x) (void)hipFree(x);
    f.stage = f.xsend = f.xrecv = nullptr;
    f.sb_d = f.rb_d = nullptr;
    f.ring = nullptr;
    f.pring = nullptr;
    h->ring = nullptr;                          // aliased the focused lane's ring
    h->pring = nullptr;
    f.vs = nullptr;
    f.in[0] = f.in[1] = nullptr;
    f.pend[0] = f.pend[1] = nullptr;
    f.ost = nullptr;
    f.ost_total = nullptr;
    f.mcnt = nullptr;
    f.info = nullptr;
    f.d_list = f.d_busy = nullptr;
    f.d_slot = nullptr;
    f.nl = 0;
    f.ns = 0;
    f.h_info.clear();
    f.root_of.clear();
    f.lane_of.clear();
    f.h_slot.clear();
    f.slot_root.clear();
    f.slot_of.clear();
    f.focus = -1;
}

void free_graph(psim_handle* h) {
    free_forest(h);
    if (!h->lanes.empty()) {
        swap_lane(h, 0);
        for (size_t j = 1; j < h->lanes.size(); j++) {
            auto& l = h->lanes[j];
            void* lp[] = {l.vs, l.in[0], l.in[1], l.pend[0], l.pend[1], l.ost, l.ring, l.pring, l.srg};
            for (void* p : lp)
                if (p) (void)hipFree(p);
            delete l.win;
        }
        h->lanes.clear();
        h->cur_lane = 0;
    }
    void* ptrs[] = {h->rowp, h->col, h->rev, h->ecol, h->memb, h->alive, h->vs, h->in[0], h->in[1],
                    h->pend[0], h->pend[1], h->ost, h->dly, h->ring, h->pring};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    h->rowp = h->col = h->rev = h->ecol = h->memb = h->alive = nullptr;
    h->vs = nullptr;
    h->in[0] = h->in[1] = nullptr;
    h->pend[0] = h->pend[1] = h->ost = nullptr;
    h->dly = h->pring = nullptr;
    h->ring = nullptr;
    delete h->win;
    h->win = nullptr;
    {
        void* wp[] = {h->w_cnt, h->w_cur, h->w_off, h->w_idx, h->w_bsum, h->w_send, h->w_counts, h->w_rcnt,
                      h->w_base, h->w_cursor};
        for (void* p : wp)
            if (p) (void)hipFree(p);
        h->w_cnt = h->w_cur = h->w_off = h->w_idx = h->w_bsum = nullptr;
        h->w_counts = h->w_rcnt = h->w_base = h->w_cursor = nullptr;
        h->w_send = nullptr;
        h->w_idx_cap = 0;
        h->w_send_cap = 0;
    }
    for (auto& x : h->due) x = 0;
    if (h->omit) (void)hipFree(h->omit);
    h->omit = nullptr;
    {
        auto& b = h->bin;
        void* bp[] = {b.rec_c, b.rec_f, b.cnt_c[0], b.cnt_c[1], b.cnt_f, b.csub, b.fslot, b.obin};
        for (void* p : bp)
            if (p) (void)hipFree(p);
        b = psim_handle::Bin();
    }
    auto& sh = h->sh;
    void* sp[] = {sh.stage, sh.rem, sh.blk, sh.send_base_d, sh.cursor, sh.slot2v, sh.recv_map, sh.xsend, sh.xrecv,
                  sh.xrs_raw, sh.xrr, sh.srg};
    for (void* p : sp)
        if (p) (void)hipFree(p);
    sh.stage = sh.rem = sh.send_base_d = sh.cursor = sh.slot2v = sh.recv_map = sh.xsend = sh.xrecv = sh.srg = nullptr;
    sh.xrs = sh.xrr = nullptr;
    sh.xrs_raw = nullptr;
    sh.xcur = nullptr;
    sh.plan_ok = false;
    sh.recv_base.clear();
    sh.pending = 0;
    sh.blk = nullptr;
    sh.nblk = 0;
    sh.send_base.clear();
    h->n = 0;
    h->E = 0;
    h->Ed = 0;
    h->ell = 0;
}

// Delay ring (psim_set_delays): the arguments of round R read ring slot
// R mod kRing (tag R) and write the words of round R + 1 + d to slot
// (R + 1 + d) mod kRing with tag R + 1 + d.
void set_round_ring(const psim_handle* h, PtArgs& a, uint64_t R) {
    const size_t ng = (size_t(h->n) + (1u << kGroupShift) - 1) >> kGroupShift;
    a.dly = h->dly;
    a.ring = h->ring;
    a.pring = h->pring;
    a.ed = (uint32_t)h->Ed;
    a.ngrp = (uint32_t)ng;
    a.rpos = uint32_t(R + 1) & (kRing - 1);
    a.in_cur = h->ring + size_t(R & (kRing - 1)) * h->Ed;
    a.in_nxt = h->ring + size_t(a.rpos) * h->Ed;
    a.pend_cur = h->pring + size_t(R & (kRing - 1)) * ng;
    a.pend_nxt = h->pring + size_t(a.rpos) * ng;
    a.ctag = uint32_t(R) & 0xFFu;
    a.wtag = uint32_t(R + 1) & 0xFFu;
    if (h->sh.srg) {            // sharded: the words the exchange after round R carries
        a.srg = h->sh.srg;
        a.stage = h->sh.srg + size_t(R & (kRing - 1)) * h->Ed;
    }
}

PtArgs make_args(const psim_handle* h, uint32_t par, uint32_t tick, unsigned long long* stats) {
    PtArgs a{};
    a.n = h->n;
    a.v_lo = h->sh.v_lo;
    a.slot_base = (uint32_t)h->sh.dev_slot_base;
    a.abi_slot_base = (uint32_t)h->sh.slot_base;
    a.stage = h->sh.stage;
    a.rowp = h->rowp;
    a.col = h->col;
    a.rev = h->rev;
    a.ecol = h->ecol;
    a.memb = h->memb;
    a.alive = h->alive;
    a.vs = h->vs;
    a.in_cur = h->in[par];
    a.in_nxt = h->in[par ^ 1];
    a.pend_cur = h->pend[par];
    a.pend_nxt = h->pend[par ^ 1];
    a.ost = h->ost;
    a.ost_total = h->ost_total;
    a.stats = stats;
    a.tick = tick;
    a.ctag = uint32_t(h->round + 1) & 0xFFu;   // the next round to run reads these words ...
    a.wtag = uint32_t(h->round + 2) & 0xFFu;   // ... and writes words for the one after it
    a.mono8 = h->serial & 0xFFu;
    a.epoch8 = h->epoch & 0xFFu;
    a.root = h->root;
    a.omit = h->omit;
    a.ell = h->ell;
    a.ell_grid = h->ell_grid;
    if (h->dly) {
        // delay ring: `par` names the round as in[] does -- h->par reads the
        // next round's words, h->par ^ 1 writes them (the origin)
        set_round_ring(h, a, par == h->par ? h->round + 1 : h->round);
        a.dhist = stats + size_t(kStatShards) * kNStat;
    }
    if (h->bin.rec_c) {
        const auto& b = h->bin;
        a.rec_c = b.rec_c;
        a.rec_f = b.rec_f;
        a.cnt_c_cur = b.cnt_c[par];
        a.cnt_c_nxt = b.cnt_c[par ^ 1];
        a.cnt_f = b.cnt_f;
        a.csub = b.csub;
        a.fslot = b.fslot;
        a.obin = b.obin;
        a.fv_shift = b.fv_shift;
        a.cv_shift = b.cv_shift;
        a.nf = b.nf;
        a.nc = b.nc;
        a.chunks = b.chunks;
    }
    return a;
}

// ---- window lanes (ptwin.hip) ----------------------------------------------
uint32_t cur_mono(const psim_handle* h) {
    const auto it = h->mono_of.find(h->root);
    return h->have_root && it != h->mono_of.end() ? it->second : 0u;
}

// Arguments of the focused window lane for the round reading records[par].
WinArgs make_win_args(const psim_handle* h, uint32_t par, uint32_t tick, unsigned long long* stats) {
    WinArgs a{};
    a.n = h->n;
    a.v_lo = h->sh.v_lo;
    a.ell = h->ell;
    a.mono = cur_mono(h);
    a.mono8 = h->serial & 0xFFu;
    a.epoch8 = h->epoch & 0xFFu;
    a.tick = tick;
    a.rowp = h->rowp;
    a.col = h->col;
    a.memb = h->memb;
    a.alive = h->alive;
    a.omit = h->omit;
    a.vs = h->vs;
    a.iset = h->win->iset;
    a.rows = h->win->rows;
    a.head = h->win->head;
    a.ost = h->ost;
    a.in = h->win->msg[par];
    a.nin = h->win->nmsg + par;
    a.off = h->w_off;
    a.idx = h->w_idx;
    a.out = h->win->msg[par ^ 1];
    a.nout = h->win->nmsg + (par ^ 1);
    a.cap = h->win->cap;
    a.stats = stats;
    return a;
}

// Window lanes need the per-message machinery of the single-GPU static
// engine (not the binned one; delay faults keep their own ring).
bool lanes_enabled(const psim_handle* h);
bool win_capable(const psim_handle* h) { return lanes_enabled(h) && !h->dly; }

// The focused static lane becomes a window lane (its root heartbeats again
// while a heartbeat is in flight).  Nothing is lost: ptwin.hip
// win_convert_kernel restates the lane's state and in-flight words.
int to_window(psim_handle* h) {
    const size_t n = h->n;
    const uint32_t cap = (uint32_t)std::min<uint64_t>(4ull * h->Ed + 4096, 0xF0000000ull);
    const size_t nb = (n + kBlock - 1) / kBlock;
    if (!h->w_cnt) {
        if (!alloc_zero((void**)&h->w_cnt, n * 4) || !alloc_zero((void**)&h->w_cur, n * 4) ||
            !alloc_zero((void**)&h->w_off, (n + 1) * 4) || !alloc_zero((void**)&h->w_bsum, nb * 4))
            return fail(h, PSIM_ENOMEM, "window lane scratch for n=%zu", n);
    }
    if (h->w_idx_cap < cap) {
        if (h->w_idx) (void)hipFree(h->w_idx);
        h->w_idx = nullptr;
        h->w_idx_cap = 0;
        if (!alloc_zero((void**)&h->w_idx, size_t(cap) * 4)) return fail(h, PSIM_ENOMEM, "window lane scratch");
        h->w_idx_cap = cap;
    }
    Win* w = new Win();
    w->cap = cap;
    if (!alloc_zero((void**)&w->iset, n * 2 * sizeof(uint4)) || !alloc_zero((void**)&w->rows, n * kWinRows * sizeof(PdRow)) ||
        !alloc_zero((void**)&w->head, n * sizeof(uint2)) || !alloc_zero((void**)&w->msg[0], size_t(cap) * sizeof(PdMsg)) ||
        !alloc_zero((void**)&w->msg[1], size_t(cap) * sizeof(PdMsg)) || !alloc_zero((void**)&w->nmsg, 16)) {
        delete w;
        return fail(h, PSIM_ENOMEM, "window lane of root %u (n=%zu)", h->root, n);
    }
    h->win = w;
    h->lanes[h->cur_lane].win = w;
    WinArgs a = make_win_args(h, h->par, 0, h->stats);
    a.out = w->msg[h->par];            // the words the next round reads become its records
    a.nout = w->nmsg + h->par;
    const PtArgs pa = make_args(h, h->par, 0, h->stats);
    HIPCHK(h, launch_win_convert(a, pa, h->stream));
    uint32_t cnt = 0;
    HIPCHK(h, hipMemcpyAsync(&cnt, w->nmsg + h->par, 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (cnt > cap) return fail(h, PSIM_EOVERFLOW, "window lane: %u in-flight messages > %u", cnt, cap);
    h->inflight = cnt;
    return PSIM_OK;
}

// Per-round message counts (psim_step / psim_run on one GPU with the
// slot-scatter engine; lane-local): round R adds its messages into slot R mod
// 4 (64 shards), reads the counts of rounds R-1 and R-2 -- none sent -> the
// round is a no-op; many sent -> the flag-free mode below -- and zeroes slot
// R+1 mod 4.  A broadcast zeroes all four (psim_handle_broadcast), so the
// rounds that read them were run back to back.
// Flag-free rounds: a round that follows >= n/4 messages expects most
// 16-vertex groups to receive words, so its senders write no group flags and
// the next round reads every group's words with its coalesced sweep (the
// same decision, taken from the same count, on both sides).
// Message count under which a round lists the groups it flags (0: no list).
// Several shards need it below the flag-free count (n / 4): psim_shard_run
// seeds its first round's predecessor-but-one with it (flag mode, no list).
uint32_t list_threshold(const psim_handle* h) {
    if (!h->wl_cap) return 0;
    // n / 128 messages (ng / 8 of 16-vertex groups), whatever the group size
    return h->wl_thr ? h->wl_thr : std::max<uint32_t>(1u, h->n / 128);
}

void set_round_slots(const psim_handle* h, PtArgs& a, uint64_t R) {
    // delays: a silent round may precede arrivals; sharded handles: only
    // psim_shard_run's rounds keep the counts (sh.mcnt_on: ingests add the
    // words received to them)
    if ((h->sh.world != 1 && !h->sh.mcnt_on) || h->bin.rec_c || h->dly) return;
    a.mcnt = h->mcnt_base + kMcntLane * size_t(h->cur_lane);
    a.m_w = uint32_t(R % 4);
    a.m_s = uint32_t((R + 3) % 4);
    a.m_r = uint32_t((R + 2) % 4);
    a.m_z = uint32_t((R + 1) % 4);
    a.dense = std::max<uint32_t>(1u, h->n / h->dense_div);
    const uint32_t thr = list_threshold(h);
    if (thr) {                // sparse rounds: the groups written are listed
        a.wlcnt = a.mcnt + 256;
        a.wl_cur = reinterpret_cast<uint32_t*>(a.pend_cur + h->wl_off);
        a.wl_nxt = reinterpret_cast<uint32_t*>(a.pend_nxt + h->wl_off);
        a.wl_cap = h->wl_cap;
        a.wl_thr = thr;
        a.wl_gpc = h->wl_gpc;
        a.wl_wgs = h->wl_wgs;
    }
}

// The row-holder ring of the focused lane (psim_internal.h kMcntHold): before
// round R runs with counts, holders(R-2) := the host's count and
// delta(R-1) := 0, so R's "row due" test starts from the exact count whatever
// ran before (rounds without counts, rewound rounds, a broadcast's memset).
// Host-side ost_cnt is exact whenever no round is pending.
hipError_t seed_hold_ring(psim_handle* h, uint64_t R) {
    PtArgs a = make_args(h, h->par, 0, h->stats);
    set_round_slots(h, a, R);
    if (!a.mcnt) return hipSuccess;
    const hipError_t e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(a.mcnt + kMcntHold + a.m_r),
                                           int(uint32_t(h->ost_cnt)), 1, h->stream);
    if (e != hipSuccess) return e;
    return hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(a.mcnt + kMcntHoldD + a.m_s), 0, 1, h->stream);
}

// ... for every lane (a driver call that may run any of them)
hipError_t seed_hold_rings(psim_handle* h, uint64_t R) {
    if (h->lanes.empty()) return seed_hold_ring(h, R);
    const int focus = h->cur_lane;
    save_lane(h);
    hipError_t e = hipSuccess;
    for (int j = 0; j < (int)h->lanes.size() && e == hipSuccess; j++) {
        load_lane(h, j);
        e = seed_hold_ring(h, R);
    }
    load_lane(h, focus);
    return e;
}

// seed_hold_rings as (address, value) pairs for pt_prep_kernel, every lane
// but `skip` (a lane whose origin kernel seeded it for this round already)
void prep_seeds(psim_handle* h, uint64_t R, PtPrep& p, int skip) {
    static_assert(kMaxLanes <= (int)kMaxPrep, "one seed per lane");
    auto one = [&]() {
        PtArgs a = make_args(h, h->par, 0, h->stats);
        set_round_slots(h, a, R);
        if (!a.mcnt) return;
        p.hold[p.k] = a.mcnt + kMcntHold + a.m_r;
        p.holdd[p.k] = a.mcnt + kMcntHoldD + a.m_s;
        p.hv[p.k] = uint32_t(h->ost_cnt);
        p.k++;
    };
    if (h->lanes.empty()) {
        if (skip < 0) one();
        return;
    }
    const int focus = h->cur_lane;
    save_lane(h);
    for (int j = 0; j < (int)h->lanes.size(); j++) {
        if (j == skip) continue;
        load_lane(h, j);
        one();
    }
    load_lane(h, focus);
}

// Round tags (psim_internal.h): a slot-scatter inbox word carries the round
// that reads it, mod 256, and consumed words stay in place.  Before a lane
// runs round `last`, every word older than 256 rounds must be gone, or its
// tag could alias: zero every word not tagged for the next round (both
// buffers; the in-flight words of round h->round + 1 are kept).
void set_round_tags(PtArgs& a, uint64_t R) {
    a.ctag = uint32_t(R) & 0xFFu;
    a.wtag = uint32_t(R + 1) & 0xFFu;
}

// A scrub at round S keeps the words tagged for the `span` rounds in flight
// (S+1 .. S+span; span 1 for the double buffer, kRing - 1 for the delay ring)
// and zeroes the rest.  A stale word written for round R' aliases round
// R' + 256, so the scrub must run while no stale word can carry a kept tag:
// before round S_prev + 256 - span + 1, i.e. when last + span reaches
// S_prev + 255.  (Until round 3 the test was last > S + 256: a one-round
// psim_step at exactly S + 256 kept the stale words of round S + 1 as live --
// found when the word format was shortened to a 64-round tag)
hipError_t scrub_if_needed(psim_handle* h, uint64_t last) {
    const uint64_t span = h->dly ? kRing - 1 : 1;
    if (h->bin.rec_c || last + span < h->scrub + kTagSpan) return hipSuccess;
    const uint32_t keep = uint32_t(h->round + 1) & 0xFFu;
    if (h->dly) {       // the ring: words for the next kRing - 1 rounds are in flight
        const hipError_t e = launch_pt_scrub(h->ring, kRing * h->Ed, keep, kRing - 1, h->stream);
        if (e != hipSuccess) return e;
    }
    for (int b = 0; b < 2 && !h->dly; b++) {
        const hipError_t e = launch_pt_scrub(h->in[b], h->Ed, keep, 1, h->stream);
        if (e != hipSuccess) return e;
    }
    h->scrub = h->round;
    return hipSuccess;
}

// ---- heartbeat-root lanes ------------------------------------------------
void save_lane(psim_handle* h) {
    if (h->lanes.empty()) return;              // a forest keeps its lanes in slabs
    auto& l = h->lanes[h->cur_lane];
    l.vs = h->vs; l.in[0] = h->in[0]; l.in[1] = h->in[1]; l.pend[0] = h->pend[0]; l.pend[1] = h->pend[1];
    l.ost = h->ost; l.ost_total = h->ost_total; l.par = h->par; l.serial = h->serial; l.root = h->root;
    l.have_root = h->have_root; l.ost_cnt = h->ost_cnt; l.live_rows = h->live_rows; l.inflight = h->inflight;
    l.scrub = h->scrub;
    l.ring = h->ring; l.pring = h->pring; l.srg = h->sh.srg;
    memcpy(l.due, h->due, sizeof l.due);
    l.win = h->win;
}
void load_lane(psim_handle* h, int j) {
    const auto& l = h->lanes[j];
    h->vs = l.vs; h->in[0] = l.in[0]; h->in[1] = l.in[1]; h->pend[0] = l.pend[0]; h->pend[1] = l.pend[1];
    h->ost = l.ost; h->ost_total = l.ost_total; h->par = l.par; h->serial = l.serial; h->root = l.root;
    h->have_root = l.have_root; h->ost_cnt = l.ost_cnt; h->live_rows = l.live_rows; h->inflight = l.inflight;
    h->scrub = l.scrub;
    h->ring = l.ring; h->pring = l.pring; h->sh.srg = l.srg;
    memcpy(h->due, l.due, sizeof h->due);
    h->win = l.win;
    h->cur_lane = j;
}
void swap_lane(psim_handle* h, int j) {
    if (h->lanes.empty() || j == h->cur_lane) return;
    save_lane(h);
    load_lane(h, j);
}
// Heartbeat lanes: one GPU with the slot-scatter engine, or a sharded
// handle whose exchange is in the library (psim_shard_broadcast_x /
// psim_shard_run / psim_shard_step); the split-phase sharded entry points
// keep one lane.
bool lanes_enabled(const psim_handle* h) { return !h->bin.rec_c && (h->sh.world == 1 || h->sh.xport); }
bool lane_quiescent(const psim_handle* h, const psim_handle::Lane& l) {
    if (h->sh.world > 1) return l.g_inflight == 0 && l.g_live == 0;
    return l.inflight == 0 && l.live_rows == 0;
}

// Binned engine geometry: fine bins of 2^fv vertices whose slots fit the LDS
// inbox, coarse bins of 2^cv vertices with about sqrt(#fine) fine bins each.
bool bin_geometry(const std::vector<uint32_t>& rp, uint32_t n, uint32_t& fv, uint32_t& cv, uint32_t& nf,
                  uint32_t& nc) {
    fv = 0;
    while ((1u << (fv + 1)) <= kBinVMax) fv++;
    for (;; fv--) {
        uint32_t mx = 0;
        for (uint64_t v = 0; v < n; v += (1u << fv)) {
            const uint64_t e = std::min<uint64_t>(n, v + (1u << fv));
            mx = std::max(mx, rp[e] - rp[v]);
        }
        if (mx <= kBinSlots) break;
        if (fv == 0) return false;
    }
    nf = uint32_t((uint64_t(n) + (1u << fv) - 1) >> fv);
    uint32_t g = 0;                                   // fine bins per coarse bin = 2^g ~ sqrt(nf)
    while ((1ull << (2 * g)) < nf) g++;
    while (g > 0 && (1u << g) > kCoarseMax) g--;
    while (((uint64_t(nf) + (1u << g) - 1) >> g) > kCoarseMax) g++;
    if ((1u << g) > kCoarseMax) return false;
    cv = fv + g;
    nc = uint32_t((uint64_t(nf) + (1u << g) - 1) >> g);
    return true;
}

void reduce_row(const unsigned long long* row, unsigned long long* out) {
    for (int i = 0; i < kNStat; i++) out[i] = 0;
    for (int s = 0; s < kStatShards; s++)
        for (int i = 0; i < kNStat; i++) {
            if (i == S_OVERFLOW) out[i] |= row[s * kNStat + i];
            else out[i] += row[s * kNStat + i];
        }
}

bool quiescent(const psim_handle* h) {
    if (h->sh.world > 1 && !h->lanes.empty()) return lane_quiescent(h, h->lanes[h->cur_lane]);
    return h->inflight == 0 && h->live_rows == 0;
}
// vertices holding rows (all shards)
int64_t rows_held(const psim_handle* h) {
    if (h->sh.world > 1 && !h->lanes.empty()) return h->lanes[h->cur_lane].g_ost;
    return h->ost_cnt;
}

int renorm_if_needed(psim_handle* h) {
    if (h->fo.on) return forest_renorm_all(h);
    const int focus = h->cur_lane;
    for (int j = 0; j < (int)h->lanes.size(); j++) {   // every lane's tags
        swap_lane(h, j);
        PtArgs a = make_args(h, h->par, 0, h->stats);
        HIPCHK(h, launch_pt_renorm(a, h->stream));
    }
    swap_lane(h, focus);
    return PSIM_OK;
}

// A lane's delay ring: kRing inbox buffers and group-flag buffers, zeroed.
int alloc_ring(psim_handle* h, uint32_t*& ring, uint8_t*& pring) {
    const size_t ng = (size_t(h->n) + (1u << kGroupShift) - 1) >> kGroupShift;
    ring = nullptr;
    pring = nullptr;
    if (hipMalloc((void**)&ring, kRing * h->Ed * 4) != hipSuccess || hipMalloc((void**)&pring, kRing * ng) != hipSuccess ||
        hipMemset(ring, 0, kRing * h->Ed * 4) != hipSuccess || hipMemset(pring, 0, kRing * ng) != hipSuccess) {
        if (ring) (void)hipFree(ring);
        if (pring) (void)hipFree(pring);
        ring = nullptr;
        pring = nullptr;
        return PSIM_ENOMEM;
    }
    return PSIM_OK;
}

// Messages of the round (or origin) `R` written per delay: pending until
// round R + 1 + d; the lane's in-flight count is what is still pending.
uint64_t add_due(uint64_t* due, uint64_t R, const unsigned long long* hist) {
    for (uint32_t d = 0; d < kRing; d++) due[(R + 1 + d) & (kRing - 1)] += hist[d];
    uint64_t s = 0;
    for (uint32_t k = 0; k < kRing; k++) s += due[k];
    return s;
}

// Focus the lane of heartbeat root `root`; with `create`, give a new root a
// lane while fewer than kMaxLanes hold a root.  A lane keeps its root's
// per-root eager / lazy sets and the backend's timestamps for that origin
// (partisan_plumtree_broadcast.erl:1240-1248, 1278-1282; backend :400-417)
// for the life of the handle: a 17th root is PSIM_ENOSPC -- reusing a
// quiescent lane would silently forget those sets.  Handles
// created with psim_config.max_roots > 16 keep every root in the forest
// (forest.hip) instead.
int focus_root(psim_handle* h, uint32_t root, bool create) {
    save_lane(h);
    auto& L = h->lanes;
    int pick = -1;
    for (int j = 0; j < (int)L.size() && pick < 0; j++)
        if (L[j].have_root && L[j].root == root) pick = j;
    if (pick < 0 && !create) return fail(h, PSIM_EINVAL, "root %u has no heartbeat lane", root);
    for (int j = 0; j < (int)L.size() && pick < 0; j++)
        if (!L[j].have_root) pick = j;
    bool fresh = false;
    if (pick < 0 && (int)L.size() < kMaxLanes) {
        psim_handle::Lane l;
        if (hipMalloc((void**)&l.vs, size_t(h->n) * 16) != hipSuccess ||
            hipMalloc((void**)&l.in[0], h->Ed * 4) != hipSuccess || hipMalloc((void**)&l.in[1], h->Ed * 4) != hipSuccess ||
            hipMalloc((void**)&l.pend[0], h->pend_bytes) != hipSuccess ||
            hipMalloc((void**)&l.pend[1], h->pend_bytes) != hipSuccess ||
            hipMalloc((void**)&l.ost, size_t(h->n) + 4) != hipSuccess) {
            void* lp[] = {l.vs, l.in[0], l.in[1], l.pend[0], l.pend[1], l.ost};
            for (void* p : lp)
                if (p) (void)hipFree(p);
            return fail(h, PSIM_ENOMEM, "heartbeat lane %zu for n=%u", L.size(), h->n);
        }
        if (h->dly && (alloc_ring(h, l.ring, l.pring) != PSIM_OK ||
                       (h->sh.world > 1 && !alloc_zero((void**)&l.srg, size_t(kRing) * h->Ed * 4)))) {
            void* lp[] = {l.vs, l.in[0], l.in[1], l.pend[0], l.pend[1], l.ost, l.ring, l.pring};
            for (void* p : lp)
                if (p) (void)hipFree(p);
            return fail(h, PSIM_ENOMEM, "delay ring of heartbeat lane %zu", L.size());
        }
        l.ost_total = h->ost_total_base + 4 * L.size();     // the lane's ost_total (stride 4 ints)
        L.push_back(l);
        pick = (int)L.size() - 1;
        fresh = true;
    }
    if (pick < 0)
        return fail(h, PSIM_ENOSPC, "root %u: all %d heartbeat lanes hold a root's trees (psim_config.max_roots "
                                    "keeps more)", root, kMaxLanes);
    if (fresh) {                                    // start_link/0 state for this lane
        auto& l = L[pick];
        const size_t ng = (size_t(h->n) + (1u << kGroupShift) - 1) >> kGroupShift;
        HIPCHK(h, hipMemsetAsync(l.vs, 0, size_t(h->n) * 16, h->stream));
        HIPCHK(h, hipMemsetAsync(l.in[0], 0, h->Ed * 4, h->stream));
        HIPCHK(h, hipMemsetAsync(l.in[1], 0, h->Ed * 4, h->stream));
        HIPCHK(h, hipMemsetAsync(l.pend[0], 0, ng, h->stream));
        HIPCHK(h, hipMemsetAsync(l.pend[1], 0, ng, h->stream));
        HIPCHK(h, hipMemsetAsync(l.ost, 0, size_t(h->n) + 4, h->stream));
        HIPCHK(h, hipMemsetAsync(l.ost_total, 0, 4 * sizeof(int), h->stream));
        if (l.ring) {
            HIPCHK(h, hipMemsetAsync(l.ring, 0, kRing * h->Ed * 4, h->stream));
            HIPCHK(h, hipMemsetAsync(l.pring, 0, kRing * ng, h->stream));
        }
        for (auto& x : l.due) x = 0;
        delete l.win;                               // a reused window lane starts static again
        l.win = nullptr;
        l.g_inflight = l.g_live = l.g_ost = 0;
        l.par = 0;
        l.serial = 0;
        l.have_root = false;
        l.ost_cnt = l.live_rows = 0;
        l.inflight = 0;
        l.scrub = h->round;
        load_lane(h, pick);
        PtArgs a = make_args(h, h->par, 0, h->stats);   // tags that match no serial / epoch
        HIPCHK(h, launch_pt_renorm(a, h->stream));
    } else {
        load_lane(h, pick);
    }
    return PSIM_OK;
}

// Launch up to max_rounds rounds in chunks; with stop_q, stop after the first
// round that leaves the system quiescent (trailing rounds of the chunk were
// no-ops and are not counted: they change no state).
// The end of a chunk's work, by polling an event instead of a blocking
// stream synchronisation: the host learns of it within a microsecond or so,
// where the blocking wait's wake-up was part of the idle time between two
// heartbeat intervals on the device.
// The poll spins for at most kSpinUs of wall time (a heartbeat interval's chunk
// is 0.1-3 ms: the spin covers the bench's waits), then yields the core between
// polls, so a long run -- or a NIF call on a dirty scheduler -- does not pin a
// core for its whole length.
hipError_t event_wait(hipEvent_t ev) {
    constexpr long kSpinUs = 5000;
    hipError_t e;
    timespec t0;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (uint32_t i = 0; (e = hipEventQuery(ev)) == hipErrorNotReady; i++) {
        if ((i & 63) != 63) continue;
        timespec t;
        clock_gettime(CLOCK_MONOTONIC, &t);
        const long us = (t.tv_sec - t0.tv_sec) * 1000000L + (t.tv_nsec - t0.tv_nsec) / 1000L;
        if (us > kSpinUs) sched_yield();
    }
    return e;
}

hipError_t chunk_wait(psim_handle* h) {
    hipError_t e = hipEventRecord(h->ev_done, h->stream);
    if (e != hipSuccess) return e;
    return event_wait(h->ev_done);
}

int drive(psim_handle* h, uint32_t max_rounds, psim_round_stats* out, size_t cap, bool stop_q,
          uint32_t* ran_out) {
    uint32_t ran = 0;
    if (!h->n) return fail(h, PSIM_ESTATE, "no overlay loaded");
    const uint32_t L = h->cfg.lazy_tick_rounds ? h->cfg.lazy_tick_rounds : 1;
    const int focus = h->cur_lane;
    save_lane(h);
    // every return (HIP error paths included) leaves the handle focused on
    // the lane it was focused on; lane fields are only changed in h->lanes
    struct Refocus {
        psim_handle* h;
        int f;
        ~Refocus() { load_lane(h, f); }
    } refocus{h, focus};
    auto all_quiet = [&]() {
        for (const auto& l : h->lanes)
            if (!lane_quiescent(h, l)) return false;
        return true;
    };
    // psim_plumtree_broadcast_run: the origin's counters arrive with the
    // first chunk's (its kernel seeded the focused lane's hold ring)
    bool pend = h->origin_pend;
    h->origin_pend = false;
    // the origin's counters into the focused lane (after the stream synchronised)
    auto settle_origin = [&]() -> int {
        unsigned long long r[kNStat];
        reduce_row(h->h_stats, r);                                   // row 0: the origin's
        if (r[S_OVERFLOW])
            return fail(h, PSIM_EOVERFLOW, "origin: overflow flags 0x%llx (4: outstanding rows of an older heartbeat)",
                        r[S_OVERFLOW]);
        auto& l = h->lanes[focus];
        l.ost_cnt += (int64_t)r[S_OST_DELTA];
        l.live_rows += (int64_t)r[S_LIVE_DELTA];
        l.inflight = r[PSIM_MSG_BROADCAST];
        return PSIM_OK;
    };
    bool done = !pend && stop_q && all_quiet();
    bool seeded = false;
    while (!done && ran < max_rounds) {
        const uint32_t k = std::min<uint32_t>(kChunk, max_rounds - ran);
        const bool per_round = !(h->cfg.flags & PSIM_CFG_CHUNK_TIMING);   // events between round kernels
        // a quiescent lane's round changes nothing: only the others run (the
        // focused lane always runs, so a plain psim_step still launches)
        std::vector<int> act;
        for (int j = 0; j < (int)h->lanes.size(); j++)
            if (j == focus || !lane_quiescent(h, h->lanes[j])) act.push_back(j);
        const size_t A = act.size();
        // the first chunk after a deferred origin keeps its rows behind the
        // origin's (row 0), so one copy brings both back
        const size_t r0 = pend ? 1u : 0u;
        // inbox parities advance on a copy, committed once every launch of the
        // chunk is enqueued (a failed launch leaves the lanes' parities alone)
        std::vector<uint32_t> par(A);
        for (size_t q = 0; q < A; q++) {
            par[q] = h->lanes[act[q]].par;
            load_lane(h, act[q]);
            HIPCHK(h, scrub_if_needed(h, h->round + k));
            h->lanes[act[q]].scrub = h->scrub;
        }
        auto lane_args = [&](size_t q, uint32_t i, uint32_t tick) {
            load_lane(h, act[q]);
            PtArgs a = make_args(h, par[q], tick, h->stats + (r0 + i * A + q) * kStatsRow);
            set_round_slots(h, a, h->round + i + 1);
            set_round_tags(a, h->round + i + 1);
            if (h->dly) set_round_ring(h, a, h->round + i + 1);
            par[q] ^= 1u;
            return a;
        };
        {   // the chunk's stats rows zeroed and (first chunk) every lane's hold ring seeded: one launch
            PtPrep pp{};
            pp.z = h->stats + r0 * kStatsRow;
            pp.nz = uint64_t(k) * A * kStatsRow;
            if (!seeded) prep_seeds(h, h->round + 1, pp, pend ? focus : -1);
            seeded = true;
            HIPCHK(h, launch_pt_prep(pp, h->stream));
        }
        bool any_win = false;
        for (size_t q = 0; q < A; q++) any_win |= h->lanes[act[q]].win != nullptr;
        // a window lane's round: bucket its records, handle them (ptwin.hip)
        auto win_round = [&](size_t q, uint32_t i, uint32_t tick) -> hipError_t {
            load_lane(h, act[q]);
            const WinArgs a = make_win_args(h, par[q], tick, h->stats + (r0 + i * A + q) * kStatsRow);
            par[q] ^= 1u;
            const hipError_t e = hipMemsetAsync(a.nout, 0, 4, h->stream);
            if (e != hipSuccess) return e;
            return launch_win_round(a, h->w_cnt, h->w_cur, h->w_bsum, h->stream);
        };
        if (A > 1 && !any_win) {
            // several lanes: one launch per round over all of them (blockIdx.y = lane)
            for (uint32_t i = 0; i < k; i++) {
                const uint32_t tick = ((h->round + i + 1) % L) == 0;
                for (size_t q = 0; q < A; q++) h->h_lane_args[i * A + q] = lane_args(q, i, tick);
            }
            HIPCHK(h, hipMemcpyAsync(h->lane_args, h->h_lane_args, k * A * sizeof(PtArgs), hipMemcpyHostToDevice,
                                     h->stream));
            for (uint32_t i = 0; i < k; i++) {
                if (per_round || i == 0) HIPCHK(h, hipEventRecord(h->ev[2 * i], h->stream));
                HIPCHK(h, launch_pt_round_lanes(h->lane_args + i * A, h->h_lane_args[i * A], (uint32_t)A, h->stream));
                if (per_round || i + 1 == k) HIPCHK(h, hipEventRecord(h->ev[per_round ? 2 * i + 1 : 1], h->stream));
            }
        } else {
            for (uint32_t i = 0; i < k; i++) {
                const uint32_t tick = ((h->round + i + 1) % L) == 0;
                if (per_round || i == 0) HIPCHK(h, hipEventRecord(h->ev[2 * i], h->stream));
                for (size_t q = 0; q < A; q++) {
                    if (h->lanes[act[q]].win) HIPCHK(h, win_round(q, i, tick));
                    else HIPCHK(h, launch_pt_round(lane_args(q, i, tick), h->stream));
                }
                if (per_round || i + 1 == k) HIPCHK(h, hipEventRecord(h->ev[per_round ? 2 * i + 1 : 1], h->stream));
            }
        }
        for (size_t q = 0; q < A; q++) h->lanes[act[q]].par = par[q];
        HIPCHK(h, hipMemcpyAsync(h->h_stats, h->stats, (r0 + k * A) * kStatsRow * sizeof(unsigned long long),
                                 hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, chunk_wait(h));
        float chunk_ms = 0.f;
        if (!per_round) HIPCHK(h, hipEventElapsedTime(&chunk_ms, h->ev[0], h->ev[1]));
        if (pend) {     // the origin's row (broadcast_common), then the rounds as if it had been read first
            pend = false;
            if (const int rc = settle_origin()) return rc;
            // a quiet origin (no live eager peer): the chunk's rounds were no-ops
            if (stop_q && all_quiet()) break;
        }
        for (uint32_t i = 0; i < k; i++) {
            float ms = chunk_ms / float(k);
            if (per_round) HIPCHK(h, hipEventElapsedTime(&ms, h->ev[2 * i], h->ev[2 * i + 1]));
            unsigned long long tot[kNStat] = {0};
            uint64_t msgs = 0;
            for (size_t q = 0; q < A; q++) {
                unsigned long long r[kNStat];
                reduce_row(h->h_stats + (r0 + i * A + q) * kStatsRow, r);
                if (r[S_OVERFLOW]) {
                    load_lane(h, focus);
                    return fail(h, PSIM_EOVERFLOW,
                                "round %llu: overflow flags 0x%llx (1: >4 msgs on one edge, 2: Round > 4095, "
                                "4: outstanding rows of an older heartbeat, 8: a bin region overran; window lanes: "
                                "16: message records full, 32: > 32 outstanding rows at a vertex, "
                                "64: a timestamp set of > 4 intervals, 128: a message off the overlay)",
                                (unsigned long long)(h->round + 1), r[S_OVERFLOW]);
                }
                auto& l = h->lanes[act[q]];
                uint64_t lm = 0;
                for (int t = 1; t <= 5; t++) lm += r[t];
                l.ost_cnt += (int64_t)r[S_OST_DELTA];
                l.live_rows += (int64_t)r[S_LIVE_DELTA];
                l.inflight = lm;
                if (h->dly) {                   // round R consumed its arrivals; the sends are pending
                    const uint64_t R = h->round + 1;
                    l.due[R & (kRing - 1)] = 0;
                    l.inflight = add_due(l.due, R, h->h_stats + (r0 + i * A + q) * kStatsRow + size_t(kStatShards) * kNStat);
                }
                msgs += lm;
                for (int t = 0; t < kNStat; t++) tot[t] += r[t];
            }
            h->round++;
            h->kernel_ms_total += ms;
            h->rounds_total++;
            if (out && ran < cap) {
                psim_round_stats& o = out[ran];
                memset(&o, 0, sizeof o);
                for (int t = 1; t <= 5; t++) o.sent[t] = tot[t];
                o.delivered_new = tot[S_DELIV];
                o.active = tot[S_ACTIVE];
                o.senders = tot[S_SENDERS];
                o.sender_degree_sum = tot[S_DEGSUM];
                int64_t ov = 0;
                for (const auto& l : h->lanes) ov += l.ost_cnt;
                o.outstanding_vertices = (uint64_t)ov;
                o.algo_bytes = 16ull * h->n * A + 8ull * tot[S_SENDERS] + 4ull * tot[S_DEGSUM] + 32ull * msgs;
                o.words_stored = tot[S_WORDS];
                o.kernel_ms = ms;
            }
            ran++;
            if (stop_q && all_quiet()) { done = true; break; }
        }
    }
    if (pend) {         // max_rounds 0: the origin's row is still to be read
        HIPCHK(h, hipMemcpyAsync(h->h_stats, h->stats, kStatsRow * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                                 h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        if (const int rc = settle_origin()) return rc;
    }
    load_lane(h, focus);
    if (ran_out) *ran_out = ran;
    return PSIM_OK;
}

// ---- the forest: every node's heartbeat tree ---------------
// partisan_plumtree_backend heartbeats from every node on a timer
// (:341-368, :421-428) and the broadcast server keeps each root's eager /
// lazy sets in its eager_sets / lazy_sets maps for good
// (partisan_plumtree_broadcast.erl:1240-1248, 1278-1282; only reset_peers
// drops them, :1320-1328).  A forest handle keeps up to max_roots roots:
// lane L of every slab is one root's copy of the single-lane arrays, a
// round is one launch over every lane, and nothing per lane crosses PCIe
// per round (the counters of all lanes add into the round's one stats row).

// bytes one lane takes in the slabs besides its root's records (16 n, one
// state slot per root)
uint64_t fo_lane_bytes(const psim_handle* h, uint64_t s_in) {
    const auto& f = h->fo;
    uint64_t b = 2 * s_in * 4 + 2 * f.s_pend + f.s_ost + 4 * sizeof(int) + kMcntLane * 4 + 8 + 8;
    if (h->sh.world > 1)        // staged words + the lane's share of the exchange buffers
        b += s_in * 4 + 4 * (h->sh.send_base[h->sh.world] + h->sh.recv_base[h->sh.world]);
    return b;
}

int forest_alloc(psim_handle* h) {
    auto& f = h->fo;
    if (!h->ell && !h->E) return fail(h, PSIM_EINVAL, "empty overlay");
    // lane slices aligned to 256 B: the ELL sweep reads a chunk's words as quads
    const uint64_t s_in = (h->Ed + 63) & ~uint64_t(63);
    f.s_pend = (h->pend_bytes + 255) & ~uint64_t(255);
    f.s_ost = (uint64_t(h->n) + 4 + 255) & ~uint64_t(255);
    const uint64_t C = f.slabs(), R = f.cap;    // lane slabs, state slots
    const uint64_t per = fo_lane_bytes(h, s_in), per_root = uint64_t(h->n) * 16, total = per * C + per_root * R;
    size_t fr = 0, tot = 0;
    HIPCHK(h, hipMemGetInfo(&fr, &tot));
    if (total + (uint64_t(1) << 30) > fr)
        return fail(h, PSIM_ENOMEM, "max_roots=%u over %u lanes needs %.2f GB of slabs (%.2f MB per root, %.2f MB per "
                                    "lane); %.2f GB free", f.cap, f.nlanes(), double(total) / 1e9,
                    double(per_root) / 1e6, double(per) / 1e6, double(fr) / 1e9);
    const uint64_t L = std::max(C, R);          // lane / slot lists
    if (!alloc_zero((void**)&f.vs, R * h->n * 16) || !alloc_zero((void**)&f.in[0], C * s_in * 4) ||
        !alloc_zero((void**)&f.in[1], C * s_in * 4) || !alloc_zero((void**)&f.pend[0], C * f.s_pend) ||
        !alloc_zero((void**)&f.pend[1], C * f.s_pend) || !alloc_zero((void**)&f.ost, C * f.s_ost) ||
        !alloc_zero((void**)&f.ost_total, C * 4 * sizeof(int)) || !alloc_zero((void**)&f.mcnt, C * kMcntLane * 4) ||
        !alloc_zero((void**)&f.info, R * 8) || !alloc_zero((void**)&f.d_list, L * 4) ||
        !alloc_zero((void**)&f.d_busy, L * 4) || (f.parking() && !alloc_zero((void**)&f.d_slot, C * 4))) {
        free_forest(h);
        return fail(h, PSIM_ENOMEM, "forest slabs for %u roots over %u lanes (%.2f GB)", f.cap, f.nlanes(),
                    double(total) / 1e9);
    }
    if (h->sh.world > 1) {
        const auto& sh = h->sh;
        const size_t W = size_t(sh.world);
        if (!alloc_zero((void**)&f.stage, C * s_in * 4) ||
            !alloc_zero((void**)&f.xsend, std::max<uint64_t>(1, C * sh.send_base[W]) * 4) ||
            !alloc_zero((void**)&f.xrecv, std::max<uint64_t>(1, C * sh.recv_base[W]) * 4) ||
            !alloc_zero((void**)&f.sb_d, (W + 1) * 8) || !alloc_zero((void**)&f.rb_d, (W + 1) * 8)) {
            free_forest(h);
            return fail(h, PSIM_ENOMEM, "sharded forest exchange buffers for %u roots", f.cap);
        }
        HIPCHK(h, hipMemcpy(f.sb_d, sh.send_base.data(), (W + 1) * 8, hipMemcpyHostToDevice));
        HIPCHK(h, hipMemcpy(f.rb_d, sh.recv_base.data(), (W + 1) * 8, hipMemcpyHostToDevice));
        f.s_stage = s_in;
    }
    f.g_inflight = f.g_live = 0;
    f.s_in = s_in;
    f.nl = 0;
    f.ns = 0;
    f.focus = -1;
    f.h_info.assign(f.cap, make_uint2(0u, 0u));
    f.serial.assign(f.cap, 0u);
    f.root_of.assign(C, kNoPeer);
    f.lane_of.clear();
    f.h_slot.assign(C, 0u);
    f.slot_root.clear();
    f.slot_of.clear();
    return PSIM_OK;
}

// The arguments of round R (tags R, counts ring R mod 4) for every lane: lane
// 0's slices here, the kernels shift them by the lane (fo_lane in plumtree.hip).
FoArgs forest_args(const psim_handle* h, uint32_t par, uint32_t tick, unsigned long long* stats, uint64_t R,
                   bool origin = false) {
    const auto& f = h->fo;
    PtArgs a = make_args(h, par, tick, stats);
    a.vs = f.vs;
    a.in_cur = f.in[par];
    a.in_nxt = f.in[par ^ 1];
    a.pend_cur = f.pend[par];
    a.pend_nxt = f.pend[par ^ 1];
    a.ost = f.ost;
    a.ost_total = f.ost_total;
    set_round_tags(a, R);
    a.mcnt = f.mcnt;
    a.m_w = uint32_t(R % 4);
    a.m_s = uint32_t((R + 3) % 4);
    a.m_r = uint32_t((R + 2) % 4);
    a.m_z = uint32_t((R + 1) % 4);
    a.dense = std::max<uint32_t>(1u, h->n / h->dense_div);
    const uint32_t thr = list_threshold(h);
    if (thr) {
        a.wlcnt = a.mcnt + 256;
        a.wl_cur = reinterpret_cast<uint32_t*>(a.pend_cur + h->wl_off);
        a.wl_nxt = reinterpret_cast<uint32_t*>(a.pend_nxt + h->wl_off);
        a.wl_cap = h->wl_cap;
        a.wl_thr = thr;
        a.wl_gpc = h->wl_gpc;
        a.wl_wgs = h->wl_wgs;
    }
    FoArgs fa{};
    fa.a = a;
    fa.s_vs = h->n;
    fa.s_in = f.s_in;
    fa.s_pend = f.s_pend;
    fa.s_ost = f.s_ost;
    fa.info = f.info;
    fa.nl = f.nl;
    fa.ns = f.ns;
    fa.slot = f.parking() ? f.d_slot : nullptr;
    fa.a.stage = f.stage;                      // null on one GPU
    fa.s_stage = f.s_stage;
    if (h->dly) {
        // delay faults: round R reads ring slot R and writes slot R + 1 + d
        // (set_round_ring's layout in each lane's ring); the origins emit as
        // round R - 1.  No per-round counts (a word may arrive rounds later):
        // flags only, every round runs.
        const uint64_t Rr = origin ? R - 1 : R;
        const size_t ng = (size_t(h->n) + (1u << kGroupShift) - 1) >> kGroupShift;
        PtArgs& b = fa.a;
        b.ring = f.ring;
        b.pring = f.pring;
        b.ed = uint32_t(h->Ed);
        b.ngrp = uint32_t(ng);
        b.rpos = uint32_t(Rr + 1) & (kRing - 1);
        b.in_cur = f.ring + size_t(Rr & (kRing - 1)) * h->Ed;
        b.in_nxt = f.ring + size_t(b.rpos) * h->Ed;
        b.pend_cur = f.pring + size_t(Rr & (kRing - 1)) * ng;
        b.pend_nxt = f.pring + size_t(b.rpos) * ng;
        b.ctag = uint32_t(Rr) & 0xFFu;
        b.wtag = uint32_t(Rr + 1) & 0xFFu;
        b.mcnt = nullptr;
        b.wlcnt = nullptr;
        b.wl_cur = b.wl_nxt = nullptr;
        b.wl_cap = b.wl_thr = 0;
        fa.s_in = f.s_ring;                    // fo_lane shifts the ring with the lane
        fa.s_pend = f.s_pring;
    }
    return fa;
}

// Sharded forest: the round just run (its arguments fa) left every lane's
// remote words staged; they travel as every lane's dense regions in ONE
// all-to-all-v and land in each lane's inbox for the next round.
// fixed_mark >= 0: the words are origins' pushes (flags + list).
int forest_exchange(psim_handle* h, const FoArgs& fa, int fixed_mark) {
    auto& f = h->fo;
    auto& sh = h->sh;
    if (sh.world == 1 || f.nl == 0) return PSIM_OK;
    const uint32_t W = uint32_t(sh.world), nl = f.nl;
    HIPCHK(h, launch_fo_pack_dense(fa, sh.rem, uint32_t(sh.send_base[W]), f.sb_d, W, f.xsend, h->stream));
    std::vector<uint64_t> so(W + 1), ro(W + 1);
    for (uint32_t d = 0; d <= W; d++) {
        so[d] = sh.send_base[d] * nl;
        ro[d] = sh.recv_base[d] * nl;
    }
    std::string err;
    const int rc = sh.xport->alltoallv(f.xsend, so.data(), f.xrecv, ro.data(), sh.rank, int(W), h->stream, &err);
    if (rc) return fail(h, rc, "forest exchange: %s", err.c_str());
    HIPCHK(h, launch_fo_ingest_dense(fa, f.xrecv, sh.recv_map, uint32_t(sh.recv_base[W]), f.rb_d, W, sh.slot2v,
                                     fixed_mark, h->stream));
    return PSIM_OK;
}

// Sharded forest: the global in-flight messages and live rows (one all-reduce
// of this shard's totals; every rank then takes the same stop decision).
int forest_globals(psim_handle* h) {
    auto& f = h->fo;
    int64_t v[2] = {(int64_t)h->inflight, h->live_rows};
    if (h->sh.world > 1) {
        std::string err;
        const int rc = h->sh.xport->allreduce(v, 2, h->stream, &err);
        if (rc) return fail(h, rc, "forest all-reduce: %s", err.c_str());
    }
    f.g_inflight = v[0];
    f.g_live = v[1];
    return PSIM_OK;
}

// The getters' view: the handle's single-lane fields alias lane `lane`
// (its root's records in the root's state slot).
void forest_view(psim_handle* h, uint32_t lane, uint32_t slot) {
    auto& f = h->fo;
    const uint64_t l = uint64_t(lane);
    h->vs = f.vs + uint64_t(slot) * h->n;
    for (int b = 0; b < 2; b++) {
        h->in[b] = f.in[b] + l * f.s_in;
        h->pend[b] = f.pend[b] + l * f.s_pend;
    }
    h->ost = f.ost + l * f.s_ost;
    h->ost_total = f.ost_total + 4 * l;
    if (f.ring) {                               // delay faults: the getters read the lane's ring
        h->ring = f.ring + l * f.s_ring;
        h->pring = f.pring + l * f.s_pring;
    }
    h->serial = f.serial[slot];
    h->have_root = true;
}

void forest_focus(psim_handle* h, int lane) {
    auto& f = h->fo;
    forest_view(h, uint32_t(lane), f.slot(uint32_t(lane)));
    h->root = f.root_of[lane];
    f.focus = lane;
}

// A parked root: its records, and the empty lane's (nothing in flight, no rows).
void forest_focus_parked(psim_handle* h, uint32_t slot) {
    auto& f = h->fo;
    forest_view(h, f.lanes, slot);
    h->root = f.slot_root[slot];
    f.focus = -2 - int(slot);
}

void forest_refocus(psim_handle* h) {
    auto& f = h->fo;
    if (f.focus >= 0) forest_focus(h, f.focus);
    else if (f.focus <= -2) forest_focus_parked(h, uint32_t(-2 - f.focus));
}

int forest_upload_info(psim_handle* h) {
    auto& f = h->fo;
    if (f.ns) HIPCHK(h, hipMemcpyAsync(f.info, f.h_info.data(), size_t(f.ns) * 8, hipMemcpyHostToDevice, h->stream));
    if (f.parking() && f.nl)
        HIPCHK(h, hipMemcpyAsync(f.d_slot, f.h_slot.data(), size_t(f.nl) * 4, hipMemcpyHostToDevice, h->stream));
    return PSIM_OK;
}

// The backend's heartbeat id of root's next heartbeat (broadcast_common's
// rule): *commit = false only checks it.
int next_mono(psim_handle* h, uint32_t root, uint32_t* out, bool commit) {
    uint32_t mono = 0;
    const auto it = h->mono_of.find(root);
    if (it != h->mono_of.end()) mono = it->second;
    const auto ne = h->next_epoch.find(root);
    if (ne != h->next_epoch.end()) {
        mono = (ne->second << 24) | 1u;
        if (commit) h->next_epoch.erase(ne);
    } else {
        if ((mono & 0xFFFFFFu) >= 0xFFFFFEu) return fail(h, PSIM_EOVERFLOW, "root %u: 2^24-2 heartbeats in one epoch", root);
        mono++;
    }
    if (commit) h->mono_of[root] = mono;
    if (out) *out = mono;
    return PSIM_OK;
}

// Heartbeats from roots[0, k) at once (backend handle_info(heartbeat) at each
// of them).  All or nothing: a root past max_roots is PSIM_ENOSPC, a root
// whose previous heartbeat is in flight or holds rows PSIM_EBUSY, before any
// state changes.
int forest_broadcast(psim_handle* h, const uint32_t* roots, size_t k, uint32_t* monos) {
    auto& f = h->fo;
    if (!h->n) return PSIM_ESTATE;
    if (!k) return PSIM_OK;
    if (!roots) return PSIM_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    std::vector<uint32_t> lanes(k), slots(k), old;
    std::unordered_map<uint32_t, int> seen;
    uint32_t fresh = 0, need = 0;
    const bool sharded = h->sh.world > 1;       // collective: every rank passes the same roots
    if (sharded && !h->sh.xport) return fail(h, PSIM_ESTATE, "sharded forest without a transport");
    for (size_t i = 0; i < k; i++) {
        if (roots[i] >= h->sh.n_global) return fail(h, PSIM_EINVAL, "root %u >= n", roots[i]);
        if (!seen.emplace(roots[i], 1).second)
            return fail(h, PSIM_EINVAL, "root %u heartbeats twice in one call", roots[i]);
        const auto is = f.slot_of.find(roots[i]);
        slots[i] = is == f.slot_of.end() ? kNoPeer : is->second;
        if (slots[i] == kNoPeer) fresh++;
        const auto it = f.lane_of.find(roots[i]);
        if (it == f.lane_of.end()) {
            lanes[i] = kNoPeer;
            need++;
        } else {
            lanes[i] = it->second;
            old.push_back(it->second);
        }
        const int rc = next_mono(h, roots[i], nullptr, false);
        if (rc) return rc;
    }
    if (uint64_t(f.ns) + fresh > f.cap)
        return fail(h, PSIM_ENOSPC, "%u roots hold trees, %u new ones exceed max_roots=%u", f.ns, fresh, f.cap);
    // lanes busy with their root's heartbeat: messages of the last round (count
    // slot round % 4, origins included) or rows held (delay faults: anything
    // pending anywhere, or rows held)
    auto busy_lanes = [&](const std::vector<uint32_t>& ls, std::vector<uint32_t>& busy) -> int {
        busy.assign(ls.size(), 0u);
        if (ls.empty()) return PSIM_OK;
        if (h->dly) {
            std::vector<int> tot(size_t(f.slabs()) * 4);
            HIPCHK(h, hipMemcpyAsync(tot.data(), f.ost_total, tot.size() * sizeof(int), hipMemcpyDeviceToHost,
                                     h->stream));
            HIPCHK(h, hipStreamSynchronize(h->stream));
            for (size_t i = 0; i < ls.size(); i++) busy[i] = (h->inflight != 0 || tot[4 * size_t(ls[i])] != 0);
            return PSIM_OK;
        }
        FoArgs fa = forest_args(h, h->par, 0, h->stats, h->round + 1);
        HIPCHK(h, hipMemcpyAsync(f.d_list, ls.data(), ls.size() * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, launch_fo_busy(fa, f.d_list, uint32_t(ls.size()), uint32_t(h->round % 4), f.d_busy, h->stream));
        HIPCHK(h, hipMemcpyAsync(busy.data(), f.d_busy, ls.size() * 4, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        if (sharded) {                            // busy on any shard
            std::vector<int64_t> b(busy.begin(), busy.end());
            std::string err;
            const int rc = h->sh.xport->allreduce(b.data(), b.size(), h->stream, &err);
            if (rc) return fail(h, rc, "forest busy all-reduce: %s", err.c_str());
            for (size_t i = 0; i < b.size(); i++) busy[i] = b[i] != 0;
        }
        return PSIM_OK;
    };
    {                                             // every heartbeating root's last one is done
        std::vector<uint32_t> busy;
        const int rc = busy_lanes(old, busy);
        if (rc) return rc;
        for (size_t i = 0; i < old.size(); i++)
            if (busy[i])
                return fail(h, PSIM_EBUSY, h->dly ? "root %u: messages are in flight or its lane holds rows (delay "
                                                    "faults: a forest root heartbeats again once nothing is pending)"
                                                  : "root %u: its last heartbeat is in flight or holds rows (a forest "
                                                    "keeps one heartbeat per root)", f.root_of[old[i]]);
    }
    // lanes for the roots without one: never-used lanes, then (parked roots)
    // lanes whose root's heartbeat is done -- that root keeps its records in
    // its slot and gives the lane up
    std::vector<uint32_t> freel;
    for (uint32_t l = f.nl; l < f.nlanes() && freel.size() < need; l++) freel.push_back(l);
    if (freel.size() < need && f.parking()) {
        std::vector<uint32_t> cand, busy;
        for (uint32_t l = 0; l < f.nl; l++)
            if (!seen.count(f.root_of[l])) cand.push_back(l);
        const int rc = busy_lanes(cand, busy);
        if (rc) return rc;
        for (size_t i = 0; i < cand.size() && freel.size() < need; i++)
            if (!busy[i]) freel.push_back(cand[i]);
    }
    if (freel.size() < need)
        return fail(h, PSIM_ENOSPC, "%u heartbeats need a lane and %zu are free: %u lanes, the others' heartbeats are "
                                    "in flight or hold rows (max_roots=%u)", need, freel.size(), f.nlanes(), f.cap);
    std::vector<uint32_t> wrap, own;            // wrap: slots; own: lanes whose root this shard holds
    size_t fi = 0;
    for (size_t i = 0; i < k; i++) {
        if (slots[i] == kNoPeer) {
            slots[i] = f.ns++;
            f.slot_of[roots[i]] = slots[i];
            f.slot_root.push_back(roots[i]);
        }
        if (lanes[i] == kNoPeer) {
            const uint32_t l = freel[fi++];
            if (l >= f.nl) f.nl = l + 1;
            else f.lane_of.erase(f.root_of[l]);   // its root is parked from now on
            lanes[i] = l;
            f.root_of[l] = roots[i];
            f.lane_of[roots[i]] = l;
            f.h_slot[l] = slots[i];
        }
        const uint32_t l = lanes[i], sl = slots[i];
        f.serial[sl]++;
        if ((f.serial[sl] & 0x7Fu) == 0) wrap.push_back(sl);
        const uint32_t lr = roots[i] - h->sh.v_lo;  // the origin's local index on its owner
        f.h_info[sl] = make_uint2(f.serial[sl] & 0xFFu, lr < h->n ? lr : kNoPeer);
        if (lr < h->n) own.push_back(l);
        uint32_t mono = 0;
        (void)next_mono(h, roots[i], &mono, true);
        if (monos) monos[i] = mono;
    }
    int rc = forest_upload_info(h);
    if (rc) return rc;
    if (!wrap.empty()) {                         // 8-bit Monotonic tags of these lanes re-based
        FoArgs fa = forest_args(h, h->par, 0, h->stats, h->round + 1);
        HIPCHK(h, hipMemcpyAsync(f.d_list, wrap.data(), wrap.size() * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, launch_fo_renorm(fa, f.d_list, uint32_t(wrap.size()), h->stream));
    }
    // the origins emit into the buffers the next round reads (broadcast_common)
    HIPCHK(h, hipMemsetAsync(h->stats, 0, kStatsRow * sizeof(unsigned long long), h->stream));
    FoArgs fa = forest_args(h, h->par ^ 1u, 0, h->stats, h->round + 1, true);
    fa.a.wtag = uint32_t(h->round + 1) & 0xFFu;
    if (!own.empty()) {
        HIPCHK(h, hipMemcpyAsync(f.d_list, own.data(), own.size() * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, launch_fo_origin(fa, f.d_list, uint32_t(own.size()), h->stream));
    }
    if (sharded) {
        // the origins' remote pushes: counted as the round before the next
        // one (the origin's count slot) and flagged + listed like its own
        FoArgs fx = fa;
        fx.a.m_w = fa.a.m_s;
        const int rc2 = forest_exchange(h, fx, fa.a.wl_nxt ? 2 : 1);
        if (rc2) return rc2;
    }
    HIPCHK(h, hipMemcpyAsync(h->h_stats, h->stats, kStatsRow * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                             h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    unsigned long long r[kNStat];
    reduce_row(h->h_stats, r);
    forest_focus(h, int(lanes[k - 1]));
    if (r[S_OVERFLOW])
        return fail(h, PSIM_EOVERFLOW, "origins: overflow flags 0x%llx", r[S_OVERFLOW]);
    h->ost_cnt += (int64_t)r[S_OST_DELTA];
    h->live_rows += (int64_t)r[S_LIVE_DELTA];
    h->inflight += r[PSIM_MSG_BROADCAST];
    // delay faults: the origins' pushes are pending until 1 + d rounds on
    if (h->dly) h->inflight = add_due(h->due, h->round, h->h_stats + size_t(kStatShards) * kNStat);
    return forest_globals(h);
}

int forest_scrub_if_needed(psim_handle* h, uint64_t last) {
    if (last + 1 < h->scrub + kTagSpan) return PSIM_OK;
    const uint32_t keep = uint32_t(h->round + 1) & 0xFFu;
    if (h->fo.ring && h->fo.nl)                 // delay rings: keep the next kRing - 1 rounds' words
        HIPCHK(h, launch_pt_scrub(h->fo.ring, uint64_t(h->fo.nl) * h->fo.s_ring, keep, kRing - 1, h->stream));
    for (int b = 0; b < 2 && h->fo.nl; b++)
        HIPCHK(h, launch_pt_scrub(h->fo.in[b], uint64_t(h->fo.nl) * h->fo.s_in, keep, 1, h->stream));
    h->scrub = h->round;
    return PSIM_OK;
}

int forest_renorm_all(psim_handle* h) {
    FoArgs fa = forest_args(h, h->par, 0, h->stats, h->round + 1);
    HIPCHK(h, launch_fo_renorm(fa, nullptr, h->fo.ns, h->stream));   // every root's records, parked or not
    return PSIM_OK;
}

// psim_step / psim_run on a forest: every lane runs every round (a lane with
// nothing in flight and no row due leaves in its first instructions).
int forest_drive(psim_handle* h, uint32_t max_rounds, psim_round_stats* out, size_t cap, bool stop_q,
                 uint32_t* ran_out) {
    auto& f = h->fo;
    uint32_t ran = 0;
    if (!h->n) return fail(h, PSIM_ESTATE, "no overlay loaded");
    const uint32_t L = h->cfg.lazy_tick_rounds ? h->cfg.lazy_tick_rounds : 1;
    const bool per_round = !(h->cfg.flags & PSIM_CFG_CHUNK_TIMING);
    const bool sharded = h->sh.world > 1;       // collective: every rank drives the same rounds
    // sharded: the stop rule reads the global totals (every rank decides alike)
    auto quiet = [&]() {
        return sharded ? (f.g_inflight == 0 && f.g_live == 0) : (h->inflight == 0 && h->live_rows == 0);
    };
    if (!h->dly) {   // every lane's row-holder ring from its exact count (seed_hold_ring; delays: no counts)
        FoArgs fa = forest_args(h, h->par, 0, h->stats, h->round + 1);
        HIPCHK(h, launch_fo_seed(fa, h->stream));
    }
    if (sharded) {
        const int rc = forest_globals(h);
        if (rc) return rc;
    }
    bool done = stop_q && quiet();
    while (!done && ran < max_rounds) {
        const uint32_t k = std::min<uint32_t>(kChunk, max_rounds - ran);
        int rc = forest_scrub_if_needed(h, h->round + k);
        if (rc) return rc;
        HIPCHK(h, hipMemsetAsync(h->stats, 0, k * kStatsRow * sizeof(unsigned long long), h->stream));
        uint32_t par = h->par;
        for (uint32_t i = 0; i < k; i++) {
            const uint32_t tick = ((h->round + i + 1) % L) == 0;
            const FoArgs fa = forest_args(h, par, tick, h->stats + i * kStatsRow, h->round + i + 1);
            if (per_round || i == 0) HIPCHK(h, hipEventRecord(h->ev[2 * i], h->stream));
            if (f.nl) HIPCHK(h, launch_fo_round(fa, f.gx, h->stream));
            if (per_round || i + 1 == k) HIPCHK(h, hipEventRecord(h->ev[per_round ? 2 * i + 1 : 1], h->stream));
            if (sharded) {                            // every lane's remote words, one all-to-all-v
                const int rc2 = forest_exchange(h, fa, -1);
                if (rc2) return rc2;
            }
            par ^= 1u;
        }
        h->par = par;
        HIPCHK(h, hipMemcpyAsync(h->h_stats, h->stats, k * kStatsRow * sizeof(unsigned long long),
                                 hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, chunk_wait(h));
        float chunk_ms = 0.f;
        if (!per_round) HIPCHK(h, hipEventElapsedTime(&chunk_ms, h->ev[0], h->ev[1]));
        // sharded: the chunk's per-round counters summed over ranks in one
        // all-reduce -- kinds, new deliveries, senders, degree sum, and this
        // shard's live rows / row holders after each round (global stop rule)
        constexpr int NK = 10;
        std::vector<int64_t> glob(size_t(k) * NK, 0);
        int overflow_rc = 0;
        {
            int64_t live = h->live_rows, ost = h->ost_cnt;
            for (uint32_t i = 0; i < k; i++) {
                unsigned long long r[kNStat];
                reduce_row(h->h_stats + i * kStatsRow, r);
                if (r[S_OVERFLOW] && !overflow_rc)
                    overflow_rc = fail(h, PSIM_EOVERFLOW, "round %llu: overflow flags 0x%llx (1: >4 msgs on one edge, 2: "
                                       "Round > 4095, 4: outstanding rows of an older heartbeat)",
                                       (unsigned long long)(h->round + 1 + i), r[S_OVERFLOW]);
                live += (int64_t)r[S_LIVE_DELTA];
                ost += (int64_t)r[S_OST_DELTA];
                int64_t* g = glob.data() + size_t(i) * NK;
                for (int t = 1; t <= 5; t++) g[t - 1] = (int64_t)r[t];
                g[5] = (int64_t)r[S_DELIV];
                g[6] = (int64_t)r[S_SENDERS];
                g[7] = (int64_t)r[S_DEGSUM];
                g[8] = live;
                g[9] = ost;
            }
        }
        if (sharded) {
            // an overflow on one shard still joins the collective; every rank returns the common code
            std::vector<int64_t> v(glob.size() + kNCodes);
            std::copy(glob.begin(), glob.end(), v.begin());
            put_code(v.data() + glob.size(), overflow_rc);
            std::string err;
            const int rc = h->sh.xport->allreduce(v.data(), v.size(), h->stream, &err);
            if (rc) return fail(h, rc, "forest counter all-reduce: %s", err.c_str());
            std::copy(v.begin(), v.begin() + glob.size(), glob.begin());
            const int frc = finish_code(h, v.data() + glob.size(), overflow_rc, "forest round");
            if (frc) return frc;
        } else if (overflow_rc) {
            return overflow_rc;
        }
        for (uint32_t i = 0; i < k; i++) {
            float ms = chunk_ms / float(k);
            if (per_round) HIPCHK(h, hipEventElapsedTime(&ms, h->ev[2 * i], h->ev[2 * i + 1]));
            unsigned long long r[kNStat];
            reduce_row(h->h_stats + i * kStatsRow, r);
            const int64_t* g = glob.data() + size_t(i) * NK;
            uint64_t msgs = 0;
            for (int t = 1; t <= 5; t++) msgs += r[t];
            h->ost_cnt += (int64_t)r[S_OST_DELTA];
            h->live_rows += (int64_t)r[S_LIVE_DELTA];
            h->inflight = msgs;
            if (h->dly) {   // round R consumed its arrivals; its sends are pending until R + 1 + d
                const uint64_t R = h->round + 1;
                h->due[R & (kRing - 1)] = 0;
                h->inflight = add_due(h->due, R, h->h_stats + i * kStatsRow + size_t(kStatShards) * kNStat);
            }
            if (sharded) {
                f.g_inflight = g[0] + g[1] + g[2] + g[3] + g[4];
                f.g_live = g[8];
            }
            h->round++;
            h->kernel_ms_total += ms;
            h->rounds_total++;
            if (out && ran < cap) {
                psim_round_stats& o = out[ran];
                memset(&o, 0, sizeof o);
                for (int t = 1; t <= 5; t++) o.sent[t] = (uint64_t)g[t - 1];   // global when sharded
                o.delivered_new = (uint64_t)g[5];
                o.active = r[S_ACTIVE];                                     // this shard's
                o.senders = (uint64_t)g[6];
                o.sender_degree_sum = (uint64_t)g[7];
                o.outstanding_vertices = (uint64_t)g[9];
                o.algo_bytes = 16ull * h->n * f.nl + 8ull * r[S_SENDERS] + 4ull * r[S_DEGSUM] + 32ull * msgs;
                o.words_stored = r[S_WORDS];
                o.kernel_ms = ms;
            }
            ran++;
            if (stop_q && quiet()) {
                done = true;
                break;
            }
        }
    }
    if (ran_out) *ran_out = ran;
    return PSIM_OK;
}

}  // namespace

namespace psim {

ModuleState*& handle_module(psim_handle* h, int slot) { return h->mods[slot]; }
const ModuleState* handle_module(const psim_handle* h, int slot) { return h->mods[slot]; }
hipStream_t handle_stream(const psim_handle* h) { return h->stream; }
Transport* handle_transport(psim_handle* h) { return h->sh.xport; }
int handle_device(const psim_handle* h) { return h->device; }
uint64_t handle_seed(const psim_handle* h) { return h->cfg.seed; }
int handle_fail(psim_handle* h, int code, const char* fmt, ...) {
    if (h) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        h->err = buf;
    }
    return code;
}
void handle_add_round(psim_handle* h, double kernel_ms) {
    h->kernel_ms_total += kernel_ms;
    h->rounds_total++;
}
hipEvent_t handle_event(psim_handle* h, int i) { return h->ev[i]; }
hipError_t handle_wait(psim_handle* h) { return chunk_wait(h); }

}  // namespace psim

extern "C" {

const char* psim_strerror(int code) {
    switch (code) {
    case PSIM_OK: return "ok";
    case PSIM_EINVAL: return "invalid argument";
    case PSIM_ENOMEM: return "out of memory";
    case PSIM_EHIP: return "HIP runtime error";
    case PSIM_ERCCL: return "RCCL error";
    case PSIM_ESTATE: return "invalid state";
    case PSIM_EOVERFLOW: return "fixed-capacity structure overflowed";
    case PSIM_EBUSY: return "previous broadcast not quiescent";
    case PSIM_ENODEV: return "no usable HIP device";
    case PSIM_ENOSPC: return "no slot left for another heartbeat root";
    case PSIM_ENOTSUP: return "not supported for this engine / feature combination";
    default: return "unknown error";
    }
}

const char* psim_last_error(const psim_handle* h) { return h ? h->err.c_str() : g_create_err.c_str(); }

int psim_create(const psim_config* cfg, psim_handle** out) {
    if (!cfg || !out) return PSIM_EINVAL;
    if (cfg->abi_version != PSIM_ABI_VERSION) return PSIM_EINVAL;
    *out = nullptr;
    int ndev = 0;
    const hipError_t de = hipGetDeviceCount(&ndev);
    if (de != hipSuccess || ndev == 0) {
        g_create_err = std::string("hipGetDeviceCount: ") + hipGetErrorString(de) + ", devices=" + std::to_string(ndev);
        return PSIM_ENODEV;
    }
    psim_handle* h = new (std::nothrow) psim_handle();
    if (!h) return PSIM_ENOMEM;
    h->cfg = *cfg;
    if (!h->cfg.lazy_tick_rounds) h->cfg.lazy_tick_rounds = 1;
    if (cfg->max_roots > uint32_t(kMaxLanes)) {          // the forest: every root's trees
        if (cfg->flags & PSIM_CFG_BINNED) {
            g_create_err = "max_roots > 16 needs the slot-scatter engine (not PSIM_CFG_BINNED)";
            delete h;
            return PSIM_EINVAL;
        }
        h->fo.on = true;
        h->fo.cap = cfg->max_roots;
        if (const char* e = getenv("PSIM_FOREST_GX")) h->fo.gx = uint32_t(strtoul(e, nullptr, 10));
    }
    h->device = cfg->device >= 0 ? cfg->device : 0;
    if (cfg->device < 0) (void)hipGetDevice(&h->device);
    if (h->device >= ndev) { delete h; return PSIM_EINVAL; }
    int rc = PSIM_OK;
    do {
        const hipError_t se = hipSetDevice(h->device);
        if (se != hipSuccess) {
            g_create_err = std::string("hipSetDevice: ") + hipGetErrorString(se);
            rc = PSIM_ENODEV;
            break;
        }
        if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) { rc = PSIM_EHIP; break; }
        h->own_stream = h->stream;
        if (hipMalloc(&h->sh.ring, 16 * kStatsRow * sizeof(unsigned long long)) != hipSuccess) { rc = PSIM_ENOMEM; break; }
        for (auto& e : h->sh.rev_)
            if (hipEventCreate(&e) != hipSuccess) { rc = PSIM_EHIP; break; }
        for (auto& e : h->sh.xev)
            if (hipEventCreate(&e) != hipSuccess) { rc = PSIM_EHIP; break; }
        if (hipMalloc(&h->stats, (kChunk * kMaxLanes + 1) * kStatsRow * sizeof(unsigned long long)) != hipSuccess) { rc = PSIM_ENOMEM; break; }
        if (hipHostMalloc(&h->h_stats, (kChunk * kMaxLanes + 1) * kStatsRow * sizeof(unsigned long long)) != hipSuccess) { rc = PSIM_ENOMEM; break; }
        if (hipMalloc(&h->lane_args, kChunk * kMaxLanes * sizeof(PtArgs)) != hipSuccess ||
            hipHostMalloc(&h->h_lane_args, kChunk * kMaxLanes * sizeof(PtArgs)) != hipSuccess) { rc = PSIM_ENOMEM; break; }
        if (hipMalloc(&h->scratch, 64) != hipSuccess) { rc = PSIM_ENOMEM; break; }
        if (hipMalloc(&h->ost_total_base, kMaxLanes * 4 * sizeof(int)) != hipSuccess) { rc = PSIM_ENOMEM; break; }
        if (hipMalloc(&h->mcnt_base, kMaxLanes * kMcntLane * sizeof(uint32_t)) != hipSuccess ||
            hipMemset(h->mcnt_base, 0, kMaxLanes * kMcntLane * sizeof(uint32_t)) != hipSuccess) { rc = PSIM_ENOMEM; break; }
        if (hipMemset(h->ost_total_base, 0, kMaxLanes * 4 * sizeof(int)) != hipSuccess ||
            hipDeviceSynchronize() != hipSuccess) { rc = PSIM_EHIP; break; }
        h->ost_total = h->ost_total_base;
        for (auto& e : h->ev)
            if (hipEventCreate(&e) != hipSuccess) { rc = PSIM_EHIP; break; }
        if (hipEventCreateWithFlags(&h->ev_done, hipEventDisableTiming) != hipSuccess) { rc = PSIM_EHIP; break; }
    } while (0);
    if (rc != PSIM_OK) { psim_destroy(h); return rc; }
    *out = h;
    return PSIM_OK;
}

int psim_destroy(psim_handle* h) {
    if (!h) return PSIM_EINVAL;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->own_stream) (void)hipStreamSynchronize(h->own_stream);
    free_graph(h);
    for (auto& m : h->mods) {
        delete m;
        m = nullptr;
    }
    if (h->stats) (void)hipFree(h->stats);
    if (h->h_stats) (void)hipHostFree(h->h_stats);
    if (h->lane_args) (void)hipFree(h->lane_args);
    if (h->h_lane_args) (void)hipHostFree(h->h_lane_args);
    if (h->scratch) (void)hipFree(h->scratch);
    if (h->ost_total_base) (void)hipFree(h->ost_total_base);
    if (h->mcnt_base) (void)hipFree(h->mcnt_base);
    if (h->scratch_buf) (void)hipFree(h->scratch_buf);
    for (auto& e : h->ev)
        if (e) (void)hipEventDestroy(e);
    if (h->ev_done) (void)hipEventDestroy(h->ev_done);
    for (auto& e : h->sh.rev_)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : h->sh.xev)
        if (e) (void)hipEventDestroy(e);
    if (h->sh.ring) (void)hipFree(h->sh.ring);
    delete h->sh.xport;
    h->sh.xport = nullptr;
    if (h->stream && h->stream != h->own_stream) (void)hipStreamSynchronize(h->stream);
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    if (h->cstream) {
        (void)hipStreamSynchronize(h->cstream);
        (void)hipStreamDestroy(h->cstream);
    }
    delete h;
    return PSIM_OK;
}

int psim_device_info(const psim_handle* h, char* buf, size_t cap) {
    if (!h || !buf || !cap) return PSIM_EINVAL;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, h->device) != hipSuccess) return PSIM_EHIP;
    // the marketing name is empty on some ROCm installs (the r04 bench line
    // printed " (gfx950...)"): the arch, CU count and HBM size name the part
    snprintf(buf, cap, "%s (%s, %d CUs, %.0f GB HBM)", p.name[0] ? p.name : "AMD Instinct GPU", p.gcnArchName,
             p.multiProcessorCount, double(p.totalGlobalMem) / 1e9);
    return PSIM_OK;
}

int psim_load_csr(psim_handle* h, uint32_t n, const uint64_t* row_ptr, const uint32_t* col, uint64_t col_len) {
    if (!h || !row_ptr || (!col && col_len)) return PSIM_EINVAL;
    if (row_ptr[0] != 0 || row_ptr[n] != col_len)
        return fail(h, PSIM_EINVAL, "row_ptr[0]=%llu, row_ptr[n]=%llu, col_len=%llu", (unsigned long long)row_ptr[0],
                    (unsigned long long)row_ptr[n], (unsigned long long)col_len);
    for (uint32_t v = 0; v < n; v++)     // before any col access: every row lies inside col[0, col_len)
        if (row_ptr[v + 1] < row_ptr[v]) return fail(h, PSIM_EINVAL, "row_ptr not monotone at %u", v);
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    free_graph(h);
    // symmetrise: peers(v) = members(v) U {u : v in members(u)}, minus self
    std::vector<uint64_t> cnt(size_t(n) + 1, 0);
    for (uint32_t v = 0; v < n; v++) {
        for (uint64_t e = row_ptr[v]; e < row_ptr[v + 1]; e++) {
            const uint32_t u = col[e];
            if (u >= n) return fail(h, PSIM_EINVAL, "col[%llu]=%u >= n", (unsigned long long)e, u);
            if (u == v) continue;
            cnt[v + 1]++;
            cnt[u + 1]++;
        }
    }
    for (uint32_t v = 0; v < n; v++) cnt[v + 1] += cnt[v];
    std::vector<uint32_t> tmp(cnt[n]);
    {
        std::vector<uint64_t> fill(cnt.begin(), cnt.end() - 1);
        for (uint32_t v = 0; v < n; v++)
            for (uint64_t e = row_ptr[v]; e < row_ptr[v + 1]; e++) {
                const uint32_t u = col[e];
                if (u == v) continue;
                tmp[fill[v]++] = u;
                tmp[fill[u]++] = v;
            }
    }
    std::vector<uint64_t> rp(size_t(n) + 1, 0);
    std::vector<uint32_t> cc;
    cc.reserve(tmp.size() / 2 + 16);
    for (uint32_t v = 0; v < n; v++) {
        uint32_t* b = tmp.data() + cnt[v];
        uint32_t* e = tmp.data() + cnt[v + 1];
        std::sort(b, e);
        uint32_t* u = std::unique(b, e);
        const uint64_t d = uint64_t(u - b);
        if (d > uint64_t(kMaxDeg))
            return fail(h, PSIM_EINVAL, "vertex %u has %llu peers (limit %d)", v, (unsigned long long)d, kMaxDeg);
        cc.insert(cc.end(), b, u);
        rp[v + 1] = rp[v] + d;
    }
    tmp.clear();
    tmp.shrink_to_fit();
    const uint64_t E = rp[n];
    if (E >= 0xFFFFFFFFull) return fail(h, PSIM_EINVAL, "too many peer slots (%llu)", (unsigned long long)E);
    std::vector<uint32_t> rp32(size_t(n) + 1), rev(E), memb(n, 0u);
    for (uint32_t v = 0; v <= n; v++) rp32[v] = uint32_t(rp[v]);
    for (uint32_t v = 0; v < n; v++)
        for (uint64_t e = rp[v]; e < rp[v + 1]; e++) {
            const uint32_t u = cc[e];
            const uint32_t* b = cc.data() + rp[u];
            const uint32_t* x = std::lower_bound(b, b + (rp[u + 1] - rp[u]), v);
            rev[e] = uint32_t(x - cc.data());
        }
    for (uint32_t v = 0; v < n; v++)
        for (uint64_t e = row_ptr[v]; e < row_ptr[v + 1]; e++) {
            const uint32_t u = col[e];
            if (u == v) continue;
            const uint32_t* b = cc.data() + rp[v];
            const uint32_t* x = std::lower_bound(b, b + (rp[v + 1] - rp[v]), u);
            memb[v] |= 1u << uint32_t(x - b);
        }
    // this process's shard: contiguous vertex range [lo, hi)
    auto& sh = h->sh;
    const uint32_t W = (uint32_t)sh.world;
    const uint32_t lo = uint32_t((uint64_t(n) * sh.rank) / W), hi = uint32_t((uint64_t(n) * (sh.rank + 1)) / W);
    const uint32_t nl = hi - lo;
    const uint64_t sbase = rp[lo], El = rp[hi] - rp[lo];
    auto owner = [&](uint32_t u) -> uint32_t {      // inverse of the range split
        uint32_t d = uint32_t((uint64_t(u) * W) / n);
        while (d + 1 < W && u >= uint32_t((uint64_t(n) * (d + 1)) / W)) d++;
        while (d > 0 && u < uint32_t((uint64_t(n) * d) / W)) d--;
        return d;
    };
    std::vector<uint32_t> rpl(size_t(nl) + 1), cl(El), rvl(El), mbl(nl), s2v(El), cl_dev, rv_dev;
    for (uint32_t v = 0; v <= nl; v++) rpl[v] = uint32_t(rp[lo + v] - sbase);
    for (uint64_t e = 0; e < El; e++) { cl[e] = cc[sbase + e]; rvl[e] = rev[sbase + e]; }
    for (uint32_t v = 0; v < nl; v++) {
        mbl[v] = memb[lo + v];
        for (uint32_t e = rpl[v]; e < rpl[v + 1]; e++) s2v[e] = v;
    }
    // ELL rows: with the slot-scatter engine and every degree
    // <= kEllMax, slot s of v is v*Wd + s (Wd = the maximum degree over the
    // WHOLE overlay, so every shard derives the same global slot ids), and the
    // round kernel finds a vertex's inbox words without reading rowp.  Device
    // slot ids are then ELL ids; the ABI keeps CSR slot ids (getters convert).
    uint32_t ell = 0;
    if (!(h->cfg.flags & (PSIM_CFG_BINNED | PSIM_CFG_CSR))) {
        uint64_t mx = 0;
        for (uint32_t v = 0; v < n; v++) mx = std::max<uint64_t>(mx, rp[v + 1] - rp[v]);
        if (mx >= 1 && mx <= kEllMax) ell = uint32_t(mx);
    }
    const uint64_t Ed = ell ? uint64_t(nl) * ell : El;
    if (ell && uint64_t(n) * ell >= 0xFFFFFFFFull)
        return fail(h, PSIM_EINVAL, "too many ELL slots (%llu)", (unsigned long long)(uint64_t(n) * ell));
    // local CSR slot e of local vertex v -> device slot (identity for CSR rows)
    auto dslot = [&](uint32_t v, uint64_t e) -> uint32_t { return ell ? v * ell + uint32_t(e - rpl[v]) : uint32_t(e); };
    // remote slots grouped by destination shard, and the compaction blocks
    std::vector<std::vector<uint32_t>> remd(W);
    if (W > 1)
        for (uint64_t e = 0; e < El; e++) {
            const uint32_t d = owner(cl[e]);
            if (d != (uint32_t)sh.rank) remd[d].push_back(dslot(s2v[e], e));
        }
    std::vector<uint32_t> remflat;
    std::vector<uint4> blks;
    std::vector<uint64_t> sbases(W + 1, 0);
    for (uint32_t d = 0; d < W; d++) {
        sbases[d] = remflat.size();
        for (size_t st = 0; st < remd[d].size(); st += kChunkV)
            blks.push_back(make_uint4(d, uint32_t(remflat.size() + st),
                                      uint32_t(std::min<size_t>(kChunkV, remd[d].size() - st)), 0u));
        remflat.insert(remflat.end(), remd[d].begin(), remd[d].end());
    }
    sbases[W] = remflat.size();
    // receive side: for each source shard in order, the local slots it feeds,
    // in the source's own slot order (= the order of its region for us)
    std::vector<uint32_t> recvflat;
    std::vector<uint64_t> rbases(W + 1, 0);
    if (W > 1)
        for (uint32_t src = 0; src < W; src++) {
            rbases[src] = recvflat.size();
            if (src == (uint32_t)sh.rank) continue;
            const uint32_t slo = uint32_t((uint64_t(n) * src) / W), shi = uint32_t((uint64_t(n) * (src + 1)) / W);
            for (uint64_t e = rp[slo]; e < rp[shi]; e++)
                if (cc[e] >= lo && cc[e] < hi) recvflat.push_back(dslot(cc[e] - lo, rev[e] - sbase));
        }
    rbases[W] = recvflat.size();
    std::vector<uint32_t> ep;
    if (ell) {
        // reverse slot of local slot e: global ELL id of (receiver cl[e], its
        // CSR position rev - rp[receiver]); packed rows hold col << 3 | position
        std::vector<uint32_t> ce(Ed, kNoPeer), re(Ed, 0u);
        for (uint32_t v = 0; v < nl; v++)
            for (uint32_t e = rpl[v]; e < rpl[v + 1]; e++) {
                const uint32_t u = cl[e];
                ce[dslot(v, e)] = u;
                re[dslot(v, e)] = u * ell + uint32_t(rvl[e] - rp[u]);
            }
        if (n < (1u << 29) - 1) {                          // packed rows for the ELL round kernel
            ep.resize(Ed);
            for (uint64_t e = 0; e < Ed; e++)
                ep[e] = ce[e] == kNoPeer ? kNoPeer : (ce[e] << 3) | (re[e] - ce[e] * ell);
        }
        cl_dev.swap(ce);
        rv_dev.swap(re);
        if (W > 1) {                                       // receiver vertex of a device slot
            s2v.resize(Ed);
            for (uint64_t e = 0; e < Ed; e++) s2v[e] = uint32_t(e / ell);
        }
    }
    const std::vector<uint32_t>& cl_up = ell ? cl_dev : cl;
    const std::vector<uint32_t>& rv_up = ell ? rv_dev : rvl;
    // device arrays
    auto alloc = [&](void** p, size_t bytes) -> hipError_t { return hipMalloc(p, bytes ? bytes : 4); };
    const size_t nw = (size_t(n) + 31) / 32;
    const size_t ng = (size_t(nl) + (1u << kGroupShift) - 1) >> kGroupShift;
    const bool binned = W == 1 && (h->cfg.flags & PSIM_CFG_BINNED);
    // worklist of the sparse rounds (ELL rows on one GPU): 64 shards of
    // ng / 16 groups each after the flag bytes; an overflowing shard only
    // sends the next round back to the flags
    const size_t wl_off = (ng + 15) & ~size_t(15);
    const bool wl_on = ell && !getenv("PSIM_NO_WORKLIST");   // A/B switch
    uint32_t wl_cap = wl_on ? std::max<uint32_t>(64u, uint32_t((ng + 15) / 16)) : 0u;
    if (wl_on && getenv("PSIM_WL_CAP"))          // test knob: tiny shards exercise the overflow fallback
        wl_cap = std::max<uint32_t>(1u, uint32_t(strtoul(getenv("PSIM_WL_CAP"), nullptr, 10)));
    const size_t pend_bytes = wl_off + size_t(64) * wl_cap * 4;
    auto& bn = h->bin;
    if (binned) {
        if (!bin_geometry(rpl, nl, bn.fv_shift, bn.cv_shift, bn.nf, bn.nc))
            return fail(h, PSIM_EINVAL, "overlay does not fit the binned engine (drop PSIM_CFG_BINNED)");
        // sub-region (c, s) holds the records fine bins f = s (mod kCoarseShards)
        // send into coarse bin c: at most their slots whose peer lies in c
        const size_t NS = size_t(bn.nc) * kCoarseShards;
        std::vector<uint32_t> cap(NS, 0u);
        for (uint32_t v = 0; v < nl; v++) {
            const uint32_t sh = (v >> bn.fv_shift) & (kCoarseShards - 1);
            for (uint32_t e = rpl[v]; e < rpl[v + 1]; e++) cap[size_t(cl[e] >> bn.cv_shift) * kCoarseShards + sh]++;
        }
        bn.h_csub.assign(NS + 1, 0u);
        uint32_t mx = 0;
        for (size_t i = 0; i < NS; i++) {
            bn.h_csub[i + 1] = bn.h_csub[i] + cap[i];
            mx = std::max(mx, cap[i]);
        }
        bn.chunks = std::max<uint32_t>(1u, (mx + kRouteK - 1) / kRouteK);
        bn.h_fslot.resize(size_t(bn.nf) + 1);
        for (uint32_t f = 0; f <= bn.nf; f++) bn.h_fslot[f] = rpl[std::min<uint64_t>(nl, uint64_t(f) << bn.fv_shift)];
    }
    const bool forest = h->fo.on;       // the per-lane arrays live in the forest's slabs
    if (alloc((void**)&h->rowp, (size_t(nl) + 1) * 4) != hipSuccess || alloc((void**)&h->col, Ed * 4) != hipSuccess ||
        alloc((void**)&h->rev, Ed * 4) != hipSuccess || alloc((void**)&h->memb, size_t(nl + 1) * 4) != hipSuccess ||
        (!ep.empty() && alloc((void**)&h->ecol, Ed * 4) != hipSuccess) ||
        alloc((void**)&h->alive, nw * 4) != hipSuccess || (!forest && alloc((void**)&h->vs, size_t(nl) * 16) != hipSuccess) ||
        (!binned && !forest &&
         (alloc((void**)&h->in[0], Ed * 4) != hipSuccess || alloc((void**)&h->in[1], Ed * 4) != hipSuccess ||
          alloc((void**)&h->pend[0], pend_bytes) != hipSuccess || alloc((void**)&h->pend[1], pend_bytes) != hipSuccess)) ||
        (binned && (alloc((void**)&bn.rec_c, El * 8) != hipSuccess || alloc((void**)&bn.rec_f, El * 8) != hipSuccess ||
                    alloc((void**)&bn.cnt_c[0], size_t(bn.nc) * kCoarseShards * 4) != hipSuccess ||
                    alloc((void**)&bn.cnt_c[1], size_t(bn.nc) * kCoarseShards * 4) != hipSuccess ||
                    alloc((void**)&bn.cnt_f, size_t(bn.nf) * 4) != hipSuccess ||
                    alloc((void**)&bn.csub, bn.h_csub.size() * 4) != hipSuccess ||
                    alloc((void**)&bn.fslot, (size_t(bn.nf) + 1) * 4) != hipSuccess ||
                    alloc((void**)&bn.obin, size_t(bn.nf) * 4) != hipSuccess)) ||
        (!forest && alloc((void**)&h->ost, size_t(nl) + 4) != hipSuccess) ||
        (W > 1 && (alloc((void**)&sh.stage, Ed * 4) != hipSuccess ||
                   alloc((void**)&sh.rem, remflat.size() * 4) != hipSuccess ||
                   alloc((void**)&sh.blk, blks.size() * 16) != hipSuccess ||
                   alloc((void**)&sh.send_base_d, W * 4) != hipSuccess ||
                   alloc((void**)&sh.cursor, W * 4) != hipSuccess ||
                   alloc((void**)&sh.slot2v, Ed * 4) != hipSuccess ||
                   alloc((void**)&sh.recv_map, recvflat.size() * 4) != hipSuccess))) {
        free_graph(h);
        return fail(h, PSIM_ENOMEM, "device allocation failed for n=%u E=%llu", nl, (unsigned long long)El);
    }
    h->n = nl;
    h->E = El;
    h->Ed = Ed;
    h->ell = ell;
    h->ell_grid = ell ? ell_round_grid(ell, h->device) : 0u;
#ifdef PSIM_ELL_GRID_ENV
    // A/B builds only (make variant DEFS=-DPSIM_ELL_GRID_ENV): the round kernel's grid from the
    // environment (0: one workgroup per chunk); the grid changes no result, only the schedule
    if (ell && getenv("PSIM_ELL_GRID")) h->ell_grid = uint32_t(strtoul(getenv("PSIM_ELL_GRID"), nullptr, 10));
#endif
    {
        uint64_t mx = 0;                               // the same on every shard: the whole overlay
        for (uint32_t v = 0; v < n; v++) mx = std::max<uint64_t>(mx, rp[v + 1] - rp[v]);
        sh.max_deg_g = uint32_t(mx);
        // a sparse round sends records while the bound stays under a quarter of
        // a peer pair's dense region (~ n deg / W^2 words): 8-byte records
        sh.rec_thr = W > 1 ? std::max<uint64_t>(64, uint64_t(n) * std::max<uint64_t>(1, mx) / (8ull * W * W)) : 0;
    }
    h->pend_bytes = pend_bytes;
    h->wl_thr = getenv("PSIM_WL_THR") ? uint32_t(strtoul(getenv("PSIM_WL_THR"), nullptr, 10)) : 0u;
    h->dense_div = std::max<uint32_t>(1u, getenv("PSIM_DENSE_DIV") ? uint32_t(strtoul(getenv("PSIM_DENSE_DIV"), nullptr, 10))
                                                                   : 4u);
    h->wl_gpc = getenv("PSIM_WL_GPC") ? uint32_t(strtoul(getenv("PSIM_WL_GPC"), nullptr, 10)) : 0u;
    h->wl_wgs = getenv("PSIM_WL_WGS") ? uint32_t(strtoul(getenv("PSIM_WL_WGS"), nullptr, 10)) : 256u;
    h->wl_off = wl_off;
    h->wl_cap = wl_cap;
    sh.n_global = n;
    sh.v_lo = lo;
    sh.slot_base = sbase;
    sh.dev_slot_base = ell ? uint64_t(lo) * ell : sbase;
    HIPCHK(h, hipMemcpy(h->rowp, rpl.data(), (size_t(nl) + 1) * 4, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(h->col, cl_up.data(), Ed * 4, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(h->rev, rv_up.data(), Ed * 4, hipMemcpyHostToDevice));
    if (!ep.empty()) HIPCHK(h, hipMemcpy(h->ecol, ep.data(), Ed * 4, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(h->memb, mbl.data(), size_t(nl) * 4, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemset(h->alive, 0xFF, nw * 4));
    // state: epoch tag 0 != h->epoch -> common sets; delivered tag never matches serial 1..
    if (!forest) HIPCHK(h, hipMemset(h->vs, 0, size_t(nl) * 16));
    if (binned) {
        HIPCHK(h, hipMemset(bn.cnt_c[0], 0, size_t(bn.nc) * kCoarseShards * 4));
        HIPCHK(h, hipMemset(bn.cnt_c[1], 0, size_t(bn.nc) * kCoarseShards * 4));
        HIPCHK(h, hipMemset(bn.cnt_f, 0, size_t(bn.nf) * 4));
        HIPCHK(h, hipMemset(bn.obin, 0, size_t(bn.nf) * 4));
        HIPCHK(h, hipMemcpy(bn.csub, bn.h_csub.data(), bn.h_csub.size() * 4, hipMemcpyHostToDevice));
        HIPCHK(h, hipMemcpy(bn.fslot, bn.h_fslot.data(), (size_t(bn.nf) + 1) * 4, hipMemcpyHostToDevice));
    } else if (!forest) {
        HIPCHK(h, hipMemset(h->in[0], 0, Ed * 4));
        HIPCHK(h, hipMemset(h->in[1], 0, Ed * 4));
        HIPCHK(h, hipMemset(h->pend[0], 0, ng));
        HIPCHK(h, hipMemset(h->pend[1], 0, ng));
    }
    if (!forest) HIPCHK(h, hipMemset(h->ost, 0, size_t(nl) + 4));
    HIPCHK(h, hipMemset(h->ost_total_base, 0, kMaxLanes * 4 * sizeof(int)));
    HIPCHK(h, hipMemset(h->mcnt_base, 0, kMaxLanes * kMcntLane * sizeof(uint32_t)));
    h->ost_total = h->ost_total_base;
    h->lanes.assign(forest ? 0 : 1, psim_handle::Lane());
    h->cur_lane = 0;
    if (W > 1) {
        std::vector<uint32_t> sb32(W);
        for (uint32_t d = 0; d < W; d++) sb32[d] = uint32_t(sbases[d]);
        HIPCHK(h, hipMemset(sh.stage, 0, Ed * 4));
        HIPCHK(h, hipMemcpy(sh.rem, remflat.data(), remflat.size() * 4, hipMemcpyHostToDevice));
        HIPCHK(h, hipMemcpy(sh.blk, blks.data(), blks.size() * 16, hipMemcpyHostToDevice));
        HIPCHK(h, hipMemcpy(sh.send_base_d, sb32.data(), W * 4, hipMemcpyHostToDevice));
        HIPCHK(h, hipMemcpy(sh.slot2v, s2v.data(), Ed * 4, hipMemcpyHostToDevice));
        if (!recvflat.empty())
            HIPCHK(h, hipMemcpy(sh.recv_map, recvflat.data(), recvflat.size() * 4, hipMemcpyHostToDevice));
        sh.nblk = uint32_t(blks.size());
    }
    sh.send_base = sbases;
    sh.recv_base = rbases;
    HIPCHK(h, hipDeviceSynchronize());
    {
        std::vector<uint64_t> rpl64(size_t(nl) + 1);
        for (uint32_t v = 0; v <= nl; v++) rpl64[v] = rpl[v];
        h->h_rowp = std::move(rpl64);
    }
    h->h_col = std::move(cl);
    h->h_memb = std::move(mbl);
    h->par = 0;
    h->round = 0;
    h->scrub = 0;
    h->serial = 0;
    h->epoch = 1;
    h->have_root = false;
    h->mono_of.clear();
    h->next_epoch.clear();
    h->ost_cnt = h->live_rows = 0;
    h->inflight = 0;
    if (forest) return forest_alloc(h);
    return PSIM_OK;
}

int psim_num_slots(const psim_handle* h, uint64_t* out) {
    if (!h || !out) return PSIM_EINVAL;
    *out = h->E;
    return PSIM_OK;
}

int psim_get_slots(const psim_handle* h, uint64_t* row_ptr, uint32_t* col) {
    if (!h || !h->n) return PSIM_EINVAL;
    if (row_ptr) memcpy(row_ptr, h->h_rowp.data(), (size_t(h->n) + 1) * 8);
    if (col) memcpy(col, h->h_col.data(), h->E * 4);
    return PSIM_OK;
}

int psim_set_alive(psim_handle* h, const uint8_t* alive, size_t n) {
    if (!h || !alive || n != h->sh.n_global || !h->n) return PSIM_EINVAL;
    std::vector<uint32_t> bm((n + 31) / 32, 0u);
    for (size_t v = 0; v < n; v++)
        if (alive[v]) bm[v >> 5] |= 1u << (v & 31);
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipMemcpyAsync(h->alive, bm.data(), bm.size() * 4, hipMemcpyHostToDevice, h->stream));
    if (h->fo.on) {                  // outstanding rows to live peers, over every root's lane
        HIPCHK(h, hipMemsetAsync(h->scratch, 0, 8, h->stream));
        const FoArgs fa = forest_args(h, h->par, 0, h->stats, h->round + 1);
        HIPCHK(h, launch_fo_count_live(fa, h->scratch, h->stream));
        unsigned long long live = 0;
        HIPCHK(h, hipMemcpyAsync(&live, h->scratch, 8, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        h->live_rows = (int64_t)live;
        return PSIM_OK;
    }
    const int focus = h->cur_lane;
    for (int j = 0; j < (int)h->lanes.size(); j++) {   // outstanding rows to live peers, per lane
        swap_lane(h, j);
        HIPCHK(h, hipMemsetAsync(h->scratch, 0, 8, h->stream));
        PtArgs a = make_args(h, h->par, 0, h->stats);
        HIPCHK(h, launch_pt_count_live(a, h->scratch, h->stream));
        unsigned long long live = 0;
        HIPCHK(h, hipMemcpyAsync(&live, h->scratch, 8, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        h->live_rows = (int64_t)live;
    }
    swap_lane(h, focus);
    return PSIM_OK;
}

int psim_plumtree_restart_backend(psim_handle* h, uint32_t v) {
    if (!h || !h->n) return PSIM_ESTATE;
    if (v >= h->sh.n_global) return PSIM_EINVAL;
    if (h->bin.rec_c) return fail(h, PSIM_ENOTSUP, "binned handles keep one epoch per root");
    HIPCHK(h, hipSetDevice(h->device));
    const auto it = h->mono_of.find(v);
    const uint32_t cur = it == h->mono_of.end() ? 0u : it->second >> 24;
    const auto ne = h->next_epoch.find(v);
    const uint32_t e = (ne == h->next_epoch.end() ? cur : ne->second) + 1u;
    if (e > 0xFFu) return fail(h, PSIM_EOVERFLOW, "vertex %u: 255 backend restarts", v);
    const uint32_t lv = v - h->sh.v_lo;
    if (h->fo.on) {
        // a static lane keeps one heartbeat per vertex: v may not forget one
        // that is still in flight (the ≤ 16-lane handles turn the lane into a
        // window lane instead)
        if (!quiescent(h)) return fail(h, PSIM_EBUSY, "forest: backend restart while heartbeats are in flight");
        const FoArgs fa = forest_args(h, h->par, 0, h->stats, h->round + 1);
        HIPCHK(h, launch_fo_forget(fa, lv, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        h->next_epoch[v] = e;
        return PSIM_OK;
    }
    const int focus = h->cur_lane;
    if (!h->lanes.empty()) save_lane(h);
    const int nl = h->lanes.empty() ? 1 : (int)h->lanes.size();
    for (int j = 0; j < nl; j++) {            // v forgets every origin: each lane's root
        if (!h->lanes.empty()) load_lane(h, j);
        if (!h->have_root) continue;
        if (!quiescent(h) && win_capable(h) && !h->win) {
            // v may deliver the heartbeat in flight again and hold a second
            // row per peer for it: the lane keeps every row from then on
            // (every shard decides alike: quiescent() is the global count)
            const int rc = to_window(h);
            if (rc) { save_lane(h); load_lane(h, focus); return rc; }
            save_lane(h);
        }
        if (lv < h->n)
            HIPCHK(h, launch_pt_forget(h->vs, h->win ? h->win->iset : nullptr, lv, (h->serial - 1u) & 0xFFu, h->stream));
    }
    if (!h->lanes.empty()) load_lane(h, focus);
    HIPCHK(h, hipStreamSynchronize(h->stream));
    h->next_epoch[v] = e;     // only once every lane forgot: a failed restart leaves the epoch alone
    return PSIM_OK;
}

int psim_plumtree_reset_trees(psim_handle* h) {
    if (!h || !h->n) return PSIM_ESTATE;
    HIPCHK(h, hipSetDevice(h->device));
    h->epoch++;
    if ((h->epoch & 0x7Fu) == 0) {
        int rc = renorm_if_needed(h);
        if (rc) return rc;
    }
    return PSIM_OK;
}

}  // extern "C"

namespace {

int ingest_dense(psim_handle* h, const void* recv_dev, bool force_flags = false);

// The split-phase sharded entry points drive the focused lane's words only.
int one_lane_only(psim_handle* h) {
    if (h->lanes.size() > 1 || h->win)
        return fail(h, PSIM_ENOTSUP, "several heartbeat lanes or a window lane: drive with psim_shard_broadcast_x / "
                                    "psim_shard_run / psim_shard_step");
    return PSIM_OK;
}

// Shared by psim_plumtree_broadcast and psim_shard_broadcast: every shard
// advances the same serial / epoch / Monotonic; only the root's owner runs
// the origin kernel.  Returns the origin's emitted-message stats row.
int broadcast_common(psim_handle* h, uint32_t root, uint32_t* mono_out, unsigned long long* r, bool defer = false) {
    if (!h || !h->n) return PSIM_ESTATE;
    if (root >= h->sh.n_global) return PSIM_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    if (lanes_enabled(h)) {                 // each root heartbeats over its own lane
        const int rc = focus_root(h, root, true);
        if (rc) return rc;
    }
    if (!quiescent(h) || (rows_held(h) > 0 && win_capable(h) && !h->win)) {
        // the root heartbeats again while its last heartbeat is in flight
        // (backend :341-368), or rows of it wait for a dead peer: its lane
        // keeps every heartbeat apart from then on
        if (!win_capable(h))
            return fail(h, PSIM_EBUSY, "previous broadcast of this root still in flight (sharded, binned or "
                                       "delay-fault handles keep one heartbeat per root)");
        if (!h->win) {
            const int rc = to_window(h);
            if (rc) return rc;
        }
    }
    if (!lanes_enabled(h) && h->have_root && root != h->root) {
        // single-root engine: the previous root's per-root sets are dropped
        // (DESIGN.md "Limitations": multi-root trees are SURVEY 8(f) row 1)
        h->epoch++;
    }
    h->root = root;
    h->have_root = true;
    h->serial++;
    if ((h->serial & 0x7Fu) == 0 || (h->epoch & 0x7Fu) == 0) {
        int rc = renorm_if_needed(h);
        if (rc) return rc;
    }
    uint32_t& mono = h->mono_of[root];
    const auto ne = h->next_epoch.find(root);
    if (ne != h->next_epoch.end()) {          // the first heartbeat of a restarted backend (init/1: monotonic 0)
        mono = (ne->second << 24) | 1u;
        h->next_epoch.erase(ne);
    } else {
        // Monotonic 2^24-1 is never an id (a probe for "the row's epoch is newer")
        if ((mono & 0xFFFFFFu) >= 0xFFFFFEu) return fail(h, PSIM_EOVERFLOW, "root %u: 2^24-2 heartbeats in one epoch", root);
        mono++;
    }
    if (mono_out) *mono_out = mono;
    for (int i = 0; i < kNStat; i++) r[i] = 0;
    const uint32_t lr = root - h->sh.v_lo;
    if (lr < h->n) {
        if (h->win) {                           // window lane: records for the next round
            HIPCHK(h, hipMemsetAsync(h->stats, 0, kStatsRow * sizeof(unsigned long long), h->stream));
            WinArgs a = make_win_args(h, h->par, 0, h->stats);
            a.out = h->win->msg[h->par];
            a.nout = h->win->nmsg + h->par;
            HIPCHK(h, launch_win_origin(a, lr, h->stream));
        } else {
            // origin emits into the buffer the next round reads; its kernel
            // first zeroes its stats row and the lane's count area and seeds
            // the hold ring with the holders before the origin's own change
            PtArgs a = make_args(h, h->par ^ 1u, 0, h->stats);      // row 0 (a deferred one: drive reads it)
            set_round_slots(h, a, h->round + 1);     // the origin's pushes count as round h->round's
            a.wtag = uint32_t(h->round + 1) & 0xFFu; // read by the next round
            a.root = lr;
            HIPCHK(h, launch_pt_origin(a, h->stream, uint32_t(kStatsRow), uint32_t(h->ost_cnt)));
            if (defer) {                        // read back with the first chunk of rounds (drive)
                h->origin_pend = true;
                return PSIM_OK;
            }
        }
        HIPCHK(h, hipMemcpyAsync(h->h_stats, h->stats, kStatsRow * sizeof(unsigned long long),
                                 hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, chunk_wait(h));
        reduce_row(h->h_stats, r);
        if (r[S_OVERFLOW])
            return fail(h, PSIM_EOVERFLOW, "origin: overflow flags 0x%llx (4: outstanding rows of an older heartbeat; "
                        "window lanes: 32: > 32 rows, 64: > 4 timestamp intervals)", r[S_OVERFLOW]);
    }
    h->ost_cnt += (int64_t)r[S_OST_DELTA];
    h->live_rows += (int64_t)r[S_LIVE_DELTA];
    h->inflight = (h->win ? h->inflight : 0) + r[PSIM_MSG_BROADCAST];
    if (h->dly) h->inflight = lr < h->n ? add_due(h->due, h->round, h->h_stats + size_t(kStatShards) * kNStat) : 0;
    return PSIM_OK;
}

// Pack this shard's staged cross-shard words into the caller's device buffer
// (regions at psim_shard_layout offsets); counts[d] = records for shard d.
int shard_pack(psim_handle* h, void* send_dev, uint64_t send_cap, uint64_t* counts) {
    auto& sh = h->sh;
    const uint32_t W = (uint32_t)sh.world;
    for (uint32_t d = 0; d < W; d++) counts[d] = 0;
    if (W == 1) return PSIM_OK;
    if (send_cap < sh.send_base[W] || (!send_dev && sh.send_base[W]))
        return fail(h, PSIM_EINVAL, "send buffer holds %llu records, layout needs %llu",
                    (unsigned long long)send_cap, (unsigned long long)sh.send_base[W]);
    HIPCHK(h, hipMemsetAsync(sh.cursor, 0, W * 4, h->stream));
    PtArgs a = make_args(h, h->par, 0, h->stats);
    HIPCHK(h, launch_pt_compact(a, sh.rem, sh.blk, sh.nblk, sh.send_base_d, sh.cursor, (uint2*)send_dev, h->stream));
    std::vector<uint32_t> c(W);
    HIPCHK(h, hipMemcpyAsync(c.data(), sh.cursor, W * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    for (uint32_t d = 0; d < W; d++) counts[d] = c[d];
    return PSIM_OK;
}

// ---- heartbeat intervals back to back (psim_plumtree_broadcast_run_n) ------
// Between two calls of psim_plumtree_broadcast_run the device idles while the
// host reads the interval back, returns to its caller and launches the next
// origin (~60 us a 10M-peer interval of ~2 ms, profiles/r05/experiments).
// Here interval i + 1 is enqueued BEFORE interval i is read back, on the
// prediction that i ends exactly after as many rounds as i - 1 did: its
// kernels carry a guard (PtArgs::spec) and its origin runs it only if the
// previous interval's last predicted round sent nothing, the one before sent
// something and no vertex holds a row -- the host's own quiescence test on
// the same counts.  The host repeats the test when it reads interval i back:
// on a miss the device has abandoned i + 1 (every kernel of it returned at
// once), the host undoes i + 1's bookkeeping, finishes i with the plain
// driver if it needs more rounds, and goes on.  Only the plain single-root
// handle pipelines (one lane on one GPU, no delays, no window lane, chunk
// timing); an interval that would renormalise tags or scrub the inbox, and
// every other handle, take the plain calls.
constexpr uint32_t kPipeRegion = 32;   // stats rows per interval slot: the origin's, then <= kChunk rounds'
static_assert(2 * kPipeRegion <= kChunk * kMaxLanes + 1, "two interval slots fit the stats rows");
static_assert(kDelayHist >= 2, "the spec words live in the origin row's delay histogram (no delays here)");

struct PipeRec {
    uint32_t region = 0, k = 0, mono = 0;
    uint64_t round0 = 0;     // h->round before the interval's first round
    bool guarded = false;
};
struct PipeSnap {
    uint32_t epoch = 0, serial = 0, mono = 0, par = 0;
};

unsigned long long* pipe_rows(psim_handle* h, uint32_t r) { return h->stats + size_t(r) * kPipeRegion * kStatsRow; }
unsigned long long* pipe_hrows(psim_handle* h, uint32_t r) { return h->h_stats + size_t(r) * kPipeRegion * kStatsRow; }
// the guard's words: the origin row's delay histogram, unused without delay
// faults -- read back with the rows, never zeroed by the origin's prep
uint32_t* pipe_spec(unsigned long long* rows) { return reinterpret_cast<uint32_t*>(rows + size_t(kStatShards) * kNStat); }

// the interval starting after round round0 with k rounds can be enqueued
// without a wait (`guarded`: before the previous one is read back)
bool pipe_ok(const psim_handle* h, uint32_t root, bool reset, uint64_t round0, uint32_t k, bool guarded) {
    if (h->sh.world != 1 || h->fo.on || h->dly || h->bin.rec_c || h->win || !h->mcnt_base) return false;
    if (!(h->cfg.flags & PSIM_CFG_CHUNK_TIMING)) return false;
    if (h->lanes.size() != 1 || h->cur_lane != 0 || !h->have_root || h->root != root) return false;
    if (root - h->sh.v_lo >= h->n || h->next_epoch.count(root)) return false;
    if (k == 0 || k > kChunk) return false;
    const uint32_t ep = h->epoch + (reset ? 1u : 0u);
    if (((h->serial + 1u) & 0x7Fu) == 0 || (ep & 0x7Fu) == 0) return false;        // would renormalise tags
    const auto it = h->mono_of.find(root);
    if (it == h->mono_of.end() || (it->second & 0xFFFFFFu) >= 0xFFFFFEu) return false;
    if (round0 + k + 1 >= h->scrub + kTagSpan) return false;                         // would scrub the inbox
    return guarded || (h->inflight == 0 && h->live_rows == 0 && h->ost_cnt == 0);   // exact state: quiescent
}

// reset_trees + the origin + k rounds + the read-back copies, with no wait
int pipe_enqueue(psim_handle* h, uint32_t root, bool reset, uint32_t k, uint32_t region, bool guarded,
                 uint64_t round0, PipeRec& rec) {
    if (reset) h->epoch++;
    h->serial++;
    uint32_t& mono = h->mono_of[root];
    mono++;
    rec.mono = mono;
    rec.region = region;
    rec.k = k;
    rec.round0 = round0;
    rec.guarded = guarded;
    unsigned long long* rows = pipe_rows(h, region);
    uint32_t* spec = pipe_spec(rows);                    // the origin writes both words (no memset)
    if (!h->cstream && hipStreamCreateWithFlags(&h->cstream, hipStreamNonBlocking) != hipSuccess) {
        h->cstream = nullptr;
        return fail(h, PSIM_EHIP, "run_n: copy stream");
    }
    const uint64_t round_now = h->round;
    h->round = round0;                                   // make_args / slots / tags of the interval's rounds
    struct Back {
        psim_handle* h;
        uint64_t r;
        ~Back() { h->round = r; }
    } back{h, round_now};
    PtArgs a = make_args(h, h->par ^ 1u, 0, rows);       // the origin: row 0, pushes for round round0 + 1
    set_round_slots(h, a, round0 + 1);
    a.wtag = uint32_t(round0 + 1) & 0xFFu;
    a.root = root - h->sh.v_lo;
    if (guarded) {
        a.spec = spec;
        a.spec_rl = uint32_t(round0 % 4);
    }
    // the interval starts with no row holder (guarded: the origin checks it);
    // its prep zeroes the row's counters, not the guard's words after them
    HIPCHK(h, launch_pt_origin(a, h->stream, uint32_t(kStatShards * kNStat), 0u));
    PtPrep pp{};
    pp.z = rows + kStatsRow;                             // the rounds' rows (the origin zeroed its own)
    pp.nz = uint64_t(k) * kStatsRow;
    HIPCHK(h, launch_pt_prep(pp, h->stream));
    const uint32_t L = h->cfg.lazy_tick_rounds ? h->cfg.lazy_tick_rounds : 1;
    HIPCHK(h, hipEventRecord(h->ev[2 * region], h->stream));
    for (uint32_t i = 0; i < k; i++) {
        const uint64_t R = round0 + i + 1;
        PtArgs ra = make_args(h, h->par, (R % L) == 0, rows + size_t(1 + i) * kStatsRow);
        set_round_slots(h, ra, R);
        set_round_tags(ra, R);
        if (guarded) ra.spec = spec;
        HIPCHK(h, launch_pt_round(ra, h->stream));
        h->par ^= 1u;
    }
    HIPCHK(h, hipEventRecord(h->ev[2 * region + 1], h->stream));
    // the read-back on a stream of its own, after the interval's last round:
    // the next interval's origin follows that round directly
    HIPCHK(h, hipStreamWaitEvent(h->cstream, h->ev[2 * region + 1], 0));
    HIPCHK(h, hipMemcpyAsync(pipe_hrows(h, region), rows, size_t(1 + k) * kStatsRow * sizeof(unsigned long long),
                             hipMemcpyDeviceToHost, h->cstream));
    HIPCHK(h, hipEventRecord(h->ev[4 + region], h->cstream));
    return PSIM_OK;
}

// Wait for an interval and read it back as drive() does: the origin's row,
// then its rounds up to the first quiescent one (the rest were no-ops).
// `before`: messages of the round before the last one counted (the origin's
// for a one-round interval) -- the guard's test, repeated on the host.
int pipe_collect(psim_handle* h, const PipeRec& rec, psim_round_stats* out, size_t cap, uint32_t& ran, bool& quiet,
                 uint64_t& before) {
    HIPCHK(h, event_wait(h->ev[4 + rec.region]));
    const unsigned long long* hr = pipe_hrows(h, rec.region);
    if (rec.guarded && pipe_spec(const_cast<unsigned long long*>(hr))[1] != 1u)
        return fail(h, PSIM_ESTATE, "pipelined heartbeat %u: the device abandoned an interval the host ran "
                                    "(guard 0x%x)", rec.mono, pipe_spec(const_cast<unsigned long long*>(hr))[1]);
    float chunk_ms = 0.f;
    HIPCHK(h, hipEventElapsedTime(&chunk_ms, h->ev[2 * rec.region], h->ev[2 * rec.region + 1]));
    unsigned long long r[kNStat];
    reduce_row(hr, r);
    if (r[S_OVERFLOW])
        return fail(h, PSIM_EOVERFLOW, "origin: overflow flags 0x%llx (4: outstanding rows of an older heartbeat)",
                    r[S_OVERFLOW]);
    h->ost_cnt += (int64_t)r[S_OST_DELTA];
    h->live_rows += (int64_t)r[S_LIVE_DELTA];
    h->inflight = r[PSIM_MSG_BROADCAST];
    ran = 0;
    quiet = quiescent(h);
    uint64_t prev = h->inflight;
    before = 0;
    for (uint32_t i = 0; i < rec.k && !quiet; i++) {
        reduce_row(hr + size_t(1 + i) * kStatsRow, r);
        if (r[S_OVERFLOW])
            return fail(h, PSIM_EOVERFLOW,
                        "round %llu: overflow flags 0x%llx (1: >4 msgs on one edge, 2: Round > 4095, "
                        "4: outstanding rows of an older heartbeat)", (unsigned long long)(h->round + 1), r[S_OVERFLOW]);
        uint64_t lm = 0;
        for (int t = 1; t <= 5; t++) lm += r[t];
        h->ost_cnt += (int64_t)r[S_OST_DELTA];
        h->live_rows += (int64_t)r[S_LIVE_DELTA];
        h->inflight = lm;
        const float ms = chunk_ms / float(rec.k);
        h->round++;
        h->kernel_ms_total += ms;
        h->rounds_total++;
        if (out && ran < cap) {
            psim_round_stats& o = out[ran];
            memset(&o, 0, sizeof o);
            for (int t = 1; t <= 5; t++) o.sent[t] = r[t];
            o.delivered_new = r[S_DELIV];
            o.active = r[S_ACTIVE];
            o.senders = r[S_SENDERS];
            o.sender_degree_sum = r[S_DEGSUM];
            o.outstanding_vertices = (uint64_t)h->ost_cnt;
            o.algo_bytes = 16ull * h->n + 8ull * r[S_SENDERS] + 4ull * r[S_DEGSUM] + 32ull * lm;
            o.words_stored = r[S_WORDS];
            o.kernel_ms = ms;
        }
        ran++;
        before = prev;
        prev = lm;
        quiet = quiescent(h);
    }
    return PSIM_OK;
}

int run_n(psim_handle* h, uint32_t root, uint32_t count, bool reset, uint32_t max_rounds, psim_round_stats* stats,
          size_t cap, uint32_t* rounds, uint32_t* monos, uint32_t* done) {
    if (!h->n) return fail(h, PSIM_ESTATE, "no overlay loaded");
    HIPCHK(h, hipSetDevice(h->device));
    size_t used = 0;
    uint32_t pred = 0;             // rounds the last interval ran (the next one's prediction)
    bool have_next = false;        // interval i + 1 enqueued, guarded, before interval i was read back
    PipeRec cur, next;
    PipeSnap snap;
    struct Sync {                  // the focused lane's record follows the handle's fields on every exit
        psim_handle* h;
        ~Sync() { if (!h->lanes.empty()) save_lane(h); }
    } sync{h};
    for (uint32_t i = 0; i < count; i++) {
        psim_round_stats* out = stats ? stats + used : nullptr;
        const size_t room = stats ? cap - used : 0;
        uint32_t ran = 0;
        if (have_next) {
            cur = next;
            have_next = false;
        } else if (pred && pred <= max_rounds && pipe_ok(h, root, reset, h->round, pred, false)) {
            const int rc = pipe_enqueue(h, root, reset, pred, i & 1u, false, h->round, cur);
            if (rc) return rc;
        } else {
            // the plain calls (the first interval, and any the pipeline does not cover)
            if (!h->lanes.empty()) save_lane(h);
            if (reset) {
                const int rc = psim_plumtree_reset_trees(h);
                if (rc) return rc;
            }
            uint32_t mono = 0;
            const int rc = psim_plumtree_broadcast_run(h, root, &mono, max_rounds, out, room, &ran);
            if (rc) return rc;
            used += std::min<size_t>(ran, room);
            if (rounds) rounds[i] = ran;
            if (monos) monos[i] = mono;
            if (done) *done = i + 1;
            pred = ran;
            continue;
        }
        // the next interval, on the prediction that this one takes cur.k rounds
        if (i + 1 < count && pipe_ok(h, root, reset, cur.round0 + cur.k, cur.k, true)) {
            const auto it = h->mono_of.find(root);
            snap = PipeSnap{h->epoch, h->serial, it->second, h->par};
            const int rc = pipe_enqueue(h, root, reset, cur.k, cur.region ^ 1u, true, cur.round0 + cur.k, next);
            if (rc) return rc;
            have_next = true;
        }
        bool quiet = false;
        uint64_t before = 0;
        int rc = pipe_collect(h, cur, out, room, ran, quiet, before);
        if (rc) return rc;
        if (have_next && !(quiet && ran == cur.k && before != 0 && h->ost_cnt == 0)) {
            // the device abandoned interval i + 1 (its guard saw the same counts): undo its bookkeeping
            h->epoch = snap.epoch;
            h->serial = snap.serial;
            h->mono_of[root] = snap.mono;
            h->par = snap.par;
            have_next = false;
            // the device must have made the same decision (spec[1] = 2: abandoned); a device
            // that ran the interval the host rolled back would leave the two states apart
            // (ADVICE r5).  Waiting for its read-back also orders it before anything later
            // writes those host rows.
            HIPCHK(h, event_wait(h->ev[4 + next.region]));
            const uint32_t dec = pipe_spec(pipe_hrows(h, next.region))[1];
            if (dec != 2u)
                return fail(h, PSIM_ESTATE, "pipelined heartbeat %u: the device ran an interval the host rolled back "
                                            "(guard 0x%x)", next.mono, dec);
        }
        if (!quiet && ran < max_rounds) {   // more rounds than predicted: the plain driver, chunk by chunk
            uint32_t more = 0;
            rc = drive(h, max_rounds - ran, out ? out + std::min<size_t>(ran, room) : nullptr,
                       room > ran ? room - ran : 0, true, &more);
            if (rc) return rc;
            ran += more;
        }
        used += std::min<size_t>(ran, room);
        if (rounds) rounds[i] = ran;
        if (monos) monos[i] = cur.mono;
        if (done) *done = i + 1;
        pred = ran;
    }
    return PSIM_OK;
}

}  // namespace

extern "C" {

int psim_plumtree_broadcast(psim_handle* h, uint32_t root, uint32_t* mono_out) {
    if (h && h->sh.world > 1) return fail(h, PSIM_ESTATE, "sharded handle: use psim_shard_broadcast");
    if (h && h->fo.on) return forest_broadcast(h, &root, 1, mono_out);
    unsigned long long r[kNStat];
    return broadcast_common(h, root, mono_out, r);
}

int psim_plumtree_broadcast_many(psim_handle* h, const uint32_t* roots, size_t k, uint32_t* monos_out) {
    if (!h) return PSIM_EINVAL;
    if (k && !roots) return PSIM_EINVAL;
    if (h->fo.on) return forest_broadcast(h, roots, k, monos_out);   // sharded: collective
    if (h->sh.world > 1) return fail(h, PSIM_ESTATE, "sharded handle: use psim_shard_broadcast_x per root");
    for (size_t i = 0; i < k; i++) {
        unsigned long long r[kNStat];
        const int rc = broadcast_common(h, roots[i], monos_out ? monos_out + i : nullptr, r);
        if (rc) return rc;
    }
    return PSIM_OK;
}

int psim_plumtree_broadcast_run(psim_handle* h, uint32_t root, uint32_t* mono_out, uint32_t max_rounds,
                                psim_round_stats* stats, size_t cap, uint32_t* rounds_run) {
    if (!h) return PSIM_EINVAL;
    if (h->sh.world > 1) return fail(h, PSIM_ESTATE, "sharded handle: use psim_shard_broadcast_x + psim_shard_run");
    if (h->fo.on) {
        const int rc = forest_broadcast(h, &root, 1, mono_out);
        if (rc) return rc;
        return forest_drive(h, max_rounds, stats, cap, true, rounds_run);
    }
    unsigned long long r[kNStat];
    // delay faults account the origin's words in the due ring: read it now
    const int rc = broadcast_common(h, root, mono_out, r, !h->dly);
    if (rc) return rc;
    HIPCHK(h, hipSetDevice(h->device));
    return drive(h, max_rounds, stats, cap, true, rounds_run);
}

int psim_plumtree_broadcast_run_n(psim_handle* h, uint32_t root, uint32_t count, uint32_t reset_trees,
                                  uint32_t max_rounds, psim_round_stats* stats, size_t cap, uint32_t* rounds,
                                  uint32_t* monos, uint32_t* done) {
    if (done) *done = 0;
    if (!h) return PSIM_EINVAL;
    return run_n(h, root, count, reset_trees != 0, max_rounds, stats, stats ? cap : 0, rounds, monos, done);
}

int psim_shard_init(psim_handle* h, int rank, int world) {
    if (!h || world < 1 || rank < 0 || rank >= world) return PSIM_EINVAL;
    if (h->n) return fail(h, PSIM_ESTATE, "psim_shard_init must precede psim_load_csr");
    h->sh.rank = rank;
    h->sh.world = world;
    return PSIM_OK;
}

int psim_shard_info(const psim_handle* h, uint32_t* v_lo, uint32_t* n_local, uint64_t* slot_base,
                    uint32_t* n_global) {
    if (!h) return PSIM_EINVAL;
    if (v_lo) *v_lo = h->sh.v_lo;
    if (n_local) *n_local = h->n;
    if (slot_base) *slot_base = h->sh.slot_base;
    if (n_global) *n_global = h->sh.n_global;
    return PSIM_OK;
}

int psim_shard_layout(const psim_handle* h, uint64_t* region_base, size_t world) {
    if (!h || !region_base || world != (size_t)h->sh.world || h->sh.send_base.size() != world + 1)
        return PSIM_EINVAL;
    memcpy(region_base, h->sh.send_base.data(), (world + 1) * 8);
    return PSIM_OK;
}

int psim_shard_broadcast(psim_handle* h, uint32_t root, uint32_t* mono_out, void* send_dev, uint64_t send_cap,
                         uint64_t* counts, int64_t* local_live) {
    if (h) h->sh.plan_ok = false;       // outside shard_drive_fast's record bound
    if (!h || !counts) return PSIM_EINVAL;
    if (int rc = one_lane_only(h)) return rc;
    unsigned long long r[kNStat];
    int rc = broadcast_common(h, root, mono_out, r);
    if (rc) return rc;
    if (local_live) *local_live = h->live_rows;
    return shard_pack(h, send_dev, send_cap, counts);
}

int psim_shard_round(psim_handle* h, void* send_dev, uint64_t send_cap, uint64_t* counts,
                     psim_round_stats* st, int64_t* local_live) {
    if (h) h->sh.plan_ok = false;       // outside shard_drive_fast's record bound
    if (!h || !counts) return PSIM_EINVAL;
    if (int rc = one_lane_only(h)) return rc;
    if (!h->n) return fail(h, PSIM_ESTATE, "no overlay loaded");
    HIPCHK(h, hipSetDevice(h->device));
    const uint32_t L = h->cfg.lazy_tick_rounds ? h->cfg.lazy_tick_rounds : 1;
    const uint32_t tick = ((h->round + 1) % L) == 0;
    HIPCHK(h, scrub_if_needed(h, h->round + 1));
    HIPCHK(h, hipMemsetAsync(h->stats, 0, kStatsRow * sizeof(unsigned long long), h->stream));
    PtArgs a = make_args(h, h->par, tick, h->stats);
    set_round_slots(h, a, h->round + 1);         // one shard: the counts every path keeps
    if (!h->sh.pending) HIPCHK(h, seed_hold_ring(h, h->round + 1));
    HIPCHK(h, hipEventRecord(h->ev[0], h->stream));
    HIPCHK(h, launch_pt_round(a, h->stream));
    HIPCHK(h, hipEventRecord(h->ev[1], h->stream));
    HIPCHK(h, hipMemcpyAsync(h->h_stats, h->stats, kStatsRow * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                             h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    h->par ^= 1u;   // the staged words were written for the round that reads in[par] now
    unsigned long long r[kNStat];
    reduce_row(h->h_stats, r);
    float ms = 0.f;
    HIPCHK(h, hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
    if (r[S_OVERFLOW])
        return fail(h, PSIM_EOVERFLOW, "round %llu: overflow flags 0x%llx", (unsigned long long)(h->round + 1),
                    r[S_OVERFLOW]);
    uint64_t msgs = 0;
    for (int t = 1; t <= 5; t++) msgs += r[t];
    h->round++;
    h->ost_cnt += (int64_t)r[S_OST_DELTA];
    h->live_rows += (int64_t)r[S_LIVE_DELTA];
    h->inflight = msgs;
    h->kernel_ms_total += ms;
    h->rounds_total++;
    if (st) {
        memset(st, 0, sizeof *st);
        for (int t = 1; t <= 5; t++) st->sent[t] = r[t];
        st->delivered_new = r[S_DELIV];
        st->active = r[S_ACTIVE];
        st->senders = r[S_SENDERS];
        st->sender_degree_sum = r[S_DEGSUM];
        st->outstanding_vertices = (uint64_t)h->ost_cnt;
        st->algo_bytes = 16ull * h->n + 8ull * r[S_SENDERS] + 4ull * r[S_DEGSUM] + 32ull * msgs;
        st->kernel_ms = ms;
    }
    if (local_live) *local_live = h->live_rows;
    return shard_pack(h, send_dev, send_cap, counts);
}

int psim_set_stream(psim_handle* h, void* stream) {
    if (!h) return PSIM_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    h->stream = stream ? (hipStream_t)stream : h->own_stream;
    return PSIM_OK;
}

int psim_shard_recv_layout(const psim_handle* h, uint64_t* recv_base, size_t world) {
    if (!h || !recv_base || world != (size_t)h->sh.world || h->sh.recv_base.size() != world + 1) return PSIM_EINVAL;
    memcpy(recv_base, h->sh.recv_base.data(), (world + 1) * 8);
    return PSIM_OK;
}

int psim_shard_broadcast_dense(psim_handle* h, uint32_t root, uint32_t* mono_out, void* send_dev) {
    if (h) h->sh.plan_ok = false;       // outside shard_drive_fast's record bound
    if (!h) return PSIM_EINVAL;
    if (int rc = one_lane_only(h)) return rc;
    if (h->sh.world > 1 && !send_dev) return PSIM_EINVAL;
    if (h->sh.pending) return fail(h, PSIM_ESTATE, "collect the async rounds first");
    unsigned long long r[kNStat];
    int rc = broadcast_common(h, root, mono_out, r);
    if (rc) return rc;
    PtArgs a = make_args(h, h->par ^ 1u, 0, h->stats);
    HIPCHK(h, launch_pt_pack_dense(a, h->sh.rem, (uint32_t)h->sh.send_base[h->sh.world], (uint32_t*)send_dev,
                                   h->stream));
    return PSIM_OK;
}

// rec_k > 0 (in-library exchange only): this round's cross-shard words go out
// as {receiver slot, word} records, rec_k per peer (sh.xrs), instead of the
// dense regions.
static int shard_round_async_k(psim_handle* h, void* send_dev, uint32_t rec_k, bool force_flags = false) {
    if (!h) return PSIM_EINVAL;
    if (int rc = one_lane_only(h)) return rc;
    if (!h->n) return fail(h, PSIM_ESTATE, "no overlay loaded");
    auto& sh = h->sh;
    if (sh.world > 1 && !send_dev) return PSIM_EINVAL;
    if (sh.pending >= 16) return fail(h, PSIM_ESTATE, "16 async rounds pending: call psim_shard_collect");
    HIPCHK(h, hipSetDevice(h->device));
    const uint32_t L = h->cfg.lazy_tick_rounds ? h->cfg.lazy_tick_rounds : 1;
    const uint32_t tick = ((h->round + 1) % L) == 0;
    unsigned long long* row = sh.ring + size_t(sh.pending) * kStatsRow;
    HIPCHK(h, scrub_if_needed(h, h->round + 1));
    const bool marks = !sh.chunk_mode;           // chunk mode: rows zeroed and timed per chunk by the driver
    if (marks) HIPCHK(h, hipMemsetAsync(row, 0, kStatsRow * sizeof(unsigned long long), h->stream));
    PtArgs a = make_args(h, h->par, tick, row);
    set_round_slots(h, a, h->round + 1);         // off unless shard_drive_fast turned the counts on
    a.force_flags = force_flags ? 1u : 0u;
    if (marks) HIPCHK(h, hipEventRecord(sh.rev_[2 * sh.pending], h->stream));
    HIPCHK(h, launch_pt_round(a, h->stream));
    if (marks) HIPCHK(h, hipEventRecord(sh.rev_[2 * sh.pending + 1], h->stream));
    if (sh.world > 1 && rec_k) {
        HIPCHK(h, hipMemsetAsync(sh.xrs_raw, 0, 256 + size_t(sh.world - 1) * rec_k * 8, h->stream));
        HIPCHK(h, launch_pt_compact(a, sh.rem, sh.blk, sh.nblk, nullptr, sh.xcur, sh.xrs, h->stream, rec_k,
                                    (uint32_t)sh.rank));
    } else if (sh.world > 1) {
        HIPCHK(h, launch_pt_pack_dense(a, sh.rem, (uint32_t)sh.send_base[sh.world], (uint32_t*)send_dev, h->stream));
    }
    h->par ^= 1u;
    h->round++;
    sh.pending++;
    return PSIM_OK;
}

int psim_shard_round_async(psim_handle* h, void* send_dev) {
    if (h) h->sh.plan_ok = false;       // split-phase rounds: the record-bound bookkeeping is off
    if (h && h->n && !h->sh.pending && h->lanes.size() <= 1 && !h->win)
        HIPCHK(h, seed_hold_ring(h, h->round + 1));
    return shard_round_async_k(h, send_dev, 0);
}

int psim_shard_ingest_dense(psim_handle* h, const void* recv_dev) {
    if (h) h->sh.plan_ok = false;       // outside shard_drive_fast's record bound
    if (!h) return PSIM_EINVAL;
    if (int rc = one_lane_only(h)) return rc;
    return ingest_dense(h, recv_dev);
}

}  // extern "C"

namespace {
// the focused lane's received words -> the inbox the next round reads
int ingest_dense(psim_handle* h, const void* recv_dev, bool force_flags) {
    auto& sh = h->sh;
    const uint64_t nr = sh.recv_base.empty() ? 0 : sh.recv_base[sh.world];
    if (nr == 0) return PSIM_OK;
    if (!recv_dev) return PSIM_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    PtArgs a = make_args(h, h->par ^ 1u, 0, h->stats);   // in_nxt / pend_nxt = what the next round reads
    set_round_slots(h, a, h->round);                      // counts: the round that sent them (m_w)
    a.force_flags = force_flags ? 1u : 0u;
    HIPCHK(h, launch_pt_ingest_dense(a, (const uint32_t*)recv_dev, sh.recv_map, (uint32_t)nr, sh.slot2v, h->stream));
    return PSIM_OK;
}
}  // namespace

extern "C" {

int psim_shard_collect(psim_handle* h, psim_round_stats* out, size_t cap, uint32_t* n_out, int64_t* local_live) {
    if (!h) return PSIM_EINVAL;
    auto& sh = h->sh;
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    const uint32_t k = sh.pending;
    std::vector<unsigned long long> hs(size_t(k) * kStatsRow);
    if (k) HIPCHK(h, hipMemcpy(hs.data(), sh.ring, hs.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    sh.pending = 0;
    sh.pend_rows.assign(k, 0);
    for (uint32_t i = 0; i < k; i++) {
        unsigned long long r[kNStat];
        reduce_row(hs.data() + size_t(i) * kStatsRow, r);
        float ms = 0.f;
        if (sh.chunk_mode) {                      // the chunk's device time (kernels + exchange) / its rounds
            HIPCHK(h, hipEventElapsedTime(&ms, sh.rev_[0], sh.rev_[1]));
            ms /= float(k);
        } else {
            HIPCHK(h, hipEventElapsedTime(&ms, sh.rev_[2 * i], sh.rev_[2 * i + 1]));
        }
        if (r[S_OVERFLOW]) return fail(h, PSIM_EOVERFLOW, "async round: overflow flags 0x%llx", r[S_OVERFLOW]);
        uint64_t msgs = 0;
        for (int t = 1; t <= 5; t++) msgs += r[t];
        h->ost_cnt += (int64_t)r[S_OST_DELTA];
        h->live_rows += (int64_t)r[S_LIVE_DELTA];
        h->inflight = msgs;
        if (h->dly) {          // round R consumed its arrivals; its sends are pending until R + 1 + d
            const uint64_t R = h->round - k + 1 + i;
            h->due[R & (kRing - 1)] = 0;
            h->inflight = add_due(h->due, R, hs.data() + size_t(i) * kStatsRow + size_t(kStatShards) * kNStat);
            sh.pend_rows[i] = (int64_t)h->inflight;
        }
        h->kernel_ms_total += ms;
        h->rounds_total++;
        if (out && i < cap) {
            psim_round_stats& o = out[i];
            memset(&o, 0, sizeof o);
            for (int t = 1; t <= 5; t++) o.sent[t] = r[t];
            o.delivered_new = r[S_DELIV];
            o.active = r[S_ACTIVE];
            o.senders = r[S_SENDERS];
            o.sender_degree_sum = r[S_DEGSUM];
            o.outstanding_vertices = (uint64_t)h->ost_cnt;
            o.algo_bytes = 16ull * h->n + 8ull * r[S_SENDERS] + 4ull * r[S_DEGSUM] + 32ull * msgs;
            o.words_stored = r[S_WORDS];
            o.kernel_ms = ms;
        }
        if (local_live && i < cap) local_live[i] = h->live_rows;
    }
    if (n_out) *n_out = k;
    return PSIM_OK;
}

int psim_shard_uncount(psim_handle* h, uint32_t rounds) {
    if (!h || rounds > h->round || h->sh.pending) return PSIM_EINVAL;
    h->round -= rounds;
    return PSIM_OK;
}

int psim_rccl_unique_id(uint8_t* id_out) {
    if (!id_out) return PSIM_EINVAL;
    return psim::rccl_unique_id(id_out);
}

int psim_shard_init_rccl(psim_handle* h, int rank, int world, const uint8_t* id) {
    if (!h || !id) return PSIM_EINVAL;
    int rc = psim_shard_init(h, rank, world);
    if (rc) return rc;
    delete h->sh.xport;
    h->sh.xport = nullptr;
    std::string err;
    rc = psim::make_rccl_transport(h->device, rank, world, id, &h->sh.xport, &err);
    return rc ? fail(h, rc, "%s", err.c_str()) : PSIM_OK;
}

int psim_shard_set_transport(psim_handle* h, const psim_transport* t) {
    if (!h || !t || !t->alltoallv || !t->allreduce) return PSIM_EINVAL;
    delete h->sh.xport;
    h->sh.xport = psim::make_callback_transport(*t);
    return h->sh.xport ? PSIM_OK : PSIM_ENOMEM;
}

}  // extern "C"

namespace {

// The dense word buffers of the in-library exchange (allocated on first use).
int x_buffers(psim_handle* h) {
    auto& sh = h->sh;
    if (sh.world > 1 && !sh.xport) return fail(h, PSIM_ESTATE, "sharded handle without a transport (psim_shard_init_rccl)");
    if (sh.xsend || sh.world == 1) return PSIM_OK;
    const size_t ns = std::max<uint64_t>(1, sh.send_base[sh.world]), nr = std::max<uint64_t>(1, sh.recv_base[sh.world]);
    const size_t nrec = std::max<uint64_t>(1, (sh.world - 1) * sh.rec_thr);
    if (hipMalloc((void**)&sh.xsend, ns * 4) != hipSuccess || hipMalloc((void**)&sh.xrecv, nr * 4) != hipSuccess ||
        hipMalloc((void**)&sh.xrs_raw, 256 + nrec * 8) != hipSuccess || hipMalloc((void**)&sh.xrr, nrec * 8) != hipSuccess)
        return fail(h, PSIM_ENOMEM, "exchange buffers");
    sh.xcur = reinterpret_cast<uint32_t*>(sh.xrs_raw);           // <= 64 shards
    sh.xrs = reinterpret_cast<uint2*>(sh.xrs_raw + 256);
    HIPCHK(h, hipMemsetAsync(sh.xsend, 0, ns * 4, h->stream));
    HIPCHK(h, hipMemsetAsync(sh.xrecv, 0, nr * 4, h->stream));
    return PSIM_OK;
}

// exchange the dense regions just packed into xsend, then ingest them
int x_exchange(psim_handle* h, int slot, psim_exchange_stats* xs, uint32_t rec_k = 0, bool force_flags = false) {
    auto& sh = h->sh;
    if (sh.world == 1) return PSIM_OK;
    std::string err;
    const bool marks = !sh.chunk_mode;
    if (marks) HIPCHK(h, hipEventRecord(sh.xev[2 * slot], h->stream));
    if (rec_k) {        // fixed-size record regions: 2 rec_k words per peer, none to self
        const int W = sh.world;
        std::vector<uint64_t> off(size_t(W) + 1, 0);
        for (int d = 0; d < W; d++) off[d + 1] = off[d] + (d == sh.rank ? 0 : 2ull * rec_k);
        int rc = sh.xport->alltoallv(reinterpret_cast<const uint32_t*>(sh.xrs), off.data(),
                                     reinterpret_cast<uint32_t*>(sh.xrr), off.data(), sh.rank, W, h->stream, &err);
        if (rc) return fail(h, rc, "exchange: %s", err.c_str());
        if (marks) HIPCHK(h, hipEventRecord(sh.xev[2 * slot + 1], h->stream));
        if (xs) xs->fabric_bytes += 8ull * rec_k * uint64_t(W - 1);
        PtArgs a = make_args(h, h->par ^ 1u, 0, h->stats);   // in_nxt / pend_nxt = what the next round reads
        set_round_slots(h, a, h->round);                      // counts: the round that sent them (m_w)
        a.force_flags = force_flags ? 1u : 0u;
        HIPCHK(h, launch_pt_ingest(a, sh.xrr, uint32_t(uint64_t(W - 1) * rec_k), sh.slot2v, h->stream));
        return PSIM_OK;
    }
    int rc = sh.xport->alltoallv(sh.xsend, sh.send_base.data(), sh.xrecv, sh.recv_base.data(), sh.rank, sh.world,
                                 h->stream, &err);
    if (rc) return fail(h, rc, "exchange: %s", err.c_str());
    if (marks) HIPCHK(h, hipEventRecord(sh.xev[2 * slot + 1], h->stream));
    if (xs) xs->fabric_bytes += 4ull * (sh.send_base[sh.world] - (sh.send_base[sh.rank + 1] - sh.send_base[sh.rank]));
    return ingest_dense(h, sh.xrecv, force_flags);
}

// Sharded window lane: the records the last round (or origin) wrote into
// msg[par] go to the shards owning their receivers -- counts all-to-all,
// records all-to-all-v -- and msg[par] ends up holding exactly this shard's
// records for the next round (own ones first, then by source rank).
int win_exchange(psim_handle* h, psim_exchange_stats* xs) {
    auto& sh = h->sh;
    const uint32_t W = (uint32_t)sh.world, R = (uint32_t)sh.rank;
    if (W == 1) return PSIM_OK;
    if (W > kWinMaxWorld) return fail(h, PSIM_EINVAL, "window lanes support up to %u shards", kWinMaxWorld);
    Win& w = *h->win;
    const uint32_t par = h->par;
    if (!h->w_counts) {
        if (!alloc_zero((void**)&h->w_counts, kWinMaxWorld * 4) || !alloc_zero((void**)&h->w_rcnt, kWinMaxWorld * 4) ||
            !alloc_zero((void**)&h->w_base, kWinMaxWorld * 4) || !alloc_zero((void**)&h->w_cursor, kWinMaxWorld * 4))
            return fail(h, PSIM_ENOMEM, "window exchange counters");
    }
    if (h->w_send_cap < w.cap) {
        if (h->w_send) (void)hipFree(h->w_send);
        h->w_send = nullptr;
        h->w_send_cap = 0;
        if (!alloc_zero((void**)&h->w_send, size_t(w.cap) * sizeof(PdMsg))) return fail(h, PSIM_ENOMEM, "window send buffer");
        h->w_send_cap = w.cap;
    }
    HIPCHK(h, hipMemsetAsync(h->w_counts, 0, W * 4, h->stream));
    HIPCHK(h, launch_win_split(w.msg[par], w.nmsg + par, w.cap, sh.n_global, W, h->w_counts, h->stream));
    std::vector<uint64_t> one(W + 1);
    for (uint32_t i = 0; i <= W; i++) one[i] = i;
    std::string err;
    int rc = sh.xport->alltoallv(h->w_counts, one.data(), h->w_rcnt, one.data(), (int)R, (int)W, h->stream, &err);
    if (rc) return fail(h, rc, "window counts exchange: %s", err.c_str());
    std::vector<uint32_t> cnt(W), rcv(W);
    HIPCHK(h, hipMemcpyAsync(cnt.data(), h->w_counts, W * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipMemcpyAsync(rcv.data(), h->w_rcnt, W * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    rcv[R] = cnt[R];
    std::vector<uint64_t> soff(W + 1, 0), roff(W + 1, 0);
    std::vector<uint32_t> base(W);
    for (uint32_t i = 0; i < W; i++) {
        base[i] = (uint32_t)soff[i];
        soff[i + 1] = soff[i] + cnt[i];
        roff[i + 1] = roff[i] + rcv[i];
    }
    if (roff[W] > w.cap) return fail(h, PSIM_EOVERFLOW, "window lane: %llu records for one shard > %u",
                                     (unsigned long long)roff[W], w.cap);
    HIPCHK(h, hipMemcpyAsync(h->w_base, base.data(), W * 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipMemsetAsync(h->w_cursor, 0, W * 4, h->stream));
    HIPCHK(h, launch_win_scatter(w.msg[par], w.nmsg + par, w.cap, sh.n_global, W, h->w_base, h->w_cursor, h->w_send,
                                 h->stream));
    if (cnt[R])     // own records (an RCCL all-to-all-v skips the own rank)
        HIPCHK(h, hipMemcpyAsync(w.msg[par] + roff[R], h->w_send + soff[R], size_t(cnt[R]) * sizeof(PdMsg),
                                 hipMemcpyDeviceToDevice, h->stream));
    constexpr uint64_t kW = sizeof(PdMsg) / 4;
    for (auto& x : soff) x *= kW;
    for (auto& x : roff) x *= kW;
    rc = sh.xport->alltoallv(reinterpret_cast<const uint32_t*>(h->w_send), soff.data(),
                             reinterpret_cast<uint32_t*>(w.msg[par]), roff.data(), (int)R, (int)W, h->stream, &err);
    if (rc) return fail(h, rc, "window records exchange: %s", err.c_str());
    const uint32_t total = uint32_t(roff[W] / kW);
    HIPCHK(h, hipMemcpyAsync(w.nmsg + par, &total, 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (xs) xs->fabric_bytes += sizeof(PdMsg) * (soff[W] / kW - cnt[R]);
    h->inflight = total;
    return PSIM_OK;
}

// After a sharded broadcast: the focused lane's global in-flight / live-row
// / row-holder counts (one all-reduce; every rank then decides alike).
int lane_globals(psim_handle* h) {
    save_lane(h);
    auto& l = h->lanes[h->cur_lane];
    int64_t v[3] = {(int64_t)h->inflight, h->live_rows, h->ost_cnt};
    if (h->sh.world > 1) {
        std::string err;
        const int rc = h->sh.xport->allreduce(v, 3, h->stream, &err);
        if (rc) return fail(h, rc, "lane all-reduce: %s", err.c_str());
    }
    l.g_inflight = v[0];
    l.g_live = v[1];
    l.g_ost = v[2];
    h->sh.plan_ok = true;      // shard_drive_fast may bound the next rounds' words from these
    return PSIM_OK;
}

// Rounds of a sharded handle with several lanes or a window lane: each round
// runs every lane with a root (round kernel, then its exchange), one
// all-reduce of every lane's counters per round.  Delay faults: each static
// lane stages its cross-shard delayed words in its own ring (Lane::srg), the
// exchange after round R carries that ring's slot R, and a lane's in-flight
// count is what its delay histogram still has pending (summed over shards).
int shard_drive_lanes(psim_handle* h, uint32_t max_rounds, psim_round_stats* out, size_t cap, bool stop_q,
                      uint32_t* ran_out, psim_exchange_stats* xs) {
    if (h) h->sh.plan_ok = false;       // outside shard_drive_fast's record bound
    const int focus = h->cur_lane;
    save_lane(h);
    struct Refocus {
        psim_handle* h;
        int f;
        ~Refocus() { load_lane(h, f); }
    } refocus{h, focus};
    const uint32_t L = h->cfg.lazy_tick_rounds ? h->cfg.lazy_tick_rounds : 1;
    constexpr int NK = 11;    // 5 kinds, delivered_new, senders, degree sum, live rows, row holders,
                              // messages still pending (delay faults)
    uint32_t ran = 0;
    auto quiet = [&]() {
        for (const auto& l : h->lanes)
            if (l.have_root && !lane_quiescent(h, l)) return false;
        return true;
    };
    bool done = stop_q && quiet();
    while (!done && ran < max_rounds) {
        std::vector<int> act;
        for (int j = 0; j < (int)h->lanes.size(); j++)
            if (h->lanes[j].have_root) act.push_back(j);
        const size_t A = act.size();
        if (A == 0) break;
        const uint32_t tick = ((h->round + 1) % L) == 0;
        HIPCHK(h, hipMemsetAsync(h->stats, 0, A * kStatsRow * sizeof(unsigned long long), h->stream));
        HIPCHK(h, hipEventRecord(h->ev[0], h->stream));
        for (size_t q = 0; q < A; q++) {
            load_lane(h, act[q]);
            unsigned long long* row = h->stats + q * kStatsRow;
            int rc;
            if (h->win) {
                const WinArgs a = make_win_args(h, h->par, tick, row);
                HIPCHK(h, hipMemsetAsync(a.nout, 0, 4, h->stream));
                HIPCHK(h, launch_win_round(a, h->w_cnt, h->w_cur, h->w_bsum, h->stream));
                h->par ^= 1u;
                rc = win_exchange(h, xs);
            } else {
                HIPCHK(h, scrub_if_needed(h, h->round + 1));
                PtArgs a = make_args(h, h->par, tick, row);
                HIPCHK(h, launch_pt_round(a, h->stream));
                if (h->sh.world > 1)
                    HIPCHK(h, launch_pt_pack_dense(a, h->sh.rem, (uint32_t)h->sh.send_base[h->sh.world], h->sh.xsend,
                                                   h->stream));
                h->par ^= 1u;
                // delays: the ingest files the words into the ring by the round just run
                if (h->dly) h->round++;
                rc = x_exchange(h, 0, xs);
                if (h->dly) h->round--;
            }
            if (rc) return rc;
            save_lane(h);
        }
        HIPCHK(h, hipEventRecord(h->ev[1], h->stream));
        HIPCHK(h, hipMemcpyAsync(h->h_stats, h->stats, A * kStatsRow * sizeof(unsigned long long),
                                 hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        float ms = 0.f;
        HIPCHK(h, hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
        h->round++;
        h->kernel_ms_total += ms;
        h->rounds_total++;
        std::vector<int64_t> flat(A * NK);
        unsigned long long loc[kNStat] = {0};
        for (size_t q = 0; q < A; q++) {
            unsigned long long r[kNStat];
            reduce_row(h->h_stats + q * kStatsRow, r);
            if (r[S_OVERFLOW])
                return fail(h, PSIM_EOVERFLOW, "round %llu: overflow flags 0x%llx", (unsigned long long)h->round,
                            r[S_OVERFLOW]);
            auto& l = h->lanes[act[q]];
            uint64_t lm = 0;
            for (int t = 1; t <= 5; t++) lm += r[t];
            l.ost_cnt += (int64_t)r[S_OST_DELTA];
            l.live_rows += (int64_t)r[S_LIVE_DELTA];
            if (h->dly && !l.win) {      // round R consumed its arrivals; its sends are pending until R + 1 + d
                const uint64_t R = h->round;
                l.due[R & (kRing - 1)] = 0;
                l.inflight = add_due(l.due, R, h->h_stats + q * kStatsRow + size_t(kStatShards) * kNStat);
            } else if (!l.win) {
                l.inflight = lm;
            }
            int64_t* f = flat.data() + q * NK;
            for (int t = 1; t <= 5; t++) f[t - 1] = (int64_t)r[t];
            f[5] = (int64_t)r[S_DELIV];
            f[6] = (int64_t)r[S_SENDERS];
            f[7] = (int64_t)r[S_DEGSUM];
            f[8] = l.live_rows;
            f[9] = l.ost_cnt;
            f[10] = h->dly ? (int64_t)l.inflight : 0;
            for (int t = 0; t < kNStat; t++) loc[t] += r[t];
        }
        if (h->sh.world > 1) {
            std::string err;
            const int rc = h->sh.xport->allreduce(flat.data(), flat.size(), h->stream, &err);
            if (rc) return fail(h, rc, "counter all-reduce: %s", err.c_str());
        }
        int64_t tot[NK] = {0};
        for (size_t q = 0; q < A; q++) {
            auto& l = h->lanes[act[q]];
            const int64_t* f = flat.data() + q * NK;
            l.g_inflight = h->dly ? f[10] : f[0] + f[1] + f[2] + f[3] + f[4];   // delays: what is still on the wire
            l.g_live = f[8];
            l.g_ost = f[9];
            for (int t = 0; t < NK - 1; t++) tot[t] += f[t];
        }
        if (out && ran < cap) {
            psim_round_stats& o = out[ran];
            memset(&o, 0, sizeof o);
            for (int t = 1; t <= 5; t++) o.sent[t] = (uint64_t)tot[t - 1];
            o.delivered_new = (uint64_t)tot[5];
            o.senders = (uint64_t)tot[6];
            o.sender_degree_sum = (uint64_t)tot[7];
            o.active = loc[S_ACTIVE];
            o.outstanding_vertices = (uint64_t)tot[9];
            uint64_t lm = 0;
            for (int t = 1; t <= 5; t++) lm += loc[t];
            o.algo_bytes = 16ull * h->n * A + 8ull * loc[S_SENDERS] + 4ull * loc[S_DEGSUM] + 32ull * lm;
            o.words_stored = loc[S_WORDS];
            o.kernel_ms = ms;
        }
        if (xs) {
            xs->rounds++;
            xs->kernel_ms += ms;
        }
        ran++;
        if (stop_q && quiet()) done = true;
    }
    if (ran_out) *ran_out = ran;
    return PSIM_OK;
}

int shard_drive_fast(psim_handle* h, uint32_t max_rounds, psim_round_stats* out, size_t cap, bool stop_q,
                     uint32_t* rounds_run, psim_exchange_stats* xs);

int shard_drive(psim_handle* h, uint32_t max_rounds, psim_round_stats* out, size_t cap, bool stop_q,
                uint32_t* rounds_run, psim_exchange_stats* xs) {
    if (!h) return PSIM_EINVAL;
    if (!h->n) return fail(h, PSIM_ESTATE, "no overlay loaded");
    HIPCHK(h, hipSetDevice(h->device));
    if (xs) memset(xs, 0, sizeof *xs);
    if (h->fo.on) {             // every root's lane in one launch, every lane's words in one exchange
        if (h->sh.world > 1 && !h->sh.xport) return fail(h, PSIM_ESTATE, "sharded forest without a transport");
        const double k0 = h->kernel_ms_total;
        const uint64_t r0 = h->rounds_total;
        uint32_t ran = 0;
        const int rc = forest_drive(h, max_rounds, out, cap, stop_q, &ran);
        if (rounds_run) *rounds_run = ran;
        if (xs) {
            xs->rounds = h->rounds_total - r0;
            xs->kernel_ms = h->kernel_ms_total - k0;
        }
        return rc;
    }
    int rc = x_buffers(h);
    if (rc) return rc;
    if (h->lanes.size() > 1 || h->win) {
        if (!h->sh.pending) HIPCHK(h, seed_hold_rings(h, h->round + 1));
        return shard_drive_lanes(h, max_rounds, out, cap, stop_q, rounds_run, xs);
    }
    return shard_drive_fast(h, max_rounds, out, cap, stop_q, rounds_run, xs);
}

// One lane of static words: rounds pipelined 4 at a time (kernel -> pack ->
// all-to-all-v -> ingest, stream-ordered), one sync + one all-reduce per chunk.
int shard_drive_fast(psim_handle* h, uint32_t max_rounds, psim_round_stats* out, size_t cap, bool stop_q,
                     uint32_t* rounds_run, psim_exchange_stats* xs) {
    int rc;
    constexpr uint32_t K = 4;                  // rounds between counter collections
    constexpr int NK = 11;                     // 5 kinds, delivered_new, senders, degree sum, live rows, row holders,
                                               // messages still pending (delay faults)
    uint32_t ran = 0;
    bool done = false;
    auto& sh = h->sh;
    // Record bound of the sparse rounds: a vertex sends at most
    // one word per slot and only when it received words or holds rows due, so
    // a round after M words in flight with H row holders sends <= D (M + H)
    // words (D = the overlay's widest row) and the next round starts with
    // <= H + M holders.  Every rank derives the same bound from the global
    // counts of the last collective, so every rank picks the same format.
    double bM = 0, bH = 0;
    if (sh.plan_ok && !h->lanes.empty()) {
        bM = double(h->lanes[h->cur_lane].g_inflight);
        bH = double(h->lanes[h->cur_lane].g_ost);
    }
    // PSIM_CFG_CHUNK_TIMING: no event marker or stats memset between a chunk's
    // launches (each cost ~10 us of idle GPU between dependent kernels); the
    // chunk's rows are zeroed at once and it is timed by one event pair
    struct ChunkMode {
        psim_handle* h;
        ~ChunkMode() { h->sh.chunk_mode = h->sh.mcnt_on = false; }
    } chunk_guard{h};
    sh.chunk_mode = (h->cfg.flags & PSIM_CFG_CHUNK_TIMING) != 0;
    // per-round counts from here on (several shards): the ring starts empty except the count the
    // first round reads as its previous round's, which is seeded 1 (words may
    // wait from a broadcast or from rounds run without counts: no no-op exit,
    // group flags written and read -- what every other path does)
    // (one shard: the counts are kept by every path, as on a plain handle)
    if (sh.world > 1 && h->bin.rec_c == nullptr && !h->dly && !h->lanes.empty()) {
        uint32_t* mc = h->mcnt_base + kMcntLane * size_t(h->cur_lane);
        HIPCHK(h, hipMemsetAsync(mc, 0, kMcntLane * sizeof(uint32_t), h->stream));
        HIPCHK(h, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(mc + (h->round % 4) * 64), 1, 1, h->stream));
        // the first round's predecessor-but-one: the list threshold, so it reads
        // the flags (its words were not listed) and clears them, and the rounds
        // after it list and read lists as their counts say
        if (const uint32_t thr = list_threshold(h))
            HIPCHK(h, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(mc + ((h->round + 3) % 4) * 64), thr, 1,
                                        h->stream));
        sh.mcnt_on = true;
    }
    if (!sh.pending) HIPCHK(h, seed_hold_ring(h, h->round + 1));   // the local holder count is exact
    while (!done && ran < max_rounds) {
        const uint32_t k = std::min<uint32_t>(K, max_rounds - ran);
        if (sh.chunk_mode) {
            if (sh.pending) return fail(h, PSIM_ESTATE, "collect the async rounds first");
            HIPCHK(h, hipMemsetAsync(sh.ring, 0, size_t(k) * kStatsRow * sizeof(unsigned long long), h->stream));
            HIPCHK(h, hipEventRecord(sh.rev_[0], h->stream));
        }
        for (uint32_t j = 0; j < k; j++) {
            uint32_t rec_k = 0;
            if (sh.plan_ok && sh.world > 1 && !h->dly) {   // delays: a round's words are not bounded by the last
                const double S = double(std::max<uint32_t>(1u, sh.max_deg_g)) * (bM + bH);
                bH += bM;
                bM = S;
                if (S <= double(sh.rec_thr)) rec_k = std::max<uint32_t>(1u, uint32_t(S));
            }
            // the last round this call may run writes group flags whatever its
            // count: whoever reads next (another call, a path without counts)
            // finds its words by the flags
            const bool last = ran + j + 1 == max_rounds;
            rc = shard_round_async_k(h, sh.xsend, rec_k, last);
            if (rc) return rc;
            rc = x_exchange(h, (int)j, xs, rec_k, last);
            if (rc) return rc;
        }
        if (sh.chunk_mode) HIPCHK(h, hipEventRecord(sh.rev_[1], h->stream));
        psim_round_stats st[K];
        int64_t live[K];
        uint32_t got = 0;
        rc = psim_shard_collect(h, st, K, &got, live);
        if (rc) return rc;
        if (xs) {
            xs->rounds += got;
            for (uint32_t j = 0; j < got; j++) {
                xs->kernel_ms += st[j].kernel_ms;
                float ms = 0.f;      // chunk mode: the exchange is inside kernel_ms (one event pair per chunk)
                if (h->sh.world > 1 && !sh.chunk_mode)
                    HIPCHK(h, hipEventElapsedTime(&ms, h->sh.xev[2 * j], h->sh.xev[2 * j + 1]));
                xs->exchange_ms += ms;
            }
        }
        std::vector<int64_t> flat(size_t(got) * NK);
        for (uint32_t j = 0; j < got; j++) {
            int64_t* f = flat.data() + size_t(j) * NK;
            for (int t = 1; t <= 5; t++) f[t - 1] = (int64_t)st[j].sent[t];
            f[5] = (int64_t)st[j].delivered_new;
            f[6] = (int64_t)st[j].senders;
            f[7] = (int64_t)st[j].sender_degree_sum;
            f[8] = live[j];
            f[9] = (int64_t)st[j].outstanding_vertices;
            f[10] = h->dly && j < sh.pend_rows.size() ? sh.pend_rows[j] : 0;
        }
        if (h->sh.world > 1) {
            std::string err;
            rc = h->sh.xport->allreduce(flat.data(), flat.size(), h->stream, &err);
            if (rc) return fail(h, rc, "counter all-reduce: %s", err.c_str());
        }
        for (uint32_t j = 0; j < got; j++) {
            const int64_t* f = flat.data() + size_t(j) * NK;
            int64_t msgs = 0;
            for (int t = 0; t < 5; t++) msgs += f[t];
            if (h->dly) msgs = f[10];                          // what is still on the wire, delayed included
            if (!h->lanes.empty()) {
                auto& l = h->lanes[h->cur_lane];
                l.g_inflight = msgs;
                l.g_live = f[8];
                l.g_ost = f[9];
            }
            if (j + 1 == got) {                                 // the next chunk's bound starts here
                bM = double(msgs);
                bH = double(f[9]);
            }
            if (out && ran < cap) {
                psim_round_stats& o = out[ran];
                const double kms = st[j].kernel_ms;
                memset(&o, 0, sizeof o);
                for (int t = 1; t <= 5; t++) o.sent[t] = (uint64_t)f[t - 1];
                o.delivered_new = (uint64_t)f[5];
                o.senders = (uint64_t)f[6];
                o.sender_degree_sum = (uint64_t)f[7];
                o.active = st[j].active;                        // this rank's
                o.outstanding_vertices = (uint64_t)f[9];
                o.algo_bytes = st[j].algo_bytes;                // this rank's (its kernel's bytes)
                o.words_stored = st[j].words_stored;            // this rank's
                o.kernel_ms = kms;
            }
            ran++;
            if (stop_q && msgs == 0 && f[8] == 0) {             // globally quiescent after this round
                done = true;
                const uint32_t extra = got - (j + 1);
                if (extra) {
                    rc = psim_shard_uncount(h, extra);
                    if (rc) return rc;
                }
                break;
            }
        }
    }
    if (rounds_run) *rounds_run = ran;
    return PSIM_OK;
}

}  // namespace

extern "C" {

int psim_shard_broadcast_x(psim_handle* h, uint32_t root, uint32_t* mono_out) {
    if (!h) return PSIM_EINVAL;
    if (h->fo.on) return forest_broadcast(h, &root, 1, mono_out);   // the forest's own exchange (collective)
    int rc = x_buffers(h);
    if (rc) return rc;
    if (h->sh.pending) return fail(h, PSIM_ESTATE, "collect the async rounds first");
    unsigned long long r[kNStat];
    rc = broadcast_common(h, root, mono_out, r);
    if (rc) return rc;
    if (h->win) {
        rc = win_exchange(h, nullptr);
    } else {
        // the origin sends at most one word per slot: records unless its row is wide
        auto& sh = h->sh;
        PtArgs a = make_args(h, h->par ^ 1u, 0, h->stats);
        const uint32_t rec_k = std::max<uint32_t>(1u, sh.max_deg_g) <= sh.rec_thr ? std::max<uint32_t>(1u, sh.max_deg_g) : 0u;
        if (sh.world > 1 && rec_k) {
            HIPCHK(h, hipMemsetAsync(sh.cursor, 0, sh.world * 4, h->stream));
            HIPCHK(h, hipMemsetAsync(sh.xrs, 0, size_t(sh.world - 1) * rec_k * 8, h->stream));
            HIPCHK(h, launch_pt_compact(a, sh.rem, sh.blk, sh.nblk, nullptr, sh.cursor, sh.xrs, h->stream, rec_k,
                                        (uint32_t)sh.rank));
        } else if (sh.world > 1) {
            HIPCHK(h, launch_pt_pack_dense(a, sh.rem, (uint32_t)sh.send_base[sh.world], sh.xsend, h->stream));
        }
        rc = x_exchange(h, 0, nullptr, rec_k);
    }
    if (rc) return rc;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return lane_globals(h);
}

int psim_shard_run(psim_handle* h, uint32_t max_rounds, psim_round_stats* out, size_t cap, uint32_t* rounds_run,
                   psim_exchange_stats* xs) {
    return shard_drive(h, max_rounds, out, cap, true, rounds_run, xs);
}

int psim_shard_step(psim_handle* h, uint32_t rounds, psim_round_stats* out, size_t cap, psim_exchange_stats* xs) {
    return shard_drive(h, rounds, out, cap, false, nullptr, xs);
}

int psim_shard_ingest(psim_handle* h, const void* recv_dev, uint64_t n_records) {
    if (h) h->sh.plan_ok = false;       // outside shard_drive_fast's record bound
    if (!h || (!recv_dev && n_records)) return PSIM_EINVAL;
    if (int rc = one_lane_only(h)) return rc;
    if (n_records == 0) return PSIM_OK;
    if (n_records > 0xFFFFFFFFull) return PSIM_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    PtArgs a = make_args(h, h->par ^ 1u, 0, h->stats);   // in_nxt/pend_nxt = the buffers the next round reads
    HIPCHK(h, launch_pt_ingest(a, (const uint2*)recv_dev, (uint32_t)n_records, h->sh.slot2v, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return PSIM_OK;
}

int psim_step(psim_handle* h, uint32_t rounds, psim_round_stats* stats, size_t cap) {
    if (!h) return PSIM_EINVAL;
    if (h->sh.world > 1) return fail(h, PSIM_ESTATE, "sharded handle: drive rounds with psim_shard_round");
    HIPCHK(h, hipSetDevice(h->device));
    if (h->fo.on) return forest_drive(h, rounds, stats, cap, false, nullptr);
    return drive(h, rounds, stats, cap, false, nullptr);
}

int psim_run(psim_handle* h, uint32_t max_rounds, psim_round_stats* stats, size_t cap, uint32_t* rounds_run) {
    if (!h) return PSIM_EINVAL;
    if (h->sh.world > 1) return fail(h, PSIM_ESTATE, "sharded handle: drive rounds with psim_shard_round");
    HIPCHK(h, hipSetDevice(h->device));
    if (h->fo.on) return forest_drive(h, max_rounds, stats, cap, true, rounds_run);
    return drive(h, max_rounds, stats, cap, true, rounds_run);
}

int psim_get_plumtree(const psim_handle* h, uint32_t* eager, uint32_t* lazy, uint32_t* outstanding,
                      uint16_t* recv_round, size_t n) {
    if (!h || n != h->n || !h->n) return PSIM_EINVAL;
    if (!h->vs) return fail(const_cast<psim_handle*>(h), PSIM_ESTATE, "forest: no root heartbeated yet (no lane to read)");
    psim_handle* hh = const_cast<psim_handle*>(h);
    std::vector<uint4> vs(n);
    HIPCHK(hh, hipSetDevice(h->device));
    HIPCHK(hh, hipStreamSynchronize(h->stream));
    HIPCHK(hh, hipMemcpy(vs.data(), h->vs, n * 16, hipMemcpyDeviceToHost));
    const uint32_t ep8 = h->epoch & 0xFFu, s8 = h->serial & 0xFFu;
    for (size_t v = 0; v < n; v++) {
        const uint4 st = vs[v];
        const bool cur = (st.w >> 24) == ep8;
        if (eager) eager[v] = cur ? st.x : h->h_memb[v];
        if (lazy) lazy[v] = cur ? st.y : 0u;
        if (outstanding) outstanding[v] = st.z;
        if (recv_round) {
            const bool got = h->serial && ((st.w >> 16) & 0xFFu) == s8;
            if (!got) recv_round[v] = 0xFFFF;
            else if (h->have_root && v + h->sh.v_lo == h->root) recv_round[v] = 0xFFFE;
            else recv_round[v] = uint16_t((st.w & 0xFFFFu) - 1u);
        }
    }
    return PSIM_OK;
}

int psim_get_messages(const psim_handle* h, uint32_t* src, uint32_t* dst, uint32_t* kind, uint32_t* round,
                      uint32_t* mono, size_t cap, size_t* count) {
    if (!h || !count || !h->n) return PSIM_EINVAL;
    psim_handle* hh = const_cast<psim_handle*>(h);
    HIPCHK(hh, hipSetDevice(h->device));
    HIPCHK(hh, hipStreamSynchronize(h->stream));
    std::vector<PdMsg> m;
    if (h->win) {
        uint32_t k = 0;
        HIPCHK(hh, hipMemcpy(&k, h->win->nmsg + h->par, 4, hipMemcpyDeviceToHost));
        k = std::min(k, h->win->cap);
        m.resize(k);
        if (k) HIPCHK(hh, hipMemcpy(m.data(), h->win->msg[h->par], size_t(k) * sizeof(PdMsg), hipMemcpyDeviceToHost));
        std::sort(m.begin(), m.end(), [](const PdMsg& x, const PdMsg& y) {
            return x.dst != y.dst ? x.dst < y.dst : (x.src != y.src ? x.src < y.src : x.seq < y.seq);
        });
    } else {
        // one heartbeat: the words' FIFOs; a graft / ignored_i_have answers
        // the receiver's own i_have, whose Round is the receiver's pushed Round
        std::vector<uint32_t> w(h->E);
        std::vector<uint4> vs(h->n);
        int rc = psim_get_inflight(h, w.data(), h->E);
        if (rc) return rc;
        HIPCHK(hh, hipMemcpy(vs.data(), h->vs, size_t(h->n) * 16, hipMemcpyDeviceToHost));
        const uint32_t mo = cur_mono(h);
        for (uint32_t v = 0; v < h->n; v++)
            for (uint64_t e = h->h_rowp[v]; e < h->h_rowp[v + 1]; e++) {
                uint32_t f = w[e] & 0xFFFFu, q = 0;
                for (; f; f >>= 4) {
                    PdMsg x;
                    x.type = f & 0xFu;
                    x.src = h->h_col[e];
                    x.dst = h->sh.v_lo + v;
                    x.seq = q++;
                    x.mono = x.type == PSIM_MSG_PRUNE ? 0u : mo;
                    x.round = (x.type == PSIM_MSG_BROADCAST || x.type == PSIM_MSG_IHAVE) ? (w[e] >> 16)
                            : (x.type == PSIM_MSG_PRUNE ? 0u : (vs[v].w & 0xFFFFu));
                    m.push_back(x);
                }
            }
    }
    *count = m.size();
    for (size_t i = 0; i < m.size() && i < cap; i++) {
        if (src) src[i] = m[i].src;
        if (dst) dst[i] = m[i].dst;
        if (kind) kind[i] = m[i].type;
        if (round) round[i] = m[i].round;
        if (mono) mono[i] = m[i].mono;
    }
    return PSIM_OK;
}

int psim_get_rows(const psim_handle* h, uint32_t v, uint32_t* peer, uint32_t* round, uint32_t* mono, size_t cap,
                  size_t* count) {
    if (!h || !count || !h->n || v >= h->n || h->bin.rec_c) return PSIM_EINVAL;
    psim_handle* hh = const_cast<psim_handle*>(h);
    HIPCHK(hh, hipSetDevice(h->device));
    HIPCHK(hh, hipStreamSynchronize(h->stream));
    std::vector<PdRow> r;
    if (h->win) {
        uint2 hd;
        HIPCHK(hh, hipMemcpy(&hd, h->win->head + v, sizeof hd, hipMemcpyDeviceToHost));
        r.resize(std::min<uint32_t>(hd.x, kWinRows));
        if (!r.empty())
            HIPCHK(hh, hipMemcpy(r.data(), h->win->rows + size_t(v) * kWinRows, r.size() * sizeof(PdRow),
                                 hipMemcpyDeviceToHost));
    } else {
        uint4 st;
        HIPCHK(hh, hipMemcpy(&st, h->vs + v, 16, hipMemcpyDeviceToHost));
        for (uint32_t m = st.z; m; m &= m - 1) {
            const uint32_t s = __builtin_ctz(m);
            r.push_back(PdRow{h->h_col[h->h_rowp[v] + s], cur_mono(h), st.w & 0xFFFFu});
        }
    }
    *count = r.size();
    for (size_t i = 0; i < r.size() && i < cap; i++) {
        if (peer) peer[i] = r[i].peer;
        if (round) round[i] = r[i].round;
        if (mono) mono[i] = r[i].mono;
    }
    return PSIM_OK;
}

int psim_get_delivered_mono(const psim_handle* h, uint32_t mono, uint8_t* delivered, size_t n) {
    if (!h || !delivered || n != h->n || !h->n) return PSIM_EINVAL;
    psim_handle* hh = const_cast<psim_handle*>(h);
    if (!h->win) {
        if (mono != cur_mono(h))
            return fail(hh, PSIM_EINVAL, "a static lane keeps the newest heartbeat (%u) only", cur_mono(h));
        return psim_get_delivered(h, delivered, n);
    }
    HIPCHK(hh, hipSetDevice(h->device));
    const size_t need = n;
    if (hh->scratch_cap < need) {
        if (hh->scratch_buf) (void)hipFree(hh->scratch_buf);
        hh->scratch_buf = nullptr;
        hh->scratch_cap = 0;
        if (hipMalloc(&hh->scratch_buf, need) != hipSuccess) return fail(hh, PSIM_ENOMEM, "delivered scratch");
        hh->scratch_cap = need;
    }
    HIPCHK(hh, launch_win_delivered(make_win_args(h, h->par, 0, h->stats), mono, (uint8_t*)hh->scratch_buf,
                                    h->stream));
    HIPCHK(hh, hipMemcpyAsync(delivered, hh->scratch_buf, n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hh, hipStreamSynchronize(h->stream));
    return PSIM_OK;
}

int psim_get_delivered_range(const psim_handle* h, uint32_t mono, uint32_t v0, size_t count, uint8_t* delivered) {
    if (!h || !h->n || (count && !delivered) || v0 > h->n || count > h->n - v0) return PSIM_EINVAL;
    if (!h->vs) return fail(const_cast<psim_handle*>(h), PSIM_ESTATE, "forest: no root heartbeated yet (no lane to read)");
    psim_handle* hh = const_cast<psim_handle*>(h);
    if (!count) return PSIM_OK;
    const uint32_t cm = cur_mono(h);
    if (mono == 0) mono = cm;
    HIPCHK(hh, hipSetDevice(h->device));
    HIPCHK(hh, hipStreamSynchronize(h->stream));
    if (mono == cm) {                          // the newest heartbeat: the records' Monotonic tags
        std::vector<uint4> vs(count);
        HIPCHK(hh, hipMemcpy(vs.data(), h->vs + v0, count * 16, hipMemcpyDeviceToHost));
        const uint32_t s8 = h->serial & 0xFFu;
        for (size_t i = 0; i < count; i++) delivered[i] = h->serial && ((vs[i].w >> 16) & 0xFFu) == s8;
        return PSIM_OK;
    }
    if (!h->win)
        return fail(hh, PSIM_EINVAL, "a static lane keeps the newest heartbeat (%u) only", cm);
    std::vector<uint4> is(2 * count);          // window lane: each vertex's timestamp interval set
    HIPCHK(hh, hipMemcpy(is.data(), h->win->iset + 2 * size_t(v0), count * 32, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < count; i++) {
        const uint32_t lo[4] = {is[2 * i].x, is[2 * i].y, is[2 * i].z, is[2 * i].w};
        const uint32_t hi[4] = {is[2 * i + 1].x, is[2 * i + 1].y, is[2 * i + 1].z, is[2 * i + 1].w};
        bool d = false;                        // is_stale (backend :229-244): same epoch -> member; else newer set
        if (lo[0] && (lo[0] >> 24) != (mono >> 24)) d = (lo[0] >> 24) > (mono >> 24);
        else
            for (int k = 0; k < 4; k++) d |= lo[k] && lo[k] <= mono && mono <= hi[k];
        delivered[i] = d;
    }
    return PSIM_OK;
}

int psim_get_delivered(const psim_handle* h, uint8_t* delivered, size_t n) {
    if (!h || !delivered || n != h->n || !h->n) return PSIM_EINVAL;
    if (!h->vs) return fail(const_cast<psim_handle*>(h), PSIM_ESTATE, "forest: no root heartbeated yet (no lane to read)");
    psim_handle* hh = const_cast<psim_handle*>(h);
    std::vector<uint4> vs(n);
    HIPCHK(hh, hipSetDevice(h->device));
    HIPCHK(hh, hipStreamSynchronize(h->stream));
    HIPCHK(hh, hipMemcpy(vs.data(), h->vs, n * 16, hipMemcpyDeviceToHost));
    const uint32_t s8 = h->serial & 0xFFu;
    for (size_t v = 0; v < n; v++) delivered[v] = h->serial && ((vs[v].w >> 16) & 0xFFu) == s8;
    return PSIM_OK;
}

int psim_get_inflight(const psim_handle* h, uint32_t* words, uint64_t n_words) {
    if (!h || !words || n_words != h->E) return PSIM_EINVAL;
    if (!h->vs) return fail(const_cast<psim_handle*>(h), PSIM_ESTATE, "forest: no root heartbeated yet (no lane to read)");
    psim_handle* hh = const_cast<psim_handle*>(h);
    if (h->win) return fail(hh, PSIM_ESTATE, "window lane (several heartbeats in flight): use psim_get_messages");
    HIPCHK(hh, hipSetDevice(h->device));
    HIPCHK(hh, hipStreamSynchronize(h->stream));
    if (!h->bin.rec_c) {
        const uint32_t tag = uint32_t(h->round + 1) & 0xFFu;   // words the next round reads
        const uint32_t* src = make_args(h, h->par, 0, h->stats).in_cur;   // in[par] or its ring slot
        if (h->ell) {                                          // ELL rows -> ABI (CSR) slots
            std::vector<uint32_t> d(h->Ed);
            HIPCHK(hh, hipMemcpy(d.data(), src, h->Ed * 4, hipMemcpyDeviceToHost));
            for (uint32_t v = 0; v < h->n; v++)
                for (uint64_t e = h->h_rowp[v]; e < h->h_rowp[v + 1]; e++) {
                    const uint32_t w = d[uint64_t(v) * h->ell + (e - h->h_rowp[v])];
                    words[e] = live_word(w, tag) ? abi_word(w) : 0u;
                }
            return PSIM_OK;
        }
        HIPCHK(hh, hipMemcpy(words, src, h->E * 4, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < h->E; i++) words[i] = live_word(words[i], tag) ? abi_word(words[i]) : 0u;
        return PSIM_OK;
    }
    // binned: the records waiting in the coarse bins the next round routes
    const auto& b = h->bin;
    const size_t NS = size_t(b.nc) * kCoarseShards;
    std::vector<uint32_t> cnt(NS);
    std::vector<uint2> rec(h->E);
    HIPCHK(hh, hipMemcpy(cnt.data(), b.cnt_c[h->par], NS * 4, hipMemcpyDeviceToHost));
    HIPCHK(hh, hipMemcpy(rec.data(), b.rec_c, h->E * 8, hipMemcpyDeviceToHost));
    memset(words, 0, h->E * 4);
    for (size_t c = 0; c < NS; c++)
        for (uint32_t i = 0; i < cnt[c]; i++) {
            const uint2 r = rec[size_t(b.h_csub[c]) + i];
            if (r.x >= h->E) return fail(hh, PSIM_ESTATE, "corrupt in-flight record");
            words[r.x] = abi_word(r.y);
        }
    return PSIM_OK;
}

}  // extern "C"

namespace {

void* scratch(psim_handle* h, size_t bytes) {
    if (bytes > h->scratch_cap) {
        if (h->scratch_buf) (void)hipFree(h->scratch_buf);
        h->scratch_buf = nullptr;
        h->scratch_cap = 0;
        if (hipMalloc(&h->scratch_buf, bytes) != hipSuccess) return nullptr;
        h->scratch_cap = bytes;
    }
    return h->scratch_buf;
}

// one batched vclock op over host buffers: A, B (or actor ids), outputs.
// op (launch_vc): 0 descends, 1 dominates, 4 equal -> outb[n]; 2 merge,
// 3 increment, 5 glb, 6 subtract_dots -> out[n][64]; 7 get_counter -> out[n]
int vc_op(psim_handle* h, int op, const uint32_t* a, const uint32_t* b, const uint32_t* actor, uint32_t* out,
          uint8_t* outb, size_t n) {
    if (!h || !a || n == 0) return n == 0 ? PSIM_OK : PSIM_EINVAL;
    const bool use_b = op != 3 && op != 7, use_act = op == 3 || op == 7;
    const bool bool_out = op == 0 || op == 1 || op == 4, clock_out = op == 2 || op == 3 || op == 5 || op == 6;
    if ((use_b && !b) || (use_act && !actor) || (!bool_out && !out) || (bool_out && !outb)) return PSIM_EINVAL;
    if (use_act)
        for (size_t i = 0; i < n; i++)
            if (actor[i] >= PSIM_VC_LANES) return fail(h, PSIM_EINVAL, "actor %u >= %d", actor[i], PSIM_VC_LANES);
    const size_t cb = n * PSIM_VC_LANES * 4;
    char* base = (char*)scratch(h, 3 * cb + n * 4 + n + 64);
    if (!base) return fail(h, PSIM_ENOMEM, "vclock scratch of %zu bytes", 3 * cb);
    uint32_t* da = (uint32_t*)base;
    uint32_t* db = (uint32_t*)(base + cb);
    uint32_t* dout = (uint32_t*)(base + 2 * cb);
    uint32_t* dact = (uint32_t*)(base + 3 * cb);
    uint8_t* doutb = (uint8_t*)(base + 3 * cb + n * 4);
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipMemcpyAsync(da, a, cb, hipMemcpyHostToDevice, h->stream));
    if (use_b) HIPCHK(h, hipMemcpyAsync(db, b, cb, hipMemcpyHostToDevice, h->stream));
    if (use_act) HIPCHK(h, hipMemcpyAsync(dact, actor, n * 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, launch_vc(op, da, db, dact, dout, doutb, n, h->stream));
    if (bool_out) HIPCHK(h, hipMemcpyAsync(outb, doutb, n, hipMemcpyDeviceToHost, h->stream));
    else HIPCHK(h, hipMemcpyAsync(out, dout, clock_out ? cb : n * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return PSIM_OK;
}

}  // namespace

extern "C" {

int psim_vclock_descends(psim_handle* h, const uint32_t* a, const uint32_t* b, uint8_t* out, size_t n) {
    return vc_op(h, 0, a, b, nullptr, nullptr, out, n);
}
int psim_vclock_dominates(psim_handle* h, const uint32_t* a, const uint32_t* b, uint8_t* out, size_t n) {
    return vc_op(h, 1, a, b, nullptr, nullptr, out, n);
}
int psim_vclock_merge(psim_handle* h, const uint32_t* a, const uint32_t* b, uint32_t* out, size_t n) {
    return vc_op(h, 2, a, b, nullptr, out, nullptr, n);
}
int psim_vclock_increment(psim_handle* h, const uint32_t* a, const uint32_t* actor, uint32_t* out, size_t n) {
    return vc_op(h, 3, a, nullptr, actor, out, nullptr, n);
}
int psim_vclock_equal(psim_handle* h, const uint32_t* a, const uint32_t* b, uint8_t* out, size_t n) {
    return vc_op(h, 4, a, b, nullptr, nullptr, out, n);
}
int psim_vclock_glb(psim_handle* h, const uint32_t* a, const uint32_t* b, uint32_t* out, size_t n) {
    return vc_op(h, 5, a, b, nullptr, out, nullptr, n);
}
int psim_vclock_subtract_dots(psim_handle* h, const uint32_t* dots, const uint32_t* clock, uint32_t* out, size_t n) {
    return vc_op(h, 6, dots, clock, nullptr, out, nullptr, n);
}
int psim_vclock_get_counter(psim_handle* h, const uint32_t* a, const uint32_t* actor, uint32_t* out, size_t n) {
    return vc_op(h, 7, a, nullptr, actor, out, nullptr, n);
}

int psim_forest_set_lanes(psim_handle* h, uint32_t lanes) {
    if (!h) return PSIM_EINVAL;
    if (!h->fo.on) return fail(h, PSIM_ESTATE, "not a forest (psim_config.max_roots <= 16)");
    if (h->n) return fail(h, PSIM_ESTATE, "set the forest's lanes before psim_load_csr");
    if (lanes > h->fo.cap) return fail(h, PSIM_EINVAL, "lanes=%u > max_roots=%u", lanes, h->fo.cap);
    h->fo.lanes = lanes;
    return PSIM_OK;
}

int psim_plumtree_focus(psim_handle* h, uint32_t root) {
    if (!h || !h->n) return PSIM_ESTATE;
    if (h->fo.on) {
        const auto it = h->fo.lane_of.find(root);
        if (it != h->fo.lane_of.end()) {
            forest_focus(h, int(it->second));
            return PSIM_OK;
        }
        const auto is = h->fo.slot_of.find(root);   // a parked root: its records, nothing in flight
        if (is == h->fo.slot_of.end()) return fail(h, PSIM_EINVAL, "root %u has no heartbeat tree", root);
        forest_focus_parked(h, is->second);
        return PSIM_OK;
    }
    if (!lanes_enabled(h)) return h->have_root && h->root == root ? PSIM_OK : PSIM_EINVAL;
    return focus_root(h, root, false);
}

int psim_set_omissions(psim_handle* h, const uint32_t* src, const uint32_t* dst, size_t k) {
    if (!h || !h->n || (k && (!src || !dst))) return PSIM_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    std::vector<uint32_t> bm((h->Ed + 31) / 32, 0u);
    size_t hit = 0;
    for (size_t i = 0; i < k; i++) {
        if (src[i] >= h->sh.n_global || dst[i] >= h->sh.n_global)
            return fail(h, PSIM_EINVAL, "omission pair (%u, %u) out of range", src[i], dst[i]);
        const uint32_t u = src[i] - h->sh.v_lo;
        if (u >= h->n) continue;                       // another shard's sender
        const auto b = h->h_col.begin() + h->h_rowp[u], e = h->h_col.begin() + h->h_rowp[u + 1];
        const auto it = std::lower_bound(b, e, dst[i]);
        if (it == e || *it != dst[i]) continue;        // not an overlay edge: nothing ever flows
        size_t s = size_t(it - h->h_col.begin());
        if (h->ell) s = size_t(u) * h->ell + (s - h->h_rowp[u]);   // device (ELL) slot
        bm[s >> 5] |= 1u << (s & 31);
        hit++;
    }
    if (h->omit) (void)hipFree(h->omit);
    h->omit = nullptr;
    if (!hit) return PSIM_OK;                          // healed (or no local edge affected)
    if (hipMalloc((void**)&h->omit, bm.size() * 4) != hipSuccess) return fail(h, PSIM_ENOMEM, "omission bitmap");
    HIPCHK(h, hipMemcpy(h->omit, bm.data(), bm.size() * 4, hipMemcpyHostToDevice));
    return PSIM_OK;
}

int psim_set_delays(psim_handle* h, const uint32_t* src, const uint32_t* dst, const uint8_t* rounds, size_t k) {
    if (h && h->fo.on && h->sh.world > 1)
        return fail(h, PSIM_ENOTSUP, "delay faults on a sharded forest (max_roots > 16 over several GPUs)");
    if (!h || !h->n || (k && (!src || !dst || !rounds))) return PSIM_EINVAL;
    if (h->bin.rec_c) return fail(h, PSIM_ENOTSUP, "delay faults need the slot-scatter engine (not the binned one)");
    if (h->sh.world > 1 && h->win)      // lane layouts are decided alike on every rank (global counts)
        return fail(h, PSIM_ENOTSUP, "delay faults on a sharded window lane (overlapping heartbeats)");
    if (h->sh.world > 1 && h->sh.pending)
        return fail(h, PSIM_ESTATE, "delay faults on a sharded handle with async rounds pending");
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    save_lane(h);
    int64_t v[1 + kNCodes];
    int64_t& busy = v[0];
    busy = 0;
    int lrc = PSIM_OK;
    for (const auto& l : h->lanes) {
        if (l.win && !lrc) lrc = fail(h, PSIM_ENOTSUP, "delay faults on a window lane (overlapping heartbeats)");
        busy += (int64_t)l.inflight;
    }
    if (h->fo.on) busy = (int64_t)h->inflight;   // the forest: every lane's messages (delays: still pending)
    if (h->sh.world > 1) {
        // collective: every rank must return the same code, and a shard's own
        // in-flight count says nothing about the others' (ADVICE r3), so the
        // decision is taken on the global sum before any state changes; a
        // rank's own refusal (a window lane) travels in the same all-reduce
        //  instead of leaving the others in it
        if (!h->sh.xport) return fail(h, PSIM_ESTATE, "delay faults on a sharded handle need the in-library exchange");
        put_code(v + 1, lrc);
        std::string err;
        const int rc = h->sh.xport->allreduce(v, 1 + kNCodes, h->stream, &err);
        if (rc) return fail(h, rc, "delay all-reduce: %s", err.c_str());
        lrc = finish_code(h, v + 1, lrc, "psim_set_delays");
    }
    if (lrc) return lrc;
    if (busy) return fail(h, PSIM_EBUSY, "messages in flight: a delay change could reorder a pair");
    // every shard installs the table (its own senders' pairs) and the ring,
    // so a delayed word from any shard finds its receiver's inbox ring
    std::vector<uint8_t> dl(h->Ed, 0);
    for (size_t i = 0; i < k; i++) {
        if (src[i] >= h->sh.n_global || dst[i] >= h->sh.n_global)
            return fail(h, PSIM_EINVAL, "delay pair (%u, %u) out of range", src[i], dst[i]);
        if (rounds[i] > kMaxDelay) return fail(h, PSIM_EINVAL, "delay %u > %u rounds", rounds[i], kMaxDelay);
        const uint32_t u = src[i] - h->sh.v_lo;
        if (u >= h->n) continue;                       // another shard's sender
        const auto b = h->h_col.begin() + h->h_rowp[u], e = h->h_col.begin() + h->h_rowp[u + 1];
        const auto it = std::lower_bound(b, e, dst[i]);
        if (it == e || *it != dst[i]) continue;        // not an overlay edge: nothing ever flows
        size_t s = size_t(it - h->h_col.begin());
        if (h->ell) s = size_t(u) * h->ell + (s - h->h_rowp[u]);   // device (ELL) slot
        dl[s] = rounds[i];
    }
    if (!h->dly) {
        // switch every lane to the ring; nothing is in flight, so no word moves
        if (hipMalloc((void**)&h->dly, h->Ed) != hipSuccess) return fail(h, PSIM_ENOMEM, "delay table");
        // (sharded: each lane also stages its cross-shard delayed words in a ring of its own)
        if (h->sh.world > 1) h->sh.plan_ok = false;
        const int focus = h->cur_lane;
        for (int j = 0; j < (int)h->lanes.size(); j++) {
            auto& l = h->lanes[j];
            if (alloc_ring(h, l.ring, l.pring) != PSIM_OK ||
                (h->sh.world > 1 && !alloc_zero((void**)&l.srg, size_t(kRing) * h->Ed * 4))) {
                load_lane(h, focus);
                return fail(h, PSIM_ENOMEM, "delay ring of heartbeat lane %d", j);
            }
            for (auto& x : l.due) x = 0;
        }
        if (h->lanes.empty() && h->sh.world > 1 && !h->fo.on &&
            !alloc_zero((void**)&h->sh.srg, size_t(kRing) * h->Ed * 4))
            return fail(h, PSIM_ENOMEM, "staging ring of the delay faults");
        if (h->fo.on) {
            // every lane's inbox becomes a ring (nothing is in flight: no word moves)
            auto& f = h->fo;
            const size_t ng = (size_t(h->n) + (1u << kGroupShift) - 1) >> kGroupShift;
            f.s_ring = (uint64_t(kRing) * h->Ed + 63) & ~uint64_t(63);
            f.s_pring = (uint64_t(kRing) * ng + 255) & ~uint64_t(255);
            size_t fr = 0, tot = 0;
            HIPCHK(h, hipMemGetInfo(&fr, &tot));
            const uint64_t need = uint64_t(f.slabs()) * (f.s_ring * 4 + f.s_pring);
            if (need + (uint64_t(1) << 30) > fr ||
                !alloc_zero((void**)&f.ring, uint64_t(f.slabs()) * f.s_ring * 4) ||
                !alloc_zero((void**)&f.pring, uint64_t(f.slabs()) * f.s_pring)) {
                if (f.ring) (void)hipFree(f.ring);
                f.ring = nullptr;
                (void)hipFree(h->dly);
                h->dly = nullptr;
                return fail(h, PSIM_ENOMEM, "forest delay rings: %.2f GB for %u lanes", double(need) / 1e9,
                            f.slabs());
            }
            for (auto& x : h->due) x = 0;
            forest_refocus(h);
        }
        if (!h->lanes.empty()) load_lane(h, focus);
    }
    HIPCHK(h, hipMemcpy(h->dly, dl.data(), h->Ed, hipMemcpyHostToDevice));
    return PSIM_OK;
}

int psim_trace_hash(const psim_handle* h, uint64_t* out) {
    if (!h || !out || !h->n) return PSIM_EINVAL;
    if (!h->vs) return fail(const_cast<psim_handle*>(h), PSIM_ESTATE, "forest: no root heartbeated yet (no lane to read)");
    psim_handle* hh = const_cast<psim_handle*>(h);
    HIPCHK(hh, hipSetDevice(h->device));
    PtArgs a = make_args(h, h->par, 0, h->stats);
    const uint32_t rl = h->have_root ? h->root - h->sh.v_lo : 0xFFFFFFFFu;
    HIPCHK(hh, hipMemsetAsync(h->scratch, 0, 32, h->stream));
    HIPCHK(hh, launch_pt_hash(a, h->serial != 0, rl < h->n ? rl : 0xFFFFFFFFu,
                              (h->bin.rec_c || h->win) ? 0ull : h->Ed, h->scratch, h->stream));
    if (h->win) HIPCHK(hh, launch_win_hash(make_win_args(h, h->par, 0, h->stats), h->scratch, h->stream));
    unsigned long long r[4];
    HIPCHK(hh, hipMemcpyAsync(r, h->scratch, 32, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hh, hipStreamSynchronize(h->stream));
    out[0] = r[0];
    out[1] = r[1];
    out[2] = r[2];
    out[3] = h->round;
    return PSIM_OK;
}

int psim_shard_transport_info(const psim_handle* h, int* kind, int* comm_world, int* comm_rank) {
    if (!h) return PSIM_EINVAL;
    const psim::Transport* t = h->sh.xport;
    if (kind) *kind = !t ? 0 : (std::string(t->name()) == "rccl" ? 1 : 2);
    if (comm_world) *comm_world = t ? t->comm_size() : -1;
    if (comm_rank) *comm_rank = t ? t->comm_rank() : -1;
    return PSIM_OK;
}

int psim_set_chunk_timing(psim_handle* h, int chunk) {
    if (!h) return PSIM_EINVAL;
    if (h->sh.pending) return fail(h, PSIM_ESTATE, "collect the async rounds first");
    if (chunk) h->cfg.flags |= PSIM_CFG_CHUNK_TIMING;
    else h->cfg.flags &= ~PSIM_CFG_CHUNK_TIMING;
    return PSIM_OK;
}

int psim_get_timing(const psim_handle* h, double* round_kernel_ms, uint64_t* rounds) {
    if (!h) return PSIM_EINVAL;
    if (round_kernel_ms) *round_kernel_ms = h->kernel_ms_total;
    if (rounds) *rounds = h->rounds_total;
    return PSIM_OK;
}

}  // extern "C"


