// psim_internal.h -- shared between the host ABI (psim_host.hip) and the
// Plumtree kernels (plumtree.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <string>

typedef struct psim_handle psim_handle;
typedef struct psim_scamp_stats psim_scamp_stats;
typedef struct psim_transport psim_transport;

namespace psim {

// hipMalloc + zero fill, finished before returning.  hipMemset runs on the
// null stream, which does not order with the handles' non-blocking streams:
// without the device sync a fill could land after work the handle's stream
// enqueues next (e.g. an upload into a freshly grown buffer).
inline bool alloc_zero(void** p, size_t bytes) {
    if (!bytes) bytes = 8;
    return hipMalloc(p, bytes) == hipSuccess && hipMemset(*p, 0, bytes) == hipSuccess &&
           hipDeviceSynchronize() == hipSuccess;
}

constexpr int kBlock = 256;          // threads per workgroup (4 waves of 64)

// One slot of a shared record queue for each calling lane: the lanes of a
// wave that reach the call together share ONE atomicAdd on the counter (the
// lowest active lane's), each taking base + its rank among them.  Record
// order in the queues never matters (every consumer re-sorts by (src, seq)),
// and one atomic per message on a single counter serialises at L2.
__device__ __forceinline__ uint32_t wave_reserve(uint32_t* counter) {
    const unsigned long long act = __ballot(1);
    const uint32_t lane = __lane_id();
    const uint32_t leader = (uint32_t)__ffsll((long long)act) - 1;
    const uint32_t rank = (uint32_t)__popcll(act & ((1ull << lane) - 1ull));
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(act));
    base = __shfl(base, (int)leader, 64);
    return base + rank;
}
// k < 2^10 consecutive slots for each calling lane, ONE atomicAdd per wave:
// the wave's exclusive prefix of k is assembled from one ballot per bit of k
// (ballots see exactly the active lanes, so it holds in divergent code).
__device__ __forceinline__ uint32_t wave_reserve_n(uint32_t* counter, uint32_t k) {
    const unsigned long long act = __ballot(1);
    const uint32_t lane = __lane_id();
    const uint32_t leader = (uint32_t)__ffsll((long long)act) - 1;
    const unsigned long long lt = (1ull << lane) - 1ull;
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t b = 0; b < 10; b++) {
        const unsigned long long m = __ballot((k >> b) & 1u);
        pre += (uint32_t)__popcll(m & lt) << b;
        tot += (uint32_t)__popcll(m) << b;
    }
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, tot);
    base = __shfl(base, (int)leader, 64);
    return base + pre;
}
// A wave's send buffer in LDS (the SCAMP and C3 handlers, which send one
// record at a time from divergent code).  A send reserves records of its
// wave's buffer with ONE LDS atomic per wave (wave_reserve's shape, on LDS)
// and stores its record there; at the kernel's end the wave moves the buffer
// to the global queue with one global atomicAdd of its exact count and
// coalesced stores.  wave_reserve cost a device-scope atomic per send call,
// whose return every sending lane waited for, on one counter every wave of
// the chip hit.  A buffer past kWq records sends straight to the global
// queue (wave_reserve).  No holes: the queue stays dense.
// Only read-modify-writes hand records out: lanes in the two arms of a branch
// run one arm after the other, and the compiler may sink an arm's plain LDS
// stores past the other arm (tools/mb/mb_wq.hip caught a count kept that way).
constexpr uint32_t kWq = 256;
template <class Rec>
struct WaveQ {
    Rec* buf;          // LDS [kWq]
    uint32_t* n;       // LDS: records reserved (may pass kWq)
};
__device__ __forceinline__ void wq_init(uint32_t* n) {
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(n, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
template <class Rec>
__device__ __forceinline__ void wq_send(WaveQ<Rec> q, uint32_t* counter, Rec* __restrict__ out, uint32_t cap,
                                        uint32_t& err, const Rec& r) {
    const unsigned long long act = __ballot(1);
    const uint32_t lane = __lane_id();
    const uint32_t leader = (uint32_t)__ffsll((long long)act) - 1;
    const uint32_t rank = (uint32_t)__popcll(act & ((1ull << lane) - 1ull));
    uint32_t k = 0;
    if (lane == leader)
        k = __hip_atomic_fetch_add(q.n, (uint32_t)__popcll(act), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    k = __shfl(k, (int)leader, 64) + rank;
    if (k < kWq) {
        q.buf[k] = r;
        return;
    }
    const uint32_t pos = wave_reserve(counter);     // the buffer is full: the global queue directly
    if (pos < cap) out[pos] = r;
    else err |= 1u;
}
// At the kernel's end, by all 64 lanes of the wave (converged).
template <class Rec>
__device__ __forceinline__ void wq_flush(WaveQ<Rec> q, uint32_t* counter, Rec* __restrict__ out, uint32_t cap,
                                         uint32_t& err) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");   // every lane's records are in LDS
    uint32_t n = __hip_atomic_load(q.n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    n = n < kWq ? n : kWq;
    if (n == 0) return;
    const uint32_t lane = __lane_id();
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(counter, n);
    base = __shfl(base, 0, 64);
    if (base + n > cap) err |= 1u;
    for (uint32_t i = lane; i < n; i += 64)
        if (base + i < cap) out[base + i] = q.buf[i];
}
// Per-lane round-count area (PtArgs::mcnt), u32 words:
//   [0, 256)    messages sent per round, [4 rounds][64 shards]
//   [256, 512)  worklist entries per round, [4][64] (PtArgs::wlcnt)
//   [512, 516)  row holders at the END of round k (k mod 4): round R writes
//               slot R-1 once (block 0) -- a value no workgroup of R reads
//   [516, 520)  change in row holders during round k (two's complement)
//   [520, 524)  1 = round k (k mod 4) wrote no group flags (its senders were
//               flag-free: the next round reads every group); written by block
//               0 of round k, read by round k + 1 (0, the zeroed state, = flags)
// Round R's "any row due" test reads holders(R-2) + delta(R-1): both written
// by earlier launches, so every workgroup of a launch takes the same decision
// (the running count PtArgs::ost_total moves while the launch runs).
constexpr size_t kMcntHold = 512;
constexpr size_t kMcntHoldD = 516;
constexpr size_t kMcntFF = 520;
constexpr size_t kMcntLane = 524;
constexpr int kMaxDeg = 32;          // peer slots per vertex (u32 masks)
constexpr int kStatShards = 64;      // counter shards (blockIdx & 63) to spread atomics
constexpr int kNStat = 16;           // counters per shard
#ifndef PSIM_GROUP_SHIFT
#define PSIM_GROUP_SHIFT 4               // A/B knob (-DPSIM_GROUP_SHIFT=2 / 3 builds, profiles/r06/experiments)
#endif
constexpr int kGroupShift = PSIM_GROUP_SHIFT;   // inbox flags cover 16-vertex groups (625 KB at 10M: L2-resident)
static_assert(kGroupShift >= 2 && kGroupShift <= 8, "a group spans whole 4-vertex thread quads");
constexpr uint32_t kChunkV = 1024;   // vertices owned by one round-kernel workgroup
// binned engine (single GPU): messages travel as {receiver
// slot, word} records through coarse then fine receiver bins
constexpr uint32_t kBinSlots = 4096;   // LDS inbox words of one fine bin (16 KB)
constexpr uint32_t kBinVMax = 512;     // vertices of a fine bin (2 per thread)
constexpr uint32_t kCoarseMax = 512;   // coarse bins; also fine bins per coarse bin
constexpr uint32_t kRouteK = 4096;     // records one route workgroup moves (16 per thread)
constexpr uint32_t kCoarseShards = 32; // sub-regions per coarse bin (fine bin f appends to f % 32):
                                       // spreads the reservation atomics over 32 counters

// counter indices (1..5 = PSIM_MSG_* kinds)
enum Stat : int {
    S_DELIV = 6,        // merge/2 returned true
    S_ACTIVE = 7,       // vertices that processed messages or a tick
    S_SENDERS = 8,      // vertices that emitted >= 1 message
    S_DEGSUM = 9,       // sum of deg over senders
    S_OST_DELTA = 10,   // change in #vertices with outstanding rows (two's complement)
    S_LIVE_DELTA = 11,  // change in #outstanding rows to live peers (two's complement)
    S_OVERFLOW = 12,    // bit0: per-edge FIFO > 4 ; bit1: Round > 4095 ; bit2: rows of an older heartbeat
    S_WORDS = 13,       // inbox words stored (random 4-byte stores; omitted words are not stored)
};

// Slot-scatter inbox word (one per receiver slot):
//   [11:0]  FIFO of <= 4 message kinds, 3 bits each (PSIM_MSG_*, first in the low bits)
//   [19:12] round tag: the round that reads the word, mod 256 -- consumed words
//           are never cleared; a word whose tag is not the reading round's is
//           stale (buffers are zeroed once at least every 256 rounds)
//   [31:20] Round carried by broadcast / i_have (< 4096)
// The ABI form (psim_get_inflight) is 4-bit kinds in [15:0], Round in [31:16].
constexpr uint32_t kKindBits = 3;
constexpr uint32_t kFifoMask = 0xFFFu;
constexpr uint32_t kTagShift = 12;
constexpr uint32_t kRoundShift = 20;
constexpr uint32_t kMaxRound = 0xFFFu;
constexpr uint32_t kTagSpan = 256;     // rounds before a tag repeats
constexpr uint32_t kNoPeer = 0xFFFFFFFFu;   // col of an ELL padding slot
constexpr uint32_t kEllMax = 8;              // widest ELL row (the round kernel's register-resident rows)
constexpr uint32_t kRing = 16;               // inbox ring with delay faults: a word is written <= kRing - 1
constexpr uint32_t kMaxDelay = kRing - 2;    // rounds ahead of the round that reads the slot being written
constexpr int kDelayHist = kRing;            // per-round stats row tail: messages per delay
__host__ __device__ inline uint32_t word_tag(uint32_t w) { return (w >> kTagShift) & 0xFFu; }
// a word carries messages for the round whose tag is `tag`
__host__ __device__ inline bool live_word(uint32_t w, uint32_t tag) { return (w & kFifoMask) && word_tag(w) == tag; }
__host__ __device__ inline uint32_t abi_word(uint32_t w) {   // inbox word -> psim_get_inflight form
    uint32_t f = w & kFifoMask, o = 0;
    for (uint32_t i = 0; f; i++, f >>= kKindBits) o |= (f & 7u) << (4 * i);
    return o | ((w >> kRoundShift) << 16);
}

// Per-vertex Plumtree state, one 16-byte record (one dwordx4 load):
//   x = eager mask, y = lazy mask, z = outstanding mask (bits = slots)
//   w = [15:0] round pushed by this vertex (accepted Round + 1; 0 at the root)
//       [23:16] low 8 bits of the Monotonic last delivered (Mod:merge/2)
//       [31:24] tree epoch (a mismatch == no per-root map entry: common sets)
struct PtArgs {
    uint32_t n;                            // vertices of this shard (all of them on one GPU)
    uint32_t v_lo;                         // global id of local vertex 0
    uint32_t slot_base;                    // global device slot id of local slot 0 (ELL: v_lo * W)
    uint32_t abi_slot_base;                // the same as an ABI (CSR) slot id
    uint32_t* __restrict__ stage;          // [E_local] words for receivers on other shards (sharded only)
    const uint32_t* __restrict__ rowp;     // [n+1] local slot row pointers
    const uint32_t* __restrict__ col;      // [E]   neighbour (global) id per slot (sorted in a row)
    const uint32_t* __restrict__ rev;      // [E]   global slot id of the reverse slot
    const uint32_t* __restrict__ ecol;     // [n*W] ELL only: col << 3 | reverse slot s' (rev = col*W + s'),
                                           //       kNoPeer for padding; null = read col / rev
    const uint32_t* __restrict__ memb;     // [n]   member mask = common_eagers
    const uint32_t* __restrict__ alive;    // [ceil(N/32)] bitmap over GLOBAL ids
    uint4* __restrict__ vs;                // [n]   state records
    uint32_t* __restrict__ in_cur;         // [E]   words read this round (receiver slots)
    uint32_t* __restrict__ in_nxt;         // [E]   words written this round
    uint8_t* __restrict__ pend_cur;        // [ceil(n/16)] 1 = some vertex of the group has words
    uint8_t* __restrict__ pend_nxt;
    uint8_t* __restrict__ ost;             // [n+3] 1 = outstanding rows exist
    int* ost_total;                        // device count of vertices with outstanding rows
    // messages sent per round, [4 rounds][64 shards] (null: no early exit, group flags always written):
    // round R adds its count into slot m_w = R mod 4, reads R-1 (m_s: no message -> no-op round; many ->
    // this round's senders write no group flags) and R-2 (m_r: the last round wrote none -> every group
    // is read), and zeroes m_z = (R+1) mod 4
    uint32_t* mcnt;
    uint32_t m_w, m_s, m_r, m_z;
    uint32_t dense;                        // a round following >= dense messages runs flag-free
    // sparse rounds (ELL, one GPU; null wl_cur: off): a round following < wl_thr messages lists the
    // groups it flags -- 64 shards of wl_cap entries, counts in wlcnt [4 rounds][64] like mcnt -- and
    // the next round reads only those groups (plumtree.hip round_counts)
    uint32_t* wlcnt;
    uint32_t* wl_cur;
    uint32_t* wl_nxt;
    uint32_t wl_cap, wl_thr;
    uint32_t wl_gpc;                       // listed groups per ELL chunk (0: spread over the grid; A/B knob)
    uint32_t wl_wgs;                       // list mode: groups spread over at most this many workgroups (0: the
                                           // grid; psim_host.hip psim_handle::wl_wgs)
    uint32_t ell_grid;                     // ELL kernel grid = resident workgroups (0: one per chunk)
    uint32_t force_flags;                  // this round writes group flags whatever its count (the last round
                                           // of a sharded psim_shard_step: readers without counts come next)
    unsigned long long* __restrict__ stats;  // [kStatShards][kNStat]
    uint32_t tick;                         // lazy tick fires at the end of this round
    uint32_t mono8;                        // current heartbeat Monotonic (low 8 bits)
    uint32_t epoch8;                       // current tree epoch (low 8 bits)
    uint32_t root;                         // local index of the current heartbeat's origin
    uint32_t ctag, wtag;                   // round tags of the words read / written this round
    uint32_t ell;                          // row width of the ELL slot layout (slot s of v = v*ell + s;
                                           // padding slots: col = kNoPeer), 0 = CSR (rowp)
    const uint32_t* __restrict__ omit;     // [ceil(E/32)] omission faults over sender slots, or null
    // delay faults (psim_set_delays; null dly: none): the inbox is a ring of
    // kRing buffers, ring slot k holding the words read by the rounds = k mod kRing
    const uint8_t* __restrict__ dly;       // [E] extra rounds per sender slot (<= kMaxDelay)
    uint32_t* __restrict__ ring;           // [kRing][ed] inbox words
    uint8_t* __restrict__ pring;           // [kRing][ngrp] group flags
    unsigned long long* __restrict__ dhist;  // [kRing] messages written this round per delay
    uint32_t rpos;                         // ring slot read by the round after this one
    // sharded handles: the staging words of remote receivers as a ring too --
    // slot k holds the words the exchange after round k (mod kRing) carries,
    // i.e. those arriving in round k + 1; `stage` points at this round's slot
    uint32_t* __restrict__ srg;            // [kRing][ed] (null: not sharded or no delays)
    uint32_t ed, ngrp;                     // words per ring slot, flags per ring slot
    // binned engine (null for the slot-scatter engine)
    uint2* __restrict__ rec_c;             // [E] coarse-bin regions: {receiver slot, word}
    uint2* __restrict__ rec_f;             // [E] fine-bin regions
    uint32_t* __restrict__ cnt_c_cur;      // [nc][kCoarseShards] records per sub-region, routed this round
    uint32_t* __restrict__ cnt_c_nxt;      // ... emitted this round
    uint32_t* __restrict__ cnt_f;          // [nf] records per fine region
    const uint32_t* __restrict__ csub;     // [nc*kCoarseShards+1] sub-region starts (record index)
    const uint32_t* __restrict__ fslot;    // [nf+1] first slot of each fine bin
    uint32_t* __restrict__ obin;           // [nf] vertices of the fine bin holding outstanding rows
    uint32_t fv_shift, cv_shift;           // fine bin = 2^fv_shift vertices, coarse = 2^cv_shift
    uint32_t nf, nc, chunks;               // bins; route chunks per sub-region
    // a heartbeat enqueued before the previous one was read back
    // (psim_plumtree_broadcast_run_n, psim_host.hip): spec[0] = 1 makes every
    // kernel of it return at once, spec[1] = its origin's decision (1 run,
    // 2 abandoned).  The origin runs it only if the previous heartbeat ended
    // exactly at its predicted last round, ring slot spec_rl (mod 4): no
    // message in that round, some in the one before, no row holder left.
    // null: no guard (every other launch).
    uint32_t* spec;
    uint32_t spec_rl;
};

// The forest (psim_config.max_roots > 16): every node's
// heartbeat tree (partisan_plumtree_backend.erl:341-368, 421-428) in one
// slab per array -- lane L of a slab is root L's copy of the single-lane
// array -- and one launch per round over every lane (blockIdx.y = lane).
// All lanes share the round clock: one inbox parity, one set of round tags,
// one count-ring position; each keeps its own counts, worklist and holders.
struct FoArgs {
    PtArgs a;                              // this round's arguments at lane 0's slices
    uint64_t s_vs, s_in, s_pend, s_ost;    // per-lane strides: uint4 records, u32 words, bytes, bytes
    uint64_t s_stage;                      // sharded forest: u32 staged words per lane (a.stage = lane 0's)
    const uint2* __restrict__ info;        // [slots] {Monotonic tag (low 8 bits), local root}
    uint32_t lane0, nl;                    // this launch: lanes [lane0, lane0 + gridDim.y) of [0, nl)
    // parked roots (psim_forest_set_lanes): a root's per-root records (vs, its
    // state slot) outlive its lane; lane L runs the root whose slot is
    // slot[L].  Null: slot = lane (every root keeps its lane for good).
    const uint32_t* __restrict__ slot;     // [lanes] state slot of each lane's root
    uint32_t ns;                           // slots holding a root (= nl without parking)
};
// one round over lanes [0, f.nl): gx workgroups per lane (0: the round kernel's own choice)
hipError_t launch_fo_round(FoArgs f, uint32_t gx, hipStream_t s);
// the origins of lanes[0, k) (one root each; a.mono8 / a.root from f.info)
hipError_t launch_fo_origin(const FoArgs& f, const uint32_t* lanes, uint32_t k, hipStream_t s);
// out[i] = lane lanes[i] has messages of its last round (count slot `slot`) or rows
hipError_t launch_fo_busy(const FoArgs& f, const uint32_t* lanes, uint32_t k, uint32_t slot, uint32_t* out,
                          hipStream_t s);
// every lane's row-holder ring from its exact count (a.m_r, a.m_s as PtArgs)
hipError_t launch_fo_seed(const FoArgs& f, hipStream_t s);
// tag re-base of state slots slots[0, k) (slots == null: slots [0, k))
hipError_t launch_fo_renorm(const FoArgs& f, const uint32_t* slots, uint32_t k, hipStream_t s);
// outstanding rows to live peers over every lane -> *out (added)
hipError_t launch_fo_count_live(const FoArgs& f, unsigned long long* out, hipStream_t s);
// sharded forest: every lane's staged remote words -> the dense send regions
// (region d = lane after lane, psim_shard_layout order; sb = the layout's
// [world + 1] bases on the device), and the received regions -> each lane's
// inbox (rb = the recv layout's bases; fixed_mark >= 0 overrides ingest_mark)
hipError_t launch_fo_pack_dense(FoArgs f, const uint32_t* rem, uint32_t nrem, const uint64_t* sb, uint32_t world,
                                uint32_t* send, hipStream_t s);
hipError_t launch_fo_ingest_dense(FoArgs f, const uint32_t* recv, const uint32_t* recv_map, uint32_t nrecv,
                                  const uint64_t* rb, uint32_t world, const uint32_t* slot2v, int fixed_mark,
                                  hipStream_t s);
// a backend restart at local vertex v: v forgets every origin (each slot's delivered tag)
hipError_t launch_fo_forget(const FoArgs& f, uint32_t v, hipStream_t s);

// Demers rumor mongering + anti-entropy (demers.hip)
constexpr uint32_t kDmPushCap = 24;   // AE pushes one vertex can receive per tick (Poisson(2) in-degree)
constexpr uint32_t kDmFastPush = 8;   // pushes handled in registers (the rest: the generic walk)
struct DmArgs {
    uint32_t n, m;                        // n = vertices of this shard (all of them on one GPU)
    uint32_t v_lo, n_global;              // global id of local vertex 0; membership size
    uint32_t sharded;                     // 1: AE pushes are listed by dm_pushscan after the snapshot all-gather
    uint2 key;                            // Philox key {seed_lo, seed_hi}
    uint32_t rm_on;
    uint32_t tick, tick_idx, prev_tick;   // AE tick at the end of this round; tick indices
    uint64_t dpc;                         // draws per select_random_sublist call (philox.h dm_draws_per_call)
    unsigned long long dm_mail;           // direct mail: rumor ids every vertex receives this round
    unsigned long long full;              // every rumor id's bit
    unsigned long long* __restrict__ seen;       // [n] the message store
    unsigned long long* __restrict__ snap;       // [n_global] AE payload taken at the tick (global ids)
    // RM inbox: rumors received this round from >= 1 / >= 2 / >= 3 senders (bit planes of a
    // saturating count; senders raise them with atomicOr cascades) -- cur [n], nxt [n_global]
    unsigned long long* __restrict__ rm_cur_any;
    unsigned long long* __restrict__ rm_cur_multi;
    unsigned long long* __restrict__ rm_cur_tri;
    unsigned long long* __restrict__ rm_nxt_any;
    unsigned long long* __restrict__ rm_nxt_multi;
    unsigned long long* __restrict__ rm_nxt_tri;
    // each vertex's RM process (its sequential draw stream): the rumors it called
    // select_random_sublist for in the last round and the calls it made before that
    // round (global ids, all vertices), and the same for this round (every vertex
    // writes its own every round)
    const unsigned long long* __restrict__ rmnew_prev;
    const uint32_t* __restrict__ ncall_prev;
    unsigned long long* __restrict__ rmnew_cur;
    uint32_t* __restrict__ ncall_cur;
    uint32_t* __restrict__ pushcnt_cur;   // [n]
    uint32_t* __restrict__ pushcnt_nxt;
    uint32_t* __restrict__ pushlist_cur;  // [n][kDmPushCap]
    uint32_t* __restrict__ pushlist_nxt;
    unsigned long long* __restrict__ pull_cur;   // [n][2]
    unsigned long long* __restrict__ pull_nxt;   // [n_global][2]
    unsigned long long* __restrict__ stats;      // [kStatShards][kNStat]: 1 rm, 2 push, 3 pull, 4 deliv, 5 complete, 6 overflow
    uint32_t push_cap;                    // AE pushes per vertex and tick before PSIM_EOVERFLOW (<= kDmPushCap;
                                          // PSIM_DM_PUSHCAP lowers it to test the overflow path)
};
hipError_t launch_dm_origins(uint2 key, uint32_t n, uint32_t m, uint32_t* origin, hipStream_t s);
hipError_t launch_dm_broadcast(const DmArgs& a, const uint32_t* origin, const uint32_t* idbit, hipStream_t s);
// sharded ingest: the RM planes of every shard's slice (saturating sum), the pull slice
hipError_t launch_dm_ingest_rm(const DmArgs& a, const unsigned long long* rm_recv, const unsigned long long* pull_recv,
                               uint32_t world, uint32_t chunk, hipStream_t s);
hipError_t launch_dm_round(const DmArgs& a, hipStream_t s);
// out[i] = sum over g < world of in[g * len + i] (the pull slots' reduce-scatter)
hipError_t launch_dm_sum_slices(const unsigned long long* in, uint32_t world, size_t len, unsigned long long* out,
                                hipStream_t s);
hipError_t launch_dm_pushscan(const DmArgs& a, uint32_t tick_idx, hipStream_t s);
hipError_t launch_dm_xcount(const unsigned long long* any, uint32_t world, uint32_t rank, uint32_t chunk,
                            const unsigned long long* rn_own, uint32_t n_own, uint32_t* cnt, hipStream_t s);
hipError_t launch_dm_xpack_rm(const unsigned long long* rm, uint32_t world, uint32_t rank, uint32_t chunk,
                              const uint32_t* off, uint32_t* cursor, uint32_t* rec, hipStream_t s);
hipError_t launch_dm_xunpack_rm(const uint32_t* rec, const uint32_t* off, uint32_t world, uint32_t chunk,
                                uint32_t nrec, unsigned long long* rm, hipStream_t s);
hipError_t launch_dm_xpack_rmx(const unsigned long long* rn, const uint32_t* ncall, uint32_t v_lo, uint32_t n_own,
                               uint32_t world, uint32_t rank, uint32_t per, uint32_t* cursor, uint32_t* rec,
                               hipStream_t s);
hipError_t launch_dm_xunpack_rmx(const uint32_t* rec, uint32_t nrec, unsigned long long* rn, uint32_t* ncall,
                                 hipStream_t s);

// HyParView (hyparview.hip)
constexpr uint32_t kHvX = 8;          // exchange list capacity (1 + k_active + k_passive)
struct HvMsg {                        // one 64-byte record
    uint8_t type, ttl, prio, nx;
    uint32_t src, dst, seq;           // seq: emission index at src (schedule order key)
    uint32_t peer, epoch, did_e, did_c;
    uint32_t x[kHvX];
};
static_assert(sizeof(HvMsg) == 64, "HvMsg is one 64-byte record");
struct HvHead {                       // per-vertex scalars
    uint8_t na, np;
    uint16_t nsent, nrecv;
    uint32_t seq;
    unsigned long long draws;
};
struct HvCfg {
    uint32_t active_max_size, active_min_size, active_rwl, passive_max_size, passive_rwl;
    uint32_t shuffle_k_active, shuffle_k_passive;
};
constexpr int kHvNStat = 16;          // [1..9] sent by kind, 10 draws, 11 error bits, 12 msgs processed, 13 active
struct HvArgs {
    uint32_t n;
    HvCfg cfg;
    uint2 key;
    uint32_t timers;                      // bit0 random_promotion, bit1 passive_view_maintenance
    uint32_t group;                       // hv_process: consecutive vertices per wave (1..64, launch_hv_round)
    const uint32_t* __restrict__ alive;   // [ceil(n/32)]
    HvHead* __restrict__ head;            // [n]
    uint32_t* __restrict__ act;           // [n][8], 0xFFFFFFFF padded
    uint32_t* __restrict__ pas;           // [n][32]
    unsigned long long* skey;             // sent_message_map table: keys (v << 32 | peer)
    uint2* sval;                          //   values {epoch, cnt}
    unsigned long long* rkey;             // recv_message_map table
    uint2* rval;
    uint32_t map_mask;                    // table size - 1 (power of two)
    const HvMsg* __restrict__ in;         // messages delivered this round
    const uint32_t* nin;                  // device count of `in`
    HvMsg* __restrict__ out;              // messages emitted this round
    uint32_t* nout;                       // device count of `out` (atomicAdd)
    uint32_t out_cap;
    uint32_t* __restrict__ cnt;           // [n] bucket sizes
    uint32_t* __restrict__ cur;           // [n] bucket cursors
    uint32_t* __restrict__ off;           // [n+1] bucket starts
    uint32_t* __restrict__ idx;           // [cap] message indices bucketed by destination
    uint32_t* __restrict__ idx2;          // [cap] a crowded bucket's indices in (src, seq) order
    uint32_t* __restrict__ bsum;          // [ceil(n/256)] scan partials
    unsigned long long* __restrict__ stats;  // [kHvNStat] for this round
};
hipError_t launch_hv_init(const HvArgs& a, hipStream_t s);
hipError_t launch_hv_join(const HvArgs& a, const uint32_t* v, const uint32_t* contact, uint32_t k, hipStream_t s);
hipError_t launch_hv_round(const HvArgs& a, hipStream_t s);

// Causal delivery (causal.hip)
constexpr uint32_t kCsLanes = 64;     // vclock lanes = emitter actors
constexpr uint32_t kCsBufCap = 256;   // buffered messages per vertex
constexpr uint32_t kCsWindow = 64;    // rounds of emitter base clocks kept
constexpr int kCsNStat = 8;           // 1 received, 2 delivered, 3 checks, 4 buffered, 5 error bits, 6 emitted
struct CsArgs {
    uint32_t n, m, period, dmax, redeliver;
    uint32_t v_lo;                        // global id of local vertex 0 (sharded)
    uint32_t n_global;
    uint2 key;
    uint32_t t;                           // the round being run (1-based)
    uint32_t* __restrict__ clk;           // [n][64] lane k = counter of emitter k's actor (0 = absent)
    uint32_t* __restrict__ self;          // [n] own counter of a non-emitter vertex
    uint32_t* __restrict__ buf;           // [n][kCsBufCap] (k << 24 | round)
    uint32_t* __restrict__ nbuf;          // [n]
    unsigned long long* __restrict__ delivered;   // [n]
    uint32_t* __restrict__ base;          // [kCsWindow][64][64] emitter clocks at their broadcasts
    unsigned long long* __restrict__ stats;
    uint32_t* __restrict__ dring;         // [n][64] or null: lane k = the delays of k's messages of the
                                          // last 8 rounds, 4 bits at r % 8 (dmax <= kCsRingMax)
    uint32_t bufcap;                      // buffered messages per vertex before PSIM_EOVERFLOW (<= kCsBufCap;
                                          // PSIM_CS_BUFCAP lowers it to test the overflow path)
};
constexpr uint32_t kCsRingMax = 8;
hipError_t launch_cs_round(const CsArgs& a, hipStream_t s);
hipError_t launch_cs_broadcast(const CsArgs& a, hipStream_t s);

// Full-membership strategy over the state_orset membership set (fullmem.hip)
constexpr uint32_t kFmMaxNW = 32;     // node bitmap words: <= 2048 nodes
constexpr uint32_t kFmMaxW = 32;      // token bitmap words: <= 2048 tokens
struct FmArgs {
    uint32_t n, W, NW;                    // nodes, token words, node words
    uint32_t S;                           // snapshots delivered this round
    uint32_t pass;                        // 0: count emissions, 1: emit and store
    uint32_t periodic;                    // periodic/1 fires at the end of this round
    const uint32_t* __restrict__ elem;    // [64 W] node of each token
    const unsigned long long* st_cur;     // [n][2W] {K words, R words} at the start of the round
    unsigned long long* st_nxt;           // [n][2W] after the round
    const uint8_t* __restrict__ alive0;   // [n] alive at the start of the round
    uint8_t* __restrict__ alive_nxt;      // [n] after the round
    const unsigned long long* __restrict__ alive0_bm;  // [NW]
    const unsigned long long* __restrict__ snap_st;    // [S][2W] delivered states, (src, seq) order
    const unsigned long long* __restrict__ snap_p;     // [S][NW] recipients
    unsigned long long* __restrict__ out_st;           // emitted this round
    unsigned long long* __restrict__ out_p;
    uint32_t* __restrict__ out_src;
    uint32_t* __restrict__ cnt;           // [n] emissions of each node (pass 0)
    const uint32_t* __restrict__ base;    // [n+1] emission offsets (pass 1)
    const uint32_t* __restrict__ jo;      // [n+1] join calls of each node
    const uint32_t* __restrict__ jp;      //   peers, in call order
    const uint32_t* __restrict__ lo;      // [n+1] leave calls of each node
    const uint32_t* __restrict__ lw;      //   leaving node
    const uint32_t* __restrict__ lt;      //   fresh token of a self-leave
    unsigned long long* __restrict__ stats;   // [8] 0 sent 1 processed 2 merges 3 updates 4 inflight 5 member_sum
};
hipError_t launch_fm_round(const FmArgs& a, hipStream_t s);
hipError_t launch_fm_scan(const uint32_t* cnt, uint32_t* base, uint32_t n, hipStream_t s);
hipError_t launch_fm_alive_bm(const uint8_t* alive, uint32_t n, unsigned long long* bm, uint32_t nw, hipStream_t s);

// SCAMP v1 / v2 membership strategies (scamp.hip)
constexpr uint32_t kScPv = 128;       // partial view capacity per vertex
static_assert(kScPv % 8 == 0, "row_has / row_find read rows as quad pairs");
// Whether t is among row[0, n) -- a 16-byte aligned row of capacity a
// multiple of 8 (the SCAMP partial view): quads, two in flight, instead of a
// dependent load per entry (the connection test of every SCAMP and C3 send).
__device__ __forceinline__ bool row_has(const uint32_t* __restrict__ row, uint32_t n, uint32_t t) {
    const uint4* q = reinterpret_cast<const uint4*>(row);
    for (uint32_t i = 0; i < n; i += 8) {
        const uint32_t k = n - i;                  // entries left, >= 1
        const uint4 x = q[i >> 2];
        const uint4 y = k > 4 ? q[(i >> 2) + 1] : make_uint4(0u, 0u, 0u, 0u);
        const bool h = (x.x == t) | (k > 1 && x.y == t) | (k > 2 && x.z == t) | (k > 3 && x.w == t) |
                       (k > 4 && y.x == t) | (k > 5 && y.y == t) | (k > 6 && y.z == t) | (k > 7 && y.w == t);
        if (h) return true;
    }
    return false;
}
// The first index of t in row[0, n), or -1 (same layout rules as row_has).
__device__ __forceinline__ int row_find(const uint32_t* __restrict__ row, uint32_t n, uint32_t t) {
    const uint4* q = reinterpret_cast<const uint4*>(row);
    for (uint32_t i = 0; i < n; i += 8) {
        const uint32_t k = n - i;
        const uint4 x = q[i >> 2];
        const uint4 y = k > 4 ? q[(i >> 2) + 1] : make_uint4(0u, 0u, 0u, 0u);
        const uint32_t m = (x.x == t ? 1u : 0u) | (k > 1 && x.y == t ? 2u : 0u) | (k > 2 && x.z == t ? 4u : 0u) |
                           (k > 3 && x.w == t ? 8u : 0u) | (k > 4 && y.x == t ? 16u : 0u) | (k > 5 && y.y == t ? 32u : 0u) |
                           (k > 6 && y.z == t ? 64u : 0u) | (k > 7 && y.w == t ? 128u : 0u);
        if (m) return int(i) + __ffs(m) - 1;
    }
    return -1;
}
constexpr uint32_t kScIv = 64;        // in-view capacity per vertex
struct ScMsg {                        // one 24-byte record
    uint32_t type, src, dst, seq;     // seq: emission index at src (schedule order key)
    uint32_t a, b;                    // node / replacement
};
struct ScHead {
    uint32_t npv, niv;
    uint32_t draws, inc;              // Philox counter {v, draws, KIND_SCAMP, inc}
    uint32_t seq;
    int32_t last_ping;                // round of the last ping handled, -1 = undefined
    uint32_t fresh, _pad;             // restarted since the last round
};
struct ScArgs {
    uint32_t n, ver, c, round, periodic;
    uint2 key;
    const uint8_t* __restrict__ alive0;   // [n] up at the start of the round
    uint8_t* __restrict__ alive;          // [n] cleared when a manager stops
    ScHead* __restrict__ head;
    uint32_t* __restrict__ pv;            // [n][kScPv]
    uint32_t* __restrict__ iv;            // [n][kScIv]
    const ScMsg* __restrict__ in;
    const uint32_t* nin;
    ScMsg* __restrict__ out;
    uint32_t* nout;
    uint32_t out_cap;
    uint32_t *cnt, *cur, *off, *idx, *bsum;
    // the join / leave calls made since the last round, sorted by vertex
    // (leaves first, then joins, each in call order): call_v[i] their vertex,
    // calls[i] bit31 = leave | node / contact; call_start[v] = 1 + index of
    // v's first call, 0 = none (set by sc_prep, cleared by sc_process)
    uint32_t* __restrict__ call_start;        // [n]
    const uint32_t* __restrict__ call_v;      // [ncalls]
    const uint32_t* __restrict__ calls;       // [ncalls]
    uint32_t ncalls;
    const uint8_t* __restrict__ alive_now;    // [n] alive, copied to alive0 by sc_prep
    unsigned long long* __restrict__ stats;   // [16]
    // partisan_peer_service_events:update(Members) as set deltas, per vertex in
    // firing order (C3: consumed by the Plumtree engine); null = not recorded
    uint32_t* __restrict__ ev_cnt;            // [n]
    uint2* __restrict__ ev;                   // [n][kScEv] {new member, removed member}, 0xFFFFFFFF = none
};
constexpr uint32_t kScEv = 32;                // update events per vertex and round

// The SCAMP engine's device state, for the C3 Plumtree engine (ptdyn.hip)
struct ScView {
    uint32_t n;
    const uint32_t* list;                 // the last psim_scamp_crash list (device)
    const uint32_t* pv;                   // [n][kScPv]
    const ScHead* head;
    uint8_t* alive;
    uint32_t* ev_cnt;
    uint2* ev;
};
int scamp_view(psim_handle* h, ScView* out, bool want_events);   // PSIM_ESTATE without psim_scamp_setup
int scamp_round(psim_handle* h, psim_scamp_stats* out);          // one SCAMP round (calls made so far)
int scamp_crash_list(psim_handle* h, const uint32_t* v, size_t k);
// a round in two halves: launch (calls uploaded, round launched, stats copy
// enqueued; no wait) and finish (after the stream passed it: stats folded,
// errors raised) -- psim_c3_step waits once for both engines' rounds
int scamp_round_launch(psim_handle* h);
int scamp_round_finish(psim_handle* h, psim_scamp_stats* out);
// psim_c3_run: a round launched with its stats rows copied to `dst` (pinned,
// kRoundStatShards * 16 u64) between events e0 / e1, the host's round count
// advanced at once (*round = its number); reported later from those rows
struct ScLaunch {
    unsigned long long* h_dst = nullptr;     // pinned row the stats rows are copied to (null: the handle's)
    hipEvent_t e0 = nullptr, e1 = nullptr;   // around the round's kernels (null: handle events 0 / 1)
    unsigned long long* d_stats = nullptr;   // device row the round's stats stay in (no copy; null: the handle's)
    const uint32_t* d_calls = nullptr;       // the round's calls, sorted, on the device: vertices then targets
    uint32_t d_ncalls = 0;
};
int scamp_round_launch_to(psim_handle* h, const ScLaunch& o, uint64_t* round);
// psim_c3_run's pieces of psim_scamp_join / _crash: a call list checked and
// sorted into `sorted` (k vertices then k targets); a crash list checked
// (range, duplicates); the restart of a crash list already on the device
int scamp_check_calls(psim_handle* h, const uint32_t* v, const uint32_t* x, size_t k, uint32_t* sorted);
int scamp_check_crash(psim_handle* h, const uint32_t* v, size_t k);
size_t scamp_calls_pending(psim_handle* h);   // joins / leaves made since the last round
int scamp_crash_dev(psim_handle* h, const uint32_t* dv, size_t k);
int scamp_round_report(psim_handle* h, const unsigned long long* rows, float ms, uint64_t round, psim_scamp_stats* out);
hipError_t launch_sc_init(const ScArgs& a, const uint32_t* list, uint32_t k, hipStream_t s);
hipError_t launch_sc_round(const ScArgs& a, hipStream_t s);

// C3: Plumtree over the SCAMP engine's changing views (ptdyn.hip)
constexpr uint32_t kPdTab = 128;      // peer-table ids per vertex (PdBits masks)
constexpr uint32_t kPdRows = 256;     // outstanding i_have rows per vertex (heartbeats every round pile them up)
constexpr uint32_t kPdSets = 5;       // masks per vertex: members, common eager/lazy, root eager/lazy
constexpr int kPdNStat = 16;
// SCAMP / C3 round counters are kept in kRoundStatShards copies (workgroup
// b adds into copy b mod kRoundStatShards; the host folds them): one copy took
// an atomic from every wave of the 1M-thread grid on the same few words, a
// ~0.2 ms serial floor under every round whatever it carried.
constexpr int kRoundStatShards = 64;
inline void fold_stat_shards(const unsigned long long* raw, unsigned long long* r, int nstat, int or_idx) {
    for (int i = 0; i < nstat; i++) r[i] = 0;
    for (int k = 0; k < kRoundStatShards; k++)
        for (int i = 0; i < nstat; i++) {
            const unsigned long long x = raw[size_t(k) * nstat + i];
            r[i] = i == or_idx ? (r[i] | x) : r[i] + x;
        }
}
struct PdHead {
    uint32_t ntab, flags;             // flags: bit0 root's eager/lazy map entries exist, bit1 restarted
    uint32_t myround, seq;            // pushed Round of the current heartbeat; emission counter
    uint32_t dbase, nrow;             // delivered window top (heartbeat serial); outstanding rows
    unsigned long long dmask;         // bit k: heartbeat dbase-k delivered (the backend's ISet)
};
// a set over a vertex's peer table: bit i <-> tab[i]
struct PdBits {
    unsigned long long w[2];
    __host__ __device__ static PdBits none() { return PdBits{{0ull, 0ull}}; }
    // selects, not w[i >> 6]: a variable index into a private array sends
    // the kernel's whole context to scratch memory
    __host__ __device__ static PdBits one(int i) {
        const unsigned long long x = i >= 0 ? 1ull << (i & 63) : 0ull;
        return PdBits{{i < 64 ? x : 0ull, i >= 64 ? x : 0ull}};
    }
    __host__ __device__ bool test(uint32_t i) const { return ((i < 64u ? w[0] : w[1]) >> (i & 63)) & 1ull; }
    __host__ __device__ bool any() const { return (w[0] | w[1]) != 0ull; }
    __host__ __device__ PdBits operator|(const PdBits& o) const { return PdBits{{w[0] | o.w[0], w[1] | o.w[1]}}; }
    __host__ __device__ PdBits operator&(const PdBits& o) const { return PdBits{{w[0] & o.w[0], w[1] & o.w[1]}}; }
    __host__ __device__ PdBits operator~() const { return PdBits{{~w[0], ~w[1]}}; }
    __host__ __device__ PdBits& operator|=(const PdBits& o) { w[0] |= o.w[0]; w[1] |= o.w[1]; return *this; }
    __host__ __device__ PdBits& operator&=(const PdBits& o) { w[0] &= o.w[0]; w[1] &= o.w[1]; return *this; }
};
struct PdRow { uint32_t peer, mono, round; };                   // {Peer, {Id, Mod, Round, Root}}
struct PdMsg { uint32_t type, src, dst, seq, round, mono; };   // 24 B
struct PdArgs {
    uint32_t n, mono, tick;
    uint32_t v_lo;                            // bucketing: receiver dst - v_lo (a shard's window lane; C3: 0)
    const uint8_t* __restrict__ alive;        // SCAMP's (a stopped manager takes its node down)
    const uint32_t* __restrict__ pv;          // SCAMP partial views: the connections
    const ScHead* __restrict__ sch;
    const uint32_t* __restrict__ ev_cnt;      // SCAMP update events of this round
    const uint2* __restrict__ ev;
    PdHead* __restrict__ head;
    uint32_t* __restrict__ tab;               // [n][kPdTab]
    PdBits* __restrict__ mask;                // [n][kPdSets]
    PdRow* __restrict__ rows;                 // [n][kPdRows], insertion order
    const PdMsg* __restrict__ in;
    const uint32_t* nin;
    PdMsg* __restrict__ out;
    uint32_t* nout;
    uint32_t out_cap;
    uint32_t *cnt, *cur, *off, *idx, *bsum;
    unsigned long long* __restrict__ stats;   // [kPdNStat]
};
// messages of a.in bucketed by destination: off[n+1], idx[] (order inside a bucket unspecified)
hipError_t launch_pd_bucket(const PdArgs& a, hipStream_t s, bool zeroed);
hipError_t launch_pd_init(const PdArgs& a, const uint32_t* list, uint32_t k, hipStream_t s);
hipError_t launch_pd_origin(const PdArgs& a, uint32_t root, hipStream_t s);
hipError_t launch_pd_round(const PdArgs& a, hipStream_t s);

// Window lanes (ptwin.hip): a heartbeat root whose previous
// heartbeat is still in flight when it heartbeats again.  The lane keeps the
// slot-mask eager / lazy sets of the static engine, and per vertex the
// backend's timestamp interval set for the root (<= kWinIs disjoint
// intervals of Monotonics), the outstanding rows {Peer, Monotonic, Round} in
// insertion order and an emission counter; messages are PdMsg records
// carrying their heartbeat's Monotonic and Round, bucketed by receiver and
// handled in (src, emission seq) order, as in the C3 engine.
constexpr uint32_t kWinIs = 4;        // intervals of a vertex's timestamp set
constexpr uint32_t kWinRows = 32;     // outstanding rows per vertex
struct WinArgs {
    uint32_t n, v_lo, ell;            // as PtArgs
    uint32_t mono;                    // Monotonic of the root's newest heartbeat
    uint32_t mono8, epoch8, tick;
    const uint32_t* __restrict__ rowp;
    const uint32_t* __restrict__ col;
    const uint32_t* __restrict__ memb;
    const uint32_t* __restrict__ alive;   // bitmap over global ids
    const uint32_t* __restrict__ omit;    // omission bitmap over sender slots, or null
    uint4* __restrict__ vs;           // eager, lazy, OR of the rows' slots, myround | rseq | epoch (as PtArgs)
    uint4* __restrict__ iset;         // [n][2]: lo[kWinIs], hi[kWinIs]; lo == 0: unused
    PdRow* __restrict__ rows;         // [n][kWinRows]
    uint2* __restrict__ head;         // [n]: rows, emission seq
    uint8_t* __restrict__ ost;        // [n] 1 = rows exist (the static engine's flag: psim_set_alive counts from it)
    const PdMsg* __restrict__ in;     // this round's messages, bucketed: off[n+1], idx
    const uint32_t* nin;
    const uint32_t* __restrict__ off;
    uint32_t* __restrict__ idx;
    PdMsg* __restrict__ out;          // messages for the next round
    uint32_t* nout;
    uint32_t cap;
    unsigned long long* __restrict__ stats;   // [kStatShards][kNStat] (the static engine's row)
};
// bucket a.in by receiver (cnt, cur: [n], bsum: [ceil(n / kBlock)] scratch), then the round
hipError_t launch_win_round(const WinArgs& a, uint32_t* cnt, uint32_t* cur, uint32_t* bsum, hipStream_t s);
hipError_t launch_win_origin(const WinArgs& a, uint32_t root_local, hipStream_t s);
// sharded window lanes: counts[r] += records whose receiver shard r owns ...
constexpr uint32_t kWinMaxWorld = 64;
hipError_t launch_win_split(const PdMsg* m, const uint32_t* nm, uint32_t cap, uint32_t n_global, uint32_t world,
                            uint32_t* counts, hipStream_t s);
// ... and the records, grouped by shard at base[r] (cursor[r] zeroed)
hipError_t launch_win_scatter(const PdMsg* m, const uint32_t* nm, uint32_t cap, uint32_t n_global, uint32_t world,
                              const uint32_t* base, uint32_t* cursor, PdMsg* out, hipStream_t s);
// a static-engine lane becomes a window lane: rows from the outstanding
// masks, the timestamp sets from the current delivery, the in-flight words
// of `pa` (the words the next round reads) as records
hipError_t launch_win_convert(const WinArgs& a, const PtArgs& pa, hipStream_t s);
// psim_trace_hash out[1] over the in-flight records
hipError_t launch_win_hash(const WinArgs& a, unsigned long long* out, hipStream_t s);
// delivered[v] = Mod:is_stale({root, epoch, mono})
hipError_t launch_win_delivered(const WinArgs& a, uint32_t mono, uint8_t* out, hipStream_t s);
// a backend restart at local vertex v of one lane (iset: the window lane's sets, or null)
hipError_t launch_pt_forget(uint4* vs, uint4* iset, uint32_t v, uint32_t bad, hipStream_t s);

// Cross-shard exchange owned by a handle (transport.hip).  Calls return
// PSIM_* codes and put a detail into *err.
struct Transport {
    virtual ~Transport() {}
    // u32 words, regions by rank (static offsets), on stream s (RCCL) or via
    // host staging (callbacks); the own-rank region is empty
    virtual int alltoallv(const uint32_t* send, const uint64_t* soff, uint32_t* recv, const uint64_t* roff, int rank,
                          int world, hipStream_t s, std::string* err) = 0;
    // host values, in place, summed over ranks (synchronous)
    virtual int allreduce(int64_t* vals, size_t n, hipStream_t s, std::string* err) = 0;
    // device buffer of world slices of `count` u32 words, in place: rank r's
    // slice [r count, (r + 1) count) to every rank
    virtual int allgather(uint32_t* buf, size_t count, int rank, int world, hipStream_t s, std::string* err) = 0;
    virtual const char* name() const = 0;
    // the transport's own view of the job: RCCL asks its communicator
    // (ncclCommCount / ncclCommUserRank); a callback transport reports -1
    virtual int comm_size() const { return -1; }
    virtual int comm_rank() const { return -1; }
};
int make_rccl_transport(int device, int rank, int world, const void* id, Transport** out, std::string* err);
// A capacity knob for tests: getenv(name) clipped to [1, cap], default cap.
inline uint32_t env_cap(const char* name, uint32_t cap) {
    const char* e = getenv(name);
    if (!e) return cap;
    const unsigned long v = strtoul(e, nullptr, 10);
    return v < 1 ? 1u : v > cap ? cap : (uint32_t)v;
}

// C3_PROF diagnostic builds (tools/c3_prof.py): the SCAMP and C3 Plumtree
// kernels clock their phases per wave (s_memtime at reconvergence points)
// and count handled messages by kind into kProfSlots device counters per
// kernel; the host folds them after every round and prints the running
// totals to stderr.  Off in the product build (no code, no counters).
#ifdef C3_PROF
constexpr int kProfSlots = 24;
__device__ __forceinline__ void prof_add(unsigned long long* p, int i, unsigned long long x) {
    const unsigned long long act = __ballot(1);
    if (__lane_id() == uint32_t(__ffsll((long long)act) - 1)) atomicAdd(&p[i], x);
}
#endif

// Collective error agreement: a rank whose local step fails must
// still enter the collective its peers wait in, and every rank must then
// return the same code.  A local code travels as one flag per PSIM_E* code
// inside an all-reduce that runs anyway (or on its own, agree_rc); the common
// code is the lowest-numbered flag set.
constexpr int kNCodes = 12;            // PSIM_EINVAL (-1) .. -12; other nonzero codes use the last slot
inline void put_code(int64_t* v, int rc) {
    for (int k = 0; k < kNCodes; k++) v[k] = 0;
    if (rc < 0 && rc >= -kNCodes) v[-rc - 1] = 1;
    else if (rc) v[kNCodes - 1] = 1;
}
inline int common_code(const int64_t* v) {
    for (int k = 0; k < kNCodes; k++)
        if (v[k]) return -(k + 1);
    return 0;
}

Transport* make_callback_transport(const psim_transport& t);
int rccl_unique_id(void* out);

// Protocol modules that keep their host state outside psim_host.hip: the
// handle owns one slot per module and deletes it on psim_destroy.
struct ModuleState {
    virtual ~ModuleState() {}
};
enum ModuleSlot : int {
    MOD_FULLMEM = 0, MOD_SCAMP = 1, MOD_DMSHARD = 2, MOD_PTDYN = 3, MOD_RELAY = 4, MOD_DEMERS = 5, MOD_HV = 6,
    MOD_CAUSAL = 7, MOD_COUNT = 8
};
ModuleState*& handle_module(psim_handle* h, int slot);
const ModuleState* handle_module(const psim_handle* h, int slot);
hipStream_t handle_stream(const psim_handle* h);
int handle_device(const psim_handle* h);
Transport* handle_transport(psim_handle* h);                // the exchange of psim_shard_init_rccl / _set_transport
uint64_t handle_seed(const psim_handle* h);
int handle_fail(psim_handle* h, int code, const char* fmt, ...);
void handle_add_round(psim_handle* h, double kernel_ms);   // psim_get_timing totals
hipEvent_t handle_event(psim_handle* h, int i);
// wait for the handle's stream by polling an event (psim_host.hip chunk_wait)
hipError_t handle_wait(psim_handle* h);            // i < 8
// The agreed code of a collective step (all-reduced flags v, this rank's
// local code lrc): 0, or the common code -- a rank that did not fail itself
// names the failure as another shard's.
inline int finish_code(psim_handle* h, const int64_t* v, int lrc, const char* what) {
    const int c = common_code(v);
    if (!c) return 0;
    if (lrc) return c;
    return handle_fail(h, c, "%s: another shard failed (code %d)", what, c);
}
// ... over an all-reduce of its own
inline int agree_rc(psim_handle* h, Transport* T, int lrc, const char* what) {
    int64_t v[kNCodes];
    put_code(v, lrc);
    std::string err;
    const int trc = T->allreduce(v, kNCodes, handle_stream(h), &err);
    if (trc) return handle_fail(h, trc, "%s: error agreement all-reduce: %s", what, err.c_str());
    return finish_code(h, v, lrc, what);
}

hipError_t launch_pt_round(const PtArgs& a, hipStream_t s);   // binned when a.rec_c is set
uint32_t ell_round_grid(uint32_t W, int device);              // resident workgroups of the ELL kernel
// one slot-scatter round for nlanes heartbeat lanes (d_args[0..nlanes) on device; a0 = d_args[0] on host)
hipError_t launch_pt_round_lanes(const PtArgs* d_args, const PtArgs& a0, uint32_t nlanes, hipStream_t s);
// op: 0 descends, 1 dominates, 2 merge, 3 increment, 4 equal, 5 glb, 6 subtract_dots, 7 get_counter
hipError_t launch_vc(int op, const uint32_t* a, const uint32_t* b, const uint32_t* actor, uint32_t* out,
                     uint8_t* outb, size_t n, hipStream_t s);
hipError_t launch_pt_origin(const PtArgs& a, hipStream_t s, uint32_t prep = 0, uint32_t hold = 0);
// the fills before a chunk of rounds: stats rows zeroed, hold rings seeded
constexpr uint32_t kMaxPrep = 16;
struct PtPrep {
    unsigned long long* z;
    uint64_t nz;
    uint32_t* hold[kMaxPrep];
    uint32_t* holdd[kMaxPrep];
    uint32_t hv[kMaxPrep];
    uint32_t k;
};
hipError_t launch_pt_prep(const PtPrep& p, hipStream_t s);
hipError_t launch_pt_count_live(const PtArgs& a, unsigned long long* out, hipStream_t s);
hipError_t launch_pt_renorm(const PtArgs& a, hipStream_t s);
// zero every inbox word whose round tag is not `keep` (psim_internal.h word format)
hipError_t launch_pt_scrub(uint32_t* words, uint64_t n, uint32_t keep, uint32_t span, hipStream_t s);
hipError_t launch_pt_hash(const PtArgs& a, uint32_t has_serial, uint32_t root_local, unsigned long long E,
                          unsigned long long* out, hipStream_t s);
hipError_t launch_pt_compact(const PtArgs& a, const uint32_t* rem, const uint4* blk, uint32_t nblk,
                             const uint32_t* send_base, uint32_t* cursor, uint2* out, hipStream_t s,
                             uint32_t cap = 0xFFFFFFFFu, uint32_t self = 0);
hipError_t launch_pt_ingest(const PtArgs& a, const uint2* rec, uint32_t nrec, const uint32_t* slot2v, hipStream_t s);
hipError_t launch_pt_pack_dense(const PtArgs& a, const uint32_t* rem, uint32_t nrem, uint32_t* send, hipStream_t s);
hipError_t launch_pt_ingest_dense(const PtArgs& a, const uint32_t* recv, const uint32_t* recv_map, uint32_t nrecv,
                                  const uint32_t* slot2v, hipStream_t s);

}  // namespace psim
