/*
 * psim.h -- C ABI of libpsim.so, the MI355X-native round-synchronous
 * simulator of Partisan's gossip hot path (loong/partisan).
 *
 * This is the drop-in boundary: the Erlang NIF `partisan_gpu_sim`
 * (erl/c_src/partisan_gpu_sim_nif.c) and the Python
 * host mirror (partisan_amd/) both bind exactly these symbols.  Plain
 * pointers and sizes only; no exceptions cross the ABI.
 *
 * Ownership: a handle owns all device memory it allocates; callers own
 * every host buffer they pass in or out (inputs are copied).
 * Threading: one handle is single-threaded (callers serialise, the NIF
 * holds a per-resource mutex); distinct handles may run concurrently.
 * Errors: 0 = PSIM_OK, negative PSIM_E* otherwise; psim_strerror() names
 * them and psim_last_error() returns a per-handle detail string.
 *
 * Each entry point names the reference interface it replaces.
 */
#ifndef PSIM_H
#define PSIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSIM_ABI_VERSION 3u   /* 2: psim_load_csr takes the col length; 3: psim_config.max_roots, psim_round_stats.words_stored */

#define PSIM_OK         0
#define PSIM_EINVAL    (-1)   /* bad argument / shape                        */
#define PSIM_ENOMEM    (-2)   /* device or host allocation failed            */
#define PSIM_EHIP      (-3)   /* HIP runtime error                           */
#define PSIM_ERCCL     (-4)   /* RCCL error (sharded handles)                */
#define PSIM_ESTATE    (-5)   /* call not valid in the current state         */
#define PSIM_EOVERFLOW (-6)   /* a fixed-capacity structure overflowed       */
#define PSIM_EBUSY     (-7)   /* previous broadcast has not reached quiescence */
#define PSIM_ENODEV    (-8)   /* no HIP device / kernel image for this GPU   */
#define PSIM_ENOSPC    (-9)   /* every heartbeat-root slot holds a root's state */
#define PSIM_ENOTSUP   (-10)  /* this combination of engine and features is not implemented */

/* Message kinds of the Plumtree protocol (partisan_plumtree_broadcast.erl
 * send sites); index of psim_round_stats.sent[]. */
#define PSIM_MSG_BROADCAST 1  /* {broadcast, Id, Payload, Mod, Round, Root, From} :965-969, :893-897 */
#define PSIM_MSG_PRUNE     2  /* {prune, Root, From}                   :849      */
#define PSIM_MSG_IHAVE     3  /* {i_have, Id, Mod, Round, Root, From}  :1030     */
#define PSIM_MSG_IGNORED   4  /* {ignored_i_have, ...}                 :863-867  */
#define PSIM_MSG_GRAFT     5  /* {graft, ...}                          :873-875  */

typedef struct psim_handle psim_handle;

/* Simulation parameters.  Timer periods are in rounds; the reference's
 * millisecond periods map onto rounds keeping their ratios (DESIGN.md
 * "Schedule"): lazy_tick_period 1000 ms (partisan.hrl:280),
 * exchange_tick_period 10000 ms (partisan.hrl:281). */
typedef struct psim_config {
    uint32_t abi_version;          /* must be PSIM_ABI_VERSION                 */
    int32_t  device;               /* HIP device ordinal; -1 = current device  */
    uint32_t lazy_tick_rounds;     /* lazy tick every k rounds (>= 1)          */
    uint32_t exchange_tick_rounds; /* accepted for config parity; no effect */
    uint32_t flags;                /* PSIM_CFG_* bits                          */
    uint32_t max_roots;            /* heartbeat roots whose per-root state the handle keeps (0 = 16); a
                                    * new root beyond them is PSIM_ENOSPC, never a silent eviction */
    uint64_t seed;                 /* Philox key for the protocols that draw   */
} psim_config;

/* psim_config.flags: PSIM_CFG_BINNED routes a single-GPU handle's Plumtree
 * messages as {receiver slot, word} records through coarse then fine
 * receiver bins instead of scattering one HBM word per
 * receiver slot (the default, and what sharded handles always run).  Both
 * give identical results; the binned engine is the slower one on MI355X today. */
#define PSIM_CFG_BINNED 1u
/* The slot-scatter engine on one GPU keeps each vertex's slots as a fixed-width
 * row (ELL, width = the maximum degree) when every degree is <= 8, so a
 * vertex's inbox words are found without reading row pointers;
 * PSIM_CFG_CSR keeps the CSR layout instead (same results; A/B and tests). */
#define PSIM_CFG_CSR 2u
/* psim_step / psim_run time each round with its own pair of hipEvents
 * (psim_round_stats.kernel_ms).  PSIM_CFG_CHUNK_TIMING records one pair per
 * chunk of up to 16 rounds instead -- each round's kernel_ms is then the
 * chunk's device time / its rounds -- so no event marker sits between two
 * round kernels (same results). */
#define PSIM_CFG_CHUNK_TIMING 4u

/* Per-round counters, reduced on device (psim_step / psim_run). */
typedef struct psim_round_stats {
    uint64_t sent[6];              /* messages emitted, by PSIM_MSG_* kind     */
    uint64_t delivered_new;        /* Mod:merge/2 returned true                */
    uint64_t active;               /* vertices that processed messages/ticks  */
    uint64_t senders;              /* vertices that emitted >= 1 message       */
    uint64_t sender_degree_sum;    /* sum of deg(v) over senders               */
    uint64_t outstanding_vertices; /* vertices holding outstanding i_have rows */
    uint64_t algo_bytes;           /* SURVEY 8(d) bytes: 16N + sum(8+4deg) + 32 msgs */
    double   kernel_ms;            /* device time of this round's kernel (hipEvent) */
    uint64_t words_stored;         /* inbox words (4-byte random stores) the round wrote; a word carries
                                    * the <= 4 messages of one sender to one receiver */
} psim_round_stats;

/* --- lifecycle -------------------------------------------------------- */
/* Replaces gen_server:start_link of partisan_plumtree_broadcast
 * (partisan_plumtree_broadcast.erl:234-260, init/1 :487-515). */
int  psim_create(const psim_config* cfg, psim_handle** out);
int  psim_destroy(psim_handle* h);
const char* psim_strerror(int code);
const char* psim_last_error(const psim_handle* h);
/* Writes the device name and arch (e.g. "gfx950") into buf. */
int  psim_device_info(const psim_handle* h, char* buf, size_t cap);

/* --- overlay / membership ------------------------------------------- */
/* Loads every vertex's membership list (the peer service's members minus
 * self: partisan_peer_service:members/0, consumed by start_link/0 :234-260)
 * as a CSR: row_ptr[n+1], col[col_len].  Copied.  Plumtree's peers of v
 * are the union of v's members and of the vertices listing v (a message can
 * only arrive over such an edge); at most 32 per vertex.  PSIM_EINVAL unless
 * row_ptr[0] == 0, row_ptr is monotone, row_ptr[n] == col_len and every id
 * is < n (nothing is read past col[col_len - 1]).  Neither array needs any
 * alignment beyond its element type's. */
int  psim_load_csr(psim_handle* h, uint32_t n, const uint64_t* row_ptr, const uint32_t* col, uint64_t col_len);
/* Number of peer slots (directed edges of the symmetrised overlay). */
int  psim_num_slots(const psim_handle* h, uint64_t* out);
/* The slot layout used by every per-vertex mask below: row_ptr[n+1], col[E]
 * (sorted by id within a row). */
int  psim_get_slots(const psim_handle* h, uint64_t* row_ptr, uint32_t* col);
/* alive[n] bytes (1 = up).  A dead vertex drops its inbox and fires no timer;
 * partisan:is_connected/1 on a dead peer is false. */
int  psim_set_alive(psim_handle* h, const uint8_t* alive, size_t n);

/* --- Plumtree --------------------------------------------------------- */
/* Every vertex handles a membership update that adds members: reset_peers/4
 * drops all per-root eager/lazy sets (partisan_plumtree_broadcast.erl:607-639,
 * :1320-1328).  O(1): sets are tagged with a tree epoch. */
int  psim_plumtree_reset_trees(psim_handle* h);
/* Vertex v's heartbeat backend restarts (its gen_server crashes and is
 * started again: partisan_plumtree_backend init/1 :316-329): a newer epoch
 * (erlang:system_time() there; here the restart count, 1..255), Monotonic
 * 0, and a new timestamp table -- v forgets every origin's heartbeats (each
 * lane's delivered tag / timestamp set at v).  v's next heartbeat is
 * {v, Epoch + 1, 1}; a heartbeat of an older epoch is then stale wherever
 * the newer one was recorded (is_stale :229-244) and the newer one replaces
 * the origin's set (add_timestamp :400-417).  Heartbeat ids are reported as
 * Epoch << 24 | Monotonic by every call that returns or takes one (epoch 0
 * until a restart: the plain Monotonic).  Sharded handles: every shard
 * calls it.  A static lane keeps one Round per vertex: a vertex that
 * re-delivers a heartbeat it forgot while still holding its rows reports
 * PSIM_EOVERFLOW (bit 4); window lanes keep every id. */
int  psim_plumtree_restart_backend(psim_handle* h, uint32_t v);
/* Heartbeat at `root`: partisan_plumtree_backend handle_info(heartbeat)
 * (:341-368) -> partisan_plumtree_broadcast:broadcast/2 (:324-326) ->
 * handle_cast({broadcast, Id, Payload, Mod}) (:565-569).  Emits round-0
 * eager pushes delivered by the next step.  *mono_out = the Monotonic of
 * the id {Root, Epoch, Monotonic}.  A root may heartbeat again while its
 * previous heartbeats are in flight (the backend's timer does not wait):
 * on one GPU with the slot-scatter engine its lane then becomes a window
 * lane (ptwin.hip) that keeps each heartbeat's messages, rows and the
 * backend's timestamp interval set apart -- the same per-root eager / lazy
 * sets, per-message ids -- from then until the lane is reused.  Sharded,
 * binned and delay-fault handles keep one heartbeat per root: PSIM_EBUSY. */
int  psim_plumtree_broadcast(psim_handle* h, uint32_t root, uint32_t* mono_out);
/* Heartbeats from k roots at once -- backend handle_info(heartbeat) at each
 * of them, as every node's timer fires (partisan_plumtree_backend.erl:341-368,
 * 421-428).  monos_out[i] = roots[i]'s id (may be NULL).  On a forest
 * (max_roots > 16) one origin launch for all of them, all or nothing:
 * PSIM_ENOSPC when new roots exceed max_roots, PSIM_EBUSY when a root's last
 * heartbeat is still in flight or holds rows, PSIM_EINVAL on a root listed
 * twice; otherwise psim_plumtree_broadcast per root, in order.  A SHARDED
 * forest (psim_shard_init, world > 1) takes it as a collective: every rank
 * passes the same roots (global ids), the owners run the origins and every
 * lane's cross-shard pushes move in one exchange before it returns; then
 * psim_shard_run / psim_shard_step drive all lanes (one launch per round,
 * every lane's words in one all-to-all-v, counters all-reduced per chunk). */
int  psim_plumtree_broadcast_many(psim_handle* h, const uint32_t* roots, size_t k, uint32_t* monos_out);
/* One heartbeat interval of one root: psim_plumtree_broadcast(root) then
 * psim_run(max_rounds) -- the same state, ids, per-round stats and codes --
 * in one call whose origin is not read back on its own: its counters come
 * back with the first chunk of rounds (one host round trip fewer).  An
 * origin overflow (PSIM_EOVERFLOW) is then reported after that chunk ran.
 * Delay-fault and window-lane heartbeats read the origin first, as the two
 * calls do; sharded handles: PSIM_ESTATE. */
int  psim_plumtree_broadcast_run(psim_handle* h, uint32_t root, uint32_t* mono_out, uint32_t max_rounds,
                                 psim_round_stats* stats, size_t cap, uint32_t* rounds_run);
/* `count` heartbeat intervals of one root back to back: each is
 * psim_plumtree_reset_trees (when reset_trees != 0) then
 * psim_plumtree_broadcast_run(root, max_rounds) -- the same state, ids,
 * per-round stats and codes as those calls in a loop, without a return to
 * the caller between intervals.  stats: the per-round rows of every interval
 * in order (up to cap rows in all); rounds[i] / monos[i] (either may be
 * null): the rounds interval i ran and its heartbeat id; *done: the
 * intervals completed (those before the first error). */
int  psim_plumtree_broadcast_run_n(psim_handle* h, uint32_t root, uint32_t count, uint32_t reset_trees,
                                   uint32_t max_rounds, psim_round_stats* stats, size_t cap, uint32_t* rounds,
                                   uint32_t* monos, uint32_t* done);
/* Several roots: on one GPU without PSIM_CFG_BINNED each
 * heartbeat root gets a lane of its own (per-root eager / lazy sets, rows,
 * delivered serials, in-flight words; up to 16 lanes -- a 17th root is
 * PSIM_ENOSPC; psim_config.max_roots keeps every root, the forest), so
 * heartbeats of different roots run concurrently and PSIM_EBUSY is per
 * root; rounds advance every lane and their stats are summed.  Sharded and
 * binned handles keep one lane: a heartbeat from a new root drops the old
 * root's sets.  The per-vertex getters (psim_get_plumtree, _delivered,
 * _inflight, psim_trace_hash) read the focused root: the last broadcast one,
 * or the one chosen here (PSIM_EINVAL if it has no lane). */
int  psim_plumtree_focus(psim_handle* h, uint32_t root);
/* Forest capacity (max_roots > 16): the per-root records that outlive a
 * heartbeat -- every vertex's eager / lazy / outstanding sets, accepted Round
 * and delivered id for that root, the reference's eager_sets / lazy_sets
 * entries kept for good (partisan_plumtree_broadcast.erl:1240-1248,
 * 1278-1282) -- take 16 B per vertex and root; a heartbeat in flight also
 * needs a lane (its inbox words, group flags, rows and counts: ~40 B per
 * vertex).  With lanes < max_roots the handle keeps max_roots roots' records
 * but only `lanes` lanes: a heartbeat takes the lane of a root whose own
 * heartbeat is done (that root is parked: its records stay, nothing of it is
 * in flight), and psim_plumtree_broadcast_many returns PSIM_ENOSPC when more
 * heartbeats are in flight at once than there are lanes.  Results are those
 * of lanes == max_roots.  0 (the default) = max_roots lanes.  Call before
 * psim_load_csr: PSIM_ESTATE after it or on a handle that is no forest,
 * PSIM_EINVAL for lanes > max_roots.  psim_plumtree_focus on a parked root
 * shows its records with nothing in flight. */
int  psim_forest_set_lanes(psim_handle* h, uint32_t lanes);
/* Runs exactly `rounds` rounds.  stats may be NULL; otherwise stats[cap]. */
int  psim_step(psim_handle* h, uint32_t rounds, psim_round_stats* stats, size_t cap);
/* Runs until quiescent (nothing in flight and no outstanding i_have row to
 * a live peer) or max_rounds; *rounds_run = rounds executed. */
int  psim_run(psim_handle* h, uint32_t max_rounds, psim_round_stats* stats, size_t cap,
              uint32_t* rounds_run);
/* Per-vertex Plumtree state for the current root, masks over the vertex's
 * slots (bit s = col[row_ptr[v] + s]): all_eager_peers / all_lazy_peers
 * (:1252-1282), outstanding rows (:1215-1219), the Round of the accepted
 * broadcast (0xFFFF: not delivered; 0xFFFE: the root).  Any pointer may be NULL. */
int  psim_get_plumtree(const psim_handle* h, uint32_t* eager, uint32_t* lazy,
                       uint32_t* outstanding, uint16_t* recv_round, size_t n);
/* delivered[n] bytes: Mod:is_stale(Id) for the current heartbeat (backend :229-244). */
int  psim_get_delivered(const psim_handle* h, uint8_t* delivered, size_t n);
/* Messages in flight (delivered by the next round), one word per slot of the
 * RECEIVER: bits 0..15 = FIFO of 4-bit PSIM_MSG_* kinds (first in the low
 * nibble), bits 16..31 = Round carried by broadcast / i_have.  words[E]. */
int  psim_get_inflight(const psim_handle* h, uint32_t* words, uint64_t n_words);
/* Every message the next round delivers to this handle's vertices, in the
 * order they are handled (receiver, then sender, then emission order): its
 * sender, receiver (global ids), PSIM_MSG_* kind, Round and Monotonic (prune
 * carries neither: 0).  Any array may be NULL; *count = total, entries past
 * cap are not written.  Works for both lane kinds (psim_get_inflight is the
 * static lanes' word view). */
int  psim_get_messages(const psim_handle* h, uint32_t* src, uint32_t* dst, uint32_t* kind, uint32_t* round,
                       uint32_t* mono, size_t cap, size_t* count);
/* Vertex v's outstanding i_have rows in insertion order (the ETS bag
 * {Peer, {Id, Mod, Round, Root}}, :1207-1219): peer, Round, Monotonic. */
int  psim_get_rows(const psim_handle* h, uint32_t v, uint32_t* peer, uint32_t* round, uint32_t* mono, size_t cap,
                   size_t* count);
/* delivered[n]: Mod:is_stale({Root, Epoch, mono}) (backend :229-244) for the
 * focused root, any Monotonic of a window lane; a static lane answers for
 * its newest heartbeat only (PSIM_EINVAL otherwise). */
int  psim_get_delivered_mono(const psim_handle* h, uint32_t mono, uint8_t* delivered, size_t n);
/* The same for local vertices [v0, v0 + count) only -- one vertex's
 * Mod:is_stale/1 without copying the whole delivered set (the NIF adapter's
 * is_stale/graft).  mono 0 = the focused root's newest heartbeat. */
int  psim_get_delivered_range(const psim_handle* h, uint32_t mono, uint32_t v0, size_t count, uint8_t* delivered);
/* Omission faults (test/prop_partisan_crash_fault_model.erl:117-196, send /
 * receive omission interposition funs): every Plumtree message over a
 * directed pair (src[i], dst[i]) is sent -- counted, the sender moves on --
 * and lost.  Replaces the whole set; k = 0 heals all ("resolve all faults").
 * Pairs that are not overlay edges are ignored; a partition is the set of
 * its cross edges (partisan_amd.Simulator.inject_partition). */
int  psim_set_omissions(psim_handle* h, const uint32_t* src, const uint32_t* dst, size_t k);
/* Delay faults (test/partisan_SUITE.erl with_egress_delay /
 * with_ingress_delay; partisan_peer_service_client.erl:148-176 and
 * partisan_peer_service_server.erl sleep before each send / after each
 * receipt): every Plumtree message over the directed pair (src[i], dst[i])
 * emitted in round t is delivered in round t + 1 + rounds[i] instead of
 * t + 1 (a fixed delay per pair keeps each pair FIFO).  rounds[i] <=
 * PSIM_MAX_DELAY.  Replaces the whole set (k = 0: every delay 0); an egress
 * (ingress) delay of a node is its out- (in-) edges.  PSIM_EBUSY while any
 * message is in flight (a change could reorder a pair); PSIM_ESTATE for the
 * binned engine.  Sharded handles: collective (every rank passes the same
 * global pairs and installs its own senders'), driven by psim_shard_run /
 * psim_shard_step, several heartbeat roots at once (each lane stages its
 * cross-shard delayed words in its own ring); PSIM_ESTATE with a window lane
 * or async rounds pending.  Pairs that are not overlay edges are ignored.
 * psim_run / psim_shard_run end only when no delayed message is pending. */
#define PSIM_MAX_DELAY 14u
int  psim_set_delays(psim_handle* h, const uint32_t* src, const uint32_t* dst, const uint8_t* rounds, size_t k);

/* Order-independent digest of the Plumtree state, to compare runs (the two
 * engines, shard counts, replays) at full size without copying state out.
 * With mix = the splitmix64 finaliser (z += 0x9E3779B97F4A7C15;
 * z = (z ^ z>>30) * 0xBF58476D1CE4E5B9; z = (z ^ z>>27) * 0x94D049BB133111EB;
 * z ^ z>>31) and sums mod 2^64:
 *   out[0] = sum over this handle's vertices (global id g) of
 *            mix(mix(mix(O) ^ (E<<32 | L)) ^ (g<<32 | R)), with E, L, O, R
 *            the psim_get_plumtree eager / lazy / outstanding masks and recv_round;
 *   out[1] = sum over in-flight words w != 0 (psim_get_inflight) at global
 *            receiver slot e of mix(e<<32 | w);
 *   out[2] = delivered vertices;  out[3] = rounds completed.
 * Shards' out[0..2] add up to the whole overlay's (SURVEY 8(b) psim_trace_hash). */
int  psim_trace_hash(const psim_handle* h, uint64_t* out);

/* --- vertex sharding over several GPUs (one process per GPU) -------- */
/* The overlay is split into `world` contiguous vertex ranges; this handle
 * owns range `rank`.  Call before psim_load_csr, which then
 * keeps only the local rows; getters (psim_get_plumtree, ...) return the
 * local range, psim_set_alive still takes all n_global vertices.  Rounds are
 * split-phase so that the transport stays the caller's (RCCL all-to-all-v
 * via torch.distributed "nccl" on a node; gloo in tests):
 *   psim_shard_broadcast / psim_shard_round  -> counts[d] records for shard d,
 *       packed in the caller's device buffer at region_base[d] (uint2
 *       {global receiver slot, word});
 *   caller exchanges the regions;  psim_shard_ingest(received records);
 *   the caller all-reduces the emitted-message and live-row counters and
 *   stops at global quiescence. */
int  psim_shard_init(psim_handle* h, int rank, int world);
int  psim_shard_info(const psim_handle* h, uint32_t* v_lo, uint32_t* n_local, uint64_t* slot_base,
                     uint32_t* n_global);
/* region_base[world + 1]: record offsets of each destination's region; the
 * last entry is the send buffer's capacity in records */
int  psim_shard_layout(const psim_handle* h, uint64_t* region_base, size_t world);
int  psim_shard_broadcast(psim_handle* h, uint32_t root, uint32_t* mono_out, void* send_dev, uint64_t send_cap,
                          uint64_t* counts, int64_t* local_live);
int  psim_shard_round(psim_handle* h, void* send_dev, uint64_t send_cap, uint64_t* counts,
                      psim_round_stats* stats, int64_t* local_live);
int  psim_shard_ingest(psim_handle* h, const void* recv_dev, uint64_t n_records);
/* Dense, host-sync-free exchange (what bench.py drives over RCCL): every
 * remote slot has a fixed word position in the send buffer (region d of
 * psim_shard_layout, in this shard's slot order; 0 = nothing sent), so the
 * caller moves fixed-size regions (all-to-all with static split sizes; the
 * receive regions are psim_shard_recv_layout) with no count exchange.
 * psim_set_stream puts the handle's work on the caller's stream (e.g. torch's
 * current stream, so kernels and RCCL are stream-ordered); rounds are
 * enqueued by psim_shard_round_async and their stats fetched, with one sync,
 * by psim_shard_collect (<= 16 pending). local_live[i] = this shard's
 * outstanding rows to live peers after pending round i. */
int  psim_set_stream(psim_handle* h, void* hip_stream);
int  psim_shard_recv_layout(const psim_handle* h, uint64_t* recv_base, size_t world);
int  psim_shard_broadcast_dense(psim_handle* h, uint32_t root, uint32_t* mono_out, void* send_words);
int  psim_shard_round_async(psim_handle* h, void* send_words);
int  psim_shard_ingest_dense(psim_handle* h, const void* recv_words);
int  psim_shard_collect(psim_handle* h, psim_round_stats* stats, size_t cap, uint32_t* n_rounds, int64_t* local_live);
/* The last `rounds` collected rounds ran after global quiescence (no-ops):
 * they do not advance the timer schedule (lazy tick phase), as in psim_run. */
int  psim_shard_uncount(psim_handle* h, uint32_t rounds);

/* --- the exchange inside the library -------------
 * A sharded handle can own its transport and run whole heartbeats itself:
 * every round is enqueued as round kernel -> pack -> exchange -> ingest on the
 * handle's stream, counters are collected (one host sync, one all-reduce)
 * every 4 rounds, and the run stops at GLOBAL quiescence with the single-GPU
 * engine's round count.  Transports:
 *   psim_shard_init_rccl: one RCCL communicator per handle (ncclCommInitRank
 *     on the handle's device), the words as one grouped ncclSend / ncclRecv
 *     per round over the static regions of psim_shard_layout /
 *     psim_shard_recv_layout, the counters as one int64 ncclAllReduce.  The
 *     unique id comes from psim_rccl_unique_id on one rank, shipped to the
 *     others by the caller (any out-of-band channel);
 *   psim_shard_set_transport: caller callbacks over HOST buffers (tests, or a
 *     fabric the library does not know). */
#define PSIM_RCCL_ID_BYTES 128
typedef struct psim_transport {
    void* ctx;
    /* all-to-all-v of u32 words: region d of send = send[send_off[d], send_off[d+1])
     * goes to rank d; what rank s sends to this rank lands at recv[recv_off[s], ...).
     * Returns 0 on success. */
    int (*alltoallv)(void* ctx, const uint32_t* send, const uint64_t* send_off, uint32_t* recv,
                     const uint64_t* recv_off, int world);
    /* in-place sum over ranks of n int64 values; returns 0 on success */
    int (*allreduce)(void* ctx, int64_t* vals, size_t n);
} psim_transport;
typedef struct psim_exchange_stats {
    uint64_t rounds;               /* rounds enqueued (the uncounted quiescent tail included) */
    uint64_t fabric_bytes;         /* bytes this rank sent to other ranks                     */
    double   exchange_ms;          /* device time inside the exchange (hipEvents)              */
    double   kernel_ms;            /* device time of the round kernels (hipEvents)             */
} psim_exchange_stats;
int  psim_rccl_unique_id(uint8_t* id_out /* PSIM_RCCL_ID_BYTES */);
/* psim_shard_init + an RCCL communicator of `world` ranks; before psim_load_csr */
int  psim_shard_init_rccl(psim_handle* h, int rank, int world, const uint8_t* id /* PSIM_RCCL_ID_BYTES */);
int  psim_shard_set_transport(psim_handle* h, const psim_transport* t);
/* The handle's exchange: kind 0 none, 1 the library's RCCL communicator,
 * 2 a caller transport; comm_world / comm_rank as the communicator itself
 * reports them (ncclCommCount / ncclCommUserRank; -1 for a caller transport). */
int  psim_shard_transport_info(const psim_handle* h, int* kind, int* comm_world, int* comm_rank);
/* heartbeat at `root` on every rank (collective): the origin's pushes are
 * exchanged before it returns.  Through this in-library path a sharded
 * handle has heartbeat lanes as on one GPU (one per root, window lanes for a
 * root heartbeating while its last heartbeat is in flight); every rank
 * decides busy / window / lane reuse on the same all-reduced counts.  The
 * split-phase entry points above return PSIM_ESTATE once a handle has more
 * than one lane or a window lane. */
int  psim_shard_broadcast_x(psim_handle* h, uint32_t root, uint32_t* mono_out);
/* collective: rounds until global quiescence (or max_rounds); stats are the
 * GLOBAL per-round counters (summed over ranks; kernel_ms this rank's),
 * *xs this rank's exchange figures (may be NULL) */
int  psim_shard_run(psim_handle* h, uint32_t max_rounds, psim_round_stats* stats, size_t cap, uint32_t* rounds_run,
                    psim_exchange_stats* xs);
/* Exactly `rounds` rounds of psim_shard_run (collective; no quiescence stop). */
int  psim_shard_step(psim_handle* h, uint32_t rounds, psim_round_stats* stats, size_t cap, psim_exchange_stats* xs);

/* --- partisan_vclock on dense lanes ----------------------------------- */
/* A clock is PSIM_VC_LANES u32 lanes, lane i = actor i (actor ids are ranks
 * in the sorted actor table, so lane order is the reference's term order).
 * Lane value 0 = actor absent, c+1 = counter c: descends/2's presence rule
 *  is then a lane-wise compare.  Batched over n clocks, one
 * wave per clock.  Host buffers, copied. */
#define PSIM_VC_LANES 64
/* partisan_vclock:descends/2 (src/partisan_vclock.erl:63-73): out[i] = A_i descends B_i */
int  psim_vclock_descends(psim_handle* h, const uint32_t* a, const uint32_t* b, uint8_t* out, size_t n);
/* partisan_vclock:dominates/2 (:75-77) */
int  psim_vclock_dominates(psim_handle* h, const uint32_t* a, const uint32_t* b, uint8_t* out, size_t n);
/* partisan_vclock:merge([A, B]) (:102-129): lane-wise max */
int  psim_vclock_merge(psim_handle* h, const uint32_t* a, const uint32_t* b, uint32_t* out, size_t n);
/* partisan_vclock:increment(Actor, A) (:140-153) */
int  psim_vclock_increment(psim_handle* h, const uint32_t* a, const uint32_t* actor, uint32_t* out, size_t n);
/* partisan_vclock:equal/2 (:163-164): lists:sort(A) =:= lists:sort(B), i.e.
 * lane-wise equality (a dense clock has one entry per actor) */
int  psim_vclock_equal(psim_handle* h, const uint32_t* a, const uint32_t* b, uint8_t* out, size_t n);
/* partisan_vclock:glb/2 (:183-198): actors of both, the smaller counter,
 * sorted = lane-wise min (absent = 0 drops out) */
int  psim_vclock_glb(psim_handle* h, const uint32_t* a, const uint32_t* b, uint32_t* out, size_t n);
/* partisan_vclock:subtract_dots(Dots, Clock) (:85-99, drop_dots): a dot
 * {Actor, C} survives iff get_counter(Actor, Clock) < C; sorted */
int  psim_vclock_subtract_dots(psim_handle* h, const uint32_t* dots, const uint32_t* clock, uint32_t* out, size_t n);
/* partisan_vclock:get_counter(Actor, A) (:132-137): out[i] = counter of lane
 * actor[i] in clock i, 0 when absent (one u32 per clock) */
int  psim_vclock_get_counter(psim_handle* h, const uint32_t* a, const uint32_t* actor, uint32_t* out, size_t n);

/* --- Demers epidemics (protocols/demers_*.erl) ------------------------ */
typedef struct psim_demers_stats {
    uint64_t rm_sent;              /* {broadcast, Id, ServerRef, Message, From} (rumor mongering) */
    uint64_t push_sent;            /* {push, From, AllMessages} (anti-entropy)    */
    uint64_t pull_sent;            /* {pull, From, AllMessages}                   */
    uint64_t delivered_new;        /* (vertex, rumor) pairs newly stored          */
    uint64_t complete;             /* vertices holding every rumor after the round */
    uint64_t algo_bytes;           /* 2*N*M/8 + pushes*6*M/8 + 32*msgs */
    double   kernel_ms;
} psim_demers_stats;
/* Full-membership Demers epidemic over n vertices with m <= 64 rumors whose
 * origins are Philox draws (stream kind 1).  rm_on: 1 = rumor mongering with
 * fanout 2 (demers_rumor_mongering.erl :92-186); 2 = direct mail, the
 * baseline: the origin sends to every other member, receivers only store
 * (demers_direct_mail.erl :91-143; not in psim_demers_shard_setup; the
 * origins' n-1 sends, like rumor mongering's, are not in the round stats);
 * 0 = off.  ae_period: anti-entropy
 * push-pull with fanout 2 every ae_period rounds (demers_anti_entropy.erl
 * :118-195; 0 = off, else >= 2).  Both on share one message store.
 * Replaces starting both gen_servers on every node (:50-76). */
int  psim_demers_setup(psim_handle* h, uint32_t n, uint32_t m, uint32_t ae_period, uint32_t rm_on);
/* handle_cast({broadcast, ServerRef, Message}) at every rumor's origin
 * (RM :92-115; AE :95-106, which only stores: ids {Node, 0}, Q20). */
int  psim_demers_broadcast_all(psim_handle* h);
int  psim_demers_step(psim_handle* h, uint32_t rounds, psim_demers_stats* stats, size_t cap);
/* Runs until every vertex stores every rumor (or max_rounds). */
int  psim_demers_run(psim_handle* h, uint32_t max_rounds, psim_demers_stats* stats, size_t cap,
                     uint32_t* rounds_run);
/* seen[n]: bit i = the rumor with store id i (i = rumor index; with
 * anti-entropy alone, rumors of one origin share the first one's id, Q20). */
int  psim_demers_get_seen(const psim_handle* h, uint64_t* seen, size_t n);
int  psim_demers_origins(const psim_handle* h, uint32_t* origins, size_t m);

/* --- vertex-sharded Demers (one process per GPU) ---------
 * Shard `rank` owns global ids [rank C, min((rank+1) C, n)), C = ceil(n/world)
 * (*chunk_out).  Rounds are split-phase; the transport is the caller's
 * (RCCL via torch.distributed "nccl" on a node, gloo in tests).  Caller-owned
 * device buffers:  rm_shadow [3][world C] u64 and pull_shadow [world C][2]
 * u64 (zeroed by the caller before each round), snap_all [world C] u64,
 * rmx_all = [world C] u64 then [world C] u32 (each RM process's calls of the
 * round and its calls before it: a receiver checks whether its own targets
 * sent it a rumor from them), rm_recv [3][world C] u64 (plane k = the world
 * slices of plane k sent to this shard, slice g from shard g), pull_recv
 * [C][2] u64.  After psim_demers_shard_broadcast_all and after each
 * psim_demers_shard_round the caller does, per plane, all_to_all(rm_shadow ->
 * rm_recv) in slices of C, reduce_scatter(sum, pull_shadow -> pull_recv) (one
 * writer per slot), all_gather of both rmx_all planes in slices of C, and
 * when *tick: all_gather(snap_all) in slices of C; then
 * psim_demers_shard_ingest.  Same workload, draws and results as
 * psim_demers_* on one GPU. */
int  psim_demers_shard_setup(psim_handle* h, uint32_t n, uint32_t m, uint32_t ae_period, uint32_t rm_on, int rank,
                             int world, uint64_t* chunk_out);
int  psim_demers_shard_info(const psim_handle* h, uint32_t* v_lo, uint32_t* n_local, uint64_t* chunk);
int  psim_demers_shard_broadcast_all(psim_handle* h, void* rm_shadow, void* rmx_all);
int  psim_demers_shard_round(psim_handle* h, void* rm_shadow, void* pull_shadow, void* snap_all, void* rmx_all,
                             psim_demers_stats* stats, uint32_t* tick);
int  psim_demers_shard_ingest(psim_handle* h, const void* rm_recv, const void* pull_recv, const void* rmx_all,
                              uint32_t tick);
int  psim_demers_shard_get_seen(const psim_handle* h, uint64_t* seen, size_t n_local);
/* The same exchange inside the library, on the handle's transport
 * (psim_shard_init_rccl: RCCL all-to-all-v / all-gather over xGMI on the
 * handle's stream; psim_shard_set_transport: the caller's callbacks) -- no
 * caller buffers, no host collectives: the broadcast of every rumor at its
 * origin, exactly `rounds` rounds, or rounds until every vertex of every
 * shard holds every rumor.  Collective; stats are GLOBAL (summed over the
 * shards; kernel_ms this shard's).  world 1 needs no transport. */
int  psim_demers_shard_broadcast_x(psim_handle* h);
int  psim_demers_shard_step(psim_handle* h, uint32_t rounds, psim_demers_stats* stats, size_t cap);
int  psim_demers_shard_run(psim_handle* h, uint32_t max_rounds, psim_demers_stats* stats, size_t cap,
                           uint32_t* rounds_run);
/* How the in-library exchange moves the RM planes and call records: 0 (the
 * default) sends a round's nonzero RM slots as {slot, any, multi, tri}
 * records and its callers as {vertex, rumors called, calls before} records
 * whenever they reach fewer than n/8 slots (counts summed over the shards
 * first, so every shard picks the same form), the dense slices otherwise;
 * 1 always dense; 2 always records.  Results are identical.  Collective
 * setting: every shard must pass the same mode.  *_exchange_stats: bytes
 * this shard sent to other shards, exchanges run, and how many of them sent
 * RM records / call records. */
int  psim_demers_shard_set_exchange(psim_handle* h, int mode);
int  psim_demers_shard_exchange_stats(const psim_handle* h, uint64_t* bytes_sent, uint32_t* rounds,
                                      uint32_t* sparse_rm_rounds, uint32_t* sparse_call_rounds);

/* --- HyParView view maintenance (partisan_hyparview_peer_service_manager.erl) */
typedef struct psim_hv_config {
    uint32_t active_max_size;      /* partisan.hrl / hyparview config: 6 (<= 8)   */
    uint32_t active_min_size;      /* 3                                            */
    uint32_t active_rwl;           /* 6 (<= 255)                                   */
    uint32_t passive_max_size;     /* 30 (<= 32)                                   */
    uint32_t passive_rwl;          /* 6                                            */
    uint32_t shuffle_k_active;     /* 3; k_active + k_passive <= 7                 */
    uint32_t shuffle_k_passive;    /* 4                                            */
    uint32_t shuffle_rounds;       /* passive_view_shuffle_period (10000 ms) in rounds */
    uint32_t promotion_rounds;     /* random_promotion_interval (5000 ms) in rounds */
} psim_hv_config;
typedef struct psim_hv_stats {
    uint64_t sent[10];             /* [k] = messages of kind k emitted (1 join .. 9 shuffle_reply;
                                      joins cast between rounds are not counted)   */
    uint64_t draws;                /* rand draws consumed in the round             */
    uint64_t error;                /* bit0 queue overflow, bit1 id-map overflow,
                                      bit2 get_next_id case_clause, bit3 2-tuple
                                      neighbor_rejected (reference crash points)  */
    uint64_t processed;            /* messages handled                             */
    uint64_t active;               /* vertices that ran a handler or a timer       */
    uint64_t algo_bytes;           /* 64 B per message read or written
                                      + 2 x 176 B per active vertex (views, head)
                                      + 12 B per vertex (bucket count/offset)      */
    double   kernel_ms;
} psim_hv_stats;
/* Fresh cluster of n vertices (init/1: Active = {self}, Passive = {},
 * epoch 1).  Replaces starting n partisan_hyparview_peer_service_manager
 * processes (:745-822).  Random draws use the handle's seed, stream kind 4. */
int  psim_hv_setup(psim_handle* h, uint32_t n, const psim_hv_config* cfg);
int  psim_hv_set_alive(psim_handle* h, const uint8_t* alive, size_t n);
/* handle_cast({join, Peer}) (:999-1016) at v[i] toward contact[i], made
 * between rounds (delivered by the next round).  The v[i] must be distinct. */
int  psim_hv_join(psim_handle* h, const uint32_t* v, const uint32_t* contact, size_t k);
int  psim_hv_step(psim_handle* h, uint32_t rounds, psim_hv_stats* stats, size_t cap);
/* Sequential joins (config C2's schedule): vertex v[i] joins contact[i],
 * then `rounds` rounds run, for i = 0..k-1 -- the same state, draws and
 * per-round stats (k * rounds rows, up to cap) as k psim_hv_join(v + i,
 * contact + i, 1) + psim_hv_step(rounds) calls, with one host wait per 16
 * rounds instead of two per join.  An error is reported with the round it
 * happened in, after the rounds enqueued with it ran (the state is then
 * spent: set up again). */
int  psim_hv_join_seq(psim_handle* h, const uint32_t* v, const uint32_t* contact, size_t k, uint32_t rounds,
                      psim_hv_stats* stats, size_t cap);
/* act[n*8], pas[n*32] padded with 0xFFFFFFFF; na/np = view sizes (active
 * includes self, as sets:to_list(Active) does). */
int  psim_hv_get_views(const psim_handle* h, uint32_t* act, uint8_t* na, uint32_t* pas, uint8_t* np, size_t n);
int  psim_hv_get_draws(const psim_handle* h, uint64_t* draws, size_t n);
/* which 0 = sent_message_map, 1 = recv_message_map of vertex v. */
int  psim_hv_get_idmap(const psim_handle* h, uint32_t v, int which, uint32_t* peer, uint32_t* epoch, uint32_t* cnt,
                       size_t cap, size_t* len);
int  psim_hv_inflight(const psim_handle* h, uint64_t* messages);

/* --- causal delivery (partisan_causality_backend.erl) ------------------ */
typedef struct psim_causal_stats {
    uint64_t emitted;              /* emit/4 calls at the end of the round      */
    uint64_t received;             /* receive_message/2 calls                   */
    uint64_t delivered;            /* deliver/5 calls                           */
    uint64_t checks;               /* dominates evaluations                     */
    uint64_t buffered;             /* buffered messages after the round         */
    uint64_t algo_bytes;           /* 1024 B per delivery + 256 B per
                                      dominates check + 32 B per message        */
    double   kernel_ms;
} psim_causal_stats;
/* Causal delivery among n vertices with m <= 64 emitters e_k = floor(k n / m)
 * (clock lanes = emitter actors; a non-emitter's own entry is its `self`
 * counter).  At the end of round t emitter k broadcasts -- emit/4 to every
 * other vertex in id order (:172-201) -- iff t % period == k % period; the
 * message to v lands in round t + 1 + mulhi(Philox({v, t, 6, k}), dmax).
 * Round t at v: receive_message/2 per arrival in (src, seq) order (:205-220),
 * then handle_info(deliver) if t % redeliver == 0 (:233-248). */
int  psim_causal_setup(psim_handle* h, uint32_t n, uint32_t m, uint32_t period, uint32_t dmax, uint32_t redeliver);
int  psim_causal_step(psim_handle* h, uint32_t rounds, psim_causal_stats* stats, size_t cap);
/* lanes[n*64] (lane k = counter of emitter k's actor, 0 = absent), self[n]. */
int  psim_causal_get_clocks(const psim_handle* h, uint32_t* lanes, uint32_t* self, size_t n);
/* buffered_messages of v in list order, as (emitter index, emission round). */
int  psim_causal_get_buffered(const psim_handle* h, uint32_t v, uint32_t* k, uint32_t* round, size_t cap,
                              size_t* len);
int  psim_causal_get_delivered(const psim_handle* h, uint64_t* delivered, size_t n);
int  psim_causal_emitters(const psim_handle* h, uint32_t* emitters, size_t m);
/* Vertex-sharded causal delivery (one process per GPU): this
 * handle owns global ids [floor(n rank/world), floor(n (rank+1)/world)); the
 * getters above then address that range (index 0 = its first vertex).  A
 * round is split-phase: psim_causal_shard_round runs the local round and the
 * broadcasts of the shard's emitters, writing their clocks into the caller's
 * device `slab` (64 x 64 u32, zero elsewhere); the caller sum-all-reduces
 * the slab (RCCL on a node) and hands it to psim_causal_shard_ingest.
 * Messages are never materialised, so that 16 KB is the whole
 * exchange. */
int  psim_causal_shard_setup(psim_handle* h, uint32_t n, uint32_t m, uint32_t period, uint32_t dmax,
                             uint32_t redeliver, int rank, int world);
int  psim_causal_shard_info(const psim_handle* h, uint32_t* v_lo, uint32_t* n_local);
int  psim_causal_shard_round(psim_handle* h, void* slab, psim_causal_stats* stats);
int  psim_causal_shard_ingest(psim_handle* h, const void* slab);
/* The same exchange inside the library, on the handle's transport
 * (psim_shard_init_rccl / psim_shard_set_transport; world 1 needs none):
 * `rounds` rounds, collective, stats GLOBAL (kernel_ms this shard's). */
int  psim_causal_shard_step(psim_handle* h, uint32_t rounds, psim_causal_stats* stats, size_t cap);

/* --- full-membership strategy (partisan_full_membership_strategy.erl) --
 * Nodes 0..n-1; node v's #full_v1{} membership (a state_orset,
 * partisan_membership_set.erl:113-237) is two bitmaps over the cluster's
 * token universe: known tokens and removed tokens (token v = v's own
 * init/1 add; a self-leave allocates the next free token).  Schedule of a
 * round: leave calls, then join calls (made since the previous round, in
 * call order; RemoteState = the peer's state at the end of the previous
 * round), then the inbox in (src, seq) order, then periodic/1 every
 * `periodic_rounds` rounds.  n <= 2048, max_tokens <= 2048. */
typedef struct psim_fm_stats {
    uint64_t sent;                 /* {membership_strategy, {Spec, State}} emitted */
    uint64_t processed;            /* handle_message/2 calls                      */
    uint64_t merges;               /* merges by join/3 or handle_message/2        */
    uint64_t updates;              /* membership changes (peer_service_events:update) */
    uint64_t inflight;             /* messages the next round delivers            */
    uint64_t member_sum;           /* sum over live nodes of |members|            */
    uint64_t algo_bytes;           /* bytes the round's kernels must move */
    double   kernel_ms;
} psim_fm_stats;
/* Replaces init/1 on n nodes (:70-74, new_state/1 :288-294). */
int  psim_fm_setup(psim_handle* h, uint32_t n, uint32_t periodic_rounds, uint32_t max_tokens);
int  psim_fm_set_alive(psim_handle* h, const uint8_t* alive, size_t n);
/* partisan_peer_service:join(Peer) at v[i] -> {connected, ...} -> join/3 (:85-96) */
int  psim_fm_join(psim_handle* h, const uint32_t* v, const uint32_t* peer, size_t k);
/* partisan_peer_service:leave(Leaving) at v[i] -> leave/2 (:177-214) */
int  psim_fm_leave(psim_handle* h, const uint32_t* v, const uint32_t* leaving, size_t k);
int  psim_fm_step(psim_handle* h, uint32_t rounds, psim_fm_stats* stats, size_t cap);
/* known[n*words], removed[n*words] token bitmaps (words = ceil(max_tokens/64)), alive[n] */
int  psim_fm_get_state(const psim_handle* h, uint64_t* known, uint64_t* removed, uint8_t* alive, size_t n,
                       size_t words);
/* token_node[t] = the node token t adds; *used = tokens allocated so far */
int  psim_fm_tokens(const psim_handle* h, uint32_t* token_node, size_t ntok, uint32_t* used);
int  psim_fm_inflight(const psim_handle* h, uint64_t* messages);
/* Full-membership messages on the wire: a node's
 * gossip leaves its manager as {membership_strategy, {NodeSpec, #full_v1{}}}
 * to every peer of its state (gossip_messages/2,
 * partisan_full_membership_strategy.erl:247-267; the manager's sends
 * partisan_pluggable_peer_service_manager.erl:1396-1407, 1764-1776) and is
 * handled by handle_message/2 (:135-166).  One record per message the next
 * round delivers, in handling order (dst, src, seq): seq = the sender's
 * emission index in its round (a put keeps its own); the #full_v1{}
 * membership of record i is known[i*words ...] / removed[i*words ...], token
 * bitmaps as psim_fm_get_state (words = ceil(max_tokens / 64)).
 * messages: *count = total, records past cap not written (cap 0: count only).
 * take: the messages for node dst, off the wire (the next round will not
 * deliver them); PSIM_EINVAL when cap is too small (nothing taken, *count =
 * what it needs).  put: onto the wire for the next round (what a node's
 * manager received); src may be any id, one outside the cluster included --
 * the schedule handles an inbox in (src, seq) order, a put after an
 * in-flight message of the same (src, seq); a state must hold only tokens
 * already allocated (psim_fm_tokens), removed ones among the known. */
typedef struct psim_fm_msg { uint32_t src, dst, seq, reserved; } psim_fm_msg;
int  psim_fm_messages(const psim_handle* h, psim_fm_msg* out, uint64_t* known, uint64_t* removed, size_t cap,
                      size_t words, size_t* count);
int  psim_fm_take(psim_handle* h, uint32_t dst, psim_fm_msg* out, uint64_t* known, uint64_t* removed, size_t cap,
                  size_t words, size_t* count);
int  psim_fm_put(psim_handle* h, const psim_fm_msg* msgs, const uint64_t* known, const uint64_t* removed, size_t k,
                 size_t words);

/* --- SCAMP membership (partisan_scamp_v{1,2}_membership_strategy.erl) ----
 * Nodes 0..n-1 run the strategy inside the pluggable peer service manager.
 * Round: leave calls, then join calls made since the last round (call
 * order), then the inbox in (src, seq) order with the manager's stop check,
 * then periodic/1 every `periodic_rounds`.  A handler at u reaches t iff
 * t != u, t was up at the start of the round and t is one of u's members
 * before or after the handler (DESIGN.md "SCAMP").  Views are rows of
 * PSIM_SCAMP_PV_CAP / PSIM_SCAMP_IV_CAP ids in the reference's list order;
 * overflowing one is PSIM_EOVERFLOW.  Draws: Philox stream (seed, v, kind 5,
 * incarnation). */
#define PSIM_SCAMP_PV_CAP 128
#define PSIM_SCAMP_IV_CAP 64
typedef struct psim_scamp_stats {
    uint64_t sent[7];              /* [k] queued messages of kind k: 1 forward_subscription, 2 keep_subscription,
                                      3 ping, 4 remove_subscription, 5 replace_subscription,
                                      6 bootstrap_remove_subscription                          */
    uint64_t dropped;              /* emitted to self, a dead or a non-connected node          */
    uint64_t processed;            /* handle_message/2 calls                                   */
    uint64_t draws;                /* rand draws                                               */
    uint64_t stopped;              /* managers that stopped this round                         */
    uint64_t error;                /* bit2: v2 bootstrap_remove lists:nth crash (Q18), bit3: v1 Q17 */
    uint64_t pv_sum;               /* sum over live nodes of |partial view| (self included)    */
    uint64_t inview_sum;           /* sum of |in-view|                                          */
    uint64_t resub;                /* isolated periodic re-subscriptions (Q19)                 */
    uint64_t algo_bytes;           /* bytes the round's kernels must move          */
    double   kernel_ms;
} psim_scamp_stats;
/* init/1 on n nodes (v2 :75-85, v1 :56-66); version 1 or 2; c = scamp_c (SCAMP_C_VALUE 5) */
int  psim_scamp_setup(psim_handle* h, uint32_t n, uint32_t version, uint32_t c, uint32_t periodic_rounds);
int  psim_scamp_set_alive(psim_handle* h, const uint8_t* alive, size_t n);
/* partisan_peer_service:join(Contact) at v[i] -> {connected, ...} -> join/3 */
int  psim_scamp_join(psim_handle* h, const uint32_t* v, const uint32_t* contact, size_t k);
/* partisan_peer_service:leave(Node) at v[i] -> leave/2 */
int  psim_scamp_leave(psim_handle* h, const uint32_t* v, const uint32_t* node, size_t k);
/* v[i] crash and restart now: init/1 state, new incarnation, in-flight messages to them lost */
int  psim_scamp_crash(psim_handle* h, const uint32_t* v, size_t k);
int  psim_scamp_step(psim_handle* h, uint32_t rounds, psim_scamp_stats* stats, size_t cap);
/* pv[n*PSIM_SCAMP_PV_CAP], iv[n*PSIM_SCAMP_IV_CAP] in list order, npv/niv = lengths; any may be NULL */
int  psim_scamp_get_views(const psim_handle* h, uint32_t* pv, uint32_t* npv, uint32_t* iv, uint32_t* niv, size_t n);
/* draws of the current incarnation, round of the last ping handled (-1 none), alive */
int  psim_scamp_get_nodes(const psim_handle* h, uint64_t* draws, int32_t* last_ping, uint8_t* alive, size_t n);
int  psim_scamp_inflight(const psim_handle* h, uint64_t* messages);
/* The membership messages on the wire: what the pluggable
 * manager sends as {membership_strategy, Msg} on ?MEMBERSHIP_CHANNEL
 * (partisan_pluggable_peer_service_manager.erl:1396-1407, 1764-1776), one
 * record per message the next round delivers.  type (PSIM_SC_*) and a / b
 * give the reference term (partisan_scamp_v{1,2}_membership_strategy.erl):
 *   FORWARD {forward_subscription, A}  KEEP {keep_subscription, A}
 *   PING {ping, A}  REMOVE {remove_subscription, A}
 *   REPLACE {replace_subscription, A, B}  BOOTSTRAP_REMOVE {bootstrap_remove_subscription, A}
 * with A, B vertex ids (node specs in the Erlang adapter); seq = the sender's
 * emission index (the schedule handles a vertex's inbox in (src, seq) order). */
enum { PSIM_SC_FORWARD = 1, PSIM_SC_KEEP = 2, PSIM_SC_PING = 3, PSIM_SC_REMOVE = 4, PSIM_SC_REPLACE = 5,
       PSIM_SC_BOOTSTRAP_REMOVE = 6 };
typedef struct psim_scamp_msg { uint32_t type, src, dst, seq, a, b; } psim_scamp_msg;
/* the messages in handling order (dst, src, seq); *count = total, entries past cap not written */
int  psim_scamp_messages(const psim_handle* h, psim_scamp_msg* out, size_t cap, size_t* count);
/* takes the messages for vertex dst off the wire (the next round will not
 * deliver them), in (src, seq) order; PSIM_EINVAL when cap is too small
 * (nothing taken; *count = what it needs) */
int  psim_scamp_take(psim_handle* h, uint32_t dst, psim_scamp_msg* out, size_t cap, size_t* count);
/* puts messages on the wire for the next round -- e.g. the ones a node's
 * manager received (handle_message/2 of the Erlang adapter); src may be any
 * id, a sender outside the simulated cluster included: the schedule orders
 * by (src, seq) */
int  psim_scamp_put(psim_handle* h, const psim_scamp_msg* msgs, size_t k);

/* --- C3: Plumtree repair over churning SCAMP v2 ------------------------
 * The pluggable manager runs SCAMP v2 (the psim_scamp_* state of this
 * handle) and the Plumtree server reacts to its {update, Members} casts
 * (partisan_plumtree_broadcast.erl:607-639); Plumtree sends need a
 * connection, i.e. the destination in the sender's partial view.  A round:
 * the SCAMP round, then the Plumtree round (the round's updates in order,
 * the inbox in (src, seq) order, the lazy tick).  A crash restarts both
 * processes (start_link/0 with members = {self}).  psim_scamp_get_views /
 * _get_nodes read the membership side.  crash / join return without waiting
 * for the device (their work is ordered before the next round and every
 * read-back); an error of a round (PSIM_EOVERFLOW) leaves the C3 state spent:
 * set it up again. */
typedef struct psim_c3_stats {
    psim_scamp_stats scamp;        /* the membership round                      */
    uint64_t pt_sent[6];           /* [k] Plumtree messages of PSIM_MSG_* kind k */
    uint64_t pt_dropped;           /* Plumtree sends without a connection        */
    uint64_t delivered_new;        /* Mod:merge/2 returned true                  */
    uint64_t active;               /* vertices that handled messages             */
    uint64_t updates;              /* {update, Members} casts applied            */
    uint64_t delivered_live;       /* live vertices holding the current heartbeat */
    uint64_t live;                 /* live vertices                              */
    uint64_t outstanding_live;     /* outstanding rows to connected live peers   */
    uint64_t pt_algo_bytes;        /* bytes the Plumtree round must move */
    double   pt_kernel_ms;
} psim_c3_stats;
int  psim_c3_setup(psim_handle* h, uint32_t n, uint32_t c, uint32_t periodic_rounds);
int  psim_c3_join(psim_handle* h, const uint32_t* v, const uint32_t* contact, size_t k);
int  psim_c3_crash(psim_handle* h, const uint32_t* v, size_t k);
/* heartbeat at `root` (backend :341-368 -> broadcast :565-569) */
int  psim_c3_heartbeat(psim_handle* h, uint32_t root, uint32_t* mono_out);
int  psim_c3_step(psim_handle* h, uint32_t rounds, psim_c3_stats* stats, size_t cap);
/* `rounds` rounds of churn in one call: round i is the heartbeat at hb_root
 * when hb_every != 0 and i % hb_every == 0, then crash of
 * crash_v[crash_off[i] .. crash_off[i+1]), join of join_v / join_c over
 * [join_off[i], join_off[i+1]), then one psim_c3_step round -- the same
 * calls and the same result as making them one by one, without the host
 * waiting for the device between rounds (offsets: rounds + 1 entries each).
 * stats[i] is round i's; the first failing round's error is returned.
 * Joins made by psim_c3_join since the last round: PSIM_ESTATE (step first,
 * or pass them in round 0's lists). */
int  psim_c3_run(psim_handle* h, uint32_t rounds, const uint32_t* crash_off, const uint32_t* crash_v,
                 const uint32_t* join_off, const uint32_t* join_v, const uint32_t* join_c, uint32_t hb_every,
                 uint32_t hb_root, psim_c3_stats* stats, size_t cap);
/* vertex v's Plumtree state: all_eager_peers / all_lazy_peers / outstanding
 * rows (sorted ids, up to cap each), the heartbeat serial it delivered (0 =
 * none) and its pushed Round */
int  psim_c3_get_plumtree(const psim_handle* h, uint32_t v, uint32_t* eager, size_t* ne, uint32_t* lazy, size_t* nl,
                          uint32_t* outstanding, size_t* no, size_t cap, uint32_t* delivered_mono,
                          uint32_t* recv_round);

/* ---- Transitive relay over Plumtree out-links -------
 * Replaces, for a batch of k sends with `transitive => true`:
 *   do_send_message/3 (src/partisan_hyparview_peer_service_manager.erl:2220-2290),
 *   do_tree_forward/4 (:2796-2842), handle_message({relay_message, ..}) (:1800-1832),
 *   retrieve_outlinks/1 (:2846-2870).
 * act = active views (CSR, the members handle_message checks), ol = each
 * vertex's out_links (its eager peers in its own tree), alive = 1 per live
 * vertex.  "Connected to P" = P live and a peer of the sender (a member of its
 * view or a vertex whose view lists it).  Round 0: origins handle their sends;
 * a copy sent in round r is handled in round r + 1; runs to quiescence.
 * Outputs delivered[k] (copies of Message that reached dst[k]),
 * first_round[k] (arrival round, UINT32_MAX = never) and per-round stats
 * (up to cap rows).  Returns the rounds run, PSIM_EOVERFLOW when one round
 * holds more than max_copies copies, PSIM_EINVAL for bad shapes (src == dst,
 * ids >= n, relay_ttl 0 or > 127, k >= 2^24, a CSR whose row pointers do not
 * start at 0 and end at its id array's length act_len / ol_len). */
typedef struct psim_relay_stats {
    uint64_t direct;    /* copies of Message sent to Node (connected)      */
    uint64_t relay;     /* relay_message copies sent                       */
    uint64_t dropped;   /* relay_message copies dropped at TTL 0           */
    uint64_t lost;      /* out-links not connected: the send fails         */
    uint64_t arrived;   /* copies of Message arriving at Node this round   */
} psim_relay_stats;
int64_t psim_relay_run(psim_handle* h, uint32_t n, const uint64_t* act_ptr, const uint32_t* act, uint64_t act_len,
                       const uint64_t* ol_ptr, const uint32_t* ol, uint64_t ol_len, const uint8_t* alive, uint32_t k,
                       const uint32_t* src, const uint32_t* dst, uint32_t relay_ttl, uint64_t* delivered,
                       uint32_t* first_round, psim_relay_stats* stats, size_t cap, size_t max_copies);

/* Totals since creation: device ms spent in round kernels and rounds run. */
int  psim_get_timing(const psim_handle* h, double* round_kernel_ms, uint64_t* rounds);
/* Switch PSIM_CFG_CHUNK_TIMING on (chunk != 0) or off after creation: one event
 * pair per chunk (round kernels back to back; on a sharded handle the chunk's
 * time includes its exchanges) or a pair per round kernel (kernel-only times,
 * at ~10 us of idle GPU per marker).  Not while async rounds are pending. */
int  psim_set_chunk_timing(psim_handle* h, int chunk);

#ifdef __cplusplus
}
#endif
#endif /* PSIM_H */
