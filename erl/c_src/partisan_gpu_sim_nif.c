/*
 * partisan_gpu_sim_nif.c -- the thin Erlang NIF over libpsim.so (include/psim.h).
 *
 * Built only where erl_nif.h exists (an erts host; this image has none):
 *   cc -O2 -shared -fPIC -I"$ERTS_INCLUDE" -I../../include \
 *      partisan_gpu_sim_nif.c -L../../partisan_amd -lpsim -Wl,-rpath,'$ORIGIN' \
 *      -o ../priv/partisan_gpu_sim.so
 *
 * Every call that launches device work runs on a dirty CPU scheduler
 * (ERL_NIF_DIRTY_JOB_CPU_BOUND).  A handle is an enif resource whose
 * destructor calls psim_destroy; a per-resource mutex serialises calls
 * (psim handles are single-threaded).  Errors map to {error, Atom}.
 */
#include <erl_nif.h>
#include <string.h>

#include "psim.h"

typedef struct {
    psim_handle* h;
    ErlNifMutex* mu;
    uint32_t n;          /* plumtree vertices (load_csr) */
    uint64_t slots;
    uint32_t hv_n;       /* hyparview vertices (hv_setup) */
    uint32_t dm_n;       /* demers vertices (demers_setup) */
    uint32_t sc_n;       /* scamp / c3 vertices (scamp_setup, c3_setup) */
    uint32_t fm_n;       /* full-membership nodes (fm_setup) */
    uint32_t fm_words;   /* token bitmap words per node */
    uint32_t cs_n;       /* causal vertices (causal_setup) */
} sim_res;

static ErlNifResourceType* SIM_RES;

static ERL_NIF_TERM mk_atom(ErlNifEnv* env, const char* a) {
    ERL_NIF_TERM t;
    return enif_make_existing_atom(env, a, &t, ERL_NIF_LATIN1) ? t : enif_make_atom(env, a);
}

static ERL_NIF_TERM err(ErlNifEnv* env, int rc) {
    const char* a = "psim_error";
    switch (rc) {
    case PSIM_EINVAL: a = "einval"; break;
    case PSIM_ENOMEM: a = "enomem"; break;
    case PSIM_EHIP: a = "ehip"; break;
    case PSIM_ERCCL: a = "erccl"; break;
    case PSIM_ESTATE: a = "estate"; break;
    case PSIM_EOVERFLOW: a = "eoverflow"; break;
    case PSIM_EBUSY: a = "ebusy"; break;
    case PSIM_ENODEV: a = "enodev"; break;
    case PSIM_ENOSPC: a = "enospc"; break;
    case PSIM_ENOTSUP: a = "enotsup"; break;
    }
    return enif_make_tuple2(env, mk_atom(env, "error"), mk_atom(env, a));
}

static void sim_dtor(ErlNifEnv* env, void* obj) {
    (void)env;
    sim_res* r = (sim_res*)obj;
    if (r->h) psim_destroy(r->h);
    if (r->mu) enif_mutex_destroy(r->mu);
}

static int load(ErlNifEnv* env, void** priv, ERL_NIF_TERM info) {
    (void)priv; (void)info;
    SIM_RES = enif_open_resource_type(env, NULL, "partisan_gpu_sim", sim_dtor, ERL_NIF_RT_CREATE, NULL);
    return SIM_RES ? 0 : -1;
}

static int get_res(ErlNifEnv* env, ERL_NIF_TERM t, sim_res** r) {
    return enif_get_resource(env, t, SIM_RES, (void**)r) && (*r)->h;
}

static unsigned map_u32(ErlNifEnv* env, ERL_NIF_TERM m, const char* key, unsigned dflt) {
    ERL_NIF_TERM v;
    unsigned x;
    if (enif_get_map_value(env, m, mk_atom(env, key), &v) && enif_get_uint(env, v, &x)) return x;
    return dflt;
}

/* new(#{lazy_tick_rounds, exchange_tick_rounds, device, seed, max_roots, forest_lanes}) -> {ok, Sim}
 * max_roots: heartbeat roots whose trees the handle keeps (every node of the
 * cluster heartbeats, partisan_plumtree_backend:341-368); 0 / absent = 16.
 * forest_lanes (max_roots > 16): lanes for the heartbeats in flight at once,
 * every root's records kept (psim_forest_set_lanes); 0 / absent = one per root */
static ERL_NIF_TERM nif_new(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    if (!enif_is_map(env, argv[0])) return enif_make_badarg(env);
    psim_config cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.abi_version = PSIM_ABI_VERSION;
    cfg.device = (int32_t)map_u32(env, argv[0], "device", (unsigned)-1);
    cfg.lazy_tick_rounds = map_u32(env, argv[0], "lazy_tick_rounds", 1);
    cfg.exchange_tick_rounds = map_u32(env, argv[0], "exchange_tick_rounds", 10);
    cfg.max_roots = map_u32(env, argv[0], "max_roots", 0);
    {
        ERL_NIF_TERM v;
        ErlNifUInt64 seed = 0;
        if (enif_get_map_value(env, argv[0], mk_atom(env, "seed"), &v)) enif_get_uint64(env, v, &seed);
        cfg.seed = (uint64_t)seed;
    }
    sim_res* r = (sim_res*)enif_alloc_resource(SIM_RES, sizeof(sim_res));
    memset(r, 0, sizeof *r);
    int rc = psim_create(&cfg, &r->h);
    if (rc != PSIM_OK) { enif_release_resource(r); return err(env, rc); }
    const unsigned lanes = map_u32(env, argv[0], "forest_lanes", 0);
    if (lanes && (rc = psim_forest_set_lanes(r->h, lanes)) != PSIM_OK) {
        psim_destroy(r->h);
        r->h = NULL;
        enif_release_resource(r);
        return err(env, rc);
    }
    r->mu = enif_mutex_create("partisan_gpu_sim");
    ERL_NIF_TERM t = enif_make_resource(env, r);
    enif_release_resource(r);
    return enif_make_tuple2(env, mk_atom(env, "ok"), t);
}

/* load_csr(Sim, RowPtr :: <<u64-little>>, Col :: <<u32-little>>) -> ok */
static ERL_NIF_TERM nif_load_csr(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    ErlNifBinary rp, col;
    if (!get_res(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &rp) ||
        !enif_inspect_binary(env, argv[2], &col) || rp.size < 8 || rp.size % 8 || col.size % 4)
        return enif_make_badarg(env);
    if (rp.size / 8 - 1 > 0xFFFFFFFFu) return enif_make_badarg(env);
    uint32_t n = (uint32_t)(rp.size / 8 - 1);
    /* binary data carries no alignment guarantee: copy the row pointers
     * (and ids) out; the library checks row_ptr against col's length */
    uint64_t* rpa = (uint64_t*)enif_alloc(rp.size);
    uint32_t* cola = (uint32_t*)enif_alloc(col.size ? col.size : 4);
    if (!rpa || !cola) {
        if (rpa) enif_free(rpa);
        if (cola) enif_free(cola);
        return err(env, PSIM_ENOMEM);
    }
    memcpy(rpa, rp.data, rp.size);
    memcpy(cola, col.data, col.size);
    enif_mutex_lock(r->mu);
    int rc = psim_load_csr(r->h, n, rpa, cola, col.size / 4);
    enif_free(rpa);
    enif_free(cola);
    if (rc == PSIM_OK) { r->n = n; psim_num_slots(r->h, &r->slots); }
    enif_mutex_unlock(r->mu);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

/* set_alive(Sim, <<0|1 per vertex>>) -> ok */
static ERL_NIF_TERM nif_set_alive(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    ErlNifBinary b;
    if (!get_res(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &b)) return enif_make_badarg(env);
    enif_mutex_lock(r->mu);
    int rc = psim_set_alive(r->h, b.data, b.size);
    enif_mutex_unlock(r->mu);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

/* reset_trees(Sim) -> ok   (update with new members at every node) */
static ERL_NIF_TERM nif_reset_trees(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
    enif_mutex_lock(r->mu);
    int rc = psim_plumtree_reset_trees(r->h);
    enif_mutex_unlock(r->mu);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

/* restart_backend(Sim, Vertex) -> ok   (the vertex's heartbeat backend
 * restarts: newer epoch, Monotonic 0, empty timestamp table; heartbeat ids
 * from then on are Epoch bsl 24 bor Monotonic) */
static ERL_NIF_TERM nif_restart_backend(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned v;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &v)) return enif_make_badarg(env);
    enif_mutex_lock(r->mu);
    int rc = psim_plumtree_restart_backend(r->h, v);
    enif_mutex_unlock(r->mu);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

/* broadcast(Sim, Root) -> {ok, Id}   (Id = Epoch bsl 24 bor Monotonic) */
static ERL_NIF_TERM nif_broadcast(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned root;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &root)) return enif_make_badarg(env);
    uint32_t mono = 0;
    enif_mutex_lock(r->mu);
    int rc = psim_plumtree_broadcast(r->h, root, &mono);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) return err(env, rc);
    return enif_make_tuple2(env, mk_atom(env, "ok"), enif_make_uint(env, mono));
}

/* broadcast_many(Sim, Roots :: <<u32-little>>) -> {ok, Ids :: <<u32-little>>}: the
 * backend's heartbeat timer firing at every listed node at once
 * (partisan_plumtree_backend.erl:341-368, 421-428; psim_plumtree_broadcast_many) */
static ERL_NIF_TERM nif_broadcast_many(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    ErlNifBinary roots;
    if (!get_res(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &roots) || roots.size % 4)
        return enif_make_badarg(env);
    const size_t k = roots.size / 4;
    uint32_t* rt = (uint32_t*)enif_alloc(roots.size + 4);      /* binary data has no alignment guarantee */
    if (!rt) return err(env, PSIM_ENOMEM);
    memcpy(rt, roots.data, roots.size);
    ERL_NIF_TERM t;
    unsigned char* ids = enif_make_new_binary(env, k * 4, &t);
    uint32_t* tmp = (uint32_t*)enif_alloc(k * 4 + 4);
    int rc = tmp ? PSIM_OK : PSIM_ENOMEM;
    if (rc == PSIM_OK) {
        enif_mutex_lock(r->mu);
        rc = psim_plumtree_broadcast_many(r->h, rt, k, tmp);
        enif_mutex_unlock(r->mu);
        if (rc == PSIM_OK) memcpy(ids, tmp, k * 4);
    }
    enif_free(rt);
    if (tmp) enif_free(tmp);
    if (rc != PSIM_OK) return err(env, rc);
    return enif_make_tuple2(env, mk_atom(env, "ok"), t);
}

static ERL_NIF_TERM stats_term(ErlNifEnv* env, const psim_round_stats* s) {
    ERL_NIF_TERM keys[9] = {mk_atom(env, "broadcast"), mk_atom(env, "prune"), mk_atom(env, "i_have"),
                            mk_atom(env, "ignored_i_have"), mk_atom(env, "graft"), mk_atom(env, "delivered"),
                            mk_atom(env, "senders"), mk_atom(env, "algo_bytes"), mk_atom(env, "kernel_us")};
    ERL_NIF_TERM vals[9] = {enif_make_uint64(env, s->sent[PSIM_MSG_BROADCAST]),
                            enif_make_uint64(env, s->sent[PSIM_MSG_PRUNE]),
                            enif_make_uint64(env, s->sent[PSIM_MSG_IHAVE]),
                            enif_make_uint64(env, s->sent[PSIM_MSG_IGNORED]),
                            enif_make_uint64(env, s->sent[PSIM_MSG_GRAFT]),
                            enif_make_uint64(env, s->delivered_new),
                            enif_make_uint64(env, s->senders),
                            enif_make_uint64(env, s->algo_bytes),
                            enif_make_uint64(env, (uint64_t)(s->kernel_ms * 1000.0))};
    ERL_NIF_TERM m;
    enif_make_map_from_arrays(env, keys, vals, 9, &m);
    return m;
}

/* run(Sim, MaxRounds) -> {ok, Rounds, [StatsMap]}   (to quiescence) */
static ERL_NIF_TERM nif_run(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned maxr;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &maxr)) return enif_make_badarg(env);
    enum { CAP = 4096 };
    psim_round_stats* st = (psim_round_stats*)enif_alloc(CAP * sizeof(psim_round_stats));
    if (!st) return err(env, PSIM_ENOMEM);
    uint32_t ran = 0;
    enif_mutex_lock(r->mu);
    int rc = psim_run(r->h, maxr, st, CAP, &ran);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) { enif_free(st); return err(env, rc); }
    ERL_NIF_TERM list = enif_make_list(env, 0);
    for (uint32_t i = ran < CAP ? ran : CAP; i > 0; i--) list = enif_make_list_cell(env, stats_term(env, &st[i - 1]), list);
    enif_free(st);
    return enif_make_tuple3(env, mk_atom(env, "ok"), enif_make_uint(env, ran), list);
}

/* broadcast_run(Sim, Root, MaxRounds) -> {ok, Id, Rounds, [StatsMap]}: one heartbeat
 * interval of one root, broadcast then rounds to quiescence in one call
 * (psim_plumtree_broadcast_run) */
static ERL_NIF_TERM nif_broadcast_run(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned root, maxr;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &root) || !enif_get_uint(env, argv[2], &maxr))
        return enif_make_badarg(env);
    enum { CAP = 4096 };
    psim_round_stats* st = (psim_round_stats*)enif_alloc(CAP * sizeof(psim_round_stats));
    if (!st) return err(env, PSIM_ENOMEM);
    uint32_t ran = 0, mono = 0;
    enif_mutex_lock(r->mu);
    int rc = psim_plumtree_broadcast_run(r->h, root, &mono, maxr, st, CAP, &ran);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) { enif_free(st); return err(env, rc); }
    ERL_NIF_TERM list = enif_make_list(env, 0);
    for (uint32_t i = ran < CAP ? ran : CAP; i > 0; i--) list = enif_make_list_cell(env, stats_term(env, &st[i - 1]), list);
    enif_free(st);
    return enif_make_tuple4(env, mk_atom(env, "ok"), enif_make_uint(env, mono), enif_make_uint(env, ran), list);
}

/* broadcast_run_n(Sim, Root, Count, Reset, MaxRounds) -> {ok, [{Id, Rounds}], [StatsMap]}:
 * Count heartbeat intervals of one root back to back, reset_trees before
 * each when Reset is 1 -- the same as Count reset_trees/1 + broadcast_run/3
 * calls (psim_plumtree_broadcast_run_n) */
static ERL_NIF_TERM nif_broadcast_run_n(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned root, count, reset, maxr;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &root) || !enif_get_uint(env, argv[2], &count) ||
        !enif_get_uint(env, argv[3], &reset) || !enif_get_uint(env, argv[4], &maxr) || count == 0 || count > 4096 ||
        reset > 1)
        return enif_make_badarg(env);
    enum { CAP = 65536 };
    psim_round_stats* st = (psim_round_stats*)enif_alloc(CAP * sizeof(psim_round_stats));
    uint32_t* rounds = (uint32_t*)enif_alloc(count * sizeof(uint32_t));
    uint32_t* monos = (uint32_t*)enif_alloc(count * sizeof(uint32_t));
    if (!st || !rounds || !monos) {
        if (st) enif_free(st);
        if (rounds) enif_free(rounds);
        if (monos) enif_free(monos);
        return err(env, PSIM_ENOMEM);
    }
    uint32_t done = 0;
    enif_mutex_lock(r->mu);
    int rc = psim_plumtree_broadcast_run_n(r->h, root, count, reset, maxr, st, CAP, rounds, monos, &done);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) {
        enif_free(st);
        enif_free(rounds);
        enif_free(monos);
        return err(env, rc);
    }
    uint64_t total = 0;
    ERL_NIF_TERM ivs = enif_make_list(env, 0);
    for (uint32_t i = count; i > 0; i--)
        ivs = enif_make_list_cell(env, enif_make_tuple2(env, enif_make_uint(env, monos[i - 1]),
                                                        enif_make_uint(env, rounds[i - 1])), ivs);
    for (uint32_t i = 0; i < count; i++) total += rounds[i];
    ERL_NIF_TERM list = enif_make_list(env, 0);
    for (uint64_t i = total < CAP ? total : CAP; i > 0; i--) list = enif_make_list_cell(env, stats_term(env, &st[i - 1]), list);
    enif_free(st);
    enif_free(rounds);
    enif_free(monos);
    return enif_make_tuple3(env, mk_atom(env, "ok"), ivs, list);
}

/* step(Sim, Rounds) -> {ok, [StatsMap]} */
static ERL_NIF_TERM nif_step(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned k;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &k) || k == 0 || k > 65536)
        return enif_make_badarg(env);
    psim_round_stats* st = (psim_round_stats*)enif_alloc(k * sizeof(psim_round_stats));
    if (!st) return err(env, PSIM_ENOMEM);
    enif_mutex_lock(r->mu);
    int rc = psim_step(r->h, k, st, k);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) { enif_free(st); return err(env, rc); }
    ERL_NIF_TERM list = enif_make_list(env, 0);
    for (unsigned i = k; i > 0; i--) list = enif_make_list_cell(env, stats_term(env, &st[i - 1]), list);
    enif_free(st);
    return enif_make_tuple2(env, mk_atom(env, "ok"), list);
}

/* peers(Sim) -> {ok, Eager, Lazy, Outstanding, RecvRound}: binaries of
 * u32-little masks over slots (and u16 Rounds) for every vertex */
static ERL_NIF_TERM nif_peers(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
    ERL_NIF_TERM te, tl, to, tr;
    unsigned char* e = enif_make_new_binary(env, (size_t)r->n * 4, &te);
    unsigned char* l = enif_make_new_binary(env, (size_t)r->n * 4, &tl);
    unsigned char* o = enif_make_new_binary(env, (size_t)r->n * 4, &to);
    unsigned char* rr = enif_make_new_binary(env, (size_t)r->n * 2, &tr);
    enif_mutex_lock(r->mu);
    int rc = psim_get_plumtree(r->h, (uint32_t*)e, (uint32_t*)l, (uint32_t*)o, (uint16_t*)rr, r->n);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) return err(env, rc);
    return enif_make_tuple5(env, mk_atom(env, "ok"), te, tl, to, tr);
}

/* slots(Sim) -> {ok, RowPtr, Col}: the slot layout the masks index */
static ERL_NIF_TERM nif_slots(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
    ERL_NIF_TERM trp, tcol;
    unsigned char* rp = enif_make_new_binary(env, ((size_t)r->n + 1) * 8, &trp);
    unsigned char* col = enif_make_new_binary(env, (size_t)r->slots * 4, &tcol);
    enif_mutex_lock(r->mu);
    int rc = psim_get_slots(r->h, (uint64_t*)rp, (uint32_t*)col);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) return err(env, rc);
    return enif_make_tuple3(env, mk_atom(env, "ok"), trp, tcol);
}

/* delivered(Sim) -> {ok, <<0|1 per vertex>>} */
static ERL_NIF_TERM nif_delivered(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
    ERL_NIF_TERM t;
    unsigned char* d = enif_make_new_binary(env, r->n, &t);
    enif_mutex_lock(r->mu);
    int rc = psim_get_delivered(r->h, d, r->n);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) return err(env, rc);
    return enif_make_tuple2(env, mk_atom(env, "ok"), t);
}

/* trace_hash(Sim) -> {ok, {StateDigest, InflightDigest, Delivered, Rounds}} (psim_trace_hash) */
static ERL_NIF_TERM nif_trace_hash(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
    uint64_t h[4];
    enif_mutex_lock(r->mu);
    int rc = psim_trace_hash(r->h, h);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) return err(env, rc);
    ERL_NIF_TERM t[4];
    for (int i = 0; i < 4; i++) t[i] = enif_make_uint64(env, h[i]);
    return enif_make_tuple2(env, mk_atom(env, "ok"), enif_make_tuple_from_array(env, t, 4));
}

/* focus(Sim, Root) -> ok: the per-vertex getters read Root's heartbeat lane */
static ERL_NIF_TERM nif_focus(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned root;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &root)) return enif_make_badarg(env);
    enif_mutex_lock(r->mu);
    int rc = psim_plumtree_focus(r->h, root);
    enif_mutex_unlock(r->mu);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

/* set_omissions(Sim, SrcU32s, DstU32s) -> ok: omission faults on the directed
 * pairs (native-endian u32 binaries of equal length; <<>> heals) */
static ERL_NIF_TERM nif_set_omissions(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    ErlNifBinary s, d;
    if (!get_res(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &s) ||
        !enif_inspect_binary(env, argv[2], &d) || s.size != d.size || s.size % 4)
        return enif_make_badarg(env);
    enif_mutex_lock(r->mu);
    int rc = psim_set_omissions(r->h, (const uint32_t*)s.data, (const uint32_t*)d.data, s.size / 4);
    enif_mutex_unlock(r->mu);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

/* set_delays(Sim, SrcU32s, DstU32s, Rounds) -> ok: delay faults on the
 * directed pairs, Rounds one byte per pair (<<>>s: no delays) */
static ERL_NIF_TERM nif_set_delays(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    ErlNifBinary s, d, k;
    if (!get_res(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &s) ||
        !enif_inspect_binary(env, argv[2], &d) || !enif_inspect_binary(env, argv[3], &k) || s.size != d.size ||
        s.size % 4 || k.size != s.size / 4)
        return enif_make_badarg(env);
    /* binary data carries no alignment guarantee: copy the ids (as pair_call does) */
    uint32_t* src = (uint32_t*)enif_alloc(s.size + 4);
    uint32_t* dst = (uint32_t*)enif_alloc(d.size + 4);
    if (src) memcpy(src, s.data, s.size);
    if (dst) memcpy(dst, d.data, d.size);
    if (!src || !dst) {
        enif_free(src);
        enif_free(dst);
        return err(env, PSIM_ENOMEM);
    }
    enif_mutex_lock(r->mu);
    int rc = psim_set_delays(r->h, src, dst, (const uint8_t*)k.data, k.size);
    enif_mutex_unlock(r->mu);
    enif_free(src);
    enif_free(dst);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

/* relay_run(Sim, ActPtr, Act, OlPtr, Ol, Alive, Src, Dst, RelayTTL, MaxCopies)
 *   -> {ok, Rounds, [{Direct, Relay, Dropped, Lost, Arrived}], Delivered, FirstRound}
 * Transitive relay over out-links (psim_relay_run).  Pointer binaries are
 * native-endian u64, id binaries u32, Alive one byte per vertex; Delivered is
 * a u64 binary and FirstRound a u32 binary, one entry per send. */
static ERL_NIF_TERM nif_relay_run(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    ErlNifBinary ap, ac, op, ol, al, s, d;
    unsigned ttl;
    ErlNifUInt64 maxc;
    if (!get_res(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &ap) ||
        !enif_inspect_binary(env, argv[2], &ac) || !enif_inspect_binary(env, argv[3], &op) ||
        !enif_inspect_binary(env, argv[4], &ol) || !enif_inspect_binary(env, argv[5], &al) ||
        !enif_inspect_binary(env, argv[6], &s) || !enif_inspect_binary(env, argv[7], &d) ||
        !enif_get_uint(env, argv[8], &ttl) || !enif_get_uint64(env, argv[9], &maxc))
        return enif_make_badarg(env);
    if (ap.size % 8 || ap.size < 16 || op.size != ap.size || ac.size % 4 || ol.size % 4 || s.size % 4 ||
        s.size != d.size || al.size != ap.size / 8 - 1)
        return enif_make_badarg(env);
    const size_t k = s.size / 4;
    enum { kCap = 256 };
    psim_relay_stats st[kCap];
    ERL_NIF_TERM dv_t, fr_t;   /* env-owned: dropped with the env on an error return */
    unsigned char* dv = enif_make_new_binary(env, k * 8, &dv_t);
    unsigned char* fr = enif_make_new_binary(env, k * 4, &fr_t);
    if (!dv || !fr) return err(env, PSIM_ENOMEM);
    enif_mutex_lock(r->mu);
    /* copies: binary data carries no alignment guarantee */
    uint64_t* apc = (uint64_t*)enif_alloc(ap.size);
    uint64_t* opc = (uint64_t*)enif_alloc(op.size);
    uint32_t* acc = (uint32_t*)enif_alloc(ac.size + 4);
    uint32_t* olc = (uint32_t*)enif_alloc(ol.size + 4);
    uint32_t* sc = (uint32_t*)enif_alloc(s.size + 4);
    uint32_t* dc = (uint32_t*)enif_alloc(d.size + 4);
    int64_t rc = PSIM_ENOMEM;
    if (apc && opc && acc && olc && sc && dc) {
        memcpy(apc, ap.data, ap.size);
        memcpy(opc, op.data, op.size);
        memcpy(acc, ac.data, ac.size);
        memcpy(olc, ol.data, ol.size);
        memcpy(sc, s.data, s.size);
        memcpy(dc, d.data, d.size);
        uint64_t* dva = (uint64_t*)enif_alloc(k * 8 + 8);
        uint32_t* fra = (uint32_t*)enif_alloc(k * 4 + 4);
        if (dva && fra) {
            rc = psim_relay_run(r->h, (uint32_t)(al.size), apc, acc, ac.size / 4, opc, olc, ol.size / 4,
                                (const uint8_t*)al.data, (uint32_t)k, sc, dc, ttl, dva, fra, st, kCap, (size_t)maxc);
            memcpy(dv, dva, k * 8);
            memcpy(fr, fra, k * 4);
        }
        if (dva) enif_free(dva);
        if (fra) enif_free(fra);
    }
    void* tmp[] = {apc, opc, acc, olc, sc, dc};
    for (int i = 0; i < 6; i++)
        if (tmp[i]) enif_free(tmp[i]);
    enif_mutex_unlock(r->mu);
    if (rc < 0) return err(env, (int)rc);
    ERL_NIF_TERM rows = enif_make_list(env, 0);
    for (int64_t i = (rc < kCap ? rc : kCap) - 1; i >= 0; i--)
        rows = enif_make_list_cell(env,
                                   enif_make_tuple5(env, enif_make_uint64(env, st[i].direct),
                                                    enif_make_uint64(env, st[i].relay),
                                                    enif_make_uint64(env, st[i].dropped),
                                                    enif_make_uint64(env, st[i].lost),
                                                    enif_make_uint64(env, st[i].arrived)),
                                   rows);
    return enif_make_tuple5(env, mk_atom(env, "ok"), enif_make_uint64(env, (ErlNifUInt64)rc), rows, dv_t, fr_t);
}

/* ---- HyParView --------------------------------------------------------- */

/* hv_setup(Sim, N, #{active_max_size, ..., promotion_rounds}) -> ok */
static ERL_NIF_TERM nif_hv_setup(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned n;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &n) || !enif_is_map(env, argv[2]))
        return enif_make_badarg(env);
    psim_hv_config c;
    c.active_max_size = map_u32(env, argv[2], "active_max_size", 6);
    c.active_min_size = map_u32(env, argv[2], "active_min_size", 3);
    c.active_rwl = map_u32(env, argv[2], "active_rwl", 6);
    c.passive_max_size = map_u32(env, argv[2], "passive_max_size", 30);
    c.passive_rwl = map_u32(env, argv[2], "passive_rwl", 6);
    c.shuffle_k_active = map_u32(env, argv[2], "shuffle_k_active", 3);
    c.shuffle_k_passive = map_u32(env, argv[2], "shuffle_k_passive", 4);
    c.shuffle_rounds = map_u32(env, argv[2], "shuffle_rounds", 10);
    c.promotion_rounds = map_u32(env, argv[2], "promotion_rounds", 5);
    enif_mutex_lock(r->mu);
    int rc = psim_hv_setup(r->h, n, &c);
    if (rc == PSIM_OK) r->hv_n = n;
    enif_mutex_unlock(r->mu);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

/* hv_join(Sim, Joiners :: <<u32-little>>, Contacts :: <<u32-little>>) -> ok
 * (one handle_cast({join, Contact}) per joiner, between two rounds) */
static ERL_NIF_TERM nif_hv_join(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    ErlNifBinary v, c;
    if (!get_res(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &v) ||
        !enif_inspect_binary(env, argv[2], &c) || v.size != c.size || v.size % 4)
        return enif_make_badarg(env);
    enif_mutex_lock(r->mu);
    int rc = psim_hv_join(r->h, (const uint32_t*)v.data, (const uint32_t*)c.data, v.size / 4);
    enif_mutex_unlock(r->mu);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

static ERL_NIF_TERM hv_stats_term(ErlNifEnv* env, const psim_hv_stats* s) {
    static const char* names[10] = {"", "join", "neighbor", "forward_join", "disconnect", "neighbor_request",
                                    "neighbor_rejected", "neighbor_accepted", "shuffle", "shuffle_reply"};
    ERL_NIF_TERM keys[13], vals[13];
    for (int k = 1; k < 10; k++) {
        keys[k - 1] = mk_atom(env, names[k]);
        vals[k - 1] = enif_make_uint64(env, s->sent[k]);
    }
    keys[9] = mk_atom(env, "draws");      vals[9] = enif_make_uint64(env, s->draws);
    keys[10] = mk_atom(env, "error");     vals[10] = enif_make_uint64(env, s->error);
    keys[11] = mk_atom(env, "processed"); vals[11] = enif_make_uint64(env, s->processed);
    keys[12] = mk_atom(env, "kernel_us"); vals[12] = enif_make_uint64(env, (uint64_t)(s->kernel_ms * 1000.0));
    ERL_NIF_TERM m;
    enif_make_map_from_arrays(env, keys, vals, 13, &m);
    return m;
}

/* hv_step(Sim, Rounds) -> {ok, [StatsMap]} */
static ERL_NIF_TERM nif_hv_step(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned k;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &k) || k == 0 || k > 65536)
        return enif_make_badarg(env);
    psim_hv_stats* st = (psim_hv_stats*)enif_alloc(k * sizeof(psim_hv_stats));
    enif_mutex_lock(r->mu);
    int rc = psim_hv_step(r->h, k, st, k);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) { enif_free(st); return err(env, rc); }
    ERL_NIF_TERM list = enif_make_list(env, 0);
    for (unsigned i = k; i > 0; i--) list = enif_make_list_cell(env, hv_stats_term(env, &st[i - 1]), list);
    enif_free(st);
    return enif_make_tuple2(env, mk_atom(env, "ok"), list);
}

/* hv_views(Sim) -> {ok, Active, ActiveLen, Passive, PassiveLen}: u32-little
 * rows of 8 / 32 ids padded with 16#FFFFFFFF, and u8 lengths */
static ERL_NIF_TERM nif_hv_views(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    if (!get_res(env, argv[0], &r) || !r->hv_n) return enif_make_badarg(env);
    const size_t n = r->hv_n;
    ERL_NIF_TERM ta, tna, tp, tnp;
    unsigned char* a = enif_make_new_binary(env, n * 32, &ta);
    unsigned char* na = enif_make_new_binary(env, n, &tna);
    unsigned char* p = enif_make_new_binary(env, n * 128, &tp);
    unsigned char* np = enif_make_new_binary(env, n, &tnp);
    enif_mutex_lock(r->mu);
    int rc = psim_hv_get_views(r->h, (uint32_t*)a, na, (uint32_t*)p, np, n);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) return err(env, rc);
    ERL_NIF_TERM out[5] = {mk_atom(env, "ok"), ta, tna, tp, tnp};
    return enif_make_tuple_from_array(env, out, 5);
}

/* ---- Demers --------------------------------------------------------------- */

/* demers_setup(Sim, N, M, AePeriod, RumorMongering :: boolean()) -> ok */
static ERL_NIF_TERM nif_demers_setup(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned n, m, ae;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &n) || !enif_get_uint(env, argv[2], &m) ||
        !enif_get_uint(env, argv[3], &ae))
        return enif_make_badarg(env);
    const int rm = enif_is_identical(argv[4], mk_atom(env, "true"));
    enif_mutex_lock(r->mu);
    int rc = psim_demers_setup(r->h, n, m, ae, rm ? 1u : 0u);
    if (rc == PSIM_OK) rc = psim_demers_broadcast_all(r->h);
    if (rc == PSIM_OK) r->dm_n = n;
    enif_mutex_unlock(r->mu);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

/* demers_run(Sim, MaxRounds) -> {ok, Rounds, Seen :: <<u64-little per vertex>>} */
static ERL_NIF_TERM nif_demers_run(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned maxr;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &maxr)) return enif_make_badarg(env);
    ERL_NIF_TERM t;
    uint32_t ran = 0;
    enif_mutex_lock(r->mu);
    /* dm_n is read under the lock: a concurrent demers_setup may change it */
    const uint32_t nl = r->dm_n;
    if (!nl) {
        enif_mutex_unlock(r->mu);
        return enif_make_badarg(env);
    }
    unsigned char* seen = enif_make_new_binary(env, (size_t)nl * 8, &t);
    int rc = psim_demers_run(r->h, maxr, NULL, 0, &ran);
    if (rc == PSIM_OK) rc = psim_demers_get_seen(r->h, (uint64_t*)seen, nl);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) return err(env, rc);
    return enif_make_tuple3(env, mk_atom(env, "ok"), enif_make_uint(env, ran), t);
}

/* ---- vclock (dense 64-lane clocks, u32-little lanes, 0 = absent) ----------- */

/* vclock(Sim, Op, A, B) -> {ok, Binary} | {error, _}
 *   Op :: descends | dominates | equal              -> <<0|1 per clock>>
 *       | merge | glb | subtract_dots               -> Clocks   (B = clocks)
 *       | increment                                 -> Clocks   (B = u32 actor lanes)
 *       | get_counter                               -> <<u32 per clock>> (B = actor lanes)
 * partisan_vclock descends/2, dominates/2, equal/2, merge/1, glb/2,
 * subtract_dots/2, increment/2, get_counter/2 (src/partisan_vclock.erl:58-198) */
static ERL_NIF_TERM nif_vclock(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    ErlNifBinary a, b;
    const size_t cb = PSIM_VC_LANES * 4;
    if (!get_res(env, argv[0], &r) || !enif_inspect_binary(env, argv[2], &a) ||
        !enif_inspect_binary(env, argv[3], &b) || a.size % cb)
        return enif_make_badarg(env);
    const size_t n = a.size / cb;
    static const char* ops[] = {"descends", "dominates", "equal", "merge", "glb", "subtract_dots", "increment",
                                "get_counter"};
    int op = -1;
    for (int i = 0; i < 8 && op < 0; i++)
        if (enif_is_identical(argv[1], mk_atom(env, ops[i]))) op = i;
    if (op < 0) return enif_make_badarg(env);
    const int by_actor = op >= 6;
    if (by_actor ? b.size != n * 4 : b.size != a.size) return enif_make_badarg(env);
    const uint32_t* pa = (const uint32_t*)a.data;
    const uint32_t* pb = (const uint32_t*)b.data;
    ERL_NIF_TERM t;
    int rc = PSIM_OK;
    unsigned char* o = enif_make_new_binary(env, op <= 2 ? n : op == 7 ? n * 4 : a.size, &t);
    enif_mutex_lock(r->mu);
    switch (op) {
    case 0: rc = psim_vclock_descends(r->h, pa, pb, o, n); break;
    case 1: rc = psim_vclock_dominates(r->h, pa, pb, o, n); break;
    case 2: rc = psim_vclock_equal(r->h, pa, pb, o, n); break;
    case 3: rc = psim_vclock_merge(r->h, pa, pb, (uint32_t*)o, n); break;
    case 4: rc = psim_vclock_glb(r->h, pa, pb, (uint32_t*)o, n); break;
    case 5: rc = psim_vclock_subtract_dots(r->h, pa, pb, (uint32_t*)o, n); break;
    case 6: rc = psim_vclock_increment(r->h, pa, pb, (uint32_t*)o, n); break;
    default: rc = psim_vclock_get_counter(r->h, pa, pb, (uint32_t*)o, n); break;
    }
    enif_mutex_unlock(r->mu);
    return rc == PSIM_OK ? enif_make_tuple2(env, mk_atom(env, "ok"), t) : err(env, rc);
}

/* ---- shared helpers for the batch entry points ------------------------------ */

/* A u32 binary copied to an aligned buffer (binary data has no alignment
 * guarantee); *k = element count.  NULL on a bad size or no memory. */
static uint32_t* u32_copy(ErlNifEnv* env, ERL_NIF_TERM t, size_t* k) {
    ErlNifBinary b;
    if (!enif_inspect_binary(env, t, &b) || b.size % 4) return NULL;
    uint32_t* p = (uint32_t*)enif_alloc(b.size + 4);
    if (p) memcpy(p, b.data, b.size);
    *k = b.size / 4;
    return p;
}

typedef int (*pair_fn)(psim_handle*, const uint32_t*, const uint32_t*, size_t);
typedef int (*list_fn)(psim_handle*, const uint32_t*, size_t);

/* Fn(Sim, As :: <<u32>>, Bs :: <<u32>>) -> ok, for the batched join / leave calls */
static ERL_NIF_TERM pair_call(ErlNifEnv* env, const ERL_NIF_TERM argv[], pair_fn fn) {
    sim_res* r;
    size_t ka = 0, kb = 0;
    if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
    uint32_t* a = u32_copy(env, argv[1], &ka);
    uint32_t* b = u32_copy(env, argv[2], &kb);
    int rc = PSIM_EINVAL;
    if (a && b && ka == kb) {
        enif_mutex_lock(r->mu);
        rc = fn(r->h, a, b, ka);
        enif_mutex_unlock(r->mu);
    }
    if (a) enif_free(a);
    if (b) enif_free(b);
    if (!a || !b || ka != kb) return enif_make_badarg(env);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

static ERL_NIF_TERM list_call(ErlNifEnv* env, const ERL_NIF_TERM argv[], list_fn fn) {
    sim_res* r;
    size_t k = 0;
    if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
    uint32_t* a = u32_copy(env, argv[1], &k);
    if (!a) return enif_make_badarg(env);
    enif_mutex_lock(r->mu);
    int rc = fn(r->h, a, k);
    enif_mutex_unlock(r->mu);
    enif_free(a);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

static ERL_NIF_TERM kv_map(ErlNifEnv* env, const char* const* names, const uint64_t* vals, int n) {
    ERL_NIF_TERM keys[24], vs[24], m;
    for (int i = 0; i < n && i < 24; i++) {
        keys[i] = mk_atom(env, names[i]);
        vs[i] = enif_make_uint64(env, vals[i]);
    }
    enif_make_map_from_arrays(env, keys, vs, (size_t)n, &m);
    return m;
}

static ERL_NIF_TERM stats_list(ErlNifEnv* env, ERL_NIF_TERM* maps, unsigned k) {
    ERL_NIF_TERM list = enif_make_list(env, 0);
    for (unsigned i = k; i > 0; i--) list = enif_make_list_cell(env, maps[i - 1], list);
    return list;
}

static int get_rounds(ErlNifEnv* env, ERL_NIF_TERM t, unsigned* k) {
    return enif_get_uint(env, t, k) && *k >= 1 && *k <= 65536;
}

/* ---- SCAMP (partisan_scamp_v{1,2}_membership_strategy) ----------------------- */

/* scamp_setup(Sim, N, Version, C, PeriodicRounds) -> ok */
static ERL_NIF_TERM nif_scamp_setup(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned n, ver, c, per;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &n) || !enif_get_uint(env, argv[2], &ver) ||
        !enif_get_uint(env, argv[3], &c) || !enif_get_uint(env, argv[4], &per))
        return enif_make_badarg(env);
    enif_mutex_lock(r->mu);
    int rc = psim_scamp_setup(r->h, n, ver, c, per);
    if (rc == PSIM_OK) r->sc_n = n;
    enif_mutex_unlock(r->mu);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

/* scamp_join(Sim, Joiners, Contacts) / scamp_leave(Sim, Vs, Leaving) -> ok; scamp_crash(Sim, Vs) -> ok */
static ERL_NIF_TERM nif_scamp_join(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    return pair_call(env, argv, psim_scamp_join);
}
static ERL_NIF_TERM nif_scamp_leave(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    return pair_call(env, argv, psim_scamp_leave);
}
static ERL_NIF_TERM nif_scamp_crash(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    return list_call(env, argv, psim_scamp_crash);
}

static ERL_NIF_TERM scamp_stats_term(ErlNifEnv* env, const psim_scamp_stats* s) {
    static const char* const names[] = {"forward_subscription", "keep_subscription", "ping", "remove_subscription",
                                        "replace_subscription", "bootstrap_remove_subscription", "dropped",
                                        "processed", "draws", "stopped", "error", "pv_sum", "inview_sum", "resub",
                                        "kernel_us"};
    uint64_t v[15];
    for (int k = 1; k <= 6; k++) v[k - 1] = s->sent[k];
    v[6] = s->dropped; v[7] = s->processed; v[8] = s->draws; v[9] = s->stopped; v[10] = s->error;
    v[11] = s->pv_sum; v[12] = s->inview_sum; v[13] = s->resub; v[14] = (uint64_t)(s->kernel_ms * 1000.0);
    return kv_map(env, names, v, 15);
}

/* scamp_step(Sim, Rounds) -> {ok, [StatsMap]} */
static ERL_NIF_TERM nif_scamp_step(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned k;
    if (!get_res(env, argv[0], &r) || !get_rounds(env, argv[1], &k)) return enif_make_badarg(env);
    psim_scamp_stats* st = (psim_scamp_stats*)enif_alloc(k * sizeof(psim_scamp_stats));
    ERL_NIF_TERM* maps = (ERL_NIF_TERM*)enif_alloc(k * sizeof(ERL_NIF_TERM));
    if (!st || !maps) {
        if (st) enif_free(st);
        if (maps) enif_free(maps);
        return err(env, PSIM_ENOMEM);
    }
    enif_mutex_lock(r->mu);
    int rc = psim_scamp_step(r->h, k, st, k);
    enif_mutex_unlock(r->mu);
    ERL_NIF_TERM out = err(env, rc);
    if (rc == PSIM_OK) {
        for (unsigned i = 0; i < k; i++) maps[i] = scamp_stats_term(env, &st[i]);
        out = enif_make_tuple2(env, mk_atom(env, "ok"), stats_list(env, maps, k));
    }
    enif_free(st);
    enif_free(maps);
    return out;
}

/* ---- membership messages on the wire ------------------
 * A SCAMP message as the pluggable manager carries it
 * (partisan_pluggable_peer_service_manager.erl:1396-1407):
 *   {Src, Dst, Seq, {membership_strategy, Msg}}
 * Msg in the strategy's own shape (partisan_scamp_v2_membership_strategy.erl
 * :101-347): {forward_subscription, A} | {keep_subscription, A} | {ping, A} |
 * {remove_subscription, A} | {replace_subscription, A, B} |
 * {bootstrap_remove_subscription, A}; A, B, Src, Dst are vertex ids (the
 * Erlang cluster maps them to node specs), Seq the sender's emission index. */
static const char* const kScTag[] = {"", "forward_subscription", "keep_subscription", "ping",
                                     "remove_subscription", "replace_subscription", "bootstrap_remove_subscription"};

static ERL_NIF_TERM sc_msg_term(ErlNifEnv* env, const psim_scamp_msg* m) {
    ERL_NIF_TERM body = m->type == PSIM_SC_REPLACE
                            ? enif_make_tuple3(env, mk_atom(env, kScTag[m->type]), enif_make_uint(env, m->a),
                                               enif_make_uint(env, m->b))
                            : enif_make_tuple2(env, mk_atom(env, kScTag[m->type]), enif_make_uint(env, m->a));
    return enif_make_tuple4(env, enif_make_uint(env, m->src), enif_make_uint(env, m->dst), enif_make_uint(env, m->seq),
                            enif_make_tuple2(env, mk_atom(env, "membership_strategy"), body));
}

static ERL_NIF_TERM sc_msg_list(ErlNifEnv* env, const psim_scamp_msg* m, size_t k) {
    ERL_NIF_TERM list = enif_make_list(env, 0);
    for (size_t i = k; i-- > 0;) list = enif_make_list_cell(env, sc_msg_term(env, &m[i]), list);
    return list;
}

/* the inverse of sc_msg_term; 0 on a malformed term */
static int sc_msg_parse(ErlNifEnv* env, ERL_NIF_TERM t, psim_scamp_msg* m) {
    int n, nb, nm;
    const ERL_NIF_TERM *f, *b, *w;
    unsigned src, dst, seq, x, y = 0;
    if (!enif_get_tuple(env, t, &n, &f) || n != 4 || !enif_get_uint(env, f[0], &src) ||
        !enif_get_uint(env, f[1], &dst) || !enif_get_uint(env, f[2], &seq) || !enif_get_tuple(env, f[3], &nm, &w) ||
        nm != 2 || !enif_is_identical(w[0], mk_atom(env, "membership_strategy")) || !enif_get_tuple(env, w[1], &nb, &b) ||
        nb < 2 || !enif_get_uint(env, b[1], &x))
        return 0;
    for (uint32_t k = PSIM_SC_FORWARD; k <= PSIM_SC_BOOTSTRAP_REMOVE; k++) {
        if (!enif_is_identical(b[0], mk_atom(env, kScTag[k]))) continue;
        if (nb != (k == PSIM_SC_REPLACE ? 3 : 2)) return 0;
        if (k == PSIM_SC_REPLACE && !enif_get_uint(env, b[2], &y)) return 0;
        m->type = k; m->src = src; m->dst = dst; m->seq = seq; m->a = x; m->b = y;
        return 1;
    }
    return 0;
}

/* scamp_messages(Sim) -> {ok, [{Src, Dst, Seq, {membership_strategy, Msg}}]}:
 * the messages the next round delivers, in handling order (psim_scamp_messages) */
static ERL_NIF_TERM nif_scamp_messages(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
    size_t k = 0;
    enif_mutex_lock(r->mu);
    int rc = psim_scamp_messages(r->h, NULL, 0, &k);
    psim_scamp_msg* m = rc == PSIM_OK ? (psim_scamp_msg*)enif_alloc((k ? k : 1) * sizeof(psim_scamp_msg)) : NULL;
    if (rc == PSIM_OK) rc = m ? psim_scamp_messages(r->h, m, k, &k) : PSIM_ENOMEM;
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) { enif_free(m); return err(env, rc); }
    ERL_NIF_TERM list = sc_msg_list(env, m, k);
    enif_free(m);
    return enif_make_tuple2(env, mk_atom(env, "ok"), list);
}

/* scamp_messages_from(Sim, Src) -> {ok, [...]}: scamp_messages/1 keeping only
 * Src's messages, filtered before any term is built (the Erlang cluster's
 * outgoing/1 renders one node's sends: ADVICE r4) */
static ERL_NIF_TERM nif_scamp_messages_from(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned src;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &src)) return enif_make_badarg(env);
    size_t k = 0;
    enif_mutex_lock(r->mu);
    int rc = psim_scamp_messages(r->h, NULL, 0, &k);
    psim_scamp_msg* m = rc == PSIM_OK ? (psim_scamp_msg*)enif_alloc((k ? k : 1) * sizeof(psim_scamp_msg)) : NULL;
    if (rc == PSIM_OK) rc = m ? psim_scamp_messages(r->h, m, k, &k) : PSIM_ENOMEM;
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) { enif_free(m); return err(env, rc); }
    size_t j = 0;
    for (size_t i = 0; i < k; i++)
        if (m[i].src == src) m[j++] = m[i];
    ERL_NIF_TERM list = sc_msg_list(env, m, j);
    enif_free(m);
    return enif_make_tuple2(env, mk_atom(env, "ok"), list);
}

/* scamp_take(Sim, Dst) -> {ok, [Message]}: takes Dst's messages off the wire
 * (psim_scamp_take) -- what a manager hands to the node they are for */
static ERL_NIF_TERM nif_scamp_take(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned dst;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &dst)) return enif_make_badarg(env);
    size_t k = 0;
    enif_mutex_lock(r->mu);
    int rc = psim_scamp_messages(r->h, NULL, 0, &k);          /* an upper bound for Dst's share */
    psim_scamp_msg* m = rc == PSIM_OK ? (psim_scamp_msg*)enif_alloc((k ? k : 1) * sizeof(psim_scamp_msg)) : NULL;
    if (rc == PSIM_OK) rc = m ? psim_scamp_take(r->h, dst, m, k, &k) : PSIM_ENOMEM;
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) { enif_free(m); return err(env, rc); }
    ERL_NIF_TERM list = sc_msg_list(env, m, k);
    enif_free(m);
    return enif_make_tuple2(env, mk_atom(env, "ok"), list);
}

/* scamp_put(Sim, [Message]) -> ok: messages onto the wire for the next round
 * (psim_scamp_put) -- what handle_message/2 of a simulated node received */
static ERL_NIF_TERM nif_scamp_put(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
    size_t k = 0, cap = 16;
    psim_scamp_msg* m = (psim_scamp_msg*)enif_alloc(cap * sizeof(psim_scamp_msg));
    ERL_NIF_TERM list = argv[1], head, tail;
    while (m && enif_get_list_cell(env, list, &head, &tail)) {
        if (k == cap) {
            psim_scamp_msg* g = (psim_scamp_msg*)enif_alloc(2 * cap * sizeof(psim_scamp_msg));
            if (g) memcpy(g, m, cap * sizeof(psim_scamp_msg));
            enif_free(m);
            m = g;
            cap *= 2;
            if (!m) break;
        }
        if (!sc_msg_parse(env, head, &m[k])) { enif_free(m); return enif_make_badarg(env); }
        k++;
        list = tail;
    }
    if (!m) return err(env, PSIM_ENOMEM);
    enif_mutex_lock(r->mu);
    int rc = psim_scamp_put(r->h, m, k);
    enif_mutex_unlock(r->mu);
    enif_free(m);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

/* scamp_views(Sim) -> {ok, PartialViews, PvLens, InViews, IvLens}: u32 rows of
 * PSIM_SCAMP_PV_CAP / PSIM_SCAMP_IV_CAP ids in the reference's list order */
static ERL_NIF_TERM nif_scamp_views(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    if (!get_res(env, argv[0], &r) || !r->sc_n) return enif_make_badarg(env);
    const size_t n = r->sc_n;
    ERL_NIF_TERM tp, tnp, ti, tni;
    unsigned char* pv = enif_make_new_binary(env, n * PSIM_SCAMP_PV_CAP * 4, &tp);
    unsigned char* npv = enif_make_new_binary(env, n * 4, &tnp);
    unsigned char* iv = enif_make_new_binary(env, n * PSIM_SCAMP_IV_CAP * 4, &ti);
    unsigned char* niv = enif_make_new_binary(env, n * 4, &tni);
    uint32_t* a = (uint32_t*)enif_alloc(n * (PSIM_SCAMP_PV_CAP + PSIM_SCAMP_IV_CAP + 2) * 4);
    if (!pv || !npv || !iv || !niv || !a) {
        if (a) enif_free(a);
        return err(env, PSIM_ENOMEM);
    }
    uint32_t *ap = a, *anp = ap + n * PSIM_SCAMP_PV_CAP, *ai = anp + n, *ani = ai + n * PSIM_SCAMP_IV_CAP;
    enif_mutex_lock(r->mu);
    int rc = psim_scamp_get_views(r->h, ap, anp, ai, ani, n);
    enif_mutex_unlock(r->mu);
    if (rc == PSIM_OK) {
        memcpy(pv, ap, n * PSIM_SCAMP_PV_CAP * 4);
        memcpy(npv, anp, n * 4);
        memcpy(iv, ai, n * PSIM_SCAMP_IV_CAP * 4);
        memcpy(niv, ani, n * 4);
    }
    enif_free(a);
    if (rc != PSIM_OK) return err(env, rc);
    ERL_NIF_TERM out[5] = {mk_atom(env, "ok"), tp, tnp, ti, tni};
    return enif_make_tuple_from_array(env, out, 5);
}

/* ---- full membership (partisan_full_membership_strategy) ---------------------- */

/* fm_setup(Sim, N, PeriodicRounds, MaxTokens) -> ok */
static ERL_NIF_TERM nif_fm_setup(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned n, per, tok;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &n) || !enif_get_uint(env, argv[2], &per) ||
        !enif_get_uint(env, argv[3], &tok))
        return enif_make_badarg(env);
    enif_mutex_lock(r->mu);
    int rc = psim_fm_setup(r->h, n, per, tok);
    if (rc == PSIM_OK) { r->fm_n = n; r->fm_words = (tok + 63) / 64; }
    enif_mutex_unlock(r->mu);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}
static ERL_NIF_TERM nif_fm_join(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    return pair_call(env, argv, psim_fm_join);
}
static ERL_NIF_TERM nif_fm_leave(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    return pair_call(env, argv, psim_fm_leave);
}

/* fm_step(Sim, Rounds) -> {ok, [StatsMap]} */
static ERL_NIF_TERM nif_fm_step(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned k;
    if (!get_res(env, argv[0], &r) || !get_rounds(env, argv[1], &k)) return enif_make_badarg(env);
    psim_fm_stats* st = (psim_fm_stats*)enif_alloc(k * sizeof(psim_fm_stats));
    ERL_NIF_TERM* maps = (ERL_NIF_TERM*)enif_alloc(k * sizeof(ERL_NIF_TERM));
    if (!st || !maps) {
        if (st) enif_free(st);
        if (maps) enif_free(maps);
        return err(env, PSIM_ENOMEM);
    }
    enif_mutex_lock(r->mu);
    int rc = psim_fm_step(r->h, k, st, k);
    enif_mutex_unlock(r->mu);
    ERL_NIF_TERM out = err(env, rc);
    if (rc == PSIM_OK) {
        static const char* const names[] = {"sent", "processed", "merges", "updates", "inflight", "member_sum",
                                            "kernel_us"};
        for (unsigned i = 0; i < k; i++) {
            const uint64_t v[7] = {st[i].sent, st[i].processed, st[i].merges, st[i].updates, st[i].inflight,
                                   st[i].member_sum, (uint64_t)(st[i].kernel_ms * 1000.0)};
            maps[i] = kv_map(env, names, v, 7);
        }
        out = enif_make_tuple2(env, mk_atom(env, "ok"), stats_list(env, maps, k));
    }
    enif_free(st);
    enif_free(maps);
    return out;
}

/* fm_state(Sim) -> {ok, Known, Removed, Alive}: per node the u64 token
 * bitmaps of its state_orset (known / removed) and one alive byte */
static ERL_NIF_TERM nif_fm_state(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    if (!get_res(env, argv[0], &r) || !r->fm_n) return enif_make_badarg(env);
    const size_t n = r->fm_n, w = r->fm_words;
    ERL_NIF_TERM tk, trm, ta;
    unsigned char* kb = enif_make_new_binary(env, n * w * 8, &tk);
    unsigned char* rb = enif_make_new_binary(env, n * w * 8, &trm);
    unsigned char* ab = enif_make_new_binary(env, n, &ta);
    uint64_t* tmp = (uint64_t*)enif_alloc(2 * n * w * 8 + 8);
    if (!kb || !rb || !ab || !tmp) {
        if (tmp) enif_free(tmp);
        return err(env, PSIM_ENOMEM);
    }
    enif_mutex_lock(r->mu);
    int rc = psim_fm_get_state(r->h, tmp, tmp + n * w, ab, n, w);
    enif_mutex_unlock(r->mu);
    if (rc == PSIM_OK) {
        memcpy(kb, tmp, n * w * 8);
        memcpy(rb, tmp + n * w, n * w * 8);
    }
    enif_free(tmp);
    if (rc != PSIM_OK) return err(env, rc);
    return enif_make_tuple4(env, mk_atom(env, "ok"), tk, trm, ta);
}

/* fm_tokens(Sim) -> {ok, TokenNodes :: <<u32 per token>>, Used}: the node each
 * state_orset token adds (token v = node v's init/1 add; a self-leave takes a
 * fresh one) */
static ERL_NIF_TERM nif_fm_tokens(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    if (!get_res(env, argv[0], &r) || !r->fm_n) return enif_make_badarg(env);
    const size_t ntok = (size_t)r->fm_words * 64;
    ERL_NIF_TERM tt;
    unsigned char* tb = enif_make_new_binary(env, ntok * 4, &tt);
    uint32_t* tmp = (uint32_t*)enif_alloc(ntok * 4 + 4);
    uint32_t used = 0;
    if (!tb || !tmp) {
        if (tmp) enif_free(tmp);
        return err(env, PSIM_ENOMEM);
    }
    enif_mutex_lock(r->mu);
    int rc = psim_fm_tokens(r->h, tmp, ntok, &used);
    enif_mutex_unlock(r->mu);
    if (rc == PSIM_OK) memcpy(tb, tmp, ntok * 4);
    enif_free(tmp);
    if (rc != PSIM_OK) return err(env, rc);
    return enif_make_tuple3(env, mk_atom(env, "ok"), tt, enif_make_uint(env, used));
}

/* ---- full membership on the wire ---------------------------- */

/* [{Src, Dst, Seq, Known, Removed}]: Known / Removed the message's state_orset
 * as token bitmaps (u64 words, little endian; the cluster module renders the
 * #full_v1{} term) */
static ERL_NIF_TERM fm_msg_list(ErlNifEnv* env, const psim_fm_msg* m, const uint64_t* k, const uint64_t* rm, size_t c,
                                size_t w) {
    ERL_NIF_TERM list = enif_make_list(env, 0);
    for (size_t i = c; i > 0; i--) {
        ERL_NIF_TERM tk, tr;
        unsigned char* kb = enif_make_new_binary(env, w * 8, &tk);
        unsigned char* rb = enif_make_new_binary(env, w * 8, &tr);
        if (kb) memcpy(kb, k + (i - 1) * w, w * 8);
        if (rb) memcpy(rb, rm + (i - 1) * w, w * 8);
        const psim_fm_msg* x = &m[i - 1];
        ERL_NIF_TERM t[5] = {enif_make_uint(env, x->src), enif_make_uint(env, x->dst), enif_make_uint(env, x->seq), tk, tr};
        list = enif_make_list_cell(env, enif_make_tuple_from_array(env, t, 5), list);
    }
    return list;
}

/* fm_messages(Sim) / fm_take(Sim, Dst) -> {ok, [{Src, Dst, Seq, Known, Removed}]}
 * in handling order (psim_fm_messages / psim_fm_take) */
/* take: 0 every message, 1 take Dst's, 2 every message from Src (argv[1]),
 * filtered before the terms are built (fm_messages_from/2) */
static ERL_NIF_TERM fm_wire(ErlNifEnv* env, const ERL_NIF_TERM argv[], int take) {
    sim_res* r;
    unsigned dst = 0;
    if (!get_res(env, argv[0], &r) || !r->fm_n || (take && !enif_get_uint(env, argv[1], &dst)))
        return enif_make_badarg(env);
    const size_t w = r->fm_words;
    size_t k = 0;
    enif_mutex_lock(r->mu);
    int rc = psim_fm_messages(r->h, NULL, NULL, NULL, 0, w, &k);     /* an upper bound for Dst's share */
    const size_t cap = k ? k : 1;
    psim_fm_msg* m = rc == PSIM_OK ? (psim_fm_msg*)enif_alloc(cap * sizeof(psim_fm_msg)) : NULL;
    uint64_t* kw = rc == PSIM_OK ? (uint64_t*)enif_alloc(2 * cap * w * 8) : NULL;
    if (rc == PSIM_OK && (!m || !kw)) rc = PSIM_ENOMEM;
    if (rc == PSIM_OK)
        rc = take == 1 ? psim_fm_take(r->h, dst, m, kw, kw + cap * w, cap, w, &k)
                       : psim_fm_messages(r->h, m, kw, kw + cap * w, cap, w, &k);
    enif_mutex_unlock(r->mu);
    if (rc == PSIM_OK && take == 2) {      /* keep Src = argv[1]'s messages, in order */
        size_t j = 0;
        for (size_t i = 0; i < k && i < cap; i++) {
            if (m[i].src != dst) continue;
            if (j != i) {
                m[j] = m[i];
                memmove(kw + j * w, kw + i * w, w * 8);
                memmove(kw + cap * w + j * w, kw + cap * w + i * w, w * 8);
            }
            j++;
        }
        k = j;
    }
    ERL_NIF_TERM out = rc == PSIM_OK ? enif_make_tuple2(env, mk_atom(env, "ok"),
                                                        fm_msg_list(env, m, kw, kw + cap * w, k < cap ? k : cap, w))
                                     : err(env, rc);
    if (m) enif_free(m);
    if (kw) enif_free(kw);
    return out;
}
static ERL_NIF_TERM nif_fm_messages(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    return fm_wire(env, argv, 0);
}
static ERL_NIF_TERM nif_fm_take(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    return fm_wire(env, argv, 1);
}
static ERL_NIF_TERM nif_fm_messages_from(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    return fm_wire(env, argv, 2);
}

/* fm_put(Sim, [{Src, Dst, Seq, Known, Removed}]) -> ok: what a simulated node's
 * manager received (handle_message/2) onto the wire for the next round */
static ERL_NIF_TERM nif_fm_put(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned len;
    if (!get_res(env, argv[0], &r) || !r->fm_n || !enif_get_list_length(env, argv[1], &len))
        return enif_make_badarg(env);
    const size_t w = r->fm_words, cap = len ? len : 1;
    psim_fm_msg* m = (psim_fm_msg*)enif_alloc(cap * sizeof(psim_fm_msg));
    uint64_t* kw = (uint64_t*)enif_alloc(2 * cap * w * 8);
    if (!m || !kw) {
        if (m) enif_free(m);
        if (kw) enif_free(kw);
        return err(env, PSIM_ENOMEM);
    }
    ERL_NIF_TERM list = argv[1], head, tail;
    size_t i = 0;
    while (enif_get_list_cell(env, list, &head, &tail)) {
        const ERL_NIF_TERM* t;
        int ar;
        ErlNifBinary kb, rb;
        unsigned src, dst, seq;
        if (!enif_get_tuple(env, head, &ar, &t) || ar != 5 || !enif_get_uint(env, t[0], &src) ||
            !enif_get_uint(env, t[1], &dst) || !enif_get_uint(env, t[2], &seq) ||
            !enif_inspect_binary(env, t[3], &kb) || !enif_inspect_binary(env, t[4], &rb) || kb.size != w * 8 ||
            rb.size != w * 8) {
            enif_free(m);
            enif_free(kw);
            return enif_make_badarg(env);
        }
        m[i].src = src; m[i].dst = dst; m[i].seq = seq; m[i].reserved = 0;
        memcpy(kw + i * w, kb.data, w * 8);
        memcpy(kw + cap * w + i * w, rb.data, w * 8);
        i++;
        list = tail;
    }
    enif_mutex_lock(r->mu);
    int rc = psim_fm_put(r->h, m, kw, kw + cap * w, i, w);
    enif_mutex_unlock(r->mu);
    enif_free(m);
    enif_free(kw);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

/* ---- C3: Plumtree repair over churning SCAMP v2 ------------------------------- */

/* c3_setup(Sim, N, C, PeriodicRounds) -> ok */
static ERL_NIF_TERM nif_c3_setup(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned n, c, per;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &n) || !enif_get_uint(env, argv[2], &c) ||
        !enif_get_uint(env, argv[3], &per))
        return enif_make_badarg(env);
    enif_mutex_lock(r->mu);
    int rc = psim_c3_setup(r->h, n, c, per);
    if (rc == PSIM_OK) r->sc_n = n;
    enif_mutex_unlock(r->mu);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}
static ERL_NIF_TERM nif_c3_join(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    return pair_call(env, argv, psim_c3_join);
}
static ERL_NIF_TERM nif_c3_crash(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    return list_call(env, argv, psim_c3_crash);
}

/* c3_heartbeat(Sim, Root) -> {ok, Monotonic} */
static ERL_NIF_TERM nif_c3_heartbeat(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned root;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &root)) return enif_make_badarg(env);
    uint32_t mono = 0;
    enif_mutex_lock(r->mu);
    int rc = psim_c3_heartbeat(r->h, root, &mono);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) return err(env, rc);
    return enif_make_tuple2(env, mk_atom(env, "ok"), enif_make_uint(env, mono));
}

/* {ok, [{PlumtreeMap, ScampMap}]} of k C3 rounds; maps: k scratch terms */
static ERL_NIF_TERM c3_stats_ok(ErlNifEnv* env, const psim_c3_stats* st, ERL_NIF_TERM* maps, unsigned k) {
    static const char* const names[] = {"broadcast", "prune", "i_have", "ignored_i_have", "graft", "pt_dropped",
                                        "delivered_new", "updates", "delivered_live", "live", "outstanding_live",
                                        "pt_kernel_us"};
    for (unsigned i = 0; i < k; i++) {
        const psim_c3_stats* x = &st[i];
        const uint64_t v[12] = {x->pt_sent[1], x->pt_sent[2], x->pt_sent[3], x->pt_sent[4], x->pt_sent[5],
                                x->pt_dropped, x->delivered_new, x->updates, x->delivered_live, x->live,
                                x->outstanding_live, (uint64_t)(x->pt_kernel_ms * 1000.0)};
        maps[i] = enif_make_tuple2(env, kv_map(env, names, v, 12), scamp_stats_term(env, &x->scamp));
    }
    return enif_make_tuple2(env, mk_atom(env, "ok"), stats_list(env, maps, k));
}

/* c3_run(Sim, CrashOff, CrashV, JoinOff, JoinV, JoinC, HbEvery, Root) -> {ok, [Stats]}
 * (psim_c3_run: R rounds of churn in one call; the offsets are <<u32>> of R + 1
 * entries, the lists <<u32>> as in c3_crash / c3_join; Stats as c3_step's) */
static ERL_NIF_TERM nif_c3_run(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned hb, root;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[6], &hb) || !enif_get_uint(env, argv[7], &root))
        return enif_make_badarg(env);
    size_t n[5] = {0, 0, 0, 0, 0};
    uint32_t* b[5];
    int ok = 1;
    for (int i = 0; i < 5; i++) {
        b[i] = u32_copy(env, argv[1 + i], &n[i]);
        ok &= b[i] != NULL;
    }
    const size_t k = n[0] ? n[0] - 1 : 0;
    /* offsets index the lists from 0 (psim_c3_run checks they never go backwards) */
    ok = ok && n[0] >= 1 && n[2] == n[0] && n[4] == n[3] && k <= 1000000 && b[0][k] <= n[1] && b[2][k] <= n[3];
    psim_c3_stats* st = ok && k ? (psim_c3_stats*)enif_alloc(k * sizeof(psim_c3_stats)) : NULL;
    ERL_NIF_TERM* maps = ok && k ? (ERL_NIF_TERM*)enif_alloc(k * sizeof(ERL_NIF_TERM)) : NULL;
    ERL_NIF_TERM out;
    if (!ok) {
        out = enif_make_badarg(env);
    } else if (k && (!st || !maps)) {
        out = err(env, PSIM_ENOMEM);
    } else {
        enif_mutex_lock(r->mu);
        int rc = psim_c3_run(r->h, (uint32_t)k, b[0], b[1], b[2], b[3], b[4], hb, root, st, k);
        enif_mutex_unlock(r->mu);
        out = rc == PSIM_OK ? c3_stats_ok(env, st, maps, (unsigned)k) : err(env, rc);
    }
    for (int i = 0; i < 5; i++)
        if (b[i]) enif_free(b[i]);
    if (st) enif_free(st);
    if (maps) enif_free(maps);
    return out;
}

/* c3_step(Sim, Rounds) -> {ok, [StatsMap]} (both protocols' counters) */
static ERL_NIF_TERM nif_c3_step(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned k;
    if (!get_res(env, argv[0], &r) || !get_rounds(env, argv[1], &k)) return enif_make_badarg(env);
    psim_c3_stats* st = (psim_c3_stats*)enif_alloc(k * sizeof(psim_c3_stats));
    ERL_NIF_TERM* maps = (ERL_NIF_TERM*)enif_alloc(k * sizeof(ERL_NIF_TERM));
    if (!st || !maps) {
        if (st) enif_free(st);
        if (maps) enif_free(maps);
        return err(env, PSIM_ENOMEM);
    }
    enif_mutex_lock(r->mu);
    int rc = psim_c3_step(r->h, k, st, k);
    enif_mutex_unlock(r->mu);
    ERL_NIF_TERM out = rc == PSIM_OK ? c3_stats_ok(env, st, maps, k) : err(env, rc);
    enif_free(st);
    enif_free(maps);
    return out;
}

/* ---- causal delivery (partisan_causality_backend) ----------------------------- */

/* causal_setup(Sim, N, M, Period, DMax, Redeliver) -> ok */
static ERL_NIF_TERM nif_causal_setup(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned n, m, per, dmax, red;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &n) || !enif_get_uint(env, argv[2], &m) ||
        !enif_get_uint(env, argv[3], &per) || !enif_get_uint(env, argv[4], &dmax) || !enif_get_uint(env, argv[5], &red))
        return enif_make_badarg(env);
    enif_mutex_lock(r->mu);
    int rc = psim_causal_setup(r->h, n, m, per, dmax, red);
    if (rc == PSIM_OK) r->cs_n = n;
    enif_mutex_unlock(r->mu);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

/* causal_step(Sim, Rounds) -> {ok, [StatsMap]} */
static ERL_NIF_TERM nif_causal_step(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned k;
    if (!get_res(env, argv[0], &r) || !get_rounds(env, argv[1], &k)) return enif_make_badarg(env);
    psim_causal_stats* st = (psim_causal_stats*)enif_alloc(k * sizeof(psim_causal_stats));
    ERL_NIF_TERM* maps = (ERL_NIF_TERM*)enif_alloc(k * sizeof(ERL_NIF_TERM));
    if (!st || !maps) {
        if (st) enif_free(st);
        if (maps) enif_free(maps);
        return err(env, PSIM_ENOMEM);
    }
    enif_mutex_lock(r->mu);
    int rc = psim_causal_step(r->h, k, st, k);
    enif_mutex_unlock(r->mu);
    ERL_NIF_TERM out = err(env, rc);
    if (rc == PSIM_OK) {
        static const char* const names[] = {"emitted", "received", "delivered", "checks", "buffered", "kernel_us"};
        for (unsigned i = 0; i < k; i++) {
            const uint64_t v[6] = {st[i].emitted, st[i].received, st[i].delivered, st[i].checks, st[i].buffered,
                                   (uint64_t)(st[i].kernel_ms * 1000.0)};
            maps[i] = kv_map(env, names, v, 6);
        }
        out = enif_make_tuple2(env, mk_atom(env, "ok"), stats_list(env, maps, k));
    }
    enif_free(st);
    enif_free(maps);
    return out;
}

/* causal_clocks(Sim) -> {ok, Lanes :: <<u32 x 64 per vertex>>, Self :: <<u32 per vertex>>} */
static ERL_NIF_TERM nif_causal_clocks(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    if (!get_res(env, argv[0], &r) || !r->cs_n) return enif_make_badarg(env);
    const size_t n = r->cs_n;
    ERL_NIF_TERM tl, ts;
    unsigned char* lb = enif_make_new_binary(env, n * PSIM_VC_LANES * 4, &tl);
    unsigned char* sb = enif_make_new_binary(env, n * 4, &ts);
    uint32_t* tmp = (uint32_t*)enif_alloc(n * (PSIM_VC_LANES + 1) * 4);
    if (!lb || !sb || !tmp) {
        if (tmp) enif_free(tmp);
        return err(env, PSIM_ENOMEM);
    }
    enif_mutex_lock(r->mu);
    int rc = psim_causal_get_clocks(r->h, tmp, tmp + n * PSIM_VC_LANES, n);
    enif_mutex_unlock(r->mu);
    if (rc == PSIM_OK) {
        memcpy(lb, tmp, n * PSIM_VC_LANES * 4);
        memcpy(sb, tmp + n * PSIM_VC_LANES, n * 4);
    }
    enif_free(tmp);
    if (rc != PSIM_OK) return err(env, rc);
    return enif_make_tuple3(env, mk_atom(env, "ok"), tl, ts);
}

/* ---- vertex sharding with the exchange inside the library (RCCL) ------------- */

/* rccl_unique_id() -> {ok, <<_:1024>>}: on one rank; ship it to the others */
static ERL_NIF_TERM nif_rccl_unique_id(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    (void)argv;
    ERL_NIF_TERM t;
    unsigned char* b = enif_make_new_binary(env, PSIM_RCCL_ID_BYTES, &t);
    if (!b) return err(env, PSIM_ENOMEM);
    int rc = psim_rccl_unique_id(b);
    return rc == PSIM_OK ? enif_make_tuple2(env, mk_atom(env, "ok"), t) : err(env, rc);
}

/* shard_init_rccl(Sim, Rank, World, UniqueId) -> ok   (before load_csr) */
static ERL_NIF_TERM nif_shard_init_rccl(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned rank, world;
    ErlNifBinary id;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &rank) || !enif_get_uint(env, argv[2], &world) ||
        !enif_inspect_binary(env, argv[3], &id) || id.size != PSIM_RCCL_ID_BYTES)
        return enif_make_badarg(env);
    enif_mutex_lock(r->mu);
    int rc = psim_shard_init_rccl(r->h, (int)rank, (int)world, id.data);
    enif_mutex_unlock(r->mu);
    return rc == PSIM_OK ? mk_atom(env, "ok") : err(env, rc);
}

/* demers_shard_setup(Sim, N, M, AePeriod, RumorMongering :: boolean(), Rank, World) -> {ok, VLo, NLocal}:
 * this rank's vertex range of a C4 epidemic sharded over World ranks (after
 * shard_init_rccl: the exchange runs on the handle's RCCL communicator) */
static ERL_NIF_TERM nif_demers_shard_setup(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned n, m, ae, rank, world;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &n) || !enif_get_uint(env, argv[2], &m) ||
        !enif_get_uint(env, argv[3], &ae) || !enif_get_uint(env, argv[5], &rank) || !enif_get_uint(env, argv[6], &world))
        return enif_make_badarg(env);
    const int rm = enif_is_identical(argv[4], mk_atom(env, "true"));
    uint32_t vlo = 0, nl = 0;
    enif_mutex_lock(r->mu);
    int rc = psim_demers_shard_setup(r->h, n, m, ae, rm ? 1u : 0u, (int)rank, (int)world, NULL);
    if (rc == PSIM_OK) rc = psim_demers_shard_info(r->h, &vlo, &nl, NULL);
    if (rc == PSIM_OK) r->dm_n = nl;
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) return err(env, rc);
    return enif_make_tuple3(env, mk_atom(env, "ok"), enif_make_uint(env, vlo), enif_make_uint(env, nl));
}

/* demers_shard_run(Sim, MaxRounds) -> {ok, Rounds, Seen :: <<u64-little per local vertex>>}:
 * every rumor from its origin, rounds until every vertex of every shard holds
 * every rumor (collective: psim_demers_shard_broadcast_x + psim_demers_shard_run) */
static ERL_NIF_TERM nif_demers_shard_run(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned maxr;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &maxr)) return enif_make_badarg(env);
    ERL_NIF_TERM t;
    uint32_t ran = 0;
    enif_mutex_lock(r->mu);
    /* dm_n read once under the lock: the binary and get_seen agree */
    const uint32_t nl = r->dm_n;
    unsigned char* seen = enif_make_new_binary(env, (size_t)nl * 8, &t);
    int rc = psim_demers_shard_broadcast_x(r->h);
    if (rc == PSIM_OK) rc = psim_demers_shard_run(r->h, maxr, NULL, 0, &ran);
    if (rc == PSIM_OK && nl) rc = psim_demers_shard_get_seen(r->h, (uint64_t*)seen, nl);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) return err(env, rc);
    return enif_make_tuple3(env, mk_atom(env, "ok"), enif_make_uint(env, ran), t);
}

/* causal_shard_setup(Sim, N, M, Period, DMax, Redeliver, Rank, World) -> {ok, VLo, NLocal}
 * (after shard_init_rccl) */
static ERL_NIF_TERM nif_causal_shard_setup(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned n, m, per, dmax, red, rank, world;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &n) || !enif_get_uint(env, argv[2], &m) ||
        !enif_get_uint(env, argv[3], &per) || !enif_get_uint(env, argv[4], &dmax) ||
        !enif_get_uint(env, argv[5], &red) || !enif_get_uint(env, argv[6], &rank) || !enif_get_uint(env, argv[7], &world))
        return enif_make_badarg(env);
    uint32_t vlo = 0, nl = 0;
    enif_mutex_lock(r->mu);
    int rc = psim_causal_shard_setup(r->h, n, m, per, dmax, red, (int)rank, (int)world);
    if (rc == PSIM_OK) rc = psim_causal_shard_info(r->h, &vlo, &nl);
    if (rc == PSIM_OK) r->cs_n = nl;
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) return err(env, rc);
    return enif_make_tuple3(env, mk_atom(env, "ok"), enif_make_uint(env, vlo), enif_make_uint(env, nl));
}

/* causal_shard_step(Sim, Rounds) -> {ok, [StatsMap]}   (collective, global counters) */
static ERL_NIF_TERM nif_causal_shard_step(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned k;
    if (!get_res(env, argv[0], &r) || !get_rounds(env, argv[1], &k)) return enif_make_badarg(env);
    psim_causal_stats* st = (psim_causal_stats*)enif_alloc(k * sizeof(psim_causal_stats));
    ERL_NIF_TERM* maps = (ERL_NIF_TERM*)enif_alloc(k * sizeof(ERL_NIF_TERM));
    if (!st || !maps) {
        if (st) enif_free(st);
        if (maps) enif_free(maps);
        return err(env, PSIM_ENOMEM);
    }
    enif_mutex_lock(r->mu);
    int rc = psim_causal_shard_step(r->h, k, st, k);
    enif_mutex_unlock(r->mu);
    ERL_NIF_TERM out = err(env, rc);
    if (rc == PSIM_OK) {
        static const char* const names[] = {"emitted", "received", "delivered", "checks", "buffered", "kernel_us"};
        for (unsigned i = 0; i < k; i++) {
            const uint64_t v[6] = {st[i].emitted, st[i].received, st[i].delivered, st[i].checks, st[i].buffered,
                                   (uint64_t)(st[i].kernel_ms * 1000.0)};
            maps[i] = kv_map(env, names, v, 6);
        }
        out = enif_make_tuple2(env, mk_atom(env, "ok"), stats_list(env, maps, k));
    }
    enif_free(st);
    enif_free(maps);
    return out;
}

/* shard_broadcast(Sim, Root) -> {ok, Monotonic}   (collective over the ranks) */
static ERL_NIF_TERM nif_shard_broadcast(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned root;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &root)) return enif_make_badarg(env);
    uint32_t mono = 0;
    enif_mutex_lock(r->mu);
    int rc = psim_shard_broadcast_x(r->h, root, &mono);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) return err(env, rc);
    return enif_make_tuple2(env, mk_atom(env, "ok"), enif_make_uint(env, mono));
}

/* shard_run(Sim, MaxRounds) -> {ok, Rounds, [StatsMap], {FabricBytes, ExchangeUs, KernelUs}}
 * (collective: global counters, stops at global quiescence) */
static ERL_NIF_TERM nif_shard_run(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned maxr;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &maxr)) return enif_make_badarg(env);
    enum { CAP = 4096 };
    psim_round_stats* st = (psim_round_stats*)enif_alloc(CAP * sizeof(psim_round_stats));
    if (!st) return err(env, PSIM_ENOMEM);
    uint32_t ran = 0;
    psim_exchange_stats xs;
    enif_mutex_lock(r->mu);
    int rc = psim_shard_run(r->h, maxr, st, CAP, &ran, &xs);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) { enif_free(st); return err(env, rc); }
    ERL_NIF_TERM list = enif_make_list(env, 0);
    for (uint32_t i = ran < CAP ? ran : CAP; i > 0; i--) list = enif_make_list_cell(env, stats_term(env, &st[i - 1]), list);
    enif_free(st);
    ERL_NIF_TERM x = enif_make_tuple3(env, enif_make_uint64(env, xs.fabric_bytes),
                                      enif_make_uint64(env, (uint64_t)(xs.exchange_ms * 1000.0)),
                                      enif_make_uint64(env, (uint64_t)(xs.kernel_ms * 1000.0)));
    ERL_NIF_TERM out[4] = {mk_atom(env, "ok"), enif_make_uint(env, ran), list, x};
    return enif_make_tuple_from_array(env, out, 4);
}

/* delivered_mono(Sim, Mono) -> {ok, Bin}: Mod:is_stale({Root, Epoch, Mono}) per
 * vertex of the focused root (psim_get_delivered_mono) */
static ERL_NIF_TERM nif_delivered_mono(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned mono;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &mono)) return enif_make_badarg(env);
    ERL_NIF_TERM t;
    unsigned char* d = enif_make_new_binary(env, r->n, &t);
    enif_mutex_lock(r->mu);
    int rc = psim_get_delivered_mono(r->h, mono, d, r->n);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) return err(env, rc);
    return enif_make_tuple2(env, mk_atom(env, "ok"), t);
}

/* is_delivered(Sim, V, Mono) -> {ok, boolean()}: Mod:is_stale({Root, Epoch,
 * Mono}) at one vertex of the focused root (Mono 0: the newest heartbeat),
 * psim_get_delivered_range over one vertex -- O(1) per call, where
 * delivered/1 copies the whole overlay's set */
static ERL_NIF_TERM nif_is_delivered(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned v, mono;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &v) || !enif_get_uint(env, argv[2], &mono) ||
        v >= r->n)
        return enif_make_badarg(env);
    uint8_t d = 0;
    enif_mutex_lock(r->mu);
    int rc = psim_get_delivered_range(r->h, mono, v, 1, &d);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) return err(env, rc);
    return enif_make_tuple2(env, mk_atom(env, "ok"), mk_atom(env, d ? "true" : "false"));
}

/* rows(Sim, V) -> {ok, [{Peer, Round, Mono}]}: v's outstanding i_have rows in
 * insertion order (psim_get_rows) */
static ERL_NIF_TERM nif_rows(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned v;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &v) || v >= r->n) return enif_make_badarg(env);
    enum { CAP = 64 };
    uint32_t p[CAP], rd[CAP], m[CAP];
    size_t k = 0;
    enif_mutex_lock(r->mu);
    int rc = psim_get_rows(r->h, v, p, rd, m, CAP, &k);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) return err(env, rc);
    ERL_NIF_TERM list = enif_make_list(env, 0);
    for (size_t i = k < CAP ? k : CAP; i > 0; i--)
        list = enif_make_list_cell(env, enif_make_tuple3(env, enif_make_uint(env, p[i - 1]), enif_make_uint(env, rd[i - 1]),
                                                         enif_make_uint(env, m[i - 1])), list);
    return enif_make_tuple2(env, mk_atom(env, "ok"), list);
}

/* messages(Sim) -> {ok, [{Src, Dst, Kind, Round, Mono}]}: the next round's
 * messages in handling order (psim_get_messages) */
static ERL_NIF_TERM nif_messages(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
    size_t k = 0;
    enif_mutex_lock(r->mu);
    int rc = psim_get_messages(r->h, NULL, NULL, NULL, NULL, NULL, 0, &k);
    uint32_t* a = NULL;
    if (rc == PSIM_OK && k) {
        a = (uint32_t*)enif_alloc(k * 5 * sizeof(uint32_t));
        if (!a) rc = PSIM_ENOMEM;
        else rc = psim_get_messages(r->h, a, a + k, a + 2 * k, a + 3 * k, a + 4 * k, k, &k);
    }
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) { if (a) enif_free(a); return err(env, rc); }
    ERL_NIF_TERM list = enif_make_list(env, 0);
    for (size_t i = k; i > 0; i--) {
        ERL_NIF_TERM e[5];
        for (int j = 0; j < 5; j++) e[j] = enif_make_uint(env, a[j * k + i - 1]);
        list = enif_make_list_cell(env, enif_make_tuple_from_array(env, e, 5), list);
    }
    if (a) enif_free(a);
    return enif_make_tuple2(env, mk_atom(env, "ok"), list);
}

/* shard_step(Sim, Rounds) -> {ok, [Stats], {FabricBytes, ExchangeUs, KernelUs}}:
 * exactly Rounds collective rounds (psim_shard_step) */
static ERL_NIF_TERM nif_shard_step(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    sim_res* r;
    unsigned rounds;
    if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &rounds) || rounds > 4096)
        return enif_make_badarg(env);
    psim_round_stats* st = (psim_round_stats*)enif_alloc((rounds ? rounds : 1) * sizeof(psim_round_stats));
    if (!st) return err(env, PSIM_ENOMEM);
    psim_exchange_stats xs;
    enif_mutex_lock(r->mu);
    int rc = psim_shard_step(r->h, rounds, st, rounds, &xs);
    enif_mutex_unlock(r->mu);
    if (rc != PSIM_OK) { enif_free(st); return err(env, rc); }
    ERL_NIF_TERM list = enif_make_list(env, 0);
    for (unsigned i = rounds; i > 0; i--) list = enif_make_list_cell(env, stats_term(env, &st[i - 1]), list);
    enif_free(st);
    ERL_NIF_TERM x = enif_make_tuple3(env, enif_make_uint64(env, xs.fabric_bytes),
                                      enif_make_uint64(env, (uint64_t)(xs.exchange_ms * 1000.0)),
                                      enif_make_uint64(env, (uint64_t)(xs.kernel_ms * 1000.0)));
    return enif_make_tuple3(env, mk_atom(env, "ok"), list, x);
}

static ErlNifFunc funcs[] = {
    {"new", 1, nif_new, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"load_csr", 3, nif_load_csr, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"set_alive", 2, nif_set_alive, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"reset_trees", 1, nif_reset_trees, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"restart_backend", 2, nif_restart_backend, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"broadcast", 2, nif_broadcast, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"broadcast_many", 2, nif_broadcast_many, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"step", 2, nif_step, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"run", 2, nif_run, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"broadcast_run", 3, nif_broadcast_run, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"broadcast_run_n", 5, nif_broadcast_run_n, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"peers", 1, nif_peers, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"slots", 1, nif_slots, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"delivered", 1, nif_delivered, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"trace_hash", 1, nif_trace_hash, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"focus", 2, nif_focus, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"set_omissions", 3, nif_set_omissions, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"set_delays", 4, nif_set_delays, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"delivered_mono", 2, nif_delivered_mono, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"is_delivered", 3, nif_is_delivered, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"rows", 2, nif_rows, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"messages", 1, nif_messages, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"shard_step", 2, nif_shard_step, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"relay_run", 10, nif_relay_run, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"hv_setup", 3, nif_hv_setup, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"hv_join", 3, nif_hv_join, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"hv_step", 2, nif_hv_step, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"hv_views", 1, nif_hv_views, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"demers_setup", 5, nif_demers_setup, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"demers_run", 2, nif_demers_run, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"vclock", 4, nif_vclock, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"scamp_setup", 5, nif_scamp_setup, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"scamp_join", 3, nif_scamp_join, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"scamp_leave", 3, nif_scamp_leave, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"scamp_crash", 2, nif_scamp_crash, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"scamp_step", 2, nif_scamp_step, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"scamp_views", 1, nif_scamp_views, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"scamp_messages", 1, nif_scamp_messages, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"scamp_messages_from", 2, nif_scamp_messages_from, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"scamp_take", 2, nif_scamp_take, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"scamp_put", 2, nif_scamp_put, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"fm_setup", 4, nif_fm_setup, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"fm_join", 3, nif_fm_join, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"fm_leave", 3, nif_fm_leave, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"fm_step", 2, nif_fm_step, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"fm_state", 1, nif_fm_state, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"fm_tokens", 1, nif_fm_tokens, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"fm_messages", 1, nif_fm_messages, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"fm_messages_from", 2, nif_fm_messages_from, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"fm_take", 2, nif_fm_take, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"fm_put", 2, nif_fm_put, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"c3_setup", 4, nif_c3_setup, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"c3_join", 3, nif_c3_join, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"c3_crash", 2, nif_c3_crash, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"c3_heartbeat", 2, nif_c3_heartbeat, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"c3_step", 2, nif_c3_step, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"c3_run", 8, nif_c3_run, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"causal_setup", 6, nif_causal_setup, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"causal_step", 2, nif_causal_step, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"causal_clocks", 1, nif_causal_clocks, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"rccl_unique_id", 0, nif_rccl_unique_id, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"shard_init_rccl", 4, nif_shard_init_rccl, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"shard_broadcast", 2, nif_shard_broadcast, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"shard_run", 2, nif_shard_run, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"demers_shard_setup", 7, nif_demers_shard_setup, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"demers_shard_run", 2, nif_demers_shard_run, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"causal_shard_setup", 8, nif_causal_shard_setup, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"causal_shard_step", 2, nif_causal_shard_step, ERL_NIF_DIRTY_JOB_CPU_BOUND},
};

ERL_NIF_INIT(partisan_gpu_sim, funcs, load, NULL, NULL, NULL)
