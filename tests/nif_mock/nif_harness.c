/* nif_harness.c -- drives the real Erlang NIF shim (erl/c_src/partisan_gpu_sim_nif.c)
 * as the BEAM would: load/3, then calls through its ErlNifFunc table with
 * terms of the mock term store (tests/nif_mock/mock_erts.c), linked with
 * libpsim.so.  TEST INFRASTRUCTURE (tests/test_nif_harness.py runs it on the
 * GPU box and checks its JSON report against the Python path).
 *
 * Scenario: config C2 in small (HyParView sequential joins + shuffle
 * periods, then a Plumtree heartbeat over the active views), Demers, SCAMP
 * v2 join waves, full membership, C3 churn, causal delivery, vclock ops and
 * the vertex-sharded run with the in-library RCCL exchange at world 1. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mock_erts.h"

static const ErlNifFunc* g_funcs;
static int g_nfuncs;
static ErlNifEnv* const ENV = (ErlNifEnv*)0x1;   /* the shim never dereferences it */

static ERL_NIF_TERM call(const char* name, unsigned arity, const ERL_NIF_TERM* argv) {
    for (int i = 0; i < g_nfuncs; i++)
        if (!strcmp(g_funcs[i].name, name) && g_funcs[i].arity == arity) return g_funcs[i].fptr(ENV, (int)arity, argv);
    fprintf(stderr, "no NIF %s/%u\n", name, arity);
    exit(2);
}

static void die(const char* what, ERL_NIF_TERM t) {
    fprintf(stderr, "FAIL %s: ", what);
    if (mock_is_badarg(t)) fprintf(stderr, "badarg\n");
    else if (mock_tuple_arity(t) == 2 && mock_is_atom(mock_elem(t, 0), "error"))
        fprintf(stderr, "{error, %s}\n", mock_atom_name(mock_elem(t, 1)));
    else fprintf(stderr, "unexpected term\n");
    exit(1);
}

static void want_ok(const char* what, ERL_NIF_TERM t) {
    if (!mock_is_atom(t, "ok")) die(what, t);
}

/* {ok, ...} -> the tuple */
static ERL_NIF_TERM want_ok_tuple(const char* what, ERL_NIF_TERM t) {
    if (mock_tuple_arity(t) < 2 || !mock_is_atom(mock_elem(t, 0), "ok")) die(what, t);
    return t;
}

#define A(...) ((const ERL_NIF_TERM[]){__VA_ARGS__})

static ERL_NIF_TERM new_sim(uint64_t seed) {
    const char* k[] = {"seed", "lazy_tick_rounds", "device"};
    const uint64_t v[] = {seed, 1, 0};
    ERL_NIF_TERM r = want_ok_tuple("new", call("new", 1, A(mock_map(3, k, v))));
    return mock_elem(r, 1);
}

static ERL_NIF_TERM u32s(const uint32_t* a, size_t n) { return mock_bin(a, n * 4); }

static uint32_t lcg(uint64_t* s) {
    *s = *s * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(*s >> 33);
}

/* the report goes to argv[1] (the libraries may write to stdout) */
static FILE* g_out;

int main(int argc, char** argv) {
    mock_nif_load_fn load;
    g_out = argc > 1 ? fopen(argv[1], "w") : stdout;
    if (!g_out) {
        fprintf(stderr, "FAIL open %s\n", argv[1]);
        return 1;
    }
    g_funcs = mock_nif_table(&g_nfuncs, &load);
    if (load(ENV, NULL, 0) != 0) {
        fprintf(stderr, "FAIL load\n");
        return 1;
    }
    fprintf(g_out, "{");
    /* ---- C2 in small: HyParView overlay, then a Plumtree heartbeat -------- */
    {
        const uint32_t n = 2000;
        ERL_NIF_TERM sim = new_sim(0x5EED0002ull);
        const char* hk[] = {"shuffle_rounds", "promotion_rounds"};
        const uint64_t hv[] = {10, 5};
        want_ok("hv_setup", call("hv_setup", 3, A(sim, mock_uint(n), mock_map(2, hk, hv))));
        uint64_t s = 2;
        for (uint32_t i = 1; i < n; i++) {       /* vertex i joins a contact in [0, i), one join per round */
            const uint32_t c = lcg(&s) % i;
            want_ok("hv_join", call("hv_join", 3, A(sim, u32s(&i, 1), u32s(&c, 1))));
            want_ok_tuple("hv_step", call("hv_step", 2, A(sim, mock_uint(1))));
        }
        want_ok_tuple("hv_step", call("hv_step", 2, A(sim, mock_uint(100))));   /* 10 shuffle periods */
        ERL_NIF_TERM views = want_ok_tuple("hv_views", call("hv_views", 1, A(sim)));
        size_t na_sz, nl_sz;
        const uint32_t* act = (const uint32_t*)mock_bin_data(mock_elem(views, 1), &na_sz);
        const unsigned char* alen = mock_bin_data(mock_elem(views, 2), &nl_sz);
        uint64_t* rp = (uint64_t*)calloc(n + 1, 8);
        uint32_t* col = (uint32_t*)calloc((size_t)n * 8, 4);
        uint64_t e = 0;
        for (uint32_t v = 0; v < n; v++) {       /* active views minus self = the members plumtree sees */
            for (uint32_t j = 0; j < alen[v]; j++)
                if (act[v * 8 + j] != v) col[e++] = act[v * 8 + j];
            rp[v + 1] = e;
        }
        want_ok("load_csr", call("load_csr", 3, A(sim, mock_bin(rp, (n + 1) * 8), u32s(col, e))));
        ERL_NIF_TERM bc = want_ok_tuple("broadcast", call("broadcast", 2, A(sim, mock_uint(0))));
        ERL_NIF_TERM run = want_ok_tuple("run", call("run", 2, A(sim, mock_uint(1000))));
        const uint64_t rounds = mock_int(mock_elem(run, 1));
        ERL_NIF_TERM stats = mock_elem(run, 2);
        uint64_t bsum = 0, x;
        for (size_t i = 0; i < mock_list_len(stats); i++)
            if (mock_map_get(mock_list_nth(stats, i), "broadcast", &x)) bsum += x;
        ERL_NIF_TERM dl = want_ok_tuple("delivered", call("delivered", 1, A(sim)));
        size_t dsz;
        const unsigned char* d = mock_bin_data(mock_elem(dl, 1), &dsz);
        uint64_t got = 0;
        for (size_t i = 0; i < dsz; i++) got += d[i];
        ERL_NIF_TERM th = mock_elem(want_ok_tuple("trace_hash", call("trace_hash", 1, A(sim))), 1);
        fprintf(g_out, "\"c2\": {\"n\": %u, \"edges\": %llu, \"mono\": %llu, \"rounds\": %llu, \"delivered\": %llu, "
               "\"broadcasts\": %llu, \"trace\": [\"%llu\", \"%llu\", \"%llu\", \"%llu\"]}",
               n, (unsigned long long)e, (unsigned long long)mock_int(mock_elem(bc, 1)), (unsigned long long)rounds,
               (unsigned long long)got, (unsigned long long)bsum, (unsigned long long)mock_int(mock_elem(th, 0)),
               (unsigned long long)mock_int(mock_elem(th, 1)), (unsigned long long)mock_int(mock_elem(th, 2)),
               (unsigned long long)mock_int(mock_elem(th, 3)));
        {   /* every node heartbeats: the same overlay on a forest handle, all n roots
             * at once through broadcast_many, twice; a 2n-th root is {error, enospc} */
            const char* k[] = {"seed", "lazy_tick_rounds", "device", "max_roots"};
            const uint64_t v[] = {0x5EED0002ull, 1, 0, n};
            ERL_NIF_TERM fs = mock_elem(want_ok_tuple("new", call("new", 1, A(mock_map(4, k, v)))), 1);
            want_ok("load_csr", call("load_csr", 3, A(fs, mock_bin(rp, (n + 1) * 8), u32s(col, e))));
            uint32_t* roots = (uint32_t*)calloc(n, 4);
            for (uint32_t i = 0; i < n; i++) roots[i] = i;
            uint64_t fr[2] = {0, 0}, fdl = 0;
            for (int it = 0; it < 2; it++) {
                ERL_NIF_TERM ids = want_ok_tuple("broadcast_many", call("broadcast_many", 2, A(fs, u32s(roots, n))));
                size_t isz;
                const uint32_t* idp = (const uint32_t*)mock_bin_data(mock_elem(ids, 1), &isz);
                if (isz != (size_t)n * 4 || idp[0] != (uint32_t)(it + 1)) { fprintf(stderr, "broadcast_many ids\n"); return 1; }
                ERL_NIF_TERM fr_run = want_ok_tuple("run", call("run", 2, A(fs, mock_uint(1000))));
                fr[it] = mock_int(mock_elem(fr_run, 1));
                ERL_NIF_TERM fst = mock_elem(fr_run, 2);
                for (size_t i = 0; i < mock_list_len(fst); i++)
                    if (it == 0 && mock_map_get(mock_list_nth(fst, i), "delivered", &x)) fdl += x;
            }
            uint32_t extra = 0;
            ERL_NIF_TERM big = call("broadcast_many", 2, A(fs, u32s(&extra, 1)));   /* root 0 again: fine */
            (void)big;
            want_ok_tuple("run", call("run", 2, A(fs, mock_uint(1000))));
            fprintf(g_out, ", \"forest\": {\"roots\": %u, \"rounds\": [%llu, %llu], \"delivered\": %llu}", n,
                    (unsigned long long)fr[0], (unsigned long long)fr[1], (unsigned long long)fdl);
            /* parked roots: the same n roots' records through 16 lanes, 16 heartbeats at a time
             * (forest_lanes => psim_forest_set_lanes); 17 at once is {error, enospc} */
            const char* kp[] = {"seed", "lazy_tick_rounds", "device", "max_roots", "forest_lanes"};
            const uint64_t vp[] = {0x5EED0002ull, 1, 0, n, 16};
            ERL_NIF_TERM ps = mock_elem(want_ok_tuple("new", call("new", 1, A(mock_map(5, kp, vp)))), 1);
            want_ok("load_csr", call("load_csr", 3, A(ps, mock_bin(rp, (n + 1) * 8), u32s(col, e))));
            ERL_NIF_TERM over = call("broadcast_many", 2, A(ps, u32s(roots, 17)));
            const int enospc = mock_tuple_arity(over) == 2 && mock_is_atom(mock_elem(over, 0), "error") &&
                               mock_is_atom(mock_elem(over, 1), "enospc");
            uint64_t pdl = 0;
            for (uint32_t b = 0; b < n; b += 16) {
                const uint32_t k16 = n - b < 16 ? n - b : 16;
                want_ok_tuple("broadcast_many", call("broadcast_many", 2, A(ps, u32s(roots + b, k16))));
                ERL_NIF_TERM pr = want_ok_tuple("run", call("run", 2, A(ps, mock_uint(1000))));
                ERL_NIF_TERM pst = mock_elem(pr, 2);
                for (size_t i = 0; i < mock_list_len(pst); i++)
                    if (mock_map_get(mock_list_nth(pst, i), "delivered", &x)) pdl += x;
            }
            fprintf(g_out, ", \"parked\": {\"roots\": %u, \"lanes\": 16, \"delivered\": %llu, \"enospc\": %d}", n,
                    (unsigned long long)pdl, enospc);
            free(roots);
        }
        {   /* window-lane-era getters on the static lane: every vertex delivered this Monotonic, nothing in flight */
            ERL_NIF_TERM dm = want_ok_tuple("delivered_mono", call("delivered_mono", 2, A(sim, mock_elem(bc, 1))));
            size_t dmz;
            const unsigned char* dmb = mock_bin_data(mock_elem(dm, 1), &dmz);
            uint64_t dmsum = 0;
            for (size_t i = 0; i < dmz; i++) dmsum += dmb[i];
            ERL_NIF_TERM ms = want_ok_tuple("messages", call("messages", 1, A(sim)));
            ERL_NIF_TERM rw = want_ok_tuple("rows", call("rows", 2, A(sim, mock_uint(0))));
            uint64_t one = 0;                    /* is_delivered/3: Mod:is_stale at one vertex, O(1) */
            for (uint32_t v = 0; v < n; v++) {
                ERL_NIF_TERM iv = want_ok_tuple("is_delivered",
                                                call("is_delivered", 3, A(sim, mock_uint(v), mock_uint(0))));
                one += mock_is_atom(mock_elem(iv, 1), "true");
            }
            fprintf(g_out, ", \"c2_getters\": {\"delivered_mono\": %llu, \"messages\": %zu, \"rows0\": %zu, "
                    "\"is_delivered\": %llu}",
                    (unsigned long long)dmsum, mock_list_len(mock_elem(ms, 1)), mock_list_len(mock_elem(rw, 1)),
                    (unsigned long long)one);
        }
        {   /* root 0's second heartbeat in one call: broadcast_run (broadcast + run to quiescence) */
            ERL_NIF_TERM br = want_ok_tuple("broadcast_run", call("broadcast_run", 3, A(sim, mock_uint(0), mock_uint(1000))));
            ERL_NIF_TERM st2 = mock_elem(br, 3);
            uint64_t b2 = 0, y;
            for (size_t i = 0; i < mock_list_len(st2); i++)
                if (mock_map_get(mock_list_nth(st2, i), "broadcast", &y)) b2 += y;
            ERL_NIF_TERM th2 = mock_elem(want_ok_tuple("trace_hash", call("trace_hash", 1, A(sim))), 1);
            fprintf(g_out, ", \"c2_hb2\": {\"mono\": %llu, \"rounds\": %llu, \"broadcasts\": %llu, "
                    "\"trace\": [\"%llu\", \"%llu\", \"%llu\", \"%llu\"]}",
                    (unsigned long long)mock_int(mock_elem(br, 1)), (unsigned long long)mock_int(mock_elem(br, 2)),
                    (unsigned long long)b2, (unsigned long long)mock_int(mock_elem(th2, 0)),
                    (unsigned long long)mock_int(mock_elem(th2, 1)), (unsigned long long)mock_int(mock_elem(th2, 2)),
                    (unsigned long long)mock_int(mock_elem(th2, 3)));
        }
        {   /* three more heartbeats of root 0 over its tree in one call: broadcast_run_n */
            ERL_NIF_TERM bn = want_ok_tuple("broadcast_run_n", call("broadcast_run_n", 5,
                                            A(sim, mock_uint(0), mock_uint(3), mock_uint(0), mock_uint(1000))));
            ERL_NIF_TERM ivs = mock_elem(bn, 1), st3 = mock_elem(bn, 2);
            uint64_t b3 = 0, y;
            for (size_t i = 0; i < mock_list_len(st3); i++)
                if (mock_map_get(mock_list_nth(st3, i), "broadcast", &y)) b3 += y;
            ERL_NIF_TERM th3 = mock_elem(want_ok_tuple("trace_hash", call("trace_hash", 1, A(sim))), 1);
            fprintf(g_out, ", \"c2_hb345\": {\"intervals\": [");
            for (size_t i = 0; i < mock_list_len(ivs); i++) {
                ERL_NIF_TERM iv = mock_list_nth(ivs, i);
                fprintf(g_out, "%s[%llu, %llu]", i ? ", " : "", (unsigned long long)mock_int(mock_elem(iv, 0)),
                        (unsigned long long)mock_int(mock_elem(iv, 1)));
            }
            fprintf(g_out, "], \"rows\": %zu, \"broadcasts\": %llu, \"trace\": [\"%llu\", \"%llu\", \"%llu\", \"%llu\"]}",
                    mock_list_len(st3), (unsigned long long)b3, (unsigned long long)mock_int(mock_elem(th3, 0)),
                    (unsigned long long)mock_int(mock_elem(th3, 1)), (unsigned long long)mock_int(mock_elem(th3, 2)),
                    (unsigned long long)mock_int(mock_elem(th3, 3)));
        }
        /* the same overlay, vertex-sharded at world 1 with the library's own RCCL communicator */
        ERL_NIF_TERM sim7 = new_sim(0x5EED0002ull);
        ERL_NIF_TERM id = mock_elem(want_ok_tuple("rccl_unique_id", call("rccl_unique_id", 0, A(0))), 1);
        want_ok("shard_init_rccl", call("shard_init_rccl", 4, A(sim7, mock_uint(0), mock_uint(1), id)));
        want_ok("load_csr", call("load_csr", 3, A(sim7, mock_bin(rp, (n + 1) * 8), u32s(col, e))));
        want_ok_tuple("shard_broadcast", call("shard_broadcast", 2, A(sim7, mock_uint(0))));
        ERL_NIF_TERM sr = want_ok_tuple("shard_run", call("shard_run", 2, A(sim7, mock_uint(1000))));
        ERL_NIF_TERM dl7 = want_ok_tuple("delivered", call("delivered", 1, A(sim7)));
        d = mock_bin_data(mock_elem(dl7, 1), &dsz);
        uint64_t got7 = 0;
        for (size_t i = 0; i < dsz; i++) got7 += d[i];
        ERL_NIF_TERM ss = want_ok_tuple("shard_step", call("shard_step", 2, A(sim7, mock_uint(2))));
        fprintf(g_out, ", \"shard_rccl_world1\": {\"rounds\": %llu, \"delivered\": %llu, \"step2\": %zu}",
               (unsigned long long)mock_int(mock_elem(sr, 1)), (unsigned long long)got7, mock_list_len(mock_elem(ss, 1)));
        free(rp);
        free(col);
    }
    /* ---- Demers rumor mongering + anti-entropy --------------------------- */
    {
        ERL_NIF_TERM sim = new_sim(0x5EED0004ull);
        want_ok("demers_setup", call("demers_setup", 5, A(sim, mock_uint(20000), mock_uint(64), mock_uint(2),
                                                          mock_atom("true"))));
        ERL_NIF_TERM r = want_ok_tuple("demers_run", call("demers_run", 2, A(sim, mock_uint(200))));
        size_t sz;
        const uint64_t* seen = (const uint64_t*)mock_bin_data(mock_elem(r, 2), &sz);
        uint64_t full = 0;
        for (size_t i = 0; i < sz / 8; i++) full += seen[i] == ~0ull;
        fprintf(g_out, ", \"demers\": {\"n\": 20000, \"rounds\": %llu, \"complete\": %llu}",
               (unsigned long long)mock_int(mock_elem(r, 1)), (unsigned long long)full);
    }
    /* ---- the same epidemic vertex-sharded at world 1, exchange on the library's RCCL communicator */
    {
        ERL_NIF_TERM sim = new_sim(0x5EED0004ull);
        ERL_NIF_TERM id = mock_elem(want_ok_tuple("rccl_unique_id", call("rccl_unique_id", 0, A(0))), 1);
        want_ok("shard_init_rccl", call("shard_init_rccl", 4, A(sim, mock_uint(0), mock_uint(1), id)));
        want_ok_tuple("demers_shard_setup", call("demers_shard_setup", 7, A(sim, mock_uint(20000), mock_uint(64),
                                                                              mock_uint(2), mock_atom("true"),
                                                                              mock_uint(0), mock_uint(1))));
        ERL_NIF_TERM r = want_ok_tuple("demers_shard_run", call("demers_shard_run", 2, A(sim, mock_uint(200))));
        size_t sz;
        const uint64_t* seen = (const uint64_t*)mock_bin_data(mock_elem(r, 2), &sz);
        uint64_t full = 0;
        for (size_t i = 0; i < sz / 8; i++) full += seen[i] == ~0ull;
        fprintf(g_out, ", \"demers_shard_rccl_world1\": {\"rounds\": %llu, \"complete\": %llu}",
               (unsigned long long)mock_int(mock_elem(r, 1)), (unsigned long long)full);
    }
    /* ---- SCAMP v2 join waves ---------------------------------------------- */
    {
        const uint32_t n = 3000;
        ERL_NIF_TERM sim = new_sim(0x5EED0003ull);
        want_ok("scamp_setup", call("scamp_setup", 5, A(sim, mock_uint(n), mock_uint(2), mock_uint(5), mock_uint(10))));
        uint64_t s = 3;
        for (uint32_t k = 1; k < n; k *= 2) {
            const uint32_t hi = 2 * k < n ? 2 * k : n;
            uint32_t* v = (uint32_t*)malloc((hi - k) * 4);
            uint32_t* c = (uint32_t*)malloc((hi - k) * 4);
            for (uint32_t i = k; i < hi; i++) {
                v[i - k] = i;
                c[i - k] = lcg(&s) % k;
            }
            want_ok("scamp_join", call("scamp_join", 3, A(sim, u32s(v, hi - k), u32s(c, hi - k))));
            want_ok_tuple("scamp_step", call("scamp_step", 2, A(sim, mock_uint(3))));
            free(v);
            free(c);
        }
        ERL_NIF_TERM st = mock_elem(want_ok_tuple("scamp_step", call("scamp_step", 2, A(sim, mock_uint(5)))), 1);
        uint64_t pv = 0;
        mock_map_get(mock_list_nth(st, 4), "pv_sum", &pv);
        ERL_NIF_TERM vw = want_ok_tuple("scamp_views", call("scamp_views", 1, A(sim)));
        size_t sz;
        const uint32_t* npv = (const uint32_t*)mock_bin_data(mock_elem(vw, 2), &sz);
        uint64_t tot = 0;
        for (size_t i = 0; i < sz / 4; i++) tot += npv[i];
        fprintf(g_out, ", \"scamp\": {\"n\": %u, \"pv_sum\": %llu, \"view_entries\": %llu}", n, (unsigned long long)pv,
               (unsigned long long)tot);
    }
    /* ---- SCAMP v2 on the wire: {membership_strategy, Msg} terms each round,
     *      and one node's messages taken off and put back */
    {
        const uint32_t n = 400;
        ERL_NIF_TERM sim = new_sim(0x5EED0004ull);
        want_ok("scamp_setup", call("scamp_setup", 5, A(sim, mock_uint(n), mock_uint(2), mock_uint(5), mock_uint(10))));
        uint64_t s = 11;
        for (uint32_t k = 1; k < n; k *= 2) {
            const uint32_t hi = 2 * k < n ? 2 * k : n;
            uint32_t v[512], c[512];
            for (uint32_t i = k; i < hi; i++) {
                v[i - k] = i;
                c[i - k] = lcg(&s) % k;
            }
            want_ok("scamp_join", call("scamp_join", 3, A(sim, u32s(v, hi - k), u32s(c, hi - k))));
            want_ok_tuple("scamp_step", call("scamp_step", 2, A(sim, mock_uint(3))));
        }
        static const char* const tags[] = {"", "forward_subscription", "keep_subscription", "ping",
                                           "remove_subscription", "replace_subscription",
                                           "bootstrap_remove_subscription"};
        fprintf(g_out, ", \"scamp_wire\": {\"n\": %u, \"rounds\": [", n);
        uint64_t taken = 0;
        for (int r = 0; r < 12; r++) {
            ERL_NIF_TERM ms = mock_elem(want_ok_tuple("scamp_messages", call("scamp_messages", 1, A(sim))), 1);
            fprintf(g_out, "%s[", r ? ", " : "");
            for (size_t i = 0; i < mock_list_len(ms); i++) {
                ERL_NIF_TERM m = mock_list_nth(ms, i);             /* {Src, Dst, Seq, {membership_strategy, Msg}} */
                ERL_NIF_TERM w = mock_elem(m, 3), body = mock_elem(w, 1);
                if (!mock_is_atom(mock_elem(w, 0), "membership_strategy")) { fprintf(stderr, "bad wire term\n"); return 1; }
                int t = 0;
                for (int k = 1; k <= 6; k++) if (mock_is_atom(mock_elem(body, 0), tags[k])) t = k;
                const uint64_t b = mock_tuple_arity(body) == 3 ? mock_int(mock_elem(body, 2)) : 0;
                fprintf(g_out, "%s[%d, %llu, %llu, %llu, %llu, %llu]", i ? ", " : "", t,
                        (unsigned long long)mock_int(mock_elem(m, 0)), (unsigned long long)mock_int(mock_elem(m, 1)),
                        (unsigned long long)mock_int(mock_elem(m, 2)), (unsigned long long)mock_int(mock_elem(body, 1)),
                        (unsigned long long)b);
            }
            fprintf(g_out, "]");
            if (mock_list_len(ms) > 0) {             /* scamp_messages_from/2 = the Src-filtered list, in order */
                const uint64_t src = mock_int(mock_elem(mock_list_nth(ms, mock_list_len(ms) / 2), 0));
                ERL_NIF_TERM f = mock_elem(want_ok_tuple("scamp_messages_from",
                                                         call("scamp_messages_from", 2, A(sim, mock_uint((uint32_t)src)))), 1);
                size_t j = 0;
                for (size_t i = 0; i < mock_list_len(ms); i++) {
                    ERL_NIF_TERM m = mock_list_nth(ms, i);
                    if ((uint64_t)mock_int(mock_elem(m, 0)) != src) continue;
                    if (j >= mock_list_len(f) || mock_int(mock_elem(mock_list_nth(f, j), 1)) != mock_int(mock_elem(m, 1)) ||
                        mock_int(mock_elem(mock_list_nth(f, j), 2)) != mock_int(mock_elem(m, 2))) {
                        fprintf(stderr, "scamp_messages_from differs at %zu\n", j);
                        return 1;
                    }
                    j++;
                }
                if (j != mock_list_len(f)) { fprintf(stderr, "scamp_messages_from: %zu vs %zu\n", j, mock_list_len(f)); return 1; }
            }
            if (r == 5 && mock_list_len(ms) > 0) {   /* a manager's round trip: take one node's messages, put them back */
                const uint64_t d = mock_int(mock_elem(mock_list_nth(ms, 0), 1));
                ERL_NIF_TERM got = mock_elem(want_ok_tuple("scamp_take", call("scamp_take", 2, A(sim, mock_uint(d)))), 1);
                taken = mock_list_len(got);
                want_ok("scamp_put", call("scamp_put", 2, A(sim, got)));
            }
            want_ok_tuple("scamp_step", call("scamp_step", 2, A(sim, mock_uint(1))));
        }
        ERL_NIF_TERM vw = want_ok_tuple("scamp_views", call("scamp_views", 1, A(sim)));
        size_t sz, szl;
        const uint32_t* pv = (const uint32_t*)mock_bin_data(mock_elem(vw, 1), &sz);
        const uint32_t* npv = (const uint32_t*)mock_bin_data(mock_elem(vw, 2), &szl);
        fprintf(g_out, "], \"taken\": %llu, \"views\": [", (unsigned long long)taken);
        for (uint32_t v = 0; v < n; v++) {
            fprintf(g_out, "%s[", v ? ", " : "");
            for (uint32_t j = 0; j < npv[v]; j++) fprintf(g_out, "%s%u", j ? ", " : "", pv[v * 128 + j]);
            fprintf(g_out, "]");
        }
        fprintf(g_out, "]}");
    }
    /* ---- full membership (C1 shape: 16 nodes join node 0) ------------------ */
    {
        const uint32_t n = 16;
        ERL_NIF_TERM sim = new_sim(0x5EED0001ull);
        want_ok("fm_setup", call("fm_setup", 4, A(sim, mock_uint(n), mock_uint(10), mock_uint(64))));
        uint32_t v[15], p[15];
        for (uint32_t i = 1; i < n; i++) {
            v[i - 1] = i;
            p[i - 1] = 0;
        }
        want_ok("fm_join", call("fm_join", 3, A(sim, u32s(v, 15), u32s(p, 15))));
        want_ok_tuple("fm_step", call("fm_step", 2, A(sim, mock_uint(30))));
        ERL_NIF_TERM fs = want_ok_tuple("fm_state", call("fm_state", 1, A(sim)));
        size_t sz;
        const uint64_t* known = (const uint64_t*)mock_bin_data(mock_elem(fs, 1), &sz);
        uint64_t full = 0;
        for (uint32_t i = 0; i < n; i++) full += (known[i] & 0xFFFFull) == 0xFFFFull;
        ERL_NIF_TERM tk = want_ok_tuple("fm_tokens", call("fm_tokens", 1, A(sim)));
        size_t tsz;
        const uint32_t* tn = (const uint32_t*)mock_bin_data(mock_elem(tk, 1), &tsz);
        uint64_t ident = 0;
        for (uint32_t i = 0; i < n; i++) ident += tn[i] == i;          /* token v = node v's init/1 add */
        fprintf(g_out, ", \"fullmem\": {\"n\": %u, \"knows_all\": %llu, \"tokens_used\": %llu, \"own_tokens\": %llu}", n,
               (unsigned long long)full, (unsigned long long)mock_int(mock_elem(tk, 2)), (unsigned long long)ident);
    }
    /* ---- full membership on the wire: {membership_strategy, {Spec, #full_v1{}}} --- */
    {
        const uint32_t n = 12;
        ERL_NIF_TERM sim = new_sim(0x5EED0001ull);
        want_ok("fm_setup", call("fm_setup", 4, A(sim, mock_uint(n), mock_uint(3), mock_uint(64))));
        uint32_t v[11], p[11];
        for (uint32_t i = 1; i < n; i++) {
            v[i - 1] = i;
            p[i - 1] = i - 1;
        }
        want_ok("fm_join", call("fm_join", 3, A(sim, u32s(v, 11), u32s(p, 11))));
        fprintf(g_out, ", \"fm_wire\": {\"n\": %u, \"rounds\": [", n);
        uint64_t taken = 0;
        for (int r = 0; r < 8; r++) {
            want_ok_tuple("fm_step", call("fm_step", 2, A(sim, mock_uint(1))));
            ERL_NIF_TERM ms = mock_elem(want_ok_tuple("fm_messages", call("fm_messages", 1, A(sim))), 1);
            fprintf(g_out, "%s[", r ? ", " : "");
            for (size_t i = 0; i < mock_list_len(ms); i++) {
                ERL_NIF_TERM m = mock_list_nth(ms, i);             /* {Src, Dst, Seq, Known, Removed} */
                size_t kz, rz;
                const uint64_t* kw = (const uint64_t*)mock_bin_data(mock_elem(m, 3), &kz);
                const uint64_t* rw = (const uint64_t*)mock_bin_data(mock_elem(m, 4), &rz);
                fprintf(g_out, "%s[%llu, %llu, %llu, %llu]", i ? ", " : "", (unsigned long long)mock_int(mock_elem(m, 0)),
                        (unsigned long long)mock_int(mock_elem(m, 1)), (unsigned long long)kw[0], (unsigned long long)rw[0]);
            }
            fprintf(g_out, "]");
            if (mock_list_len(ms) > 0) {             /* fm_messages_from/2 = the Src-filtered list, in order */
                const uint64_t src = mock_int(mock_elem(mock_list_nth(ms, mock_list_len(ms) / 2), 0));
                ERL_NIF_TERM f = mock_elem(want_ok_tuple("fm_messages_from",
                                                         call("fm_messages_from", 2, A(sim, mock_uint((uint32_t)src)))), 1);
                size_t j = 0;
                for (size_t i = 0; i < mock_list_len(ms); i++) {
                    ERL_NIF_TERM m = mock_list_nth(ms, i);
                    if ((uint64_t)mock_int(mock_elem(m, 0)) != src) continue;
                    size_t z1, z2;
                    const uint64_t* a = (const uint64_t*)mock_bin_data(mock_elem(m, 3), &z1);
                    const uint64_t* b = j < mock_list_len(f) ? (const uint64_t*)mock_bin_data(mock_elem(mock_list_nth(f, j), 3), &z2) : NULL;
                    if (!b || z1 != z2 || memcmp(a, b, z1) != 0 ||
                        mock_int(mock_elem(mock_list_nth(f, j), 1)) != mock_int(mock_elem(m, 1))) {
                        fprintf(stderr, "fm_messages_from differs at %zu\n", j);
                        return 1;
                    }
                    j++;
                }
                if (j != mock_list_len(f)) { fprintf(stderr, "fm_messages_from: %zu vs %zu\n", j, mock_list_len(f)); return 1; }
            }
            if (r == 3 && mock_list_len(ms) > 0) {   /* a manager's round trip: take one node's messages, put them back */
                const uint64_t d = mock_int(mock_elem(mock_list_nth(ms, 0), 1));
                ERL_NIF_TERM got = mock_elem(want_ok_tuple("fm_take", call("fm_take", 2, A(sim, mock_uint(d)))), 1);
                taken = mock_list_len(got);
                want_ok("fm_put", call("fm_put", 2, A(sim, got)));
            }
            if (r == 5) {                             /* node 2's state from a node outside the cluster, to node 4 */
                ERL_NIF_TERM fs = want_ok_tuple("fm_state", call("fm_state", 1, A(sim)));
                size_t sz;
                const uint64_t* kn = (const uint64_t*)mock_bin_data(mock_elem(fs, 1), &sz);
                const uint64_t* rm = (const uint64_t*)mock_bin_data(mock_elem(fs, 2), &sz);
                ERL_NIF_TERM el[5] = {mock_uint(n), mock_uint(4), mock_uint(0), mock_bin(&kn[2], 8), mock_bin(&rm[2], 8)};
                ERL_NIF_TERM msg = enif_make_tuple_from_array(NULL, el, 5);
                want_ok("fm_put", call("fm_put", 2, A(sim, enif_make_list_cell(NULL, msg, enif_make_list(NULL, 0)))));
            }
        }
        ERL_NIF_TERM fs = want_ok_tuple("fm_state", call("fm_state", 1, A(sim)));
        size_t sz;
        const uint64_t* kn = (const uint64_t*)mock_bin_data(mock_elem(fs, 1), &sz);
        const uint64_t* rm = (const uint64_t*)mock_bin_data(mock_elem(fs, 2), &sz);
        fprintf(g_out, "], \"taken\": %llu, \"known\": [", (unsigned long long)taken);
        for (uint32_t i = 0; i < n; i++) fprintf(g_out, "%s%llu", i ? ", " : "", (unsigned long long)kn[i]);
        fprintf(g_out, "], \"removed\": [");
        for (uint32_t i = 0; i < n; i++) fprintf(g_out, "%s%llu", i ? ", " : "", (unsigned long long)rm[i]);
        fprintf(g_out, "]}");
    }
    /* ---- C3: SCAMP v2 churn + Plumtree repair ------------------------------- */
    {
        const uint32_t n = 2000;
        ERL_NIF_TERM sim = new_sim(0x5EED0003ull);
        want_ok("c3_setup", call("c3_setup", 4, A(sim, mock_uint(n), mock_uint(5), mock_uint(10))));
        uint64_t s = 5;
        for (uint32_t k = 1; k < n; k *= 2) {
            const uint32_t hi = 2 * k < n ? 2 * k : n;
            uint32_t* v = (uint32_t*)malloc((hi - k) * 4);
            uint32_t* c = (uint32_t*)malloc((hi - k) * 4);
            for (uint32_t i = k; i < hi; i++) {
                v[i - k] = i;
                c[i - k] = lcg(&s) % k;
            }
            want_ok("c3_join", call("c3_join", 3, A(sim, u32s(v, hi - k), u32s(c, hi - k))));
            want_ok_tuple("c3_step", call("c3_step", 2, A(sim, mock_uint(3))));
            free(v);
            free(c);
        }
        want_ok_tuple("c3_heartbeat", call("c3_heartbeat", 2, A(sim, mock_uint(0))));
        ERL_NIF_TERM st = mock_elem(want_ok_tuple("c3_step", call("c3_step", 2, A(sim, mock_uint(10)))), 1);
        uint64_t dl = 0, live = 0;
        ERL_NIF_TERM last = mock_elem(mock_list_nth(st, 9), 0);
        mock_map_get(last, "delivered_live", &dl);
        mock_map_get(last, "live", &live);
        uint32_t crash[20];
        for (int i = 0; i < 20; i++) crash[i] = 100 + 17 * i;
        want_ok("c3_crash", call("c3_crash", 2, A(sim, u32s(crash, 20))));
        want_ok_tuple("c3_step", call("c3_step", 2, A(sim, mock_uint(2))));
        /* c3_run: 3 rounds in one call -- round 0 a heartbeat and a crash list, round 1 those vertices rejoin */
        uint32_t coff[4] = {0, 10, 10, 10}, joff[4] = {0, 0, 10, 10}, cv[10], jv[10], jc[10];
        for (int i = 0; i < 10; i++) { cv[i] = jv[i] = 1000 + 31 * i; jc[i] = 7; }
        ERL_NIF_TERM rs = mock_elem(want_ok_tuple("c3_run", call("c3_run", 8, A(sim, u32s(coff, 4), u32s(cv, 10),
                                                                                 u32s(joff, 4), u32s(jv, 10), u32s(jc, 10),
                                                                                 mock_uint(3), mock_uint(0)))), 1);
        uint64_t run_live = 0;
        mock_map_get(mock_elem(mock_list_nth(rs, 2), 0), "live", &run_live);
        fprintf(g_out, ", \"c3\": {\"n\": %u, \"delivered_live\": %llu, \"live\": %llu, \"run_rounds\": %zu, "
                "\"run_live\": %llu}", n, (unsigned long long)dl, (unsigned long long)live, mock_list_len(rs),
                (unsigned long long)run_live);
    }
    /* ---- causal delivery ------------------------------------------------------ */
    {
        ERL_NIF_TERM sim = new_sim(0x5EED0005ull);
        want_ok("causal_setup", call("causal_setup", 6, A(sim, mock_uint(1000), mock_uint(8), mock_uint(1), mock_uint(2),
                                                          mock_uint(1))));
        ERL_NIF_TERM st = mock_elem(want_ok_tuple("causal_step", call("causal_step", 2, A(sim, mock_uint(10)))), 1);
        uint64_t delivered = 0, x;
        for (size_t i = 0; i < mock_list_len(st); i++)
            if (mock_map_get(mock_list_nth(st, i), "delivered", &x)) delivered += x;
        want_ok_tuple("causal_clocks", call("causal_clocks", 1, A(sim)));
        fprintf(g_out, ", \"causal\": {\"n\": 1000, \"delivered\": %llu}", (unsigned long long)delivered);
    }
    /* ---- causal delivery sharded at world 1 over the library's RCCL communicator */
    {
        ERL_NIF_TERM sim = new_sim(0x5EED0005ull);
        ERL_NIF_TERM id = mock_elem(want_ok_tuple("rccl_unique_id", call("rccl_unique_id", 0, A(0))), 1);
        want_ok("shard_init_rccl", call("shard_init_rccl", 4, A(sim, mock_uint(0), mock_uint(1), id)));
        want_ok_tuple("causal_shard_setup", call("causal_shard_setup", 8, A(sim, mock_uint(1000), mock_uint(8),
                                                                              mock_uint(1), mock_uint(2), mock_uint(1),
                                                                              mock_uint(0), mock_uint(1))));
        ERL_NIF_TERM st = mock_elem(want_ok_tuple("causal_shard_step", call("causal_shard_step", 2, A(sim, mock_uint(10)))), 1);
        uint64_t delivered = 0, x;
        for (size_t i = 0; i < mock_list_len(st); i++)
            if (mock_map_get(mock_list_nth(st, i), "delivered", &x)) delivered += x;
        fprintf(g_out, ", \"causal_shard_rccl_world1\": {\"delivered\": %llu}", (unsigned long long)delivered);
    }
    /* ---- vclock merge on dense lanes ------------------------------------------ */
    {
        ERL_NIF_TERM sim = new_sim(1);
        uint32_t a[64] = {0}, b[64] = {0};
        a[0] = 3; a[5] = 1; b[0] = 1; b[7] = 4;
        ERL_NIF_TERM m = want_ok_tuple("vclock", call("vclock", 4, A(sim, mock_atom("merge"), u32s(a, 64), u32s(b, 64))));
        size_t sz;
        const uint32_t* o = (const uint32_t*)mock_bin_data(mock_elem(m, 1), &sz);
        fprintf(g_out, ", \"vclock_merge\": [%u, %u, %u]", o[0], o[5], o[7]);
    }
    fprintf(g_out, "}\n");
    if (g_out != stdout) fclose(g_out);
    mock_drop_terms();      /* resource destructors: psim_destroy on every handle */
    return 0;
}
