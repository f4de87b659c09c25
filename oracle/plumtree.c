/*
 * plumtree.c -- round-synchronous restatement of
 *   src/partisan_plumtree_broadcast.erl  (gen_server, protocol 487-1328)
 *   src/partisan_plumtree_backend.erl    (heartbeat handler 180-417)
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  This is the checker the HIP
 * path (partisan_amd/csrc/plumtree.hip) is compared against; it is written
 * independently of the kernel, in the reference's own data model:
 * ordsets, a map Root -> ordset for eager/lazy sets, the outstanding ETS
 * duplicate_bag as an insertion-ordered row list, and the backend's
 * per-origin {Epoch, IntervalSet} table.
 *
 * Schedule (DESIGN.md "Schedule"; one admissible interleaving of the
 * asynchronous reference, which only guarantees per-pair FIFO):
 *   - round t delivers every message emitted in round t-1 (or by an API
 *     call made between rounds t-1 and t);
 *   - a vertex processes its inbox sorted by (src id, src emission seq);
 *   - after all inboxes, each live vertex fires its lazy tick when
 *     t % lazy_tick_rounds == 0 (handle_info(lazy_tick), :646-649);
 *   - messages to a dead vertex are dropped; dead vertices do nothing.
 * The exchange tick (:651-654) only consumes draws of the plumtree
 * process's UNSEEDED rand state and calls the backend's
 * exchange/1, which returns `ignore` (backend:292-293); it has no
 * observable effect and is not simulated.
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>

/* ---------------- ordsets of u32 (term order == id order) --- */
typedef struct { uint32_t* a; uint32_t n, cap; } oset;

static void os_free(oset* s) { free(s->a); s->a = NULL; s->n = s->cap = 0; }
static void os_reserve(oset* s, uint32_t c) {
    if (c <= s->cap) return;
    uint32_t nc = s->cap ? s->cap * 2 : 4;
    while (nc < c) nc *= 2;
    s->a = (uint32_t*)realloc(s->a, nc * sizeof(uint32_t));
    s->cap = nc;
}
static void os_copy(oset* d, const oset* s) { d->n = 0; os_reserve(d, s->n); memcpy(d->a, s->a, s->n * sizeof(uint32_t)); d->n = s->n; }
static int os_find(const oset* s, uint32_t x, uint32_t* pos) {
    uint32_t lo = 0, hi = s->n;
    while (lo < hi) { uint32_t m = (lo + hi) / 2; if (s->a[m] < x) lo = m + 1; else hi = m; }
    *pos = lo;
    return lo < s->n && s->a[lo] == x;
}
static int os_member(const oset* s, uint32_t x) { uint32_t p; return os_find(s, x, &p); }
/* ordsets:add_element/2 */
static void os_add(oset* s, uint32_t x) {
    uint32_t p;
    if (os_find(s, x, &p)) return;
    os_reserve(s, s->n + 1);
    memmove(&s->a[p + 1], &s->a[p], (s->n - p) * sizeof(uint32_t));
    s->a[p] = x; s->n++;
}
/* ordsets:del_element/2 */
static void os_del(oset* s, uint32_t x) {
    uint32_t p;
    if (!os_find(s, x, &p)) return;
    memmove(&s->a[p], &s->a[p + 1], (s->n - p - 1) * sizeof(uint32_t));
    s->n--;
}
/* ordsets:subtract/2 in place */
static void os_subtract(oset* s, const oset* r) {
    uint32_t k = 0;
    for (uint32_t i = 0; i < s->n; i++) if (!os_member(r, s->a[i])) s->a[k++] = s->a[i];
    s->n = k;
}
/* ordsets:union/2 in place */
static void os_union(oset* s, const oset* r) { for (uint32_t i = 0; i < r->n; i++) os_add(s, r->a[i]); }

/* ---------------- maps Root -> ordset ----------------------------------- */
typedef struct { uint32_t root; oset s; } rootset;
typedef struct { rootset* e; uint32_t n, cap; } rootmap;

static oset* rm_find(rootmap* m, uint32_t root) {
    for (uint32_t i = 0; i < m->n; i++) if (m->e[i].root == root) return &m->e[i].s;
    return NULL;
}
static void rm_clear(rootmap* m) { for (uint32_t i = 0; i < m->n; i++) os_free(&m->e[i].s); m->n = 0; }
/* maps:put(Root, Set, Map) */
static void rm_put(rootmap* m, uint32_t root, const oset* s) {
    oset* d = rm_find(m, root);
    if (!d) {
        if (m->n == m->cap) { m->cap = m->cap ? m->cap * 2 : 2; m->e = (rootset*)realloc(m->e, m->cap * sizeof(rootset)); }
        m->e[m->n].root = root; memset(&m->e[m->n].s, 0, sizeof(oset));
        d = &m->e[m->n].s; m->n++;
    }
    os_copy(d, s);
}

/* ---------------- outstanding ETS duplicate_bag ------------------------- */
typedef struct { uint32_t peer, id_node, id_epoch, id_mono, round, root; } outrow;

/* ---------------- backend ETS {Node, Epoch, ISet} ------------------------ */
typedef struct { uint32_t node, epoch; orc_iel* is; size_t n, cap; } tsrow;
typedef struct { uint32_t node, epoch, mono, round; } recvrec;   /* instrumentation only */

typedef struct {
    oset all_members, common_eagers, common_lazys;
    rootmap eager_sets, lazy_sets;
    outrow* out; size_t nout, capout;
    tsrow* ts; size_t nts, capts;
    recvrec* rr; size_t nrr, caprr;
    uint32_t hb_epoch, hb_monotonic;      /* backend #state{epoch, monotonic} */
    uint64_t seq;                         /* emission counter (FIFO order)    */
    uint32_t* upd; size_t nupd, capupd;   /* queued {update, Members}: [len, ids...] records */
    uint8_t fresh;                        /* restarted since the last round: inbox dropped */
} node_t;

struct orc_plumtree {
    uint32_t n, lazy_tick_rounds;
    uint64_t round;                        /* rounds completed */
    node_t* nodes;
    uint8_t* alive;
    orc_msg* cur; size_t ncur, capcur;    /* being processed this round */
    orc_msg* nxt; size_t nnxt, capnxt;    /* emitted, delivered next round */
    orc_round_stats* st;                   /* stats of the running round */
    orc_pt_conn_fn conn;                   /* partisan:cast_message needs a connection (C3) */
    void* conn_ctx;
    uint64_t dropped;                      /* sends to a non-connected peer */
    uint64_t* omit; size_t nomit;          /* omission faults: sorted (src << 32 | dst) keys */
    uint64_t omitted;                      /* messages they dropped */
    uint64_t* dkey; uint8_t* dval; size_t ndly;   /* delay faults: sorted (src << 32 | dst) -> rounds */
    orc_msg* dq; uint64_t* dqa; size_t ndq, capdq; /* delayed messages and their arrival rounds */
    uint64_t emit_round;                   /* the round whose emissions are being made (0: before round 1) */
};

void orc_pt_set_conn(orc_plumtree* s, orc_pt_conn_fn fn, void* ctx) { s->conn = fn; s->conn_ctx = ctx; }
uint64_t orc_pt_dropped(const orc_plumtree* s) { return s->dropped; }

static int cmp_u64(const void* x, const void* y) {
    const uint64_t a = *(const uint64_t*)x, b = *(const uint64_t*)y;
    return a < b ? -1 : a > b;
}
/* Send / receive omission faults (test/prop_partisan_crash_fault_model.erl
 * :117-196): an interposition fun in the manager's forward_message (sender
 * side) or receive_message (receiver side) path returns undefined for the
 * directed pair, so the message is sent -- counted, the sender's state moves
 * on -- and lost.  Replaces the whole set; k = 0 heals every fault. */
void orc_pt_set_omissions(orc_plumtree* s, const uint32_t* src, const uint32_t* dst, size_t k) {
    free(s->omit);
    s->omit = NULL;
    s->nomit = 0;
    if (!k) return;
    s->omit = (uint64_t*)malloc(k * sizeof(uint64_t));
    for (size_t i = 0; i < k; i++) s->omit[i] = ((uint64_t)src[i] << 32) | dst[i];
    qsort(s->omit, k, sizeof(uint64_t), cmp_u64);
    s->nomit = k;
}
uint64_t orc_pt_omitted(const orc_plumtree* s) { return s->omitted; }

/* Delay faults (test/partisan_SUITE.erl groups with_egress_delay /
 * with_ingress_delay; partisan_peer_service_client.erl:148-176 sleeps
 * egress_delay ms before each send, partisan_peer_service_server.erl the
 * same on receipt): in rounds, a message emitted in round t over the
 * directed pair (src, dst) with delay d is delivered in round t + 1 + d
 * instead of t + 1.  A fixed per-pair delay keeps every pair FIFO, which is
 * all the reference guarantees.  Replaces the whole set (k = 0: no delays);
 * refused with ORC_BADARG while any message is in flight, as a change could
 * reorder a pair's messages. */
int orc_pt_set_delays(orc_plumtree* s, const uint32_t* src, const uint32_t* dst, const uint8_t* d, size_t k) {
    if (s->nnxt || s->ndq) return ORC_BADARG;
    free(s->dkey); free(s->dval);
    s->dkey = NULL; s->dval = NULL; s->ndly = 0;
    if (!k) return ORC_OK;
    uint64_t* kv = (uint64_t*)malloc(k * sizeof(uint64_t));   /* key << 8 | delay, sorted by key */
    for (size_t i = 0; i < k; i++) kv[i] = ((((uint64_t)src[i] << 32) | dst[i]) << 8) | d[i];
    qsort(kv, k, sizeof(uint64_t), cmp_u64);
    s->dkey = (uint64_t*)malloc(k * sizeof(uint64_t));
    s->dval = (uint8_t*)malloc(k);
    for (size_t i = 0; i < k; i++) {           /* a repeated pair: the last listed wins */
        const uint64_t key = kv[i] >> 8;
        if (s->ndly && s->dkey[s->ndly - 1] == key) { s->dval[s->ndly - 1] = (uint8_t)kv[i]; continue; }
        s->dkey[s->ndly] = key; s->dval[s->ndly] = (uint8_t)kv[i]; s->ndly++;
    }
    free(kv);
    return ORC_OK;
}
static uint32_t delay_of(const orc_plumtree* s, uint32_t src, uint32_t dst) {
    if (!s->ndly) return 0;
    const uint64_t key = ((uint64_t)src << 32) | dst;
    size_t lo = 0, hi = s->ndly;
    while (lo < hi) { size_t m = (lo + hi) / 2; if (s->dkey[m] < key) lo = m + 1; else hi = m; }
    return lo < s->ndly && s->dkey[lo] == key ? s->dval[lo] : 0;
}
/* messages in flight: delivered next round + delayed beyond it */
uint64_t orc_pt_inflight(const orc_plumtree* s) { return s->nnxt + s->ndq; }

static int omitted(const orc_plumtree* s, uint32_t src, uint32_t dst) {
    if (!s->nomit) return 0;
    const uint64_t key = ((uint64_t)src << 32) | dst;
    return bsearch(&key, s->omit, s->nomit, sizeof(uint64_t), cmp_u64) != NULL;
}

/* ---------------- message emission: partisan:cast_message via send/3 ---- */
static void emit(orc_plumtree* s, uint32_t src, uint32_t dst, uint32_t type,
                 uint32_t round, uint32_t root, uint32_t idn, uint32_t ide, uint32_t idm) {
    if (s->conn && !s->conn(s->conn_ctx, src, dst)) {    /* do_send_message: no connection, dropped */
        s->dropped++;
        return;
    }
    if (omitted(s, src, dst)) {                         /* interposition: sent, then lost */
        s->nodes[src].seq++;
        if (s->st) s->st->sent[type]++;
        s->omitted++;
        return;
    }
    const uint32_t d = delay_of(s, src, dst);
    orc_msg* m;
    if (d) {                                             /* delivered in round emit_round + 1 + d */
        if (s->ndq == s->capdq) {
            s->capdq = s->capdq ? s->capdq * 2 : 1024;
            s->dq = (orc_msg*)realloc(s->dq, s->capdq * sizeof(orc_msg));
            s->dqa = (uint64_t*)realloc(s->dqa, s->capdq * sizeof(uint64_t));
        }
        s->dqa[s->ndq] = s->emit_round + 1 + d;
        m = &s->dq[s->ndq++];
    } else {
        if (s->nnxt == s->capnxt) { s->capnxt = s->capnxt ? s->capnxt * 2 : 1024; s->nxt = (orc_msg*)realloc(s->nxt, s->capnxt * sizeof(orc_msg)); }
        m = &s->nxt[s->nnxt++];
    }
    m->type = type; m->src = src; m->dst = dst; m->round = round; m->root = root;
    m->id_node = idn; m->id_epoch = ide; m->id_mono = idm;
    m->seq = s->nodes[src].seq++;
    if (s->st) s->st->sent[type]++;
}

/* ---------------- heartbeat backend (partisan_plumtree_backend.erl) ------ */
static tsrow* ts_lookup(node_t* nd, uint32_t origin) {
    for (size_t i = 0; i < nd->nts; i++) if (nd->ts[i].node == origin) return &nd->ts[i];
    return NULL;
}
static void ts_set_single(tsrow* r, uint32_t epoch, uint32_t mono) {
    /* partisan_interval_sets:from_list([Monotonic]) */
    orc_iel e = {mono, mono, 0, 0};
    if (r->cap < 1) { r->cap = 4; r->is = (orc_iel*)realloc(r->is, r->cap * sizeof(orc_iel)); }
    size_t k;
    orc_iset_from_list(&e, 1, r->is, r->cap, &k);
    r->n = k; r->epoch = epoch;
}
/* add_timestamp/1 (:400-417) */
static void add_timestamp(node_t* nd, uint32_t origin, uint32_t epoch, uint32_t mono) {
    tsrow* r = ts_lookup(nd, origin);
    if (!r) {
        if (nd->nts == nd->capts) { nd->capts = nd->capts ? nd->capts * 2 : 2; nd->ts = (tsrow*)realloc(nd->ts, nd->capts * sizeof(tsrow)); }
        r = &nd->ts[nd->nts++];
        memset(r, 0, sizeof(*r)); r->node = origin;
        ts_set_single(r, epoch, mono);
    } else if (r->epoch < epoch) {
        ts_set_single(r, epoch, mono);
    } else if (r->epoch == epoch) {
        orc_iel e = {mono, mono, 0, 0};
        size_t cap = r->n + 2, k;
        orc_iel* o = (orc_iel*)malloc(cap * sizeof(orc_iel));
        orc_iset_add_element(&e, r->is, r->n, o, cap, &k);
        if (r->cap < k) { r->cap = cap; r->is = (orc_iel*)realloc(r->is, r->cap * sizeof(orc_iel)); }
        memcpy(r->is, o, k * sizeof(orc_iel)); r->n = k;
        free(o);
    } /* Epoch0 > Epoch: old message, ignored */
}
/* is_stale/1 (:229-244) */
static int is_stale(node_t* nd, uint32_t origin, uint32_t epoch, uint32_t mono) {
    tsrow* r = ts_lookup(nd, origin);
    if (!r) return 0;
    if (r->epoch == epoch) { orc_iel e = {mono, mono, 0, 0}; return orc_iset_is_element(&e, r->is, r->n) == 1; }
    return r->epoch > epoch;
}
/* merge/2 (:205-215): not stale -> add_timestamp, true */
static int backend_merge(node_t* nd, uint32_t origin, uint32_t epoch, uint32_t mono) {
    if (is_stale(nd, origin, epoch, mono)) return 0;
    add_timestamp(nd, origin, epoch, mono);
    return 1;
}
/* graft/1 (:254-280): 0 = {ok, M}, 1 = stale, 2 = {error, not_found} */
static int backend_graft(node_t* nd, uint32_t origin, uint32_t epoch, uint32_t mono) {
    tsrow* r = ts_lookup(nd, origin);
    if (!r) return 2;
    if (r->epoch == epoch) { orc_iel e = {mono, mono, 0, 0}; return orc_iset_is_element(&e, r->is, r->n) == 1 ? 0 : 2; }
    if (r->epoch > epoch) return 1;
    return 2;
}

/* ---------------- plumtree state helpers (:1207-1328) -------------------- */
/* all_peers/3 (:1278-1282) */
static const oset* all_peers(node_t* nd, uint32_t root, int lazy) {
    oset* s = rm_find(lazy ? &nd->lazy_sets : &nd->eager_sets, root);
    return s ? s : (lazy ? &nd->common_lazys : &nd->common_eagers);
}
/* update_peers/5 + set_peers/4 (:1233-1248); add_eager/add_lazy (:1223-1229) */
static void update_peers(node_t* nd, uint32_t from, uint32_t root, int to_lazy) {
    oset e = {0}, l = {0};
    os_copy(&e, all_peers(nd, root, 0));
    os_copy(&l, all_peers(nd, root, 1));
    if (to_lazy) { os_del(&e, from); os_add(&l, from); }
    else { os_add(&e, from); os_del(&l, from); }
    rm_put(&nd->eager_sets, root, &e);
    rm_put(&nd->lazy_sets, root, &l);
    os_free(&e); os_free(&l);
}
/* add_all_outstanding/5 (:1215-1219) */
static void add_outstanding(node_t* nd, uint32_t peer, uint32_t idn, uint32_t ide, uint32_t idm,
                            uint32_t round, uint32_t root) {
    if (nd->nout == nd->capout) { nd->capout = nd->capout ? nd->capout * 2 : 4; nd->out = (outrow*)realloc(nd->out, nd->capout * sizeof(outrow)); }
    outrow* r = &nd->out[nd->nout++];
    r->peer = peer; r->id_node = idn; r->id_epoch = ide; r->id_mono = idm; r->round = round; r->root = root;
}
/* ack_outstanding/5 (:1207-1211): ets:delete_object removes every identical row (Q26) */
static void ack_outstanding(node_t* nd, uint32_t idn, uint32_t ide, uint32_t idm,
                            uint32_t round, uint32_t root, uint32_t from) {
    size_t k = 0;
    for (size_t i = 0; i < nd->nout; i++) {
        outrow* r = &nd->out[i];
        int match = r->peer == from && r->id_node == idn && r->id_epoch == ide && r->id_mono == idm &&
                    r->round == round && r->root == root;
        if (!match) nd->out[k++] = *r;
    }
    nd->nout = k;
}
/* eager_push/7 (:962-970): send to eager_peers(Root, From) = all eagers -- From */
static void eager_push(orc_plumtree* s, uint32_t v, uint32_t idn, uint32_t ide, uint32_t idm,
                       uint32_t round, uint32_t root, uint32_t from) {
    node_t* nd = &s->nodes[v];
    const oset* e = all_peers(nd, root, 0);
    for (uint32_t i = 0; i < e->n; i++)
        if (e->a[i] != from) emit(s, v, e->a[i], ORC_MSG_BROADCAST, round, root, idn, ide, idm);
}
/* schedule_lazy_push/6 (:974-988) */
static void schedule_lazy_push(orc_plumtree* s, uint32_t v, uint32_t idn, uint32_t ide, uint32_t idm,
                               uint32_t round, uint32_t root, uint32_t from) {
    node_t* nd = &s->nodes[v];
    const oset* l = all_peers(nd, root, 1);
    for (uint32_t i = 0; i < l->n; i++)
        if (l->a[i] != from) add_outstanding(nd, l->a[i], idn, ide, idm, round, root);
}
/* reset_peers/4 (:1320-1328) */
static void reset_peers(node_t* nd, uint32_t self, const oset* all, const oset* eagers, const oset* lazys) {
    os_copy(&nd->common_eagers, eagers); os_del(&nd->common_eagers, self);
    os_copy(&nd->common_lazys, lazys); os_del(&nd->common_lazys, self);
    rm_clear(&nd->eager_sets);
    rm_clear(&nd->lazy_sets);
    os_copy(&nd->all_members, all);
}

/* ---------------- handle_cast clauses (:565-639) ------------------------ */
static void handle(orc_plumtree* s, uint32_t v, const orc_msg* m) {
    node_t* nd = &s->nodes[v];
    switch (m->type) {
    case ORC_MSG_BROADCAST: {                       /* :571-578 -> handle_broadcast/8 :843-857 */
        int valid = backend_merge(nd, m->id_node, m->id_epoch, m->id_mono);
        if (!valid) {
            update_peers(nd, m->src, m->root, 1);    /* add_lazy(From, Root) */
            emit(s, v, m->src, ORC_MSG_PRUNE, 0, m->root, 0, 0, 0);
        } else {
            if (s->st) s->st->delivered_new++;
            if (nd->nrr == nd->caprr) { nd->caprr = nd->caprr ? nd->caprr * 2 : 2; nd->rr = (recvrec*)realloc(nd->rr, nd->caprr * sizeof(recvrec)); }
            nd->rr[nd->nrr].node = m->id_node; nd->rr[nd->nrr].epoch = m->id_epoch; nd->rr[nd->nrr].mono = m->id_mono;
            nd->rr[nd->nrr].round = m->round; nd->nrr++;
            update_peers(nd, m->src, m->root, 0);    /* add_eager(From, Root) */
            eager_push(s, v, m->id_node, m->id_epoch, m->id_mono, m->round + 1, m->root, m->src);
            schedule_lazy_push(s, v, m->id_node, m->id_epoch, m->id_mono, m->round + 1, m->root, m->src);
        }
        break;
    }
    case ORC_MSG_PRUNE:                             /* :580-584 */
        update_peers(nd, m->src, m->root, 1);
        break;
    case ORC_MSG_IHAVE: {                           /* :586-590 -> handle_ihave/7 :861-876 */
        int stale = is_stale(nd, m->id_node, m->id_epoch, m->id_mono);
        if (stale) {
            emit(s, v, m->src, ORC_MSG_IGNORED, m->round, m->root, m->id_node, m->id_epoch, m->id_mono);
        } else {
            emit(s, v, m->src, ORC_MSG_GRAFT, m->round, m->root, m->id_node, m->id_epoch, m->id_mono);
            update_peers(nd, m->src, m->root, 0);
        }
        break;
    }
    case ORC_MSG_IGNORED:                           /* :592-598 */
        ack_outstanding(nd, m->id_node, m->id_epoch, m->id_mono, m->round, m->root, m->src);
        break;
    case ORC_MSG_GRAFT: {                           /* :600-605 -> handle_graft/7 :880-906 */
        int r = backend_graft(nd, m->id_node, m->id_epoch, m->id_mono);
        if (r == 1) {
            ack_outstanding(nd, m->id_node, m->id_epoch, m->id_mono, m->round, m->root, m->src);
        } else if (r == 0) {
            update_peers(nd, m->src, m->root, 0);
            emit(s, v, m->src, ORC_MSG_BROADCAST, m->round, m->root, m->id_node, m->id_epoch, m->id_mono);
        } /* {error, _}: logged only */
        break;
    }
    default: break;
    }
}

/* send_lazy/0 (:992-1019): every outstanding row, to connected peers; rows persist */
static void send_lazy(orc_plumtree* s, uint32_t v) {
    node_t* nd = &s->nodes[v];
    for (size_t i = 0; i < nd->nout; i++) {
        outrow r = nd->out[i];
        if (!s->alive[r.peer]) continue;           /* partisan:is_connected(Peer) (Q5, Q30) */
        if (s->conn && !s->conn(s->conn_ctx, v, r.peer)) continue;
        emit(s, v, r.peer, ORC_MSG_IHAVE, r.round, r.root, r.id_node, r.id_epoch, r.id_mono);
    }
}

/* ---------------- public API -------------------------------------------- */
orc_plumtree* orc_pt_create(uint32_t n, const uint64_t* row_ptr, const uint32_t* col, uint32_t lazy_tick_rounds) {
    orc_plumtree* s = (orc_plumtree*)calloc(1, sizeof(*s));
    s->n = n;
    s->lazy_tick_rounds = lazy_tick_rounds ? lazy_tick_rounds : 1;
    s->nodes = (node_t*)calloc(n, sizeof(node_t));
    s->alive = (uint8_t*)malloc(n);
    memset(s->alive, 1, n);
    for (uint32_t v = 0; v < n; v++) {
        /* start_link/0 (:234-260): InitEagers = Members, InitLazys = [];
         * init/1 (:487-515) -> reset_peers(AllMembers, InitEagers, InitLazys) */
        oset members = {0}, empty = {0};
        for (uint64_t e = row_ptr[v]; e < row_ptr[v + 1]; e++) os_add(&members, col[e]);
        os_add(&members, v);                        /* the peer service lists self too (Q29) */
        reset_peers(&s->nodes[v], v, &members, &members, &empty);
        os_free(&members);
    }
    return s;
}

void orc_pt_destroy(orc_plumtree* s) {
    if (!s) return;
    free(s->omit); free(s->dkey); free(s->dval); free(s->dq); free(s->dqa);
    for (uint32_t v = 0; v < s->n; v++) {
        node_t* nd = &s->nodes[v];
        os_free(&nd->all_members); os_free(&nd->common_eagers); os_free(&nd->common_lazys);
        rm_clear(&nd->eager_sets); rm_clear(&nd->lazy_sets);
        free(nd->eager_sets.e); free(nd->lazy_sets.e);
        free(nd->out);
        for (size_t i = 0; i < nd->nts; i++) free(nd->ts[i].is);
        free(nd->ts); free(nd->rr); free(nd->upd);
    }
    free(s->nodes); free(s->alive); free(s->cur); free(s->nxt);
    free(s);
}

void orc_pt_set_alive(orc_plumtree* s, const uint8_t* alive) { memcpy(s->alive, alive, s->n); }

/* handle_info(heartbeat) in the backend (:341-368) followed by the plumtree
 * cast {broadcast, Id, Payload, Mod} (:565-569): eager_push/4 + schedule_lazy_push/3
 * with Round = 0, Root = From = node().  Runs between rounds. */
uint32_t orc_pt_heartbeat(orc_plumtree* s, uint32_t root) {
    node_t* nd = &s->nodes[root];
    uint32_t mono = ++nd->hb_monotonic;
    add_timestamp(nd, root, nd->hb_epoch, mono);
    if (nd->nrr == nd->caprr) { nd->caprr = nd->caprr ? nd->caprr * 2 : 2; nd->rr = (recvrec*)realloc(nd->rr, nd->caprr * sizeof(recvrec)); }
    nd->rr[nd->nrr].node = root; nd->rr[nd->nrr].epoch = nd->hb_epoch; nd->rr[nd->nrr].mono = mono;
    nd->rr[nd->nrr].round = 0xFFFFFFFEu; nd->nrr++;
    orc_round_stats* saved = s->st; s->st = NULL;
    eager_push(s, root, root, nd->hb_epoch, mono, 0, root, root);
    schedule_lazy_push(s, root, root, nd->hb_epoch, mono, 0, root, root);
    s->st = saved;
    return mono;
}

/* handle_cast({update, MemberList}) (:607-639) + neighbors_down/2 (:910-951) */
int orc_pt_update(orc_plumtree* s, uint32_t v, const uint32_t* members, size_t n) {
    node_t* nd = &s->nodes[v];
    oset m = {0}, nw = {0}, removed = {0};
    for (size_t i = 0; i < n; i++) os_add(&m, members[i]);
    os_copy(&nw, &m); os_subtract(&nw, &nd->all_members);
    os_copy(&removed, &nd->all_members); os_subtract(&removed, &m);
    if (nw.n > 0) {
        oset eag = {0}, laz = {0};
        os_copy(&eag, &nd->common_eagers); os_union(&eag, &nw);
        os_copy(&laz, &nd->common_lazys);
        reset_peers(nd, v, &m, &eag, &laz);
        os_free(&eag); os_free(&laz);
    }
    /* neighbors_down(Removed, State1) */
    os_subtract(&nd->all_members, &removed);
    os_subtract(&nd->common_eagers, &removed);
    os_subtract(&nd->common_lazys, &removed);
    for (uint32_t i = 0; i < nd->eager_sets.n; i++) os_subtract(&nd->eager_sets.e[i].s, &removed);
    for (uint32_t i = 0; i < nd->lazy_sets.n; i++) os_subtract(&nd->lazy_sets.e[i].s, &removed);
    size_t k = 0;                                    /* ets:delete(?PLUMTREE_OUTSTANDING, Peer) */
    for (size_t i = 0; i < nd->nout; i++) if (!os_member(&removed, nd->out[i].peer)) nd->out[k++] = nd->out[i];
    nd->nout = k;
    os_free(&m); os_free(&nw); os_free(&removed);
    return 0;
}

/* crash + restart: start_link/0 with the peer service's members = {self};
 * the backend's timestamp table is lost (a new node) */
void orc_pt_restart(orc_plumtree* s, uint32_t v) {
    node_t* nd = &s->nodes[v];
    oset self = {0}, empty = {0};
    os_add(&self, v);
    reset_peers(nd, v, &self, &self, &empty);
    os_free(&self);
    nd->nout = 0;
    for (size_t i = 0; i < nd->nts; i++) free(nd->ts[i].is);
    nd->nts = 0;
    nd->nrr = 0;
    nd->nupd = 0;
    nd->fresh = 1;
}

/* The heartbeat backend of v restarts (its gen_server crashes and the
 * supervisor starts it again, backend init/1 :316-329): a newer epoch
 * (erlang:system_time() at init: later than every earlier one), Monotonic 0,
 * and a new ETS table -- v forgets every origin's timestamps.  The
 * plumtree server keeps its state.  recv records are instrumentation of the
 * table, so they go with it. */
void orc_pt_restart_backend(orc_plumtree* s, uint32_t v) {
    node_t* nd = &s->nodes[v];
    nd->hb_epoch++;
    nd->hb_monotonic = 0;
    for (size_t i = 0; i < nd->nts; i++) free(nd->ts[i].is);
    nd->nts = 0;
    nd->nrr = 0;
}
uint32_t orc_pt_epoch(const orc_plumtree* s, uint32_t v) { return s->nodes[v].hb_epoch; }

void orc_pt_queue_update(orc_plumtree* s, uint32_t v, const uint32_t* members, size_t n) {
    node_t* nd = &s->nodes[v];
    if (nd->nupd + n + 1 > nd->capupd) {
        nd->capupd = (nd->nupd + n + 1) * 2;
        nd->upd = (uint32_t*)realloc(nd->upd, nd->capupd * 4);
    }
    nd->upd[nd->nupd++] = (uint32_t)n;
    memcpy(nd->upd + nd->nupd, members, n * 4);
    nd->nupd += n;
}

void orc_pt_reset_peers_all(orc_plumtree* s) {
    for (uint32_t v = 0; v < s->n; v++) {
        node_t* nd = &s->nodes[v];
        oset all = {0}, e = {0}, l = {0};
        os_copy(&all, &nd->all_members); os_copy(&e, &nd->common_eagers); os_copy(&l, &nd->common_lazys);
        reset_peers(nd, v, &all, &e, &l);
        os_free(&all); os_free(&e); os_free(&l);
    }
}

static int msg_cmp(const void* x, const void* y) {
    const orc_msg* a = (const orc_msg*)x; const orc_msg* b = (const orc_msg*)y;
    if (a->dst != b->dst) return a->dst < b->dst ? -1 : 1;
    if (a->src != b->src) return a->src < b->src ? -1 : 1;
    if (a->seq != b->seq) return a->seq < b->seq ? -1 : 1;
    return 0;
}

static void one_round(orc_plumtree* s, orc_round_stats* st) {
    memset(st, 0, sizeof(*st));
    s->st = st;
    /* swap: cur <- nxt */
    orc_msg* t = s->cur; size_t tc = s->capcur;
    s->cur = s->nxt; s->ncur = s->nnxt; s->capcur = s->capnxt;
    s->nxt = t; s->nnxt = 0; s->capnxt = tc;
    s->emit_round = s->round + 1;
    {                                                   /* delayed messages due this round */
        size_t k = 0;
        for (size_t i = 0; i < s->ndq; i++) {
            if (s->dqa[i] == s->emit_round) {
                if (s->ncur == s->capcur) { s->capcur = s->capcur ? s->capcur * 2 : 1024; s->cur = (orc_msg*)realloc(s->cur, s->capcur * sizeof(orc_msg)); }
                s->cur[s->ncur++] = s->dq[i];
            } else {
                s->dq[k] = s->dq[i]; s->dqa[k] = s->dqa[i]; k++;
            }
        }
        s->ndq = k;
    }
    qsort(s->cur, s->ncur, sizeof(orc_msg), msg_cmp);
    /* {update, Members} casts queued since the last round, in order (C3) */
    for (uint32_t v = 0; v < s->n; v++) {
        node_t* nd = &s->nodes[v];
        size_t i = 0;
        while (i < nd->nupd) {
            const uint32_t k = nd->upd[i];
            if (s->alive[v]) orc_pt_update(s, v, nd->upd + i + 1, k);
            i += 1 + k;
        }
        nd->nupd = 0;
    }
    uint64_t maxe = 0, run = 0;
    uint32_t last_dst = 0xFFFFFFFFu;
    for (size_t i = 0; i < s->ncur; i++) {
        const orc_msg* m = &s->cur[i];
        if (i > 0 && s->cur[i - 1].dst == m->dst && s->cur[i - 1].src == m->src) run++; else run = 1;
        if (run > maxe) maxe = run;
        if (!s->alive[m->dst] || s->nodes[m->dst].fresh) continue;   /* lost on the wire */
        if (m->dst != last_dst) { st->active++; last_dst = m->dst; }
        handle(s, m->dst, m);
    }
    for (uint32_t v = 0; v < s->n; v++) s->nodes[v].fresh = 0;
    s->round++;
    if (s->round % s->lazy_tick_rounds == 0) {      /* handle_info(lazy_tick) */
        for (uint32_t v = 0; v < s->n; v++) {
            if (!s->alive[v] || s->nodes[v].nout == 0) continue;
            send_lazy(s, v);
        }
    }
    uint64_t outst = 0, live = 0;
    for (uint32_t v = 0; v < s->n; v++) {
        outst += s->nodes[v].nout;
        for (size_t i = 0; i < s->nodes[v].nout; i++) live += s->alive[s->nodes[v].out[i].peer] && s->alive[v];
    }
    st->outstanding = outst;
    st->outstanding_live = live;
    st->max_per_edge = maxe;
    s->st = NULL;
}

uint32_t orc_pt_step(orc_plumtree* s, uint32_t rounds, orc_round_stats* stats) {
    for (uint32_t r = 0; r < rounds; r++) one_round(s, &stats[r]);
    return rounds;
}

uint32_t orc_pt_run(orc_plumtree* s, uint32_t max_rounds, orc_round_stats* stats, size_t cap) {
    uint32_t r = 0;
    orc_round_stats tmp;
    while (r < max_rounds) {
        if (s->nnxt == 0 && s->ndq == 0) {
            uint64_t live = 0;
            for (uint32_t v = 0; v < s->n && !live; v++) {
                if (!s->alive[v]) continue;
                for (size_t i = 0; i < s->nodes[v].nout; i++) live += s->alive[s->nodes[v].out[i].peer];
            }
            if (live == 0) break;
        }
        one_round(s, r < cap ? &stats[r] : &tmp);
        r++;
    }
    return r;
}

/* the messages the next round delivers (delayed ones due then included) */
size_t orc_pt_pending(const orc_plumtree* s, orc_msg* out, size_t cap) {
    size_t n = 0;
    for (size_t i = 0; i < s->nnxt; i++, n++) if (n < cap) out[n] = s->nxt[i];
    for (size_t i = 0; i < s->ndq; i++)
        if (s->dqa[i] == s->round + 1) { if (n < cap) out[n] = s->dq[i]; n++; }
    qsort(out, n < cap ? n : cap, sizeof(orc_msg), msg_cmp);
    return n;
}

int orc_pt_get_peers(const orc_plumtree* s, uint32_t v, uint32_t root,
                     uint32_t* eager, size_t* ne, uint32_t* lazy, size_t* nl, size_t cap) {
    node_t* nd = &s->nodes[v];
    const oset* e = all_peers(nd, root, 0);
    const oset* l = all_peers(nd, root, 1);
    if (e->n > cap || l->n > cap) return ORC_NOSPACE;
    memcpy(eager, e->a, e->n * sizeof(uint32_t)); *ne = e->n;
    memcpy(lazy, l->a, l->n * sizeof(uint32_t)); *nl = l->n;
    return ORC_OK;
}

size_t orc_pt_get_outstanding(const orc_plumtree* s, uint32_t v, uint32_t* peers,
                              uint32_t* rounds, uint32_t* monos, size_t cap) {
    node_t* nd = &s->nodes[v];
    for (size_t i = 0; i < nd->nout && i < cap; i++) {
        /* the id as psim reports it: epoch << 24 | Monotonic (epoch 0 until a backend restart) */
        peers[i] = nd->out[i].peer; rounds[i] = nd->out[i].round;
        monos[i] = (nd->out[i].id_epoch << 24) | nd->out[i].id_mono;
    }
    return nd->nout;
}

/* id = epoch << 24 | Monotonic (psim's form): out[v] = is_stale(id) at v */
void orc_pt_get_delivered(const orc_plumtree* s, uint32_t origin, uint32_t id, uint8_t* out) {
    for (uint32_t v = 0; v < s->n; v++)
        out[v] = (uint8_t)is_stale((node_t*)&s->nodes[v], origin, id >> 24, id & 0xFFFFFFu);
}

/* slot of peer p in v's row of the given slot layout, or -1 */
static int64_t row_slot(const uint64_t* row_ptr, const uint32_t* col, uint32_t v, uint32_t p) {
    for (uint64_t e = row_ptr[v]; e < row_ptr[v + 1]; e++)
        if (col[e] == p) return (int64_t)(e - row_ptr[v]);
    return -1;
}

static int set_mask(const oset* x, const uint64_t* row_ptr, const uint32_t* col, uint32_t v, uint32_t* m) {
    *m = 0;
    for (uint32_t i = 0; i < x->n; i++) {
        const int64_t q = row_slot(row_ptr, col, v, x->a[i]);
        if (q < 0 || q >= 32) return ORC_NOSPACE;
        *m |= 1u << q;
    }
    return ORC_OK;
}

int orc_pt_dump_state(const orc_plumtree* s, uint32_t root, uint32_t mono, const uint64_t* row_ptr,
                      const uint32_t* col, uint32_t lo, uint32_t hi, uint32_t* eager, uint32_t* lazy,
                      uint32_t* outst, uint16_t* rr) {
    for (uint32_t v = lo; v < hi && v < s->n; v++) {
        node_t* nd = &s->nodes[v];
        const uint32_t i = v - lo;
        if (set_mask(all_peers(nd, root, 0), row_ptr, col, v, &eager[i]) ||
            set_mask(all_peers(nd, root, 1), row_ptr, col, v, &lazy[i]))
            return ORC_NOSPACE;
        outst[i] = 0;
        for (size_t k = 0; k < nd->nout; k++) {
            const int64_t q = row_slot(row_ptr, col, v, nd->out[k].peer);
            if (q < 0 || q >= 32) return ORC_NOSPACE;
            outst[i] |= 1u << q;
        }
        rr[i] = 0xFFFFu;
        for (size_t k = 0; k < nd->nrr; k++)
            if (nd->rr[k].node == root && nd->rr[k].epoch == mono >> 24 && nd->rr[k].mono == (mono & 0xFFFFFFu)) {
                rr[i] = (uint16_t)nd->rr[k].round;
                break;
            }
    }
    return ORC_OK;
}

int orc_pt_inflight_words(const orc_plumtree* s, const uint64_t* row_ptr, const uint32_t* col, uint32_t lo,
                          uint32_t hi, uint32_t* words) {
    const uint64_t base = row_ptr[lo];
    memset(words, 0, (size_t)(row_ptr[hi] - base) * sizeof(uint32_t));
    const size_t k = s->nnxt + s->ndq;              /* FIFO order per pair = emission (seq) order */
    orc_msg* m = (orc_msg*)malloc((k ? k : 1) * sizeof(orc_msg));
    size_t got = orc_pt_pending(s, m, k);
    int rc = ORC_OK;
    for (size_t i = 0; i < got && i < k && rc == ORC_OK; i++) {
        if (m[i].dst < lo || m[i].dst >= hi) continue;
        const int64_t q = row_slot(row_ptr, col, m[i].dst, m[i].src);
        if (q < 0) { rc = ORC_NOSPACE; break; }
        uint32_t* w = &words[row_ptr[m[i].dst] + (uint64_t)q - base];
        uint32_t nk = 0;
        while (nk < 4 && ((*w >> (4 * nk)) & 0xFu)) nk++;
        if (nk == 4) { rc = ORC_NOSPACE; break; }
        *w |= m[i].type << (4 * nk);
        if (m[i].type == ORC_MSG_BROADCAST || m[i].type == ORC_MSG_IHAVE) *w = (*w & 0xFFFFu) | (m[i].round << 16);
    }
    free(m);
    return rc;
}

void orc_pt_get_recv_round(const orc_plumtree* s, uint32_t origin, uint32_t mono, uint32_t* out) {
    for (uint32_t v = 0; v < s->n; v++) {
        node_t* nd = &s->nodes[v];
        out[v] = 0xFFFFFFFFu;
        for (size_t i = 0; i < nd->nrr; i++)
            if (nd->rr[i].node == origin && nd->rr[i].epoch == mono >> 24 && nd->rr[i].mono == (mono & 0xFFFFFFu)) {
                out[v] = nd->rr[i].round;
                break;
            }
    }
}
