/*
 * scamp.c -- round-synchronous restatement of the SCAMP membership
 * strategies run by the pluggable peer service manager:
 *   v2: src/partisan_scamp_v2_membership_strategy.erl:75-374
 *   v1: src/partisan_scamp_v1_membership_strategy.erl:56-329
 *   glue: src/partisan_pluggable_peer_service_manager.erl (periodic
 *   :1386-1419, {connected,..} -> join :1532-1597, handle_message
 *   {membership_strategy,..} :1739-1808, internal_leave :2059-2109,
 *   do_send_message :1938-1987).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Checker for csrc/scamp.hip.
 * Trajectories are parity unpinned by reference vectors (no reference test
 * pins them); the tests check the view invariants the
 * protocol guarantees (a kept subscription is in the keeper's partial view
 * and the keeper is in the subscriber's in-view, v2).
 *
 * Simulation contract (DESIGN.md "SCAMP"):
 *  - node_spec() <-> vertex id; sets v2 / usort order = id order (Q28);
 *    the v2 partial view and in-view are lists (prepend order kept);
 *  - a message emitted by a handler at u reaches t iff t != u, t was alive
 *    at the start of the round, and u holds an outbound connection to t:
 *    connections are made to members only (establish_connections
 *    :1638-1669 skips self) and killed for non-members after every
 *    membership message (pending_leavers :2041-2054, cast after the
 *    sends), so the connected set of a handler's sends is
 *    members-before U members-after (connect/1 succeeds iff the peer is up,
 *    Q30).  Anything else is dropped (do_send_message :1971-1985);
 *  - rand: one Philox stream per vertex and incarnation (kind 5, counter
 *    {v, draw index, 5, incarnation}); rand:uniform(N) = 1 + floor(r N / 2^64)
 *    on a 64-bit draw; rand:uniform() = (r >> 11) 2^-53, so shuffle/1
 *    (lists:sort of {Float, N}) orders by (r >> 11, N);
 *  - round t at v: a vertex restarted since the last round drops its inbox
 *    (messages addressed to the crashed incarnation); then leave calls,
 *    then join calls ({connected, Contact, ...} -> join/3), both in call
 *    order; then the inbox in (src, emission seq) order, each
 *    handle_message followed by the manager's stop check (:1791-1803: a
 *    node whose members no longer contain itself shuts down); then
 *    periodic/1 when t % periodic_rounds == 0;
 *  - isolation (Q19): last_message_time = the round of the last ping
 *    handled; periodic/1 finds the node isolated iff it handled a ping
 *    before and none in the current round (100 ms window vs a 10 s period);
 *  - crash(v): the node restarts with init/1 state and a new incarnation
 *    (its rand stream restarts); messages in flight to it are lost.
 *  - reference crash points are reported, not emulated: v2
 *    bootstrap_remove_subscription reaching lists:nth(0) or past the list
 *    end (Q18) and the v1 remove_subscription badarg (Q17, the swapped
 *    sets:del_element arguments turn the membership into the node_spec
 *    map, whose keys are not the node: the manager stops) stop the vertex
 *    and set an error bit.
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>

enum { SC_FWD = 1, SC_KEEP, SC_PING, SC_REMOVE, SC_REPLACE, SC_BOOT };
#define SC_KIND 5u
#define SC_ERR_BOOT 4u
#define SC_ERR_Q17 8u

typedef struct { uint32_t* a; uint32_t n, cap; } ulist;

static void lpush_front(ulist* l, uint32_t x) {
    if (l->n == l->cap) { l->cap = l->cap ? 2 * l->cap : 8; l->a = (uint32_t*)realloc(l->a, l->cap * 4); }
    memmove(l->a + 1, l->a, l->n * 4);
    l->a[0] = x;
    l->n++;
}
static int lhas(const ulist* l, uint32_t x) { for (uint32_t i = 0; i < l->n; i++) if (l->a[i] == x) return 1; return 0; }
static void lsadd(ulist* l, uint32_t x) {          /* sorted-set insert (v1 sets, id order) */
    if (lhas(l, x)) return;
    if (l->n == l->cap) { l->cap = l->cap ? 2 * l->cap : 8; l->a = (uint32_t*)realloc(l->a, l->cap * 4); }
    uint32_t i = l->n;
    while (i > 0 && l->a[i - 1] > x) { l->a[i] = l->a[i - 1]; i--; }
    l->a[i] = x;
    l->n++;
}
static void ldel_first(ulist* l, uint32_t x) {     /* L -- [X] / sets:del_element */
    for (uint32_t i = 0; i < l->n; i++)
        if (l->a[i] == x) { memmove(l->a + i, l->a + i + 1, (l->n - i - 1) * 4); l->n--; return; }
}
static void lcopy(ulist* d, const ulist* s) {
    if (d->cap < s->n) { d->cap = s->n; d->a = (uint32_t*)realloc(d->a, (d->cap ? d->cap : 1) * 4); }
    memcpy(d->a, s->a, s->n * 4);
    d->n = s->n;
}

typedef struct { uint32_t type, src, dst, a, b; uint64_t seq; } scmsg;
typedef struct { uint32_t kind, v, x; } sccall;   /* kind 0 join (x = contact), 1 leave (x = node) */

typedef struct {
    ulist pv, iv;
    int64_t last_ping;        /* -1 = undefined */
    uint64_t draws, seq;
    uint32_t inc;
    uint8_t fresh;
} scnode;

struct orc_scamp {
    uint32_t n, ver, c, periodic;
    uint64_t seed, round;
    scnode* nd;
    uint8_t* alive;
    uint8_t* alive0;
    scmsg* cur; size_t ncur, capcur;
    scmsg* nxt; size_t nnxt, capnxt;
    sccall* calls; size_t ncalls, capcalls;
    orc_scamp_stats* st;
    ulist before;             /* members of the vertex before the running handler */
    orc_scamp_update_fn upd;  /* partisan_peer_service_events:update/1 listener (Plumtree, C3) */
    void* upd_ctx;
};

void orc_scamp_set_update_hook(orc_scamp* s, orc_scamp_update_fn fn, void* ctx) { s->upd = fn; s->upd_ctx = ctx; }

/* the manager fires update(Members) when the members list changed after a
 * join (:1574-1579) or a membership message (:1756-1761), and always after a
 * leave (:2107) */
static void fire_update(orc_scamp* s, uint32_t v, int always) {
    if (!s->upd) return;
    const ulist* pv = &s->nd[v].pv;
    int same = pv->n == s->before.n && memcmp(pv->a, s->before.a, pv->n * 4) == 0;
    if (!same || always) s->upd(s->upd_ctx, v, pv->a, pv->n);
}

static void node_init(scnode* x, uint32_t v) {      /* init/1: [Myself] / sets {Myself} */
    x->pv.n = 0;
    x->iv.n = 0;
    lpush_front(&x->pv, v);
    x->last_ping = -1;
    x->draws = 0;
    x->fresh = 0;
}

orc_scamp* orc_scamp_create(uint32_t n, uint32_t version, uint32_t c, uint32_t periodic_rounds, uint64_t seed) {
    if (version != 1 && version != 2) return NULL;
    orc_scamp* s = (orc_scamp*)calloc(1, sizeof(orc_scamp));
    s->n = n; s->ver = version; s->c = c; s->periodic = periodic_rounds; s->seed = seed;
    s->nd = (scnode*)calloc(n, sizeof(scnode));
    s->alive = (uint8_t*)malloc(n);
    s->alive0 = (uint8_t*)malloc(n);
    memset(s->alive, 1, n);
    for (uint32_t v = 0; v < n; v++) node_init(&s->nd[v], v);
    return s;
}

void orc_scamp_destroy(orc_scamp* s) {
    if (!s) return;
    for (uint32_t v = 0; v < s->n; v++) { free(s->nd[v].pv.a); free(s->nd[v].iv.a); }
    free(s->nd); free(s->alive); free(s->alive0); free(s->cur); free(s->nxt); free(s->calls); free(s->before.a);
    free(s);
}

void orc_scamp_set_alive(orc_scamp* s, const uint8_t* alive) { memcpy(s->alive, alive, s->n); }

static void push_call(orc_scamp* s, uint32_t kind, uint32_t v, uint32_t x) {
    if (s->ncalls == s->capcalls) { s->capcalls = s->capcalls ? 2 * s->capcalls : 64; s->calls = (sccall*)realloc(s->calls, s->capcalls * sizeof(sccall)); }
    s->calls[s->ncalls].kind = kind; s->calls[s->ncalls].v = v; s->calls[s->ncalls].x = x; s->ncalls++;
}
void orc_scamp_join(orc_scamp* s, uint32_t v, uint32_t contact) { push_call(s, 0, v, contact); }
void orc_scamp_leave(orc_scamp* s, uint32_t v, uint32_t node) { push_call(s, 1, v, node); }

void orc_scamp_crash(orc_scamp* s, uint32_t v) {
    scnode* x = &s->nd[v];
    node_init(x, v);
    x->inc++;
    x->fresh = 1;
    s->alive[v] = 1;
}

/* ---------------- rand ------------------------------------------------------ */
static uint64_t draw64(orc_scamp* s, uint32_t v) {
    scnode* x = &s->nd[v];
    uint32_t ctr[4] = {v, (uint32_t)x->draws, SC_KIND, x->inc};
    uint32_t key[2] = {(uint32_t)s->seed, (uint32_t)(s->seed >> 32)}, r[4];
    orc_philox4x32_10(ctr, key, r);
    x->draws++;
    if (s->st) s->st->draws++;
    return (uint64_t)r[0] | ((uint64_t)r[1] << 32);
}
/* random_0_or_1/0 (v2 :367-374, v1 :322-329): rand:uniform(10) >= 5 */
static int random_0_or_1(orc_scamp* s, uint32_t v) {
    uint32_t r = 1u + (uint32_t)(((unsigned __int128)draw64(s, v) * 10u) >> 64);
    return r >= 5 ? 1 : 0;
}
/* select_random_sublist(L, K) = lists:sublist(shuffle(L), K) (v2 :354-364):
 * one uniform() per element in list order; the K smallest (float, N) */
static uint32_t select_random_sublist(orc_scamp* s, uint32_t v, const ulist* l, uint32_t k, uint32_t* out) {
    uint32_t m = l->n;
    if (m == 0) return 0;
    uint64_t* key = (uint64_t*)malloc(m * 8);
    uint8_t* used = (uint8_t*)calloc(m, 1);
    for (uint32_t i = 0; i < m; i++) key[i] = draw64(s, v) >> 11;
    uint32_t got = 0;
    while (got < k && got < m) {
        uint32_t best = UINT32_MAX;
        for (uint32_t i = 0; i < m; i++) {
            if (used[i]) continue;
            if (best == UINT32_MAX || key[i] < key[best] || (key[i] == key[best] && l->a[i] < l->a[best])) best = i;
        }
        used[best] = 1;
        out[got++] = l->a[best];
    }
    free(key); free(used);
    return got;
}

/* ---------------- emission ------------------------------------------------- */
static int connected(orc_scamp* s, uint32_t u, uint32_t t) {
    return t != u && s->alive0[t] && (lhas(&s->before, t) || lhas(&s->nd[u].pv, t));
}
static void emit(orc_scamp* s, uint32_t u, uint32_t t, uint32_t type, uint32_t a, uint32_t b) {
    if (!connected(s, u, t)) { if (s->st) s->st->dropped++; return; }
    if (s->nnxt == s->capnxt) { s->capnxt = s->capnxt ? 2 * s->capnxt : 1024; s->nxt = (scmsg*)realloc(s->nxt, s->capnxt * sizeof(scmsg)); }
    scmsg* m = &s->nxt[s->nnxt++];
    m->type = type; m->src = u; m->dst = t; m->a = a; m->b = b;
    m->seq = s->nd[u].seq++;
    if (s->st) s->st->sent[type]++;
}
static void begin_handler(orc_scamp* s, uint32_t v) { lcopy(&s->before, &s->nd[v].pv); }

/* ---------------- membership_strategy callbacks ------------------------- */
/* join/3 (v2 :89-137, v1 :69-119) */
static void do_join(orc_scamp* s, uint32_t v, uint32_t node) {
    scnode* x = &s->nd[v];
    begin_handler(s, v);
    ulist pv0 = {0, 0, 0};
    lcopy(&pv0, &x->pv);
    uint32_t k = s->ver == 2 ? s->c - 1 : s->c;   /* Q15 */
    uint32_t sel[64];
    if (s->ver == 2) lpush_front(&x->pv, node); else lsadd(&x->pv, node);
    emit(s, v, node, SC_FWD, v, 0);                          /* forward_subscription(Myself) */
    for (uint32_t i = 0; i < pv0.n; i++) emit(s, v, pv0.a[i], SC_FWD, node, 0);
    uint32_t ns = select_random_sublist(s, v, &pv0, k < 64 ? k : 64, sel);
    for (uint32_t i = 0; i < ns; i++) emit(s, v, sel[i], SC_FWD, node, 0);
    free(pv0.a);
}

/* leave/2 (v2 :140-146, v1 :122-142) */
static void do_leave(orc_scamp* s, uint32_t v, uint32_t node) {
    scnode* x = &s->nd[v];
    begin_handler(s, v);
    if (s->ver == 2) {
        for (uint32_t i = 0; i < x->pv.n; i++) emit(s, v, x->pv.a[i], SC_BOOT, node, 0);
    } else {
        ldel_first(&x->pv, node);
        for (uint32_t i = 0; i < s->before.n; i++) emit(s, v, s->before.a[i], SC_REMOVE, node, 0);
    }
}

/* periodic/1 (v2 :180-221, v1 :174-216) */
static void do_periodic(orc_scamp* s, uint32_t v) {
    scnode* x = &s->nd[v];
    begin_handler(s, v);
    int isolated = x->last_ping >= 0 && (uint64_t)x->last_ping < s->round;
    if (isolated) {
        uint32_t sel[1];
        uint32_t ns = select_random_sublist(s, v, &x->pv, 1, sel);
        if (s->st) s->st->resub++;
        for (uint32_t i = 0; i < ns; i++) emit(s, v, sel[i], SC_FWD, v, 0);
    }
    for (uint32_t i = 0; i < x->pv.n; i++) emit(s, v, x->pv.a[i], SC_PING, v, 0);
}

/* handle_message/2; returns 0 when the manager stops (stop check :1791-1803) */
static int do_message(orc_scamp* s, uint32_t v, const scmsg* m) {
    scnode* x = &s->nd[v];
    begin_handler(s, v);
    switch (m->type) {
    case SC_PING:                                            /* v2 :224-229, v1 :219-227 */
        x->last_ping = (int64_t)s->round;
        break;
    case SC_FWD: {                                           /* v2 :313-341, v1 :264-297 */
        uint32_t node = m->a;
        int keep = random_0_or_1(s, v) == 0 && !lhas(&x->pv, node);
        if (keep) {
            if (s->ver == 2) {
                lpush_front(&x->pv, node);
                emit(s, v, node, SC_KEEP, v, 0);
            } else {
                lsadd(&x->pv, node);
            }
        } else {
            uint32_t sel[1];
            uint32_t ns = select_random_sublist(s, v, &s->before, 1, sel);
            for (uint32_t i = 0; i < ns; i++) emit(s, v, sel[i], SC_FWD, node, 0);
        }
        break;
    }
    case SC_KEEP:                                            /* v2 :342-347 */
        lpush_front(&x->iv, m->a);
        break;
    case SC_REMOVE: {                                        /* v2 :295-312, v1 :230-262 */
        uint32_t node = m->a;
        if (!lhas(&x->pv, node)) break;
        if (s->ver == 1) {                                   /* Q17: the manager stops */
            if (s->st) s->st->error |= SC_ERR_Q17;
            return 0;
        }
        ldel_first(&x->pv, node);
        for (uint32_t i = 0; i < s->before.n; i++) emit(s, v, s->before.a[i], SC_REMOVE, node, 0);
        break;
    }
    case SC_REPLACE:                                         /* v2 :275-294 */
        for (uint32_t i = 0; i < x->pv.n; i++) if (x->pv.a[i] == m->a) x->pv.a[i] = m->b;
        break;
    case SC_BOOT: {                                          /* v2 :230-274 */
        if (m->a != v) break;
        int32_t L = (int32_t)x->iv.n, P = (int32_t)x->pv.n;
        int32_t num = L - (int32_t)(s->c - 1);
        int32_t rem = L - num;
        /* lists:nth/2 needs 1 <= N <= length (Q18): check every index first */
        int crash = 0;
        if (num > 0)
            for (int32_t N = 1; N <= num && !crash; N++)
                if (P == 0 || N / P < 1 || N / P > P) crash = 1;
        if (!crash && rem > L) crash = 1;
        if (crash) {
            if (s->st) s->st->error |= SC_ERR_BOOT;
            return 0;
        }
        ulist iv0 = {0, 0, 0}, pv0 = {0, 0, 0};
        lcopy(&iv0, &x->iv);
        lcopy(&pv0, &x->pv);
        x->pv.n = 0;
        x->iv.n = 0;
        if (num > 0)
            for (int32_t N = 1; N <= num; N++) emit(s, v, iv0.a[N - 1], SC_REPLACE, v, pv0.a[N / P - 1]);
        if (rem > 0)
            for (int32_t N = 1; N <= rem; N++) emit(s, v, iv0.a[N - 1], SC_REMOVE, v, 0);
        free(iv0.a); free(pv0.a);
        break;
    }
    default:
        break;
    }
    return lhas(&x->pv, v);
}

static int cmp_msg(const void* a, const void* b) {
    const scmsg *x = (const scmsg*)a, *y = (const scmsg*)b;
    if (x->dst != y->dst) return x->dst < y->dst ? -1 : 1;
    if (x->src != y->src) return x->src < y->src ? -1 : 1;
    return x->seq < y->seq ? -1 : x->seq > y->seq;
}

static void one_round(orc_scamp* s) {
    s->round++;
    scmsg* t = s->cur; s->cur = s->nxt; s->nxt = t;
    size_t tc = s->capcur; s->capcur = s->capnxt; s->capnxt = tc;
    s->ncur = s->nnxt; s->nnxt = 0;
    qsort(s->cur, s->ncur, sizeof(scmsg), cmp_msg);
    memcpy(s->alive0, s->alive, s->n);

    /* calls made between rounds: leaves, then joins, each in call order */
    for (int kind = 1; kind >= 0; kind--)
        for (size_t i = 0; i < s->ncalls; i++) {
            sccall* c = &s->calls[i];
            if ((int)c->kind != kind || !s->alive[c->v]) continue;
            if (kind == 1) { do_leave(s, c->v, c->x); fire_update(s, c->v, 1); }
            else if (c->x != c->v && s->alive0[c->x]) {                        /* connect/1 to a live peer */
                do_join(s, c->v, c->x);
                fire_update(s, c->v, 0);
            }
        }
    s->ncalls = 0;

    for (size_t i = 0; i < s->ncur; i++) {
        scmsg* m = &s->cur[i];
        uint32_t v = m->dst;
        if (!s->alive[v] || s->nd[v].fresh) continue;
        if (s->st) s->st->processed++;
        const int up = do_message(s, v, m);
        fire_update(s, v, 0);
        if (!up) {
            s->alive[v] = 0;
            if (s->st) s->st->stopped++;
        }
    }
    for (uint32_t v = 0; v < s->n; v++) s->nd[v].fresh = 0;
    if (s->periodic && s->round % s->periodic == 0)
        for (uint32_t v = 0; v < s->n; v++)
            if (s->alive[v]) do_periodic(s, v);
}

uint32_t orc_scamp_step(orc_scamp* s, uint32_t rounds, orc_scamp_stats* st) {
    for (uint32_t r = 0; r < rounds; r++) {
        s->st = st ? &st[r] : NULL;
        if (s->st) memset(s->st, 0, sizeof(*s->st));
        one_round(s);
        if (s->st)
            for (uint32_t v = 0; v < s->n; v++)
                if (s->alive[v]) { s->st->pv_sum += s->nd[v].pv.n; s->st->inview_sum += s->nd[v].iv.n; }
    }
    s->st = NULL;
    return rounds;
}

size_t orc_scamp_inflight(const orc_scamp* s) { return s->nnxt; }

static int scmsg_cmp(const void* x, const void* y) {
    const scmsg* p = (const scmsg*)x; const scmsg* q = (const scmsg*)y;
    if (p->dst != q->dst) return p->dst < q->dst ? -1 : 1;
    if (p->src != q->src) return p->src < q->src ? -1 : 1;
    return p->seq < q->seq ? -1 : p->seq > q->seq;
}
/* the messages the next round delivers, in handling order (dst, src, seq):
 * the wire the pluggable manager carries ({membership_strategy, Msg},
 * partisan_pluggable_peer_service_manager.erl:1396-1407) -- test view */
size_t orc_scamp_pending(const orc_scamp* s, uint32_t* out6, size_t cap) {
    scmsg* m = (scmsg*)malloc((s->nnxt ? s->nnxt : 1) * sizeof(scmsg));
    memcpy(m, s->nxt, s->nnxt * sizeof(scmsg));
    qsort(m, s->nnxt, sizeof(scmsg), scmsg_cmp);
    for (size_t i = 0; i < s->nnxt && i < cap; i++) {
        uint32_t* o = out6 + 6 * i;
        o[0] = m[i].type; o[1] = m[i].src; o[2] = m[i].dst; o[3] = (uint32_t)m[i].seq; o[4] = m[i].a; o[5] = m[i].b;
    }
    free(m);
    return s->nnxt;
}

size_t orc_scamp_view(const orc_scamp* s, uint32_t v, int which, uint32_t* out, size_t cap) {
    const ulist* l = which ? &s->nd[v].iv : &s->nd[v].pv;
    for (uint32_t i = 0; i < l->n && i < cap; i++) out[i] = l->a[i];
    return l->n;
}

uint64_t orc_scamp_draws(const orc_scamp* s, uint32_t v) { return s->nd[v].draws; }
int orc_scamp_alive(const orc_scamp* s, uint32_t v) { return s->alive[v]; }
int64_t orc_scamp_last_ping(const orc_scamp* s, uint32_t v) { return s->nd[v].last_ping; }
int orc_scamp_has_member(const orc_scamp* s, uint32_t v, uint32_t t) { return lhas(&s->nd[v].pv, t); }
