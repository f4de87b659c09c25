/*
 * hyparview.c -- round-synchronous restatement of the HyParView view
 * maintenance of src/partisan_hyparview_peer_service_manager.erl
 * (init 745-822; join cast 999-1016; handle_message join 1234-1338,
 * neighbor 1340-1379, forward_join 1381-1563, disconnect 1565-1617,
 * neighbor_request/rejected/accepted 1619-1748, shuffle/shuffle_reply
 * 1750-1798; random_promotion 1046-1067; passive_view_maintenance
 * 1078-1111; helpers 2291-2697).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Checker for csrc/hyparview.hip.
 * Trajectories are parity unpinned by reference vectors (no reference test
 * pins them); the view invariants of test/partisan_SUITE.erl
 * :2331-2395 (symmetry, connectivity) are checked by the tests.
 *
 * Simulation contract (DESIGN.md "HyParView"):
 *  - node_spec() <-> vertex id; sets v2 / ordsets / usort order = id order (Q28);
 *  - connect/1 is synchronous and succeeds iff the peer is alive (Q30); every
 *    send is preceded by a connect to its destination, so a message to a live
 *    peer is delivered and one to a dead peer is lost;
 *  - every node starts at round 0 with epoch 1 (fresh data dir: 0 + 1, :761);
 *    no reservations, tag undefined;
 *  - rand: one Philox stream per vertex (kind 4), counter = the process's
 *    draw index; rand:uniform(N) = 1 + floor(r * N / 2^64); rand:uniform()
 *    consumes one draw; rand:uniform(0) raises before drawing (Q13);
 *  - round t: inbox sorted by (src, emission seq); then the timers due at
 *    the end of round t: random_promotion every promotion_rounds, then
 *    passive_view_maintenance every shuffle_rounds;
 *  - joins are casts made between rounds (their join message is delivered
 *    in the next round).
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>

enum { HV_JOIN = 1, HV_NEIGHBOR, HV_FORWARD_JOIN, HV_DISCONNECT, HV_NEIGHBOR_REQUEST,
       HV_NEIGHBOR_REJECTED, HV_NEIGHBOR_ACCEPTED, HV_SHUFFLE, HV_SHUFFLE_REPLY };

#define HV_KIND 4u
#define XMAX 8

typedef struct { uint32_t peer, epoch, cnt; } idrow;
typedef struct { idrow* a; size_t n, cap; } idmap;

typedef struct {
    uint32_t type, src, dst, peer, epoch, ttl, did_e, did_c, prio, nx;
    uint32_t x[XMAX];
    uint64_t seq;
} hvmsg;

typedef struct {
    uint32_t act[8]; uint32_t na;       /* sets:to_list(Active) incl. self, sorted */
    uint32_t pas[32]; uint32_t np;      /* passive view, sorted */
    idmap sent, recv;                   /* sent_message_map / recv_message_map */
    uint32_t epoch;
    uint64_t draws, seq;
} hvnode;

struct orc_hyparview {
    uint32_t n;
    orc_hv_config cfg;
    uint64_t seed, round;
    hvnode* nd;
    uint8_t* alive;
    hvmsg* cur; size_t ncur, capcur;
    hvmsg* nxt; size_t nnxt, capnxt;
    orc_hv_stats* st;
    int error;                          /* a reference crash (function/case clause) */
};

/* ---------------- rand --------------------------------------------------- */
static uint64_t draw64(orc_hyparview* s, uint32_t v) {
    hvnode* x = &s->nd[v];
    uint32_t ctr[4] = {v, (uint32_t)x->draws, HV_KIND, (uint32_t)(x->draws >> 32)};
    uint32_t key[2] = {(uint32_t)s->seed, (uint32_t)(s->seed >> 32)}, r[4];
    orc_philox4x32_10(ctr, key, r);
    x->draws++;
    if (s->st) s->st->draws++;
    return (uint64_t)r[0] | ((uint64_t)r[1] << 32);
}
static uint32_t uniform(orc_hyparview* s, uint32_t v, uint32_t n) {   /* rand:uniform(N), N >= 1 */
    return 1u + (uint32_t)(((unsigned __int128)draw64(s, v) * n) >> 64);
}

/* ---------------- sorted small sets ------------------------------------- */
static int has(const uint32_t* a, uint32_t n, uint32_t x) { for (uint32_t i = 0; i < n; i++) if (a[i] == x) return 1; return 0; }
static void sadd(uint32_t* a, uint32_t* n, uint32_t x) {
    if (has(a, *n, x)) return;
    uint32_t i = *n;
    while (i > 0 && a[i - 1] > x) { a[i] = a[i - 1]; i--; }
    a[i] = x; (*n)++;
}
static void sdel(uint32_t* a, uint32_t* n, uint32_t x) {
    uint32_t k = 0;
    for (uint32_t i = 0; i < *n; i++) if (a[i] != x) a[k++] = a[i];
    *n = k;
}

/* ---------------- id maps ------------------------------------------------ */
static idrow* mfind(idmap* m, uint32_t p) { for (size_t i = 0; i < m->n; i++) if (m->a[i].peer == p) return &m->a[i]; return NULL; }
static void mput(idmap* m, uint32_t p, uint32_t e, uint32_t c) {
    idrow* r = mfind(m, p);
    if (!r) {
        if (m->n == m->cap) { m->cap = m->cap ? m->cap * 2 : 4; m->a = (idrow*)realloc(m->a, m->cap * sizeof(idrow)); }
        r = &m->a[m->n++];
        r->peer = p;
    }
    r->epoch = e; r->cnt = c;
}

/* ---------------- emission ------------------------------------------------ */
static hvmsg* emit(orc_hyparview* s, uint32_t src, uint32_t dst, uint32_t type) {
    if (s->nnxt == s->capnxt) { s->capnxt = s->capnxt ? s->capnxt * 2 : 1024; s->nxt = (hvmsg*)realloc(s->nxt, s->capnxt * sizeof(hvmsg)); }
    hvmsg* m = &s->nxt[s->nnxt++];
    memset(m, 0, sizeof(*m));
    m->type = type; m->src = src; m->dst = dst;
    m->seq = s->nd[src].seq++;
    if (s->st) s->st->sent[type]++;
    return m;
}

/* ---------------- helpers (:2291-2697) ---------------------------------- */
/* pick_random(View, Omit) (:2291-2301): List = members(View) -- Omit */
static int pick_random(orc_hyparview* s, uint32_t v, const uint32_t* view, uint32_t nv,
                       const uint32_t* omit, uint32_t no, uint32_t* out) {
    uint32_t lst[40], k = 0;
    for (uint32_t i = 0; i < nv; i++) if (!has(omit, no, view[i])) lst[k++] = view[i];
    if (k == 0) return 0;                 /* rand:uniform(0) raises: undefined, no draw (Q13) */
    *out = lst[uniform(s, v, k) - 1];
    return 1;
}
/* select_peers_for_exchange/1 (:2324-2333): [Myself | shuffle(Active, ka)] ++
 * shuffle(Passive, kp), usort.  shuffle/2 (:2309-2316) draws one float per
 * element of L and keeps the first K (term order, Q8). */
static uint32_t select_exchange(orc_hyparview* s, uint32_t v, uint32_t* out) {
    hvnode* x = &s->nd[v];
    for (uint32_t i = 0; i < x->na; i++) (void)draw64(s, v);
    for (uint32_t i = 0; i < x->np; i++) (void)draw64(s, v);
    uint32_t n = 0;
    sadd(out, &n, v);
    for (uint32_t i = 0; i < x->na && i < s->cfg.shuffle_k_active; i++) sadd(out, &n, x->act[i]);
    for (uint32_t i = 0; i < x->np && i < s->cfg.shuffle_k_passive; i++) sadd(out, &n, x->pas[i]);
    return n;
}
static void get_current_id(hvnode* x, uint32_t p, uint32_t* e, uint32_t* c) {     /* :2618-2627 */
    idrow* r = mfind(&x->recv, p);
    if (r) { *e = r->epoch; *c = r->cnt; } else { *e = 1; *c = 0; }
}
static int is_addable_did(hvnode* x, uint32_t ie, uint32_t ic, uint32_t p) {     /* :2652-2665 */
    idrow* r = mfind(&x->sent, p);
    if (!r) return 1;
    if (ie > r->epoch) return 1;
    if (ie == r->epoch) return ic >= r->cnt;
    return 0;
}
static int is_addable_epoch(hvnode* x, uint32_t pe, uint32_t p) {                 /* :2667-2674 */
    idrow* r = mfind(&x->sent, p);
    return !r || pe >= r->epoch;
}
static int is_valid_disconnect(hvnode* x, uint32_t ie, uint32_t ic, uint32_t p) { /* :2639-2650 */
    idrow* r = mfind(&x->recv, p);
    if (!r) return 1;
    if (ie > r->epoch) return 1;
    return ic > r->cnt;
}

/* add_to_passive_view/2 (:2418-2449) */
static void add_to_passive(orc_hyparview* s, uint32_t v, uint32_t p) {
    hvnode* x = &s->nd[v];
    if (p == v || has(x->act, x->na, p) || has(x->pas, x->np, p)) return;
    if (x->np >= s->cfg.passive_max_size) {
        uint32_t r, om[1] = {v};
        if (pick_random(s, v, x->pas, x->np, om, 1, &r)) sdel(x->pas, &x->np, r);
    }
    sadd(x->pas, &x->np, p);
}

/* drop_random_element_from_active_view/1 (:2476-2525) */
static void drop_random_active(orc_hyparview* s, uint32_t v) {
    hvnode* x = &s->nd[v];
    uint32_t r, om[1] = {v};
    if (!pick_random(s, v, x->act, x->na, om, 1, &r)) return;
    sdel(x->act, &x->na, r);
    add_to_passive(s, v, r);
    idrow* sr = mfind(&x->sent, r);                  /* get_next_id/3 (:2630-2636) */
    uint32_t ne, nc;
    if (sr && sr->epoch == x->epoch) { ne = x->epoch; nc = sr->cnt + 1; }
    else if (!sr) { ne = x->epoch; nc = 1; }
    else { s->error = 1; return; }                   /* case_clause in the reference */
    mput(&x->sent, r, ne, nc);
    if (s->alive[r]) {                               /* connect + send {disconnect, Myself, NextId} */
        hvmsg* m = emit(s, v, r, HV_DISCONNECT);
        m->peer = v; m->did_e = ne; m->did_c = nc;
    }
}

/* add_to_active_view/3 (:2344-2410) */
static void add_to_active(orc_hyparview* s, uint32_t v, uint32_t p) {
    hvnode* x = &s->nd[v];
    if (p == v || has(x->act, x->na, p)) return;
    sdel(x->pas, &x->np, p);
    if (x->na >= s->cfg.active_max_size) drop_random_active(s, v);   /* is_full (no reservations) */
    sadd(x->act, &x->na, p);
}

/* merge_exchange/2 (:2569-2576) */
static void merge_exchange(orc_hyparview* s, uint32_t v, const uint32_t* ex, uint32_t nx) {
    hvnode* x = &s->nd[v];
    uint32_t to[XMAX + 1], k = 0;
    for (uint32_t i = 0; i < nx; i++) if (ex[i] != v && !has(x->act, x->na, ex[i])) sadd(to, &k, ex[i]);
    for (uint32_t i = 0; i < k; i++) add_to_passive(s, v, to[i]);
}

/* promote_peer/2 (:2675-2697) */
static void promote_peer(orc_hyparview* s, uint32_t v, uint32_t p) {
    hvnode* x = &s->nd[v];
    uint32_t ex[XMAX];
    uint32_t nx = select_exchange(s, v, ex);
    uint32_t e, c;
    get_current_id(x, p, &e, &c);
    if (!s->alive[p]) return;
    hvmsg* m = emit(s, v, p, HV_NEIGHBOR_REQUEST);
    m->peer = v; m->prio = 1; m->did_e = e; m->did_c = c; m->nx = nx;
    memcpy(m->x, ex, nx * 4);
}

static void send_neighbor(orc_hyparview* s, uint32_t v, uint32_t p) {
    uint32_t e, c;
    get_current_id(&s->nd[v], p, &e, &c);
    hvmsg* m = emit(s, v, p, HV_NEIGHBOR);          /* {neighbor, Myself, Tag, LastDisconnectId, Peer} */
    m->peer = v; m->did_e = e; m->did_c = c;
}

/* ---------------- handle_message clauses -------------------------------- */
static void handle(orc_hyparview* s, uint32_t v, const hvmsg* m) {
    hvnode* x = &s->nd[v];
    uint32_t P = m->peer;
    switch (m->type) {
    case HV_JOIN: {                                          /* :1234-1338 */
        if (is_addable_epoch(x, m->epoch, P) && !has(x->act, x->na, P)) {
            if (s->alive[P]) {
                add_to_active(s, v, P);
                send_neighbor(s, v, P);
                for (uint32_t i = 0; i < x->na; i++) {         /* (members -- [Myself]) -- [Peer] */
                    uint32_t q = x->act[i];
                    if (q == v || q == P) continue;
                    if (!s->alive[q]) continue;
                    hvmsg* f = emit(s, v, q, HV_FORWARD_JOIN);
                    f->peer = P; f->epoch = m->epoch; f->ttl = s->cfg.active_rwl;
                }
            }
        }
        break;
    }
    case HV_NEIGHBOR:                                        /* :1340-1379 */
        if (is_addable_did(x, m->did_e, m->did_c, P) && s->alive[P]) add_to_active(s, v, P);
        break;
    case HV_FORWARD_JOIN: {                                  /* :1381-1563 */
        uint32_t S = m->src;
        if (m->ttl == 0 || x->na == 1) {
            if (is_addable_epoch(x, m->epoch, P) && !has(x->act, x->na, P) && s->alive[P]) {
                add_to_active(s, v, P);
                send_neighbor(s, v, P);
            }
        } else {
            uint32_t act0[8], na0 = x->na;
            memcpy(act0, x->act, sizeof(act0));
            hvnode save = *x;                                 /* State0 / State2 for the `false` branch */
            uint32_t spas[32]; memcpy(spas, x->pas, sizeof(spas));
            if (m->ttl == s->cfg.passive_rwl) add_to_passive(s, v, P);
            uint32_t om[3] = {S, v, P}, r;
            if (!pick_random(s, v, act0, na0, om, 3, &r)) {
                if (is_addable_epoch(x, m->epoch, P) && !has(act0, na0, P)) {
                    if (s->alive[P]) {
                        add_to_active(s, v, P);
                        send_neighbor(s, v, P);
                    } else {                                  /* `false -> State0`: drops the passive add */
                        memcpy(x->pas, spas, sizeof(spas));
                        x->np = save.np;
                    }
                }
            } else if (s->alive[r]) {
                hvmsg* f = emit(s, v, r, HV_FORWARD_JOIN);
                f->peer = P; f->epoch = m->epoch; f->ttl = m->ttl - 1;
            }
        }
        break;
    }
    case HV_DISCONNECT: {                                    /* :1565-1617 */
        if (!is_valid_disconnect(x, m->did_e, m->did_c, P)) break;
        uint32_t pas0[32], np0 = x->np;
        memcpy(pas0, x->pas, sizeof(pas0));
        sdel(x->act, &x->na, P);
        add_to_passive(s, v, P);
        mput(&x->recv, P, m->did_e, m->did_c);
        if (x->na == 1) {
            uint32_t om[2] = {v, P}, r;
            if (pick_random(s, v, pas0, np0, om, 2, &r)) promote_peer(s, v, r);
        }
        break;
    }
    case HV_NEIGHBOR_REQUEST: {                              /* :1619-1711 */
        uint32_t ack[XMAX];
        uint32_t nack = select_exchange(s, v, ack);
        if (!m->prio && x->na >= s->cfg.active_max_size) {
            /* would send the 2-tuple {neighbor_rejected, Myself}, which matches
             * no handle_message clause at the receiver (never reached: every
             * neighbor_request is sent with priority high, :2692-2695) */
            s->error = 1;
        } else if (is_addable_did(x, m->did_e, m->did_c, P)) {
            if (s->alive[P]) {
                uint32_t e, c;
                get_current_id(x, P, &e, &c);
                hvmsg* a = emit(s, v, P, HV_NEIGHBOR_ACCEPTED);
                a->peer = v; a->did_e = e; a->did_c = c; a->nx = nack;
                memcpy(a->x, ack, nack * 4);
                add_to_active(s, v, P);
            }
        } else if (s->alive[P]) {
            hvmsg* a = emit(s, v, P, HV_NEIGHBOR_REJECTED);
            a->peer = v; a->nx = nack;
            memcpy(a->x, ack, nack * 4);
        }
        merge_exchange(s, v, m->x, m->nx);
        break;
    }
    case HV_NEIGHBOR_REJECTED:                               /* :1713-1724 */
        merge_exchange(s, v, m->x, m->nx);
        break;
    case HV_NEIGHBOR_ACCEPTED:                               /* :1726-1748 */
        if (is_addable_did(x, m->did_e, m->did_c, P)) add_to_active(s, v, P);
        merge_exchange(s, v, m->x, m->nx);
        break;
    case HV_SHUFFLE_REPLY:                                   /* :1750-1752 */
        merge_exchange(s, v, m->x, m->nx);
        break;
    case HV_SHUFFLE: {                                       /* :1754-1798 */
        uint32_t S = m->peer;                                /* Sender field */
        if (m->ttl > 0 && x->na > 1) {
            uint32_t om[2] = {S, v}, r;
            if (pick_random(s, v, x->act, x->na, om, 2, &r) && s->alive[r]) {
                hvmsg* f = emit(s, v, r, HV_SHUFFLE);
                f->peer = v; f->ttl = m->ttl - 1; f->nx = m->nx;
                memcpy(f->x, m->x, m->nx * 4);
            }
        } else {
            for (uint32_t i = 0; i < x->np; i++) (void)draw64(s, v);   /* shuffle(Passive, |Exchange|) */
            uint32_t k = x->np < m->nx ? x->np : m->nx;
            if (s->alive[S]) {
                hvmsg* f = emit(s, v, S, HV_SHUFFLE_REPLY);
                f->peer = v; f->nx = k;
                memcpy(f->x, x->pas, k * 4);
            }
            merge_exchange(s, v, m->x, m->nx);
        }
        break;
    }
    default: break;
    }
}

/* ---------------- timers -------------------------------------------------- */
static void random_promotion(orc_hyparview* s, uint32_t v) {                 /* :1046-1067 */
    hvnode* x = &s->nd[v];
    if (x->na >= s->cfg.active_min_size) return;     /* has_reached_limit */
    uint32_t om[1] = {v}, r;
    if (pick_random(s, v, x->pas, x->np, om, 1, &r)) promote_peer(s, v, r);
}
static void passive_view_maintenance(orc_hyparview* s, uint32_t v) {         /* :1078-1111 */
    hvnode* x = &s->nd[v];
    uint32_t ex[XMAX];
    uint32_t nx = select_exchange(s, v, ex);
    uint32_t om[1] = {v}, r;
    if (!pick_random(s, v, x->act, x->na, om, 1, &r)) return;
    if (!s->alive[r]) return;
    hvmsg* f = emit(s, v, r, HV_SHUFFLE);
    f->peer = v; f->ttl = s->cfg.active_rwl; f->nx = nx;
    memcpy(f->x, ex, nx * 4);
}

/* ---------------- API ----------------------------------------------------- */
orc_hyparview* orc_hv_create(uint32_t n, uint64_t seed, const orc_hv_config* cfg) {
    orc_hyparview* s = (orc_hyparview*)calloc(1, sizeof(*s));
    s->n = n; s->seed = seed; s->cfg = *cfg;
    s->nd = (hvnode*)calloc(n, sizeof(hvnode));
    s->alive = (uint8_t*)malloc(n);
    memset(s->alive, 1, n);
    for (uint32_t v = 0; v < n; v++) {               /* init/1: Active = {self}, Passive = {} */
        s->nd[v].act[0] = v; s->nd[v].na = 1;
        s->nd[v].epoch = 1;
    }
    return s;
}

void orc_hv_destroy(orc_hyparview* s) {
    if (!s) return;
    for (uint32_t v = 0; v < s->n; v++) { free(s->nd[v].sent.a); free(s->nd[v].recv.a); }
    free(s->nd); free(s->alive); free(s->cur); free(s->nxt); free(s);
}

void orc_hv_set_alive(orc_hyparview* s, const uint8_t* alive) { memcpy(s->alive, alive, s->n); }

/* handle_cast({join, Peer}) (:999-1016) at `v`: connect + send join */
void orc_hv_join(orc_hyparview* s, uint32_t v, uint32_t contact) {
    if (!s->alive[contact]) return;
    orc_hv_stats* saved = s->st; s->st = NULL;
    hvmsg* m = emit(s, v, contact, HV_JOIN);
    m->peer = v; m->epoch = s->nd[v].epoch;
    s->st = saved;
}

static int cmp_msg(const void* a_, const void* b_) {
    const hvmsg* a = (const hvmsg*)a_; const hvmsg* b = (const hvmsg*)b_;
    if (a->dst != b->dst) return a->dst < b->dst ? -1 : 1;
    if (a->src != b->src) return a->src < b->src ? -1 : 1;
    return a->seq < b->seq ? -1 : (a->seq > b->seq ? 1 : 0);
}

static void one_round(orc_hyparview* s, orc_hv_stats* st) {
    memset(st, 0, sizeof(*st));
    s->st = st;
    hvmsg* t = s->cur; size_t tc = s->capcur;
    s->cur = s->nxt; s->ncur = s->nnxt; s->capcur = s->capnxt;
    s->nxt = t; s->nnxt = 0; s->capnxt = tc;
    qsort(s->cur, s->ncur, sizeof(hvmsg), cmp_msg);
    for (size_t i = 0; i < s->ncur; i++) {
        if (!s->alive[s->cur[i].dst]) continue;
        handle(s, s->cur[i].dst, &s->cur[i]);
    }
    s->round++;
    int prom = s->cfg.promotion_rounds && s->round % s->cfg.promotion_rounds == 0;
    int shuf = s->cfg.shuffle_rounds && s->round % s->cfg.shuffle_rounds == 0;
    if (prom || shuf)
        for (uint32_t v = 0; v < s->n; v++) {
            if (!s->alive[v]) continue;
            if (prom) random_promotion(s, v);
            if (shuf) passive_view_maintenance(s, v);
        }
    st->error = s->error;
    s->st = NULL;
}

uint32_t orc_hv_step(orc_hyparview* s, uint32_t rounds, orc_hv_stats* st) {
    for (uint32_t r = 0; r < rounds; r++) one_round(s, &st[r]);
    return rounds;
}

size_t orc_hv_inflight(const orc_hyparview* s) { return s->nnxt; }

void orc_hv_views(const orc_hyparview* s, uint32_t v, uint32_t* act, uint32_t* na, uint32_t* pas, uint32_t* np) {
    const hvnode* x = &s->nd[v];
    memcpy(act, x->act, x->na * 4); *na = x->na;
    memcpy(pas, x->pas, x->np * 4); *np = x->np;
}

uint64_t orc_hv_draws(const orc_hyparview* s, uint32_t v) { return s->nd[v].draws; }

size_t orc_hv_idmap(const orc_hyparview* s, uint32_t v, int which, uint32_t* peer, uint32_t* ep, uint32_t* cnt, size_t cap) {
    const idmap* m = which ? &s->nd[v].recv : &s->nd[v].sent;
    for (size_t i = 0; i < m->n && i < cap; i++) { peer[i] = m->a[i].peer; ep[i] = m->a[i].epoch; cnt[i] = m->a[i].cnt; }
    return m->n;
}
