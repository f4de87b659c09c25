/*
 * fullmem.c -- restatement of the full-membership strategy
 * (src/partisan_full_membership_strategy.erl:70-268) over the OR-set of
 * src/partisan_membership_set.erl:113-237, whose arithmetic lives in the
 * un-vendored dependency `types 0.1.8` (rebar.lock:9), module state_orset.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Checker for csrc/fullmem.hip.
 *
 * state_orset (types 0.1.8), restated from its published algorithm:
 *   payload  = orddict Elem -> orddict Token -> Active :: boolean()
 *   {add, E} = a fresh unique token for E, active (other tokens of E kept)
 *   {rmv, E} = every token of E inactive; precondition error when E is
 *              absent (partisan_membership_set:remove/3 :136-138 matches
 *              {ok, _}, so the reference crashes there: ORC_BADARG here)
 *   merge    = union of elements and of their tokens; a token present on
 *              both sides is active iff active on both (remove wins per
 *              token, a concurrent add with a fresh token survives)
 *   query    = elements with at least one active token
 *   equal    = payload equality
 * Tokens are random in the reference; here the caller supplies them (any
 * unique u64).  No query, merge or equality result depends on token values,
 * only on their identity.  Pinned by the eunit tests of
 * partisan_membership_set.erl:269-522 (tests/golden/membership_set_kat.json).
 *
 * Round schedule of the full-membership simulation (DESIGN.md "Full
 * membership"):
 *  - node v's actor is v; init/1 (:70-74) = add(v) with token v (fresh data
 *    dir; persisting to disk has no effect on the simulation);
 *  - partisan_peer_service:join is a call made between rounds; the
 *    {connected, Peer, _, _, RemoteState} event (pluggable manager
 *    :1532-1597) is handled at the start of the next round in call order,
 *    with RemoteState = the peer's state at the end of the previous round;
 *    join/3 (:85-96) merges it and gossips to to_peer_list of the result
 *    (:247-268); a join toward a dead peer never connects and is dropped;
 *  - leave(V) at v (internal_leave, pluggable :2059-2109 -> leave/2
 *    :177-214) is also a call between rounds, handled before the joins:
 *    remove V's tokens, gossip StateToGossip to the peers of the OLD state
 *    (V included); V == v restarts v from new_state/1 with a fresh token;
 *  - then the inbox in (src, emission seq) order: handle_message/2
 *    (:135-167) -- equal states: nothing; else merge and re-gossip;
 *  - after each handled message the manager stops when its own spec is no
 *    longer a member (:1791-1803): the vertex becomes dead;
 *  - periodic/1 (:106-111) at the end of rounds t with t % periodic == 0:
 *    gossip the state to every peer, unconditionally (Q27);
 *  - a message carries the sender's state at emission (term_to_binary of
 *    #full_v1{}); a message to a vertex dead at the start of the round is
 *    lost; one to a vertex that stops later in the round is dropped when it
 *    would be handled.
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>

typedef struct { uint64_t tok; uint8_t act; } otok;
typedef struct { uint32_t elem; uint32_t nt, capt; otok* t; } oel;
struct orc_orset { uint32_t ne, cap; oel* e; };

orc_orset* orc_orset_new(void) { return (orc_orset*)calloc(1, sizeof(orc_orset)); }

void orc_orset_free(orc_orset* s) {
    if (!s) return;
    for (uint32_t i = 0; i < s->ne; i++) free(s->e[i].t);
    free(s->e);
    free(s);
}

orc_orset* orc_orset_clone(const orc_orset* s) {
    orc_orset* c = orc_orset_new();
    c->ne = c->cap = s->ne;
    c->e = (oel*)calloc(s->ne ? s->ne : 1, sizeof(oel));
    for (uint32_t i = 0; i < s->ne; i++) {
        c->e[i] = s->e[i];
        c->e[i].capt = s->e[i].nt;
        c->e[i].t = (otok*)malloc((s->e[i].nt ? s->e[i].nt : 1) * sizeof(otok));
        memcpy(c->e[i].t, s->e[i].t, s->e[i].nt * sizeof(otok));
    }
    return c;
}

static oel* find_el(const orc_orset* s, uint32_t elem) {
    for (uint32_t i = 0; i < s->ne; i++) if (s->e[i].elem == elem) return &s->e[i];
    return NULL;
}

/* orddict:store keeps keys sorted */
static oel* insert_el(orc_orset* s, uint32_t elem) {
    oel* f = find_el(s, elem);
    if (f) return f;
    if (s->ne == s->cap) { s->cap = s->cap ? 2 * s->cap : 4; s->e = (oel*)realloc(s->e, s->cap * sizeof(oel)); }
    uint32_t i = s->ne;
    while (i > 0 && s->e[i - 1].elem > elem) { s->e[i] = s->e[i - 1]; i--; }
    memset(&s->e[i], 0, sizeof(oel));
    s->e[i].elem = elem;
    s->ne++;
    return &s->e[i];
}

static void put_tok(oel* e, uint64_t tok, uint8_t act) {
    for (uint32_t i = 0; i < e->nt; i++) if (e->t[i].tok == tok) { e->t[i].act = act; return; }
    if (e->nt == e->capt) { e->capt = e->capt ? 2 * e->capt : 2; e->t = (otok*)realloc(e->t, e->capt * sizeof(otok)); }
    uint32_t i = e->nt;
    while (i > 0 && e->t[i - 1].tok > tok) { e->t[i] = e->t[i - 1]; i--; }
    e->t[i].tok = tok; e->t[i].act = act;
    e->nt++;
}

/* one (Elem, Token, Active) entry of a payload, as a received state carries it */
int orc_orset_put(orc_orset* s, uint32_t elem, uint64_t token, uint8_t active) {
    put_tok(insert_el(s, elem), token, active ? 1 : 0);
    return ORC_OK;
}

/* state_orset:mutate({add, Elem}, Actor, S) via partisan_membership_set:add/3 (:125-127) */
int orc_orset_add(orc_orset* s, uint32_t elem, uint64_t token) {
    put_tok(insert_el(s, elem), token, 1);
    return ORC_OK;
}

/* state_orset:mutate({rmv, Elem}, Actor, S) via partisan_membership_set:remove/3 (:136-138) */
int orc_orset_remove(orc_orset* s, uint32_t elem) {
    oel* e = find_el(s, elem);
    if (!e) return ORC_BADARG;
    for (uint32_t i = 0; i < e->nt; i++) e->t[i].act = 0;
    return ORC_OK;
}

/* state_orset:merge/2 via partisan_membership_set:merge/2 (:170-171) */
orc_orset* orc_orset_merge(const orc_orset* a, const orc_orset* b) {
    orc_orset* m = orc_orset_clone(a);
    for (uint32_t i = 0; i < b->ne; i++) {
        oel* e = insert_el(m, b->e[i].elem);
        for (uint32_t j = 0; j < b->e[i].nt; j++) {
            const otok* t = &b->e[i].t[j];
            int found = 0;
            for (uint32_t k = 0; k < e->nt; k++)
                if (e->t[k].tok == t->tok) { e->t[k].act = e->t[k].act && t->act; found = 1; break; }
            if (!found) put_tok(e, t->tok, t->act);
        }
    }
    return m;
}

/* state_orset:equal/2 via partisan_membership_set:equal/2 (:180-181) */
int orc_orset_equal(const orc_orset* a, const orc_orset* b) {
    if (a->ne != b->ne) return 0;
    for (uint32_t i = 0; i < a->ne; i++) {
        const oel *x = &a->e[i], *y = &b->e[i];
        if (x->elem != y->elem || x->nt != y->nt) return 0;
        for (uint32_t j = 0; j < x->nt; j++)
            if (x->t[j].tok != y->t[j].tok || x->t[j].act != y->t[j].act) return 0;
    }
    return 1;
}

/* to_list/1 (:190-192): lists:sort(sets:to_list(query(T))) -- id order (Q28) */
size_t orc_orset_to_list(const orc_orset* s, uint32_t* out, size_t cap) {
    size_t k = 0;
    for (uint32_t i = 0; i < s->ne; i++) {
        int any = 0;
        for (uint32_t j = 0; j < s->e[i].nt; j++) any |= s->e[i].t[j].act;
        if (any) { if (out && k < cap) out[k] = s->e[i].elem; k++; }
    }
    return k;
}

/* the payload, for inspection: (elem, token, active) rows in orddict order */
size_t orc_orset_dump(const orc_orset* s, uint32_t* elem, uint64_t* tok, uint8_t* act, size_t cap) {
    size_t k = 0;
    for (uint32_t i = 0; i < s->ne; i++)
        for (uint32_t j = 0; j < s->e[i].nt; j++) {
            if (k < cap) { elem[k] = s->e[i].elem; tok[k] = s->e[i].t[j].tok; act[k] = s->e[i].t[j].act; }
            k++;
        }
    return k;
}

static int is_member(const orc_orset* s, uint32_t v) {
    oel* e = find_el(s, v);
    if (!e) return 0;
    for (uint32_t j = 0; j < e->nt; j++) if (e->t[j].act) return 1;
    return 0;
}

/* ------------------------------------------------------------------------ */
/* the round-synchronous full-membership simulation                          */
/* ------------------------------------------------------------------------ */
typedef struct { uint32_t src, dst; uint64_t seq, ord; orc_orset* st; } fmmsg;   /* ord: arrival, breaks (src, seq) ties */
typedef struct { uint32_t v, peer; uint64_t tok; } fmpair;

struct orc_fullmem {
    uint32_t n, periodic;
    uint64_t round, next_token;
    orc_orset** st;
    uint8_t* alive;
    uint8_t* alive0;                 /* alive at the start of the round */
    uint64_t* seq;
    fmmsg* cur; size_t ncur, capcur;
    fmmsg* nxt; size_t nnxt, capnxt;
    uint64_t nord;
    fmpair* jq; size_t njq, capjq;
    fmpair* lq; size_t nlq, caplq;
    orc_fm_stats* stt;
};

orc_fullmem* orc_fm_create(uint32_t n, uint32_t periodic_rounds) {
    orc_fullmem* s = (orc_fullmem*)calloc(1, sizeof(orc_fullmem));
    s->n = n;
    s->periodic = periodic_rounds;
    s->next_token = n;
    s->st = (orc_orset**)calloc(n, sizeof(orc_orset*));
    s->alive = (uint8_t*)malloc(n);
    s->alive0 = (uint8_t*)malloc(n);
    s->seq = (uint64_t*)calloc(n, sizeof(uint64_t));
    memset(s->alive, 1, n);
    for (uint32_t v = 0; v < n; v++) {       /* init/1 -> new_state/1 (:288-294) */
        s->st[v] = orc_orset_new();
        orc_orset_add(s->st[v], v, v);
    }
    return s;
}

static void free_msgs(fmmsg* m, size_t n) { for (size_t i = 0; i < n; i++) orc_orset_free(m[i].st); }

void orc_fm_destroy(orc_fullmem* s) {
    if (!s) return;
    for (uint32_t v = 0; v < s->n; v++) orc_orset_free(s->st[v]);
    free_msgs(s->cur, s->ncur);
    free_msgs(s->nxt, s->nnxt);
    free(s->cur); free(s->nxt); free(s->jq); free(s->lq);
    free(s->st); free(s->alive); free(s->alive0); free(s->seq);
    free(s);
}

void orc_fm_set_alive(orc_fullmem* s, const uint8_t* alive) { memcpy(s->alive, alive, s->n); }

static void push_pair(fmpair** q, size_t* n, size_t* cap, uint32_t v, uint32_t p, uint64_t tok) {
    if (*n == *cap) { *cap = *cap ? 2 * *cap : 64; *q = (fmpair*)realloc(*q, *cap * sizeof(fmpair)); }
    (*q)[*n].v = v; (*q)[*n].peer = p; (*q)[*n].tok = tok; (*n)++;
}

void orc_fm_join(orc_fullmem* s, uint32_t v, uint32_t peer) { push_pair(&s->jq, &s->njq, &s->capjq, v, peer, 0); }
/* a self-leave's fresh token is allocated at call time, in call order */
void orc_fm_leave(orc_fullmem* s, uint32_t v, uint32_t leaving) {
    push_pair(&s->lq, &s->nlq, &s->caplq, v, leaving, leaving == v ? s->next_token++ : 0);
}

/* gossip_messages(State0, State) (:247-268): State to to_peer_list(State0) */
static void gossip(orc_fullmem* s, uint32_t v, const orc_orset* peers_of, const orc_orset* st) {
    for (uint32_t i = 0; i < peers_of->ne; i++) {
        uint32_t p = peers_of->e[i].elem;
        if (p == v || !is_member(peers_of, p)) continue;
        if (s->stt) s->stt->sent++;
        uint64_t q = s->seq[v]++;
        if (!s->alive0[p]) continue;                 /* lost (never connected) */
        if (s->nnxt == s->capnxt) { s->capnxt = s->capnxt ? 2 * s->capnxt : 256; s->nxt = (fmmsg*)realloc(s->nxt, s->capnxt * sizeof(fmmsg)); }
        fmmsg* m = &s->nxt[s->nnxt++];
        m->src = v; m->dst = p; m->seq = q; m->ord = s->nord++; m->st = orc_orset_clone(st);
    }
}

static int members_changed(const orc_orset* a, const orc_orset* b) {
    size_t na = orc_orset_to_list(a, NULL, 0), nb = orc_orset_to_list(b, NULL, 0);
    if (na != nb) return 1;
    for (uint32_t i = 0; i < a->ne; i++)
        if (is_member(a, a->e[i].elem) != is_member(b, a->e[i].elem)) return 1;
    return 0;
}

static void replace_state(orc_fullmem* s, uint32_t v, orc_orset* nst) {
    if (s->stt && members_changed(s->st[v], nst)) s->stt->updates++;
    orc_orset_free(s->st[v]);
    s->st[v] = nst;
}

static int cmp_msg(const void* a, const void* b) {
    const fmmsg *x = (const fmmsg*)a, *y = (const fmmsg*)b;
    if (x->dst != y->dst) return x->dst < y->dst ? -1 : 1;
    if (x->src != y->src) return x->src < y->src ? -1 : 1;
    if (x->seq != y->seq) return x->seq < y->seq ? -1 : 1;
    return x->ord < y->ord ? -1 : x->ord > y->ord;
}

static void one_round(orc_fullmem* s) {
    s->round++;
    /* messages emitted in round t-1 (and between rounds) are delivered now */
    free_msgs(s->cur, s->ncur);
    fmmsg* t = s->cur; s->cur = s->nxt; s->nxt = t;
    size_t tc = s->capcur; s->capcur = s->capnxt; s->capnxt = tc;
    s->ncur = s->nnxt; s->nnxt = 0;
    qsort(s->cur, s->ncur, sizeof(fmmsg), cmp_msg);

    memcpy(s->alive0, s->alive, s->n);
    /* RemoteState of a join = the peer's state at the end of the previous round */
    orc_orset** snap = (orc_orset**)calloc(s->n, sizeof(orc_orset*));
    for (size_t i = 0; i < s->njq; i++) {
        uint32_t p = s->jq[i].peer;
        if (!snap[p]) snap[p] = orc_orset_clone(s->st[p]);
    }
    /* leaves, then joins, made between rounds */
    for (size_t i = 0; i < s->nlq; i++) {
        uint32_t v = s->lq[i].v, who = s->lq[i].peer;
        if (!s->alive[v]) continue;
        orc_orset* g = orc_orset_clone(s->st[v]);
        if (find_el(g, who)) orc_orset_remove(g, who);
        gossip(s, v, s->st[v], g);                   /* peers of State0 (:212) */
        if (who == v) {                              /* new_state(Actor) */
            orc_orset* f = orc_orset_new();
            orc_orset_add(f, v, s->lq[i].tok);
            orc_orset_free(g);
            replace_state(s, v, f);
        } else {
            replace_state(s, v, g);
        }
    }
    s->nlq = 0;
    for (size_t i = 0; i < s->njq; i++) {
        uint32_t v = s->jq[i].v, p = s->jq[i].peer;
        if (!s->alive[v] || !s->alive0[p] || v == p) continue;
        orc_orset* m = orc_orset_merge(s->st[v], snap[p]);   /* join/3 (:85-96) */
        replace_state(s, v, m);
        if (s->stt) s->stt->merges++;
        gossip(s, v, s->st[v], s->st[v]);
    }
    for (uint32_t v = 0; v < s->n; v++) orc_orset_free(snap[v]);
    free(snap);
    s->njq = 0;

    for (size_t i = 0; i < s->ncur; i++) {           /* handle_message/2 (:135-167) */
        fmmsg* m = &s->cur[i];
        uint32_t v = m->dst;
        if (!s->alive[v]) continue;
        if (s->stt) s->stt->processed++;
        if (orc_orset_equal(s->st[v], m->st)) continue;
        orc_orset* nst = orc_orset_merge(s->st[v], m->st);
        replace_state(s, v, nst);
        if (s->stt) s->stt->merges++;
        gossip(s, v, s->st[v], s->st[v]);
        if (!is_member(s->st[v], v)) s->alive[v] = 0;   /* {stop, normal} (:1791-1803) */
    }
    if (s->periodic && s->round % s->periodic == 0)      /* handle_info(periodic) :1386-1419 */
        for (uint32_t v = 0; v < s->n; v++)
            if (s->alive[v]) gossip(s, v, s->st[v], s->st[v]);
}

uint32_t orc_fm_step(orc_fullmem* s, uint32_t rounds, orc_fm_stats* st) {
    for (uint32_t r = 0; r < rounds; r++) {
        s->stt = st ? &st[r] : NULL;
        if (s->stt) memset(s->stt, 0, sizeof(*s->stt));
        one_round(s);
        if (s->stt) {
            s->stt->inflight = s->nnxt;
            for (uint32_t v = 0; v < s->n; v++)
                if (s->alive[v]) s->stt->member_sum += orc_orset_to_list(s->st[v], NULL, 0);
        }
    }
    s->stt = NULL;
    return rounds;
}

size_t orc_fm_inflight(const orc_fullmem* s) { return s->nnxt; }

/* The messages on the wire (the pluggable manager's {membership_strategy,
 * {NodeSpec, #full_v1{}}} sends, partisan_full_membership_strategy.erl:247-267)
 * in handling order (dst, src, seq); their states via orc_fm_message_state. */
size_t orc_fm_messages(orc_fullmem* s, uint32_t* src, uint32_t* dst, uint64_t* seq, size_t cap) {
    qsort(s->nxt, s->nnxt, sizeof(fmmsg), cmp_msg);
    for (size_t i = 0; i < s->nnxt && i < cap; i++) {
        if (src) src[i] = s->nxt[i].src;
        if (dst) dst[i] = s->nxt[i].dst;
        if (seq) seq[i] = s->nxt[i].seq;
    }
    return s->nnxt;
}

const orc_orset* orc_fm_message_state(const orc_fullmem* s, size_t i) { return i < s->nnxt ? s->nxt[i].st : NULL; }

/* dst's messages off the wire, in handling order; the caller owns st[i].
 * More than cap: nothing is taken. */
size_t orc_fm_take(orc_fullmem* s, uint32_t dst, uint32_t* src, uint64_t* seq, orc_orset** st, size_t cap) {
    qsort(s->nxt, s->nnxt, sizeof(fmmsg), cmp_msg);
    size_t c = 0;
    for (size_t i = 0; i < s->nnxt; i++) c += s->nxt[i].dst == dst;
    if (c > cap) return c;
    size_t k = 0, o = 0;
    for (size_t i = 0; i < s->nnxt; i++) {
        if (s->nxt[i].dst == dst) {
            src[k] = s->nxt[i].src; seq[k] = s->nxt[i].seq; st[k] = s->nxt[i].st;
            k++;
        } else {
            s->nxt[o++] = s->nxt[i];
        }
    }
    s->nnxt = o;
    return c;
}

/* a message a manager received, onto the wire for the next round (the state is copied) */
void orc_fm_put(orc_fullmem* s, uint32_t src, uint32_t dst, uint64_t seq, const orc_orset* st) {
    if (s->nnxt == s->capnxt) { s->capnxt = s->capnxt ? 2 * s->capnxt : 256; s->nxt = (fmmsg*)realloc(s->nxt, s->capnxt * sizeof(fmmsg)); }
    fmmsg* m = &s->nxt[s->nnxt++];
    m->src = src; m->dst = dst; m->seq = seq; m->ord = s->nord++; m->st = orc_orset_clone(st);
}

size_t orc_fm_members(const orc_fullmem* s, uint32_t v, uint32_t* out, size_t cap) {
    return orc_orset_to_list(s->st[v], out, cap);
}

const orc_orset* orc_fm_state(const orc_fullmem* s, uint32_t v) { return s->st[v]; }

int orc_fm_alive(const orc_fullmem* s, uint32_t v) { return s->alive[v]; }
