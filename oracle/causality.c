/*
 * causality.c -- restatement of the causal delivery backend
 * (src/partisan_causality_backend.erl: emit 172-201, receive_message
 * 205-220, handle_info(deliver) 233-248, deliver 265-300,
 * internal_receive_message 309-344) over the sparse clocks of vclock.c.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Checker for csrc/causal.hip.
 *
 * Pinned by test/partisan_SUITE.erl:500-586 (causal_test, transcribed as
 * tests/golden/causal_kat.json) through the primitive API below; the
 * round-driven workload (C5) is parity unpinned by reference vectors.
 *
 * Quirks kept: every emit increments the sender's own entry (so the clocks
 * of one broadcast differ per destination); the order buffer ships only the
 * destination's entry; deliver discards the orddict:merge of order buffers
 * (Q24); the delivery test is strict dominates; a buffer fold tries every
 * buffered message once, in buffer order, so a message unblocked by a later
 * one waits for the next fold (Q25).
 *
 * Round workload (DESIGN.md "Causal delivery"): M <= 64 emitters
 * e_k = floor(k * N / M).  At the end of round t, emitter k broadcasts
 * (emit to every other vertex in id order) iff t % P == k % P.  The message
 * to v emitted at round t arrives in round t + d, d = 1 + mulhi(draw, D),
 * draw = Philox({v, t, 6, k}).  Round t at v: arrivals in (src, seq) order,
 * each a receive_message; then handle_info(deliver) if t % redeliver == 0.
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>

#define KIND_CAUSAL 6u

typedef struct { orc_dot* d; size_t n; } clk;

typedef struct cmsg {
    uint32_t src, dest, k, round;
    uint64_t seq;
    clk clock;          /* MessageClock */
    int has_dep;        /* IncomingOrderBuffer has MyNode (the destination) */
    clk dep;
    struct cmsg* next;  /* arrival bucket chain */
} cmsg;

typedef struct {
    clk local;
    clk* ob;            /* order buffer: dest -> clock (emitters / primitive API) */
    uint8_t* ob_has;
    cmsg** buf; size_t nbuf, capbuf;     /* buffered_messages, list order */
    cmsg** log; size_t nlog, caplog;     /* deliveries (primitive API) */
    uint64_t seq, delivered;
} cnode;

struct orc_causal {
    uint32_t n, m, period, dmax, redeliver;
    uint64_t seed, round;
    cnode* nd;
    uint32_t* emitter;                   /* [m] */
    int32_t* kof;                        /* [n] emitter index or -1 */
    cmsg** bucket;                       /* [dmax + 1] ring of arrival chains */
    int keep_log;
    orc_causal_stats* st;
};

static clk clk_copy(const clk* c) {
    clk r;
    r.n = c->n;
    r.d = (orc_dot*)malloc((c->n + 1) * sizeof(orc_dot));
    memcpy(r.d, c->d, c->n * sizeof(orc_dot));
    return r;
}
static void clk_free(clk* c) { free(c->d); c->d = NULL; c->n = 0; }

/* partisan_vclock:increment/2 */
static void clk_increment(clk* c, uint32_t actor) {
    orc_dot* out = (orc_dot*)malloc((c->n + 2) * sizeof(orc_dot));
    size_t k = 0;
    orc_vc_increment(actor, c->d, c->n, out, c->n + 2, &k);
    free(c->d);
    c->d = out; c->n = k;
}
/* partisan_vclock:merge([A, B]) */
static void clk_merge(clk* a, const clk* b) {
    size_t lens[2] = {a->n, b->n};
    orc_dot* flat = (orc_dot*)malloc((a->n + b->n + 1) * sizeof(orc_dot));
    memcpy(flat, a->d, a->n * sizeof(orc_dot));
    memcpy(flat + a->n, b->d, b->n * sizeof(orc_dot));
    orc_dot* out = (orc_dot*)malloc((a->n + b->n + 1) * sizeof(orc_dot));
    size_t k = 0;
    orc_vc_merge(flat, lens, 2, out, a->n + b->n + 1, &k);
    free(flat); free(a->d);
    a->d = out; a->n = k;
}

static void push(cmsg*** arr, size_t* n, size_t* cap, cmsg* x) {
    if (*n == *cap) { *cap = *cap ? *cap * 2 : 8; *arr = (cmsg**)realloc(*arr, *cap * sizeof(cmsg*)); }
    (*arr)[(*n)++] = x;
}

orc_causal* orc_causal_create(uint32_t n, uint32_t m, uint32_t period, uint32_t dmax, uint32_t redeliver,
                              uint64_t seed) {
    orc_causal* s = (orc_causal*)calloc(1, sizeof(*s));
    s->n = n; s->m = m; s->period = period ? period : 1; s->dmax = dmax ? dmax : 1;
    s->redeliver = redeliver; s->seed = seed;
    s->nd = (cnode*)calloc(n, sizeof(cnode));
    s->kof = (int32_t*)malloc(n * sizeof(int32_t));
    for (uint32_t v = 0; v < n; v++) s->kof[v] = -1;
    s->emitter = (uint32_t*)calloc(m ? m : 1, sizeof(uint32_t));
    for (uint32_t k = 0; k < m; k++) {
        s->emitter[k] = (uint32_t)(((uint64_t)k * n) / m);
        s->kof[s->emitter[k]] = (int32_t)k;
    }
    s->bucket = (cmsg**)calloc(s->dmax + 1, sizeof(cmsg*));
    s->keep_log = (m == 0);              /* primitive API: keep delivery logs */
    return s;
}

static void free_msg(cmsg* x) { clk_free(&x->clock); clk_free(&x->dep); free(x); }

void orc_causal_destroy(orc_causal* s) {
    if (!s) return;
    for (uint32_t b = 0; b <= s->dmax; b++)
        for (cmsg* x = s->bucket[b]; x;) { cmsg* nx = x->next; free_msg(x); x = nx; }
    for (uint32_t v = 0; v < s->n; v++) {
        cnode* x = &s->nd[v];
        clk_free(&x->local);
        if (x->ob) { for (uint32_t d = 0; d < s->n; d++) clk_free(&x->ob[d]); free(x->ob); free(x->ob_has); }
        for (size_t i = 0; i < x->nbuf; i++) free_msg(x->buf[i]);
        free(x->buf);
        if (s->keep_log) for (size_t i = 0; i < x->nlog; i++) free_msg(x->log[i]);
        free(x->log);
    }
    free(s->nd); free(s->kof); free(s->emitter); free(s->bucket); free(s);
}

/* handle_call({emit, Node, ServerRef, Message}) (:172-201) at `v` toward `dest` */
static cmsg* emit(orc_causal* s, uint32_t v, uint32_t dest) {
    cnode* x = &s->nd[v];
    clk_increment(&x->local, v);                         /* LocalClock = increment(MyNode, LocalClock0) */
    if (!x->ob) { x->ob = (clk*)calloc(s->n, sizeof(clk)); x->ob_has = (uint8_t*)calloc(s->n, 1); }
    cmsg* m = (cmsg*)calloc(1, sizeof(cmsg));
    m->src = v; m->dest = dest; m->seq = x->seq++;
    m->clock = clk_copy(&x->local);
    if (x->ob_has[dest]) { m->has_dep = 1; m->dep = x->ob[dest]; }    /* FilteredOrderBuffer = [{Node, Clock}] */
    x->ob[dest] = clk_copy(&x->local);                   /* orddict:store(Node, LocalClock, OrderBuffer0) */
    x->ob_has[dest] = 1;
    if (s->st) s->st->emitted++;
    return m;
}

/* deliver/5 (:265-300): the orddict:merge of order buffers is discarded (Q24) */
static void deliver(orc_causal* s, uint32_t v, cmsg* m) {
    cnode* x = &s->nd[v];
    clk_merge(&x->local, &m->clock);                     /* merge([LocalClock, MessageClock]) */
    clk_increment(&x->local, v);
    x->delivered++;
    if (s->st) s->st->delivered++;
    if (s->keep_log) push(&x->log, &x->nlog, &x->caplog, m);
    else free_msg(m);
}

/* internal_receive_message/2 (:309-344): returns 1 if delivered */
static int try_deliver(orc_causal* s, uint32_t v, cmsg* m) {
    cnode* x = &s->nd[v];
    if (m->has_dep) {
        if (s->st) s->st->checks++;
        if (!orc_vc_dominates(x->local.d, x->local.n, m->dep.d, m->dep.n)) return 0;
    }
    /* buffered_messages = BufferedMessages -- [FullMessage] */
    for (size_t i = 0; i < x->nbuf; i++)
        if (x->buf[i] == m) { memmove(&x->buf[i], &x->buf[i + 1], (x->nbuf - i - 1) * sizeof(cmsg*)); x->nbuf--; break; }
    deliver(s, v, m);
    return 1;
}

/* one lists:foldl over a snapshot of the buffer */
static void fold(orc_causal* s, uint32_t v) {
    cnode* x = &s->nd[v];
    size_t k = x->nbuf;
    if (!k) return;
    cmsg** snap = (cmsg**)malloc(k * sizeof(cmsg*));
    memcpy(snap, x->buf, k * sizeof(cmsg*));
    for (size_t i = 0; i < k; i++) try_deliver(s, v, snap[i]);
    free(snap);
}

/* handle_call({receive_message, M}) (:205-220) */
static void receive(orc_causal* s, uint32_t v, cmsg* m) {
    cnode* x = &s->nd[v];
    push(&x->buf, &x->nbuf, &x->capbuf, m);              /* BufferedMessages0 ++ [FullMessage] */
    if (s->st) s->st->received++;
    fold(s, v);
}

/* ---------------- primitive API (the partisan_SUITE causal_test) ---------- */
static cmsg** g_handles = NULL;    /* not thread-safe: test helper only */
static size_t g_nh = 0, g_caph = 0;

uint32_t orc_causal_emit(orc_causal* s, uint32_t node, uint32_t dest) {
    cmsg* m = emit(s, node, dest);
    push(&g_handles, &g_nh, &g_caph, m);
    return (uint32_t)(g_nh - 1);
}
void orc_causal_receive(orc_causal* s, uint32_t node, uint32_t msg) { receive(s, node, g_handles[msg]); }
void orc_causal_tick(orc_causal* s, uint32_t node) { fold(s, node); }
size_t orc_causal_log(const orc_causal* s, uint32_t node, uint32_t* msgs, size_t cap) {
    const cnode* x = &s->nd[node];
    size_t k = 0;
    for (size_t i = 0; i < x->nlog; i++)
        for (size_t h = 0; h < g_nh; h++)
            if (g_handles[h] == x->log[i]) { if (k < cap) msgs[k] = (uint32_t)h; k++; break; }
    return k;
}
void orc_causal_reset_handles(void) { free(g_handles); g_handles = NULL; g_nh = g_caph = 0; }

/* ---------------- round workload ------------------------------------------ */
static uint32_t delay_of(const orc_causal* s, uint32_t v, uint64_t t, uint32_t k) {
    uint32_t ctr[4] = {v, (uint32_t)t, KIND_CAUSAL, k}, key[2] = {(uint32_t)s->seed, (uint32_t)(s->seed >> 32)}, r[4];
    orc_philox4x32_10(ctr, key, r);
    const uint64_t x = (uint64_t)r[0] | ((uint64_t)r[1] << 32);
    return 1u + (uint32_t)(((unsigned __int128)x * s->dmax) >> 64);
}

static int cmp_arrival(const void* a_, const void* b_) {
    const cmsg* a = *(cmsg* const*)a_; const cmsg* b = *(cmsg* const*)b_;
    if (a->dest != b->dest) return a->dest < b->dest ? -1 : 1;
    if (a->src != b->src) return a->src < b->src ? -1 : 1;
    return a->seq < b->seq ? -1 : (a->seq > b->seq);
}

static void one_round(orc_causal* s, orc_causal_stats* st) {
    memset(st, 0, sizeof(*st));
    s->st = st;
    const uint64_t t = ++s->round;
    /* arrivals of round t */
    cmsg** arr = NULL; size_t na = 0, capa = 0;
    const uint32_t slot = (uint32_t)(t % (s->dmax + 1));
    for (cmsg* x = s->bucket[slot]; x; x = x->next) push(&arr, &na, &capa, x);
    s->bucket[slot] = NULL;
    if (na) qsort(arr, na, sizeof(cmsg*), cmp_arrival);
    size_t i = 0;
    for (uint32_t v = 0; v < s->n; v++) {
        while (i < na && arr[i]->dest == v) receive(s, v, arr[i++]);
        if (s->redeliver && t % s->redeliver == 0) fold(s, v);
    }
    free(arr);
    /* broadcasts at the end of round t */
    for (uint32_t k = 0; k < s->m; k++) {
        if (t % s->period != k % s->period) continue;
        const uint32_t e = s->emitter[k];
        for (uint32_t d = 0; d < s->n; d++) {
            if (d == e) continue;
            cmsg* m = emit(s, e, d);
            m->k = k; m->round = (uint32_t)t;
            const uint32_t dl = delay_of(s, d, t, k);
            const uint32_t b = (uint32_t)((t + dl) % (s->dmax + 1));
            m->next = s->bucket[b];
            s->bucket[b] = m;
        }
    }
    for (uint32_t v = 0; v < s->n; v++) st->buffered += s->nd[v].nbuf;
    s->st = NULL;
}

uint32_t orc_causal_step(orc_causal* s, uint32_t rounds, orc_causal_stats* st) {
    for (uint32_t r = 0; r < rounds; r++) one_round(s, &st[r]);
    return rounds;
}

size_t orc_causal_clock(const orc_causal* s, uint32_t v, orc_dot* out, size_t cap) {
    const clk* c = &s->nd[v].local;
    for (size_t i = 0; i < c->n && i < cap; i++) out[i] = c->d[i];
    return c->n;
}
size_t orc_causal_buffered(const orc_causal* s, uint32_t v, uint32_t* k, uint32_t* round, size_t cap) {
    const cnode* x = &s->nd[v];
    for (size_t i = 0; i < x->nbuf && i < cap; i++) { k[i] = x->buf[i]->k; round[i] = x->buf[i]->round; }
    return x->nbuf;
}
uint64_t orc_causal_delivered(const orc_causal* s, uint32_t v) { return s->nd[v].delivered; }
uint32_t orc_causal_emitter(const orc_causal* s, uint32_t k) { return s->emitter[k]; }
