/*
 * demers.c -- round-synchronous restatement of
 *   protocols/demers_rumor_mongering.erl (:92-186)
 *   protocols/demers_anti_entropy.erl    (:95-227)
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Checker for
 * partisan_amd/csrc/demers.hip.  Parity of Demers trajectories is
 * unpinned by reference vectors (only the convergence
 * postcondition is pinned, test/prop_partisan_reliable_broadcast.erl:127-172).
 *
 * Simulation contract (DESIGN.md "Demers"):
 *  - full membership: members = all vertices incl. self (membership/1 =
 *    lists:usort(Members), :177-178) -- implicit ids 0..N-1;
 *  - each process has its own sequential draw stream, as Erlang's per-process
 *    `rand` state (partisan_config.erl:701-716 seeds each process): Philox
 *    stream (seed, vertex, kind) -- kind RM for demers_rumor_mongering, AE for
 *    demers_anti_entropy -- whose j-th draw is the u64 {x, y} of Philox
 *    counter {vertex, j_lo, kind, j_hi}; the process's counter advances by the
 *    draws each call consumes, in the order the process makes its calls;
 *  - select_random_sublist(usort(Members), 2) (:179-186, :222-227) =
 *    lists:sublist(shuffle(L), 2), shuffle/1 = sort of {rand:uniform(), N}:
 *    FAITHFUL mode (n <= DM_FAITHFUL_MAX): one draw per member in list order,
 *    the two smallest (draw >> 11, member) -- rand:uniform()'s 53-bit float and
 *    the tuple order; n draws per call.  SCALED mode (larger n): the same
 *    distribution -- a uniform ordered pair of distinct members -- from 2
 *    draws, i1 = floor(d0 n / 2^64), i2 = floor(d1 (n-1) / 2^64) (+1 if >= i1);
 *  - rumor m originates at origin(m) = uniform draw of the workload stream;
 *  - the two processes share one message store (Demers et al.'s rumor
 *    mongering backed by anti-entropy; run alone, each is the reference
 *    module: rm only = ae_period 0, ae only = rm off, with Q20's id reuse);
 *  - round t: RM messages (sorted by rumor, then senders that are not among
 *    the receiver's own forward targets for that rumor, then those that are,
 *    each by id), then AE push (by sender), then AE pull (by sender); the AE
 *    tick fires at the end of rounds t with t % ae_period == 0.
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>

/* Philox4x32-10 (Random123), independent of the product's device copy. */
void orc_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static uint64_t mulhi64(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) >> 64); }

/* draw j of process (v, kind)'s stream */
static uint64_t draw64(uint64_t seed, uint32_t v, uint32_t kind, uint64_t j) {
    uint32_t ctr[4] = {v, (uint32_t)j, kind, (uint32_t)(j >> 32)}, key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)}, r[4];
    orc_philox4x32_10(ctr, key, r);
    return (uint64_t)r[0] | ((uint64_t)r[1] << 32);
}

/* draws one select_random_sublist(usort(Members), 2) call consumes over n members */
static uint64_t dm_draws_per_call(uint32_t n) { return n <= DM_FAITHFUL_MAX ? n : 2; }

/* select_random_sublist(usort(Members), 2) over members 0..n-1 (n >= 2), the
 * call whose first draw is draw j of process (v, kind) */
static void select2(uint64_t seed, uint32_t v, uint32_t kind, uint32_t n, uint64_t j, uint32_t out[2]) {
    if (n <= DM_FAITHFUL_MAX) {                      /* lists:sort([{rand:uniform(), N} || N <- L]) */
        uint64_t k0 = ~0ull, k1 = ~0ull;
        uint32_t i0 = 0, i1 = 0;
        for (uint32_t i = 0; i < n; i++) {
            const uint64_t k = draw64(seed, v, kind, j + i) >> 11;
            if (k < k0) { k1 = k0; i1 = i0; k0 = k; i0 = i; }
            else if (k < k1) { k1 = k; i1 = i; }
        }
        out[0] = i0; out[1] = i1;
        return;
    }
    out[0] = (uint32_t)mulhi64(draw64(seed, v, kind, j), n);
    uint32_t i2 = (uint32_t)mulhi64(draw64(seed, v, kind, j + 1), n - 1);
    if (i2 >= out[0]) i2++;
    out[1] = i2;
}

int orc_dm_select2(uint64_t seed, uint32_t v, uint32_t kind, uint32_t n, uint64_t j, uint32_t* out) {
    if (n < 2) return 0;
    select2(seed, v, kind, n, j, out);
    return 2;
}

uint64_t orc_dm_draws_per_call(uint32_t n) { return dm_draws_per_call(n); }

enum { DM_RM = 1, DM_PUSH = 2, DM_PULL = 3 };
enum { KIND_WORKLOAD = 1, KIND_RM = 2, KIND_AE = 3 };

typedef struct { uint32_t type, src, dst, m; uint64_t payload, seq; uint32_t cls; uint32_t _pad; } dmsg;

struct orc_demers {
    uint32_t n, m, ae_period, rm_on;
    uint64_t seed, round;
    uint64_t* seen;              /* ETS ?MODULE of each process (shared store) */
    uint64_t* emitted;           /* per-vertex emission counter (FIFO seq)     */
    uint64_t* rmdraw;            /* draws taken by each vertex's RM process     */
    uint64_t* aedraw;            /* draws taken by each vertex's AE process     */
    uint64_t* newrm;             /* scratch: rumors new at v among this round's RM messages */
    uint64_t dpc;                /* draws per select_random_sublist call        */
    uint32_t* origin;            /* origin of rumor m                           */
    uint32_t* idbit;             /* store bit of rumor m (Q20 in ae-only mode)  */
    uint64_t full;
    dmsg* cur; size_t ncur, capcur;
    dmsg* nxt; size_t nnxt, capnxt;
    orc_dm_stats* st;
};

static void emit(orc_demers* s, uint32_t type, uint32_t src, uint32_t dst, uint32_t m, uint64_t payload) {
    if (s->nnxt == s->capnxt) { s->capnxt = s->capnxt ? s->capnxt * 2 : 4096; s->nxt = (dmsg*)realloc(s->nxt, s->capnxt * sizeof(dmsg)); }
    dmsg* x = &s->nxt[s->nnxt++];
    x->type = type; x->src = src; x->dst = dst; x->m = m; x->payload = payload; x->seq = s->emitted[src]++;
    x->cls = 0;
    if (s->st) {
        if (type == DM_RM) s->st->rm_sent++;
        else if (type == DM_PUSH) s->st->push_sent++;
        else s->st->pull_sent++;
    }
}

orc_demers* orc_dm_create(uint32_t n, uint32_t m, uint64_t seed, uint32_t ae_period, uint32_t rm_on) {
    if (m == 0 || m > 64 || n < 2) return NULL;
    orc_demers* s = (orc_demers*)calloc(1, sizeof(*s));
    s->n = n; s->m = m; s->seed = seed; s->ae_period = ae_period; s->rm_on = rm_on;
    s->seen = (uint64_t*)calloc(n, 8);
    s->emitted = (uint64_t*)calloc(n, 8);
    s->rmdraw = (uint64_t*)calloc(n, 8);
    s->aedraw = (uint64_t*)calloc(n, 8);
    s->newrm = (uint64_t*)calloc(n, 8);
    s->dpc = dm_draws_per_call(n);
    s->origin = (uint32_t*)calloc(m, 4);
    s->idbit = (uint32_t*)calloc(m, 4);
    for (uint32_t i = 0; i < m; i++) {
        uint32_t ctr[4] = {i, 0, KIND_WORKLOAD, 0}, key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)}, r[4];
        orc_philox4x32_10(ctr, key, r);
        s->origin[i] = (uint32_t)mulhi64((uint64_t)r[0] | ((uint64_t)r[1] << 32), n);
        s->idbit[i] = i;
        if (!rm_on)   /* anti-entropy alone: next_id never increments, ids {Node, 0} (Q20) */
            for (uint32_t j = 0; j < i; j++) if (s->origin[j] == s->origin[i]) { s->idbit[i] = s->idbit[j]; break; }
        s->full |= 1ull << s->idbit[i];
    }
    return s;
}

void orc_dm_destroy(orc_demers* s) {
    if (!s) return;
    free(s->seen); free(s->emitted); free(s->rmdraw); free(s->aedraw); free(s->newrm); free(s->origin); free(s->idbit); free(s->cur); free(s->nxt);
    free(s);
}

uint32_t orc_dm_origin(const orc_demers* s, uint32_t m) { return s->origin[m]; }
uint64_t orc_dm_full_mask(const orc_demers* s) { return s->full; }

/* handle_cast({broadcast, ServerRef, Message}) at every origin, rumor order.
 * RM (:92-115): deliver, store, forward to select_random_sublist(..) -- [MyNode].
 * AE (:95-106): deliver and store only.
 * Direct mail (rm_on == 2, demers_direct_mail.erl:91-121): deliver, store,
 * forward to every member but MyNode. */
void orc_dm_broadcast_all(orc_demers* s) {
    for (uint32_t i = 0; i < s->m; i++) {
        uint32_t o = s->origin[i];
        s->seen[o] |= 1ull << s->idbit[i];
        if (!s->rm_on) continue;
        if (s->rm_on == 2) {
            for (uint32_t t = 0; t < s->n; t++) if (t != o) emit(s, DM_RM, o, t, i, 0);
            continue;
        }
        uint32_t t[2];
        select2(s->seed, o, KIND_RM, s->n, s->rmdraw[o], t);   /* the origin's RM process calls once per rumor */
        s->rmdraw[o] += s->dpc;
        for (int j = 0; j < 2; j++) if (t[j] != o) emit(s, DM_RM, o, t[j], i, 0);
    }
}

static int cmp_msg(const void* x, const void* y) {
    const dmsg* a = (const dmsg*)x; const dmsg* b = (const dmsg*)y;
    if (a->dst != b->dst) return a->dst < b->dst ? -1 : 1;
    if (a->type != b->type) return a->type < b->type ? -1 : 1;
    if (a->type == DM_RM) {
        if (a->m != b->m) return a->m < b->m ? -1 : 1;
        if (a->cls != b->cls) return a->cls < b->cls ? -1 : 1;
    }
    if (a->src != b->src) return a->src < b->src ? -1 : 1;
    if (a->seq != b->seq) return a->seq < b->seq ? -1 : 1;
    return 0;
}

static void one_round(orc_demers* s, orc_dm_stats* st) {
    memset(st, 0, sizeof(*st));
    s->st = st;
    dmsg* t = s->cur; size_t tc = s->capcur;
    s->cur = s->nxt; s->ncur = s->nnxt; s->capcur = s->capnxt;
    s->nxt = t; s->nnxt = 0; s->capnxt = tc;
    /* class of an RM message: is the sender one of the receiver's own targets
     * for the rumor, i.e. of the call the receiver's RM process makes when it
     * accepts it -- its (rank + 1)-th call this round, rank = the new rumors
     * with smaller ids (RM messages are handled by rumor first) */
    for (size_t i = 0; i < s->ncur; i++) {
        const dmsg* x = &s->cur[i];
        if (x->type == DM_RM && !(s->seen[x->dst] & (1ull << s->idbit[x->m]))) s->newrm[x->dst] |= 1ull << x->m;
    }
    for (size_t i = 0; i < s->ncur; i++) {
        dmsg* x = &s->cur[i];
        x->cls = 0;
        if (x->type != DM_RM || s->rm_on == 2 || !((s->newrm[x->dst] >> x->m) & 1ull)) continue;
        const uint64_t below = s->newrm[x->dst] & ((1ull << x->m) - 1ull);
        uint32_t tg[2];
        select2(s->seed, x->dst, KIND_RM, s->n, s->rmdraw[x->dst] + s->dpc * (uint64_t)__builtin_popcountll(below), tg);
        for (int j = 0; j < 2; j++) if (tg[j] == x->src) x->cls = 1;
    }
    for (size_t i = 0; i < s->ncur; i++) s->newrm[s->cur[i].dst] = 0;
    qsort(s->cur, s->ncur, sizeof(dmsg), cmp_msg);
    for (size_t i = 0; i < s->ncur; i++) {
        const dmsg* x = &s->cur[i];
        uint32_t v = x->dst;
        if (x->type == DM_RM) {                      /* handle_info({broadcast, Id, ..., FromNode}) :127-158 */
            uint64_t b = 1ull << s->idbit[x->m];
            if (s->seen[v] & b) continue;            /* ets:lookup -> [_] */
            s->seen[v] |= b;                         /* deliver + ets:insert */
            st->delivered_new++;
            if (s->rm_on == 2) continue;             /* direct mail :127-143: store only */
            uint32_t tg[2];
            select2(s->seed, v, KIND_RM, s->n, s->rmdraw[v], tg);
            s->rmdraw[v] += s->dpc;
            for (int j = 0; j < 2; j++)              /* AntiEntropyMembers -- [MyNode, FromNode] */
                if (tg[j] != v && tg[j] != x->src) emit(s, DM_RM, v, tg[j], x->m, 0);
        } else if (x->type == DM_PUSH) {             /* handle_info({push, FromNode, TheirMessages}) :143-176 */
            uint64_t nw = x->payload & ~s->seen[v];
            st->delivered_new += (uint64_t)__builtin_popcountll(nw);
            s->seen[v] |= x->payload;
            emit(s, DM_PULL, v, x->src, 0, s->seen[v]);
        } else {                                     /* handle_info({pull, _, Messages}) :178-195 */
            uint64_t nw = x->payload & ~s->seen[v];
            st->delivered_new += (uint64_t)__builtin_popcountll(nw);
            s->seen[v] |= x->payload;
        }
    }
    s->round++;
    if (s->ae_period && s->round % s->ae_period == 0) {   /* handle_info(antientropy) :118-141 */
        for (uint32_t v = 0; v < s->n; v++) {
            uint32_t tg[2];
            select2(s->seed, v, KIND_AE, s->n, s->aedraw[v], tg);   /* one call per tick: (tick - 1) dpc draws before */
            s->aedraw[v] += s->dpc;
            for (int j = 0; j < 2; j++) if (tg[j] != v) emit(s, DM_PUSH, v, tg[j], 0, s->seen[v]);
        }
    }
    uint64_t done = 0;
    for (uint32_t v = 0; v < s->n; v++) done += (s->seen[v] & s->full) == s->full;
    st->complete = done;
    s->st = NULL;
}

uint32_t orc_dm_step(orc_demers* s, uint32_t rounds, orc_dm_stats* st) {
    for (uint32_t r = 0; r < rounds; r++) one_round(s, &st[r]);
    return rounds;
}

uint32_t orc_dm_run(orc_demers* s, uint32_t max_rounds, orc_dm_stats* st, size_t cap) {
    orc_dm_stats tmp;
    uint32_t r = 0;
    for (;;) {
        uint64_t done = 0;
        for (uint32_t v = 0; v < s->n; v++) done += (s->seen[v] & s->full) == s->full;
        if (done == s->n || r >= max_rounds) break;
        one_round(s, r < cap ? &st[r] : &tmp);
        r++;
    }
    return r;
}

void orc_dm_get_seen(const orc_demers* s, uint64_t* out) { memcpy(out, s->seen, (size_t)s->n * 8); }

size_t orc_dm_pending(const orc_demers* s, uint32_t* type, uint32_t* src, uint32_t* dst, uint32_t* m,
                      uint64_t* payload, size_t cap) {
    for (size_t i = 0; i < s->nnxt && i < cap; i++) {
        type[i] = s->nxt[i].type; src[i] = s->nxt[i].src; dst[i] = s->nxt[i].dst; m[i] = s->nxt[i].m;
        payload[i] = s->nxt[i].payload;
    }
    return s->nnxt;
}
