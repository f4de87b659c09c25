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
 *  - select_random_sublist(Members, 2) = the first two of shuffle/1, i.e. a
 *    uniformly random ordered pair of distinct members; drawn from Philox
 *    stream (seed, vertex, event, kind): RM event = rumor id, AE event = tick;
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

/* select_random_sublist(usort(Members), 2) over members 0..n-1 */
static int sample2(uint64_t seed, uint32_t v, uint32_t event, uint32_t kind, uint32_t n, uint32_t out[2]) {
    uint32_t ctr[4] = {v, event, kind, 0}, key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)}, r[4];
    orc_philox4x32_10(ctr, key, r);
    uint64_t r0 = (uint64_t)r[0] | ((uint64_t)r[1] << 32), r1 = (uint64_t)r[2] | ((uint64_t)r[3] << 32);
    if (n == 0) return 0;
    out[0] = (uint32_t)mulhi64(r0, n);
    if (n == 1) return 1;
    uint32_t i2 = (uint32_t)mulhi64(r1, n - 1);
    if (i2 >= out[0]) i2++;
    out[1] = i2;
    return 2;
}

int orc_dm_sample2(uint64_t seed, uint32_t v, uint32_t event, uint32_t kind, uint32_t n, uint32_t* out) {
    return sample2(seed, v, event, kind, n, out);
}

enum { DM_RM = 1, DM_PUSH = 2, DM_PULL = 3 };
enum { KIND_WORKLOAD = 1, KIND_RM = 2, KIND_AE = 3 };

typedef struct { uint32_t type, src, dst, m; uint64_t payload, seq; uint32_t cls; uint32_t _pad; } dmsg;

struct orc_demers {
    uint32_t n, m, ae_period, rm_on;
    uint64_t seed, round;
    uint64_t* seen;              /* ETS ?MODULE of each process (shared store) */
    uint64_t* emitted;           /* per-vertex emission counter (FIFO seq)     */
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
    free(s->seen); free(s->emitted); free(s->origin); free(s->idbit); free(s->cur); free(s->nxt);
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
        int k = sample2(s->seed, o, i, KIND_RM, s->n, t);
        for (int j = 0; j < k; j++) if (t[j] != o) emit(s, DM_RM, o, t[j], i, 0);
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
    /* class of an RM message: is the sender one of the receiver's own targets */
    for (size_t i = 0; i < s->ncur; i++) {
        dmsg* x = &s->cur[i];
        if (x->type != DM_RM || s->rm_on == 2) continue;
        uint32_t tg[2];
        int k = sample2(s->seed, x->dst, x->m, KIND_RM, s->n, tg);
        x->cls = 0;
        for (int j = 0; j < k; j++) if (tg[j] == x->src) x->cls = 1;
    }
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
            int k = sample2(s->seed, v, x->m, KIND_RM, s->n, tg);
            for (int j = 0; j < k; j++)              /* AntiEntropyMembers -- [MyNode, FromNode] */
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
        uint32_t tick = (uint32_t)(s->round / s->ae_period);
        for (uint32_t v = 0; v < s->n; v++) {
            uint32_t tg[2];
            int k = sample2(s->seed, v, tick, KIND_AE, s->n, tg);
            for (int j = 0; j < k; j++) if (tg[j] != v) emit(s, DM_PUSH, v, tg[j], 0, s->seen[v]);
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
