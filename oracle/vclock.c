/*
 * vclock.c -- restatement of partisan_vclock (src/partisan_vclock.erl:58-198).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * A clock is the Erlang list [{Actor, Counter}] with its order preserved:
 * increment/2 prepends, merge/1 of one clock returns it unsorted, merge of
 * two or more returns a keysorted list.  Actors are
 * u32 ids whose integer order equals the Erlang term order of the names.
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>

#define PUSH(arr, n, cap, v) do { if ((n) >= (cap)) return ORC_NOSPACE; (arr)[(n)++] = (v); } while (0)

/* lists:keyfind(Actor, 1, Clock): first match */
static const orc_dot* keyfind(uint32_t actor, const orc_dot* a, size_t na) {
    for (size_t i = 0; i < na; i++) if (a[i].actor == actor) return &a[i];
    return NULL;
}

/* descends/2 (:63-73): every {NodeB, CtrB} in B has NodeB in A with CtrA >= CtrB.
 * An actor of B missing from A fails even when CtrB == 0 (Q22). */
int orc_vc_descends(const orc_dot* a, size_t na, const orc_dot* b, size_t nb) {
    for (size_t i = 0; i < nb; i++) {
        const orc_dot* x = keyfind(b[i].actor, a, na);
        if (!x) return 0;
        if (!(x->ctr >= b[i].ctr)) return 0;
    }
    return 1;
}

/* dominates/2 (:75-77) */
int orc_vc_dominates(const orc_dot* a, size_t na, const orc_dot* b, size_t nb) {
    return orc_vc_descends(a, na, b, nb) && !orc_vc_descends(b, nb, a, na);
}

/* lists:keysort(1, L): stable sort on the actor */
static void keysort(orc_dot* l, size_t n) {
    for (size_t i = 1; i < n; i++) {
        orc_dot x = l[i];
        size_t j = i;
        while (j > 0 && l[j - 1].actor > x.actor) { l[j] = l[j - 1]; j--; }
        l[j] = x;
    }
}

/* merge/3 (:111-129): merge two keysorted clocks, max of equal actors
 * (compare(Ctr1, Ctr2) =:= lt -> Ctr2 ; _ -> Ctr1). */
static size_t merge2(const orc_dot* v, size_t nv, const orc_dot* w, size_t nw, orc_dot* out) {
    size_t i = 0, j = 0, k = 0;
    while (i < nv && j < nw) {
        if (v[i].actor < w[j].actor) out[k++] = v[i++];
        else if (v[i].actor > w[j].actor) out[k++] = w[j++];
        else {
            orc_dot d = v[i];
            d.ctr = v[i].ctr < w[j].ctr ? w[j].ctr : v[i].ctr;
            out[k++] = d;
            i++; j++;
        }
    }
    while (i < nv) out[k++] = v[i++];
    while (j < nw) out[k++] = w[j++];
    return k;
}

/* merge/1 (:102-105) and merge/2 (:107-109) */
int orc_vc_merge(const orc_dot* flat, const size_t* lens, size_t nclocks,
                 orc_dot* out, size_t cap, size_t* out_n) {
    *out_n = 0;
    if (nclocks == 0) return ORC_OK;
    size_t total = 0;
    for (size_t c = 0; c < nclocks; c++) total += lens[c];
    if (nclocks == 1) {                                   /* merge([Single]) -> Single, unsorted */
        if (lens[0] > cap) return ORC_NOSPACE;
        memcpy(out, flat, lens[0] * sizeof(orc_dot));
        *out_n = lens[0];
        return ORC_OK;
    }
    orc_dot* acc = (orc_dot*)malloc((total + 1) * sizeof(orc_dot));
    orc_dot* tmp = (orc_dot*)malloc((total + 1) * sizeof(orc_dot));
    orc_dot* srt = (orc_dot*)malloc((total + 1) * sizeof(orc_dot));
    size_t nacc = lens[0];
    memcpy(acc, flat, lens[0] * sizeof(orc_dot));
    keysort(acc, nacc);                                   /* lists:keysort(1, First) */
    size_t off = lens[0];
    for (size_t c = 1; c < nclocks; c++) {                /* merge([AClock|VClocks], NClock) */
        memcpy(srt, flat + off, lens[c] * sizeof(orc_dot));
        keysort(srt, lens[c]);
        size_t k = merge2(srt, lens[c], acc, nacc, tmp);
        memcpy(acc, tmp, k * sizeof(orc_dot));
        nacc = k;
        off += lens[c];
    }
    int rc = ORC_OK;
    if (nacc > cap) rc = ORC_NOSPACE;
    else { memcpy(out, acc, nacc * sizeof(orc_dot)); *out_n = nacc; }
    free(acc); free(tmp); free(srt);
    return rc;
}

/* get_counter/2 (:132-137) */
int64_t orc_vc_get_counter(uint32_t actor, const orc_dot* a, size_t na) {
    const orc_dot* x = keyfind(actor, a, na);
    return x ? x->ctr : 0;
}

/* increment/2 (:140-153): keytake the first match, prepend {Node, C+1} */
int orc_vc_increment(uint32_t actor, const orc_dot* a, size_t na,
                     orc_dot* out, size_t cap, size_t* out_n) {
    size_t k = 0;
    int64_t ctr = 1;
    size_t skip = (size_t)-1;
    for (size_t i = 0; i < na; i++) if (a[i].actor == actor) { ctr = a[i].ctr + 1; skip = i; break; }
    orc_dot head = {actor, 0, ctr};
    PUSH(out, k, cap, head);
    for (size_t i = 0; i < na; i++) if (i != skip) PUSH(out, k, cap, a[i]);
    *out_n = k;
    return ORC_OK;
}

/* lists:sort/1 on {Actor, Ctr} tuples */
static int dot_cmp(const void* x, const void* y) {
    const orc_dot* a = (const orc_dot*)x; const orc_dot* b = (const orc_dot*)y;
    if (a->actor != b->actor) return a->actor < b->actor ? -1 : 1;
    if (a->ctr != b->ctr) return a->ctr < b->ctr ? -1 : 1;
    return 0;
}

/* equal/2 (:163-164): lists:sort(VA) =:= lists:sort(VB) */
int orc_vc_equal(const orc_dot* a, size_t na, const orc_dot* b, size_t nb) {
    if (na != nb) return 0;
    orc_dot* sa = (orc_dot*)malloc((na + 1) * sizeof(orc_dot));
    orc_dot* sb = (orc_dot*)malloc((nb + 1) * sizeof(orc_dot));
    memcpy(sa, a, na * sizeof(orc_dot)); memcpy(sb, b, nb * sizeof(orc_dot));
    qsort(sa, na, sizeof(orc_dot), dot_cmp); qsort(sb, nb, sizeof(orc_dot), dot_cmp);
    int eq = 1;
    for (size_t i = 0; i < na; i++) if (dot_cmp(&sa[i], &sb[i]) != 0) { eq = 0; break; }
    free(sa); free(sb);
    return eq;
}

/* all_nodes/1 (:157-159): [X || {X, _} <- sort(VClock)] */
int orc_vc_all_nodes(const orc_dot* a, size_t na, uint32_t* out, size_t cap, size_t* out_n) {
    if (na > cap) return ORC_NOSPACE;
    orc_dot* s = (orc_dot*)malloc((na + 1) * sizeof(orc_dot));
    memcpy(s, a, na * sizeof(orc_dot));
    qsort(s, na, sizeof(orc_dot), dot_cmp);
    for (size_t i = 0; i < na; i++) out[i] = s[i].actor;
    *out_n = na;
    free(s);
    return ORC_OK;
}

/* glb/2 (:183-198) */
int orc_vc_glb(const orc_dot* a, size_t na, const orc_dot* b, size_t nb,
               orc_dot* out, size_t cap, size_t* out_n) {
    size_t k = 0;
    for (size_t i = 0; i < na; i++) {
        const orc_dot* x = keyfind(a[i].actor, b, nb);
        if (!x) continue;
        orc_dot d = a[i];
        if (!(x->ctr >= a[i].ctr)) d.ctr = x->ctr;
        PUSH(out, k, cap, d);
    }
    qsort(out, k, sizeof(orc_dot), dot_cmp);
    *out_n = k;
    return ORC_OK;
}

/* subtract_dots/2 + drop_dots/3 (:85-99) */
int orc_vc_subtract_dots(const orc_dot* dots, size_t nd, const orc_dot* clock, size_t nc,
                         orc_dot* out, size_t cap, size_t* out_n) {
    size_t k = 0;
    for (size_t i = 0; i < nd; i++) {
        int64_t c = orc_vc_get_counter(dots[i].actor, clock, nc);
        if (c >= dots[i].ctr) continue;
        PUSH(out, k, cap, dots[i]);
    }
    qsort(out, k, sizeof(orc_dot), dot_cmp);
    *out_n = k;
    return ORC_OK;
}
