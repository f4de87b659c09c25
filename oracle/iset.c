/*
 * iset.c -- restatement of partisan_interval_sets (src/partisan_interval_sets.erl).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Sets are ordered lists of elements; an element is an integer or a closed
 * interval {H, T}.  Each helper below cites the Erlang clause(s) it follows.
 * Recursion over the list is kept as a loop that builds the same list.
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>

static orc_iel mk_int(int64_t n) { orc_iel e = {n, n, 0, 0}; return e; }
static orc_iel mk_iv(int64_t h, int64_t t) { orc_iel e = {h, t, 1, 0}; return e; }

/* validate_element/1, is_element_type/1 (:~536-549): integers, or {X,Y} with X =< Y */
static int valid(const orc_iel* e) { return !e->iv || e->lo <= e->hi; }

/* simplify/1: {N, N} -> N */
static orc_iel simplify(orc_iel e) { if (e.iv && e.lo == e.hi) e.iv = 0; return e; }

/* exact term equality (=:=): 4 and {4,4} are different terms */
static int term_eq(const orc_iel* a, const orc_iel* b) {
    return a->iv == b->iv && a->lo == b->lo && a->hi == b->hi;
}

/* equal/2: {_,_}=A,A ; N,{N,N} ; {N,N},N ; N,N  ==> same closed range */
static int equal(const orc_iel* a, const orc_iel* b) { return a->lo == b->lo && a->hi == b->hi; }

/* element_includes/2, element_included/2 */
static int includes(const orc_iel* a, const orc_iel* b) { return a->lo <= b->lo && a->hi >= b->hi; }
static int included(const orc_iel* a, const orc_iel* b) { return includes(b, a); }
/* element_precedes/2: tail(A) < head(B) (all four clauses) */
static int precedes(const orc_iel* a, const orc_iel* b) { return a->hi < b->lo; }
static int succeeds(const orc_iel* a, const orc_iel* b) { return precedes(b, a); }
/* element_starts_before/2 */
static int starts_before(const orc_iel* a, const orc_iel* b) { return a->lo < b->lo; }
/* element_overlaps/2 (integers via interval/1; N,N -> A =:= B) */
static int overlaps(const orc_iel* a, const orc_iel* b) { return a->lo <= b->hi && b->lo <= a->hi; }
/* element_meets/2: (precedes(A,B) andalso H2 =:= T1+1) orelse (precedes(B,A) andalso H1 =:= T2+1);
 * integers: abs(A-B) == 1 */
static int meets(const orc_iel* a, const orc_iel* b) {
    return (precedes(a, b) && b->lo == a->hi + 1) || (precedes(b, a) && a->lo == b->hi + 1);
}
/* unsafe_element_union/2: always returns a tuple */
static orc_iel uunion(const orc_iel* a, const orc_iel* b) {
    return mk_iv(a->lo < b->lo ? a->lo : b->lo, a->hi > b->hi ? a->hi : b->hi);
}
/* unsafe_element_intersection/2: always a tuple */
static orc_iel uinter(const orc_iel* a, const orc_iel* b) {
    return mk_iv(a->lo > b->lo ? a->lo : b->lo, a->hi < b->hi ? a->hi : b->hi);
}

int orc_iset_element_precedes(const orc_iel* a, const orc_iel* b) { return precedes(a, b); }
int orc_iset_element_meets(const orc_iel* a, const orc_iel* b) { return meets(a, b); }

#define PUSH(arr, n, cap, v) do { if ((n) >= (cap)) return ORC_NOSPACE; (arr)[(n)++] = (v); } while (0)

/* element_subtract/2 + do_element_subtract/2 (:~606-636).
 * Note (faithful): Empty = precedes orelse included orelse succeeds, so a
 * DISJOINT A yields [] rather than [A]. */
int orc_iset_element_subtract(const orc_iel* a, const orc_iel* b, orc_iel* out, size_t cap, size_t* out_n) {
    size_t n = 0;
    *out_n = 0;
    if (precedes(a, b) || included(a, b) || succeeds(a, b)) return ORC_OK;
    int64_t H1 = a->lo, T1 = a->hi, H2 = b->lo, T2 = b->hi;
    if (a->iv && b->iv) {
        if (H1 >= H2 && T1 > T2) {
            PUSH(out, n, cap, mk_iv(T2 + 1 > H1 ? T2 + 1 : H1, T1));
        } else if (H1 < H2 && T1 <= T2) {
            PUSH(out, n, cap, mk_iv(H1, H2 - 1 < T1 ? H2 - 1 : T1));
        } else if (H1 < H2 && T1 > T2) {
            PUSH(out, n, cap, mk_iv(H1, H2 - 1));
            PUSH(out, n, cap, mk_iv(T2 + 1, T1));
        } else {
            return ORC_BADARG;
        }
    } else if (a->iv || b->iv) {
        orc_iel A = mk_iv(H1, T1), B = mk_iv(H2, T2);
        return orc_iset_element_subtract(&A, &B, out, cap, out_n);
    } else {
        return ORC_BADARG;
    }
    *out_n = n;
    return ORC_OK;
}

/* compact/1,2,3 (:~552-590), clause by clause */
static int compact(const orc_iel* l, size_t n, orc_iel* out, size_t cap, size_t* out_n) {
    size_t k = 0;
    *out_n = 0;
    if (n == 0) return ORC_OK;
    orc_iel cur = l[0];
    for (size_t i = 1; i < n; i++) {
        orc_iel e2 = l[i];
        if (term_eq(&e2, &cur)) {                                   /* [E|Es], Acc, E */
            continue;
        }
        if (e2.iv && cur.iv) {
            int64_t V1 = cur.lo, V2 = cur.hi, V3 = e2.lo, V4 = e2.hi;
            if (V2 + 1 >= V3 && V2 <= V4) { cur = mk_iv(V1, V4); continue; }
            if (V2 + 1 >= V3 && V2 > V4) { cur = mk_iv(V1, V2); continue; }
            PUSH(out, k, cap, simplify(cur)); cur = e2; continue;   /* gap */
        }
        if (e2.iv && !cur.iv) {
            int64_t E1 = cur.lo, V1 = e2.lo, V2 = e2.hi;
            if (E1 + 1 >= V1 && E1 <= V2) { cur = mk_iv(E1, V2); continue; }
            PUSH(out, k, cap, simplify(cur)); cur = e2; continue;
        }
        if (!e2.iv && cur.iv) {
            int64_t E2 = e2.lo, V1 = cur.lo, V2 = cur.hi;
            if (E2 - 1 <= V2) { cur = mk_iv(V1, E2 > V2 ? E2 : V2); continue; }
            if (E2 <= V2) { PUSH(out, k, cap, simplify(cur)); cur = e2; continue; } /* unreachable */
            PUSH(out, k, cap, simplify(cur)); cur = e2; continue;
        }
        /* both integers */
        if (cur.lo + 1 == e2.lo) { cur = mk_iv(cur.lo, e2.lo); continue; }
        PUSH(out, k, cap, simplify(cur)); cur = e2;
    }
    PUSH(out, k, cap, simplify(cur));
    *out_n = k;
    return ORC_OK;
}

/* The ordering fun handed to lists:usort/2 in from_list/1 (:184-208).
 * Returns 1 when Fun(E1, E2) is true. */
static int usort_le(const orc_iel* e1, const orc_iel* e2) {
    if (e1->iv && e2->iv) return e1->hi <= e2->lo || e1->lo <= e2->lo;
    if (e1->iv && !e2->iv) return e1->lo <= e2->lo;
    if (!e1->iv && e2->iv) return e1->lo <= e2->lo;
    return e1->lo < e2->lo;
}

/* from_list/1 (:184-208).  lists:usort/2 with the fun above, then compact.
 * For inputs whose elements do not overlap the fun is a total order and
 * usort is a stable sort dropping elements that compare equal both ways;
 * that is the domain the eunit KATs pin (:852-860).  For overlapping
 * inputs OTP's merge-sort result is implementation-defined; we apply the
 * same stable insertion order. */
int orc_iset_from_list(const orc_iel* in, size_t n, orc_iel* out, size_t cap, size_t* out_n) {
    for (size_t i = 0; i < n; i++) if (!valid(&in[i])) return ORC_BADARG;
    orc_iel* tmp = (orc_iel*)malloc((n ? n : 1) * sizeof(orc_iel));
    size_t m = 0;
    for (size_t i = 0; i < n; i++) {
        orc_iel e = in[i];
        /* insertion: find first j with not Fun(tmp[j], e) */
        size_t j = 0;
        int dup = 0;
        while (j < m && usort_le(&tmp[j], &e)) {
            if (usort_le(&e, &tmp[j])) { dup = 1; break; }     /* compares equal: keep first */
            j++;
        }
        if (dup) continue;
        memmove(&tmp[j + 1], &tmp[j], (m - j) * sizeof(orc_iel));
        tmp[j] = e;
        m++;
    }
    int rc = compact(tmp, m, out, cap, out_n);
    free(tmp);
    return rc;
}

/* is_element/2 + do_is_element/2 (:219-235) */
int orc_iset_is_element(const orc_iel* a, const orc_iel* set, size_t n) {
    if (!valid(a)) return ORC_BADARG;
    for (size_t i = 0; i < n; i++) {
        const orc_iel* b = &set[i];
        if (starts_before(a, b) || precedes(a, b)) return 0;
        if (included(a, b)) return 1;
        if (!succeeds(a, b)) return 0;
    }
    return 0;
}

/* add_element/2 (:244-279) */
int orc_iset_add_element(const orc_iel* a0, const orc_iel* set, size_t n,
                         orc_iel* out, size_t cap, size_t* out_n) {
    size_t k = 0;
    orc_iel a = *a0;
    size_t i = 0;
    *out_n = 0;
    for (;;) {
        if (!valid(&a)) return ORC_BADARG;
        if (i == n) { PUSH(out, k, cap, a); break; }           /* add_element(E, []) -> [E] */
        const orc_iel* b = &set[i];
        if (equal(&a, b)) {                                     /* -> Set */
            for (; i < n; i++) PUSH(out, k, cap, set[i]);
            break;
        }
        if (meets(&a, b)) { a = uunion(&a, b); i++; continue; }  /* add_element(E, Es) */
        if (precedes(&a, b)) {                                  /* [simplify(A)|Set] */
            PUSH(out, k, cap, simplify(a));
            for (; i < n; i++) PUSH(out, k, cap, set[i]);
            break;
        }
        if (succeeds(&a, b)) { PUSH(out, k, cap, *b); i++; continue; } /* [B|add_element(A, Es)] */
        if (overlaps(&a, b)) { a = uunion(&a, b); i++; continue; }
        return ORC_BADARG;
    }
    *out_n = k;
    return ORC_OK;
}

/* del_element/2 (:~288-322).  Faithful quirk: after an overlap the remainder
 * R = element_subtract(A, I) is a LIST and is passed back as the element;
 * validate_element(R) then raises unless the tail is empty. */
int orc_iset_del_element(const orc_iel* a0, const orc_iel* set, size_t n,
                         orc_iel* out, size_t cap, size_t* out_n) {
    size_t k = 0;
    orc_iel a = *a0;
    *out_n = 0;
    for (size_t i = 0; i < n; i++) {
        const orc_iel* b = &set[i];
        if (!valid(&a)) return ORC_BADARG;
        if (equal(&a, b)) {                                     /* -> Es */
            for (size_t j = i + 1; j < n; j++) PUSH(out, k, cap, set[j]);
            *out_n = k;
            return ORC_OK;
        }
        if (precedes(&a, b)) {                                  /* -> Set */
            for (size_t j = i; j < n; j++) PUSH(out, k, cap, set[j]);
            *out_n = k;
            return ORC_OK;
        }
        if (succeeds(&a, b)) { PUSH(out, k, cap, *b); continue; }
        if (overlaps(&a, b)) {
            orc_iel I = uinter(&a, b);                          /* element_intersection */
            orc_iel tmp[2];
            size_t nt;
            int rc = orc_iset_element_subtract(b, &I, tmp, 2, &nt);
            if (rc) return rc;
            for (size_t j = 0; j < nt; j++) PUSH(out, k, cap, simplify(tmp[j]));
            /* del_element(R, Es) with R a list: [] when Es == [], else badarg */
            if (i + 1 < n) return ORC_BADARG;
            *out_n = k;
            return ORC_OK;
        }
        return ORC_BADARG;
    }
    *out_n = k;                                                 /* del_element(_, []) -> [] */
    return ORC_OK;
}

/* flat_size/1, min/1, max/1 */
int64_t orc_iset_flat_size(const orc_iel* s, size_t n) {
    int64_t c = 0;
    for (size_t i = 0; i < n; i++) c += s[i].iv ? 1 + s[i].hi - s[i].lo : 1;
    return c;
}
int64_t orc_iset_min(const orc_iel* s, size_t n) { (void)n; return s[0].lo; }
int64_t orc_iset_max(const orc_iel* s, size_t n) { return s[n - 1].hi; }

/* is_type/1,2 (integer-valued domain; non-integer terms are not representable
 * here).  Faithful quirks: only the FIRST element is checked by
 * is_element_type/1; after {_, E2} followed by an integer the clause recurses
 * with E2 (the interval's tail), not with the integer. */
int orc_iset_is_type(const orc_iel* s, size_t n) {
    if (n == 0) return 1;
    if (!valid(&s[0])) return 0;
    orc_iel prev = s[0];
    for (size_t i = 1; i < n; i++) {
        const orc_iel* e = &s[i];
        if (e->iv && prev.iv) { if (!(prev.hi <= e->lo)) return 0; prev = *e; }
        else if (e->iv && !prev.iv) { if (!(prev.lo <= e->lo)) return 0; prev = *e; }
        else if (!e->iv && prev.iv) { if (!(prev.hi <= e->lo)) return 0; prev = mk_int(prev.hi); }
        else { if (!(prev.lo < e->lo)) return 0; prev = *e; }
    }
    return 1;
}

/* seq/1 */
int orc_iset_seq(const orc_iel* s, size_t n, int64_t* out, size_t cap, size_t* out_n) {
    size_t k = 0;
    for (size_t i = 0; i < n; i++)
        for (int64_t v = s[i].lo; v <= s[i].hi; v++) PUSH(out, k, cap, v);
    *out_n = k;
    return ORC_OK;
}

/* union/2, intersection/2, subtract/2: compact(ordsets:OP(seq(A), seq(B))) */
static int setop(int op, const orc_iel* a, size_t na, const orc_iel* b, size_t nb,
                 orc_iel* out, size_t cap, size_t* out_n) {
    int64_t fa = orc_iset_flat_size(a, na), fb = orc_iset_flat_size(b, nb);
    int64_t* sa = (int64_t*)malloc((size_t)(fa + 1) * sizeof(int64_t));
    int64_t* sb = (int64_t*)malloc((size_t)(fb + 1) * sizeof(int64_t));
    orc_iel* r = (orc_iel*)malloc((size_t)(fa + fb + 1) * sizeof(orc_iel));
    size_t la, lb, i = 0, j = 0, k = 0;
    orc_iset_seq(a, na, sa, (size_t)fa, &la);
    orc_iset_seq(b, nb, sb, (size_t)fb, &lb);
    while (i < la || j < lb) {
        if (j == lb || (i < la && sa[i] < sb[j])) { if (op != 1) r[k++] = mk_int(sa[i]); i++; }
        else if (i == la || sb[j] < sa[i]) { if (op == 0) r[k++] = mk_int(sb[j]); j++; }
        else { if (op == 0 || op == 1) r[k++] = mk_int(sa[i]); i++; j++; }
    }
    int rc = compact(r, k, out, cap, out_n);
    free(sa); free(sb); free(r);
    return rc;
}
int orc_iset_union(const orc_iel* a, size_t na, const orc_iel* b, size_t nb, orc_iel* o, size_t c, size_t* n) { return setop(0, a, na, b, nb, o, c, n); }
int orc_iset_intersection(const orc_iel* a, size_t na, const orc_iel* b, size_t nb, orc_iel* o, size_t c, size_t* n) { return setop(1, a, na, b, nb, o, c, n); }
int orc_iset_subtract(const orc_iel* a, size_t na, const orc_iel* b, size_t nb, orc_iel* o, size_t c, size_t* n) { return setop(2, a, na, b, nb, o, c, n); }
