/*
 * c3.c -- configuration C3: Plumtree broadcast repaired by
 * graft/prune over churning SCAMP v2 membership, composed from the two
 * restatements (scamp.c, plumtree.c) the way the reference wires them:
 *  - the pluggable manager runs the SCAMP strategy and fires
 *    partisan_peer_service_events:update(Members) after a join / membership
 *    message that changed the members list (:1574-1579, :1756-1761); the
 *    plumtree server receives each as a {update, Members} cast
 *    (partisan_plumtree_broadcast.erl:607-639);
 *  - plumtree sends go through partisan:cast_message -> the manager's
 *    do_send_message, which needs an outbound connection: only members have
 *    one (pluggable :1638-1669, :1938-1987); is_connected/1 likewise;
 *  - a crash restarts both processes (start_link/0 with members = {self}).
 * Round t = the SCAMP round t, then the plumtree round t, whose updates
 * (queued in order by the SCAMP round) are applied before its inbox.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Checker for csrc/ptdyn.hip.
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>

struct orc_c3 {
    uint32_t n;
    orc_scamp* sc;
    orc_plumtree* pt;
    uint64_t updates;
    uint32_t root, mono;
    int have_hb;
    uint8_t* alive;
};

static void on_update(void* ctx, uint32_t v, const uint32_t* members, size_t n) {
    orc_c3* s = (orc_c3*)ctx;
    s->updates++;
    orc_pt_queue_update(s->pt, v, members, n);
}

static int connected(void* ctx, uint32_t u, uint32_t t) {
    orc_c3* s = (orc_c3*)ctx;
    return t != u && orc_scamp_has_member(s->sc, u, t);
}

orc_c3* orc_c3_create(uint32_t n, uint32_t c, uint32_t periodic_rounds, uint64_t seed) {
    orc_c3* s = (orc_c3*)calloc(1, sizeof(orc_c3));
    s->n = n;
    s->sc = orc_scamp_create(n, 2, c, periodic_rounds, seed);
    uint64_t* rp = (uint64_t*)calloc((size_t)n + 1, sizeof(uint64_t));   /* members = {self} */
    uint32_t dummy = 0;
    s->pt = orc_pt_create(n, rp, &dummy, 1);
    free(rp);
    s->alive = (uint8_t*)malloc(n);
    orc_scamp_set_update_hook(s->sc, on_update, s);
    orc_pt_set_conn(s->pt, connected, s);
    return s;
}

void orc_c3_destroy(orc_c3* s) {
    if (!s) return;
    orc_scamp_destroy(s->sc);
    orc_pt_destroy(s->pt);
    free(s->alive);
    free(s);
}

orc_scamp* orc_c3_scamp(orc_c3* s) { return s->sc; }
orc_plumtree* orc_c3_plumtree(orc_c3* s) { return s->pt; }

void orc_c3_join(orc_c3* s, uint32_t v, uint32_t contact) { orc_scamp_join(s->sc, v, contact); }

void orc_c3_crash(orc_c3* s, uint32_t v) {
    orc_scamp_crash(s->sc, v);
    orc_pt_restart(s->pt, v);
}

uint32_t orc_c3_heartbeat(orc_c3* s, uint32_t root) {
    s->root = root;
    s->have_hb = 1;
    s->mono = orc_pt_heartbeat(s->pt, root);
    return s->mono;
}

uint32_t orc_c3_step(orc_c3* s, uint32_t rounds, orc_c3_stats* st) {
    uint8_t* dl = (uint8_t*)malloc(s->n);
    for (uint32_t r = 0; r < rounds; r++) {
        orc_c3_stats* o = st ? &st[r] : NULL;
        orc_scamp_stats ss;
        orc_round_stats ps;
        s->updates = 0;
        const uint64_t d0 = orc_pt_dropped(s->pt);
        orc_scamp_step(s->sc, 1, &ss);
        for (uint32_t v = 0; v < s->n; v++) s->alive[v] = (uint8_t)orc_scamp_alive(s->sc, v);
        orc_pt_set_alive(s->pt, s->alive);
        orc_pt_step(s->pt, 1, &ps);
        if (o) {
            memset(o, 0, sizeof(*o));
            o->scamp = ss;
            o->pt = ps;
            o->updates = s->updates;
            o->pt_dropped = orc_pt_dropped(s->pt) - d0;
            if (s->have_hb) {
                orc_pt_get_delivered(s->pt, s->root, s->mono, dl);
                for (uint32_t v = 0; v < s->n; v++)
                    if (s->alive[v]) { o->live++; o->delivered_live += dl[v]; }
            } else {
                for (uint32_t v = 0; v < s->n; v++) o->live += s->alive[v];
            }
        }
    }
    free(dl);
    return rounds;
}
