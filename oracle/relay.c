/*
 * relay.c -- transitive relay over Plumtree out-links.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restates, one message copy at a time (the reference keeps no relay state
 * and no dedup, so every copy is handled on its own):
 *   do_send_message/3 with transitive => true
 *       (src/partisan_hyparview_peer_service_manager.erl:2220-2290):
 *       connected to Node -> send; else, with broadcast and transitive set,
 *       do_tree_forward(Node, Message, Options, relay_ttl);
 *   do_tree_forward/4 (:2796-2842): for every out-link (minus self) send
 *       {relay_message, Node, Message, TTL - 1} without `transitive`, so a
 *       relay that is not connected is simply not reached;
 *   handle_message({relay_message, Node, Message, TTL}) (:1800-1832): Node in
 *       the active members -> do_send_message(Node, Message, transitive);
 *       TTL == 0 -> drop; else do_tree_forward(Node, Message, Opts, TTL)
 *       with Opts.out_links = this node's out_links;
 *   retrieve_outlinks/1 (:2846-2870) / handle_info(tree_refresh) (:1069-1076):
 *       out_links = the node's eager peers in its OWN broadcast tree
 *       (partisan_plumtree_broadcast:debug_get_peers(Node, Node)), which are
 *       its common eagers when it has no per-root entry for itself.
 *
 * Simulation contract: a message sent in round r is handled
 * in round r+1; the sends of the batch are handled by their origins in
 * round 0 in batch order.  "Connected to P" = P is live and a peer of the
 * sender: a member of its active view or a vertex whose view lists it
 * (connections are symmetric).  The active members that handle_message
 * checks are the view itself (act), live ones only: a dead peer's 'EXIT'
 * has been processed.  out_links are the snapshot the
 * caller passes (tree_refresh fired after the last tree change).
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct { uint32_t kind, k, at, ttl; } rl_msg;   /* kind 0 = relay_message, 1 = Message to Node */

static int member(const uint64_t* ptr, const uint32_t* ids, uint32_t v, uint32_t x) {
    for (uint64_t i = ptr[v]; i < ptr[v + 1]; i++)
        if (ids[i] == x) return 1;
    return 0;
}

typedef struct { rl_msg* m; size_t n, cap; } rl_q;

static int push(rl_q* q, rl_msg m, size_t limit) {
    if (q->n == q->cap) {
        size_t c = q->cap ? 2 * q->cap : 1024;
        if (c > limit) c = limit;
        if (q->n == c) return -1;
        rl_msg* p = (rl_msg*)realloc(q->m, c * sizeof(rl_msg));
        if (!p) return -1;
        q->m = p;
        q->cap = c;
    }
    q->m[q->n++] = m;
    return 0;
}

/* The handler of one copy at vertex v (origin: ttl = relay_ttl, the TTL that
 * do_send_message passes to do_tree_forward; relay: the message's TTL). */
static int handle(uint32_t v, uint32_t k, uint32_t ttl, int at_origin, const uint32_t* dst,
                  const uint64_t* act_ptr, const uint32_t* act, const uint64_t* peer_ptr, const uint32_t* peer,
                  const uint64_t* ol_ptr, const uint32_t* ol,
                  const uint8_t* alive, rl_q* out, orc_relay_round* st, size_t limit) {
    const uint32_t d = dst[k];
    /* origin: do_send_message -> connected?  relay: lists:member(Node, ActiveMembers)
     * then do_send_message(Node, Message, transitive) (connected: a member is a peer) */
    const int direct = alive[d] && (at_origin ? member(peer_ptr, peer, v, d) : member(act_ptr, act, v, d));
    if (direct) {                                            /* send Message to Node */
        st->direct++;
        return push(out, (rl_msg){1, k, d, 0}, limit);
    }
    if (!at_origin && ttl == 0) {                            /* TTL expired: drop */
        st->dropped++;
        return 0;
    }
    for (uint64_t i = ol_ptr[v]; i < ol_ptr[v + 1]; i++) {   /* do_tree_forward: every out-link */
        const uint32_t p = ol[i];
        if (p == v) continue;                                /* OutLinks -- [MyNode] */
        if (!(alive[p] && member(peer_ptr, peer, v, p))) {   /* not connected: send fails, no retry */
            st->lost++;
            continue;
        }
        st->relay++;
        if (push(out, (rl_msg){0, k, p, ttl - 1}, limit)) return -1;
    }
    return 0;
}

int64_t orc_relay_run(uint32_t n, const uint64_t* act_ptr, const uint32_t* act, const uint64_t* ol_ptr,
                      const uint32_t* ol, const uint8_t* alive, uint32_t k, const uint32_t* src,
                      const uint32_t* dst, uint32_t relay_ttl, uint64_t* delivered, uint32_t* first_round,
                      orc_relay_round* stats, size_t cap, size_t max_copies) {
    if (relay_ttl == 0) return ORC_BADARG;
    for (uint32_t i = 0; i < k; i++) {
        if (src[i] >= n || dst[i] >= n || src[i] == dst[i]) return ORC_BADARG;
        delivered[i] = 0;
        first_round[i] = UINT32_MAX;
    }
    /* peers = members ∪ vertices listing v (the overlay's symmetric connections) */
    uint64_t* peer_ptr = (uint64_t*)calloc((size_t)n + 1, sizeof(uint64_t));
    const uint64_t na = act_ptr[n];
    uint32_t* peer = (uint32_t*)malloc((size_t)(2 * na + 1) * sizeof(uint32_t));
    uint32_t* fill = (uint32_t*)calloc((size_t)n + 1, sizeof(uint32_t));
    if (!peer_ptr || !peer || !fill) {
        free(peer_ptr);
        free(peer);
        free(fill);
        return ORC_NOSPACE;
    }
    for (uint32_t v = 0; v < n; v++)
        for (uint64_t i = act_ptr[v]; i < act_ptr[v + 1]; i++) {
            peer_ptr[v + 1]++;
            peer_ptr[act[i] + 1]++;
        }
    for (uint32_t v = 0; v < n; v++) peer_ptr[v + 1] += peer_ptr[v];
    for (uint32_t v = 0; v < n; v++)
        for (uint64_t i = act_ptr[v]; i < act_ptr[v + 1]; i++) {
            peer[peer_ptr[v] + fill[v]++] = act[i];
            peer[peer_ptr[act[i]] + fill[act[i]]++] = v;
        }
    free(fill);

    rl_q cur = {0}, nxt = {0};
    int64_t rounds = 0;
    int err = 0;
    orc_relay_round st;
    memset(&st, 0, sizeof st);
    for (uint32_t i = 0; i < k && !err; i++)                 /* round 0: the origins */
        if (alive[src[i]])
            err = handle(src[i], i, relay_ttl, 1, dst, act_ptr, act, peer_ptr, peer, ol_ptr, ol, alive, &cur, &st,
                         max_copies);
    if ((size_t)rounds < cap) stats[rounds] = st;
    rounds++;
    while (!err && cur.n) {
        memset(&st, 0, sizeof st);
        nxt.n = 0;
        for (size_t j = 0; j < cur.n && !err; j++) {          /* arrival round = rounds */
            const rl_msg m = cur.m[j];
            if (m.kind == 1) {
                delivered[m.k]++;
                if (first_round[m.k] == UINT32_MAX) first_round[m.k] = (uint32_t)rounds;
                st.arrived++;
                continue;
            }
            err = handle(m.at, m.k, m.ttl, 0, dst, act_ptr, act, peer_ptr, peer, ol_ptr, ol, alive, &nxt, &st,
                         max_copies);
        }
        if ((size_t)rounds < cap) stats[rounds] = st;
        rounds++;
        rl_q t = cur;
        cur = nxt;
        nxt = t;
    }
    free(cur.m);
    free(nxt.m);
    free(peer_ptr);
    free(peer);
    return err ? ORC_NOSPACE : rounds;
}
