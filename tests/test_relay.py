"""Transitive relay over Plumtree out-links.

Oracle: oracle/relay.c (restates do_send_message/3, do_tree_forward/4 and
handle_message({relay_message, ..}) of
src/partisan_hyparview_peer_service_manager.erl:2220-2290, 2796-2842,
1800-1832).  Parity unpinned against the reference itself: its suites only
exercise relay through live multi-node runs (no golden vectors), so the C
oracle is cross-checked here against an independent pure-Python statement of
the same clauses on small cases.  GPU: csrc/relay.hip through the C ABI,
bit-exact against the oracle (per-round counters, copies delivered per send,
first arrival round).
"""
import numpy as np
import pytest

import pyoracle as O

NEVER = 0xFFFFFFFF


def random_views(n, rng, deg=3):
    """Directed active views (not necessarily symmetric), no self entries."""
    ptr = [0]
    ids = []
    for v in range(n):
        k = int(rng.integers(1, deg + 1))
        cand = rng.choice(n - 1, size=min(k, n - 1), replace=False)
        row = sorted(int(c + (c >= v)) for c in cand)
        ids.extend(row)
        ptr.append(len(ids))
    return np.asarray(ptr, np.uint64), np.asarray(ids, np.uint32)


def peers_of(ptr, ids, n):
    peers = [set() for _ in range(n)]
    for v in range(n):
        for i in range(int(ptr[v]), int(ptr[v + 1])):
            peers[v].add(int(ids[i]))
            peers[int(ids[i])].add(v)
    return peers


def random_out_links(n, peers, rng, p_stranger=0.15, p_self=0.05, cap=8):
    """Out-links: mostly peers (eager sets are peers), some strangers (their
    send fails: not connected) and occasionally the vertex itself (skipped)."""
    ptr = [0]
    ids = []
    for v in range(n):
        row = [p for p in sorted(peers[v]) if rng.random() < 0.8]
        if rng.random() < p_stranger:
            row.append(int(rng.integers(n)))
        if rng.random() < p_self:
            row.append(v)
        ids.extend(row[:cap])
        ptr.append(len(ids))
    return np.asarray(ptr, np.uint64), np.asarray(ids, np.uint32)


def random_sends(n, k, rng):
    src = rng.integers(0, n, size=k).astype(np.uint32)
    dst = rng.integers(0, n - 1, size=k).astype(np.uint32)
    dst = np.where(dst >= src, dst + 1, dst).astype(np.uint32)
    return src, dst


def py_relay(n, act_ptr, act, ol_ptr, ol, alive, src, dst, ttl0):
    """Pure-Python statement of the same clauses (small cases only)."""
    act_l = [set(int(x) for x in act[int(act_ptr[v]):int(act_ptr[v + 1])]) for v in range(n)]
    peers = peers_of(act_ptr, act, n)
    ol_l = [[int(x) for x in ol[int(ol_ptr[v]):int(ol_ptr[v + 1])]] for v in range(n)]
    k = len(src)
    deliv = [0] * k
    first = [NEVER] * k
    rows = []

    def handle(v, i, ttl, origin, out, st):
        d = int(dst[i])
        connected = alive[d] and (d in peers[v] if origin else d in act_l[v])
        if connected:                       # do_send_message: connected -> send
            st["direct"] += 1
            out.append(("msg", i, d, 0))
            return
        if not origin and ttl == 0:         # handle_message: TTL 0 -> drop
            st["dropped"] += 1
            return
        for p in ol_l[v]:                   # do_tree_forward(Node, Message, Opts, TTL)
            if p == v:
                continue
            if alive[p] and p in peers[v]:
                st["relay"] += 1
                out.append(("relay", i, p, ttl - 1))
            else:
                st["lost"] += 1

    keys = ("direct", "relay", "dropped", "lost", "arrived")
    st = dict.fromkeys(keys, 0)
    cur = []
    for i in range(k):
        if alive[int(src[i])]:
            handle(int(src[i]), i, ttl0, True, cur, st)
    rows.append(st)
    r = 1
    while cur:
        st = dict.fromkeys(keys, 0)
        nxt = []
        for kind, i, at, ttl in cur:
            if kind == "msg":
                deliv[i] += 1
                first[i] = min(first[i], r)
                st["arrived"] += 1
            else:
                handle(at, i, ttl, False, nxt, st)
        rows.append(st)
        cur = nxt
        r += 1
    return rows, np.asarray(deliv, np.uint64), np.asarray(first, np.uint32)


def make_case(n, k, seed, dead_frac=0.1):
    rng = np.random.default_rng(seed)
    ap, ai = random_views(n, rng)
    op, oi = random_out_links(n, peers_of(ap, ai, n), rng)
    alive = (rng.random(n) >= dead_frac).astype(np.uint8)
    src, dst = random_sends(n, k, rng)
    return ap, ai, op, oi, alive, src, dst


# ---------------------------------------------------------------- CPU: oracle
@pytest.mark.parametrize("seed,ttl", [(1, 1), (2, 2), (3, 5), (4, 3)])
def test_oracle_matches_python_statement(seed, ttl):
    n, k = 60, 25
    ap, ai, op, oi, alive, src, dst = make_case(n, k, seed)
    rows, dv, fr = O.relay_run(ap, ai, op, oi, alive, src, dst, relay_ttl=ttl)
    prow, pdv, pfr = py_relay(n, ap, ai, op, oi, alive, src, dst, ttl)
    assert rows == prow
    assert np.array_equal(dv, pdv) and np.array_equal(fr, pfr)


def test_oracle_line_hand_case():
    # 0 - 1 - 2 - 3 (views point right), out-links = peers: 0 -> 3 needs relays
    ap = np.array([0, 1, 2, 3, 3], np.uint64)
    ai = np.array([1, 2, 3], np.uint32)
    op = np.array([0, 1, 3, 5, 6], np.uint64)
    oi = np.array([1, 0, 2, 1, 3, 2], np.uint32)
    alive = np.ones(4, np.uint8)
    rows, dv, fr = O.relay_run(ap, ai, op, oi, alive, [0], [3], relay_ttl=5)
    # r0: origin 0 relays to 1; r1: 1 relays to 0, 2; r2: 0 relays to 1 (ttl 2),
    # 2 has 3 in its view -> direct; r3: 1 relays to 0, 2 and Message arrives
    assert rows[0] == {"direct": 0, "relay": 1, "dropped": 0, "lost": 0, "arrived": 0}
    assert rows[1] == {"direct": 0, "relay": 2, "dropped": 0, "lost": 0, "arrived": 0}
    assert rows[2] == {"direct": 1, "relay": 1, "dropped": 0, "lost": 0, "arrived": 0}
    assert rows[3]["arrived"] == 1 and rows[3]["relay"] == 2
    assert fr[0] == 3 and dv[0] >= 1
    # dead destination: never delivered, relays stop at TTL 0
    alive[3] = 0
    rows, dv, fr = O.relay_run(ap, ai, op, oi, alive, [0], [3], relay_ttl=3)
    assert dv[0] == 0 and fr[0] == NEVER
    assert sum(r["dropped"] for r in rows) > 0


def test_oracle_edge_cases():
    n = 10
    ap, ai, op, oi, alive, src, dst = make_case(n, 5, 9, dead_frac=0.0)
    rows, dv, fr = O.relay_run(ap, ai, op, oi, alive, np.zeros(0, np.uint32), np.zeros(0, np.uint32))
    assert len(rows) == 1 and len(dv) == 0
    with pytest.raises(ValueError):
        O.relay_run(ap, ai, op, oi, alive, [1], [1])                 # src == dst
    with pytest.raises(ValueError):
        O.relay_run(ap, ai, op, oi, alive, [1], [2], relay_ttl=0)
    with pytest.raises(ValueError):
        O.relay_run(ap, ai, op, oi, alive, src, dst, max_copies=1)  # a round overflows
    dead = np.zeros(n, np.uint8)
    rows, dv, fr = O.relay_run(ap, ai, op, oi, dead, src, dst)        # dead origins send nothing
    assert len(rows) == 1 and not dv.any()


# ---------------------------------------------------------------- GPU parity
@pytest.fixture(scope="module")
def sim():
    import partisan_amd as pa
    s = pa.Simulator(device=0)
    yield s
    s.close()


def _both(sim, case, ttl, max_copies=50_000_000):
    from partisan_amd.relay import relay_run
    ap, ai, op, oi, alive, src, dst = case
    g = relay_run(sim, ap, ai, op, oi, alive, src, dst, relay_ttl=ttl, max_copies=max_copies)
    o = O.relay_run(ap, ai, op, oi, alive, src, dst, relay_ttl=ttl, max_copies=max_copies)
    return g, o


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,ttl,seed", [(60, 25, 1, 1), (60, 25, 5, 3), (2000, 500, 3, 5),
                                          (20000, 3000, 5, 7), (200000, 20000, 4, 11)])
def test_relay_gpu_parity(sim, n, k, ttl, seed):
    case = make_case(n, k, seed)
    (grows, gdv, gfr), (orows, odv, ofr) = _both(sim, case, ttl)
    assert grows == orows
    assert np.array_equal(gdv, odv)
    assert np.array_equal(gfr, ofr)


@pytest.mark.gpu
def test_relay_gpu_edges(sim):
    import partisan_amd as pa
    from partisan_amd.relay import relay_run
    ap, ai, op, oi, alive, src, dst = make_case(500, 200, 21, dead_frac=0.0)
    g = relay_run(sim, ap, ai, op, oi, alive, src[:0], dst[:0])
    assert len(g[0]) == 1 and len(g[1]) == 0
    dead = np.zeros(500, np.uint8)
    rows, dv, _ = relay_run(sim, ap, ai, op, oi, dead, src, dst)
    assert len(rows) == 1 and not dv.any()
    with pytest.raises(pa.PsimError) as e:
        relay_run(sim, ap, ai, op, oi, alive, src, dst, max_copies=3)
    assert e.value.name == "PSIM_EOVERFLOW"
    with pytest.raises(ValueError):
        O.relay_run(ap, ai, op, oi, alive, src, dst, max_copies=3)
    with pytest.raises(pa.PsimError):
        relay_run(sim, ap, ai, op, oi, alive, [3], [3])
    # the handle stays usable after errors
    (grows, gdv, gfr), (orows, odv, ofr) = _both(sim, (ap, ai, op, oi, alive, src, dst), 5)
    assert grows == orows and np.array_equal(gdv, odv) and np.array_equal(gfr, ofr)


@pytest.mark.gpu
def test_relay_over_plumtree_out_links(sim):
    """Out-links read from the device Plumtree (retrieve_outlinks/1): roots that
    heartbeat use their own tree's eager peers, the rest their members."""
    import partisan_amd as pa
    from partisan_amd.relay import out_links_from
    n = 3000
    rp, col = pa.overlay.random_regular(n, 5, 77)
    pt = pa.Simulator(lazy_tick_rounds=1, device=0)
    pt.load_overlay(rp, col)
    roots = [0, 17, 123, 2999]
    for r in roots:
        pt.broadcast(r)
        pt.run()
    op, oi = out_links_from(pt, rp, col, roots)
    pt.close()
    # the tree of a root that broadcast prunes: fewer out-links than members
    assert int(op[1] - op[0]) <= int(rp[1] - rp[0])
    rng = np.random.default_rng(5)
    alive = (rng.random(n) >= 0.05).astype(np.uint8)
    src, dst = random_sends(n, 400, rng)
    src[:4] = roots
    case = (np.asarray(rp, np.uint64), np.asarray(col, np.uint32), op, oi, alive, src, dst)
    (grows, gdv, gfr), (orows, odv, ofr) = _both(sim, case, 5)
    assert grows == orows and np.array_equal(gdv, odv) and np.array_equal(gfr, ofr)
    assert (gdv > 0).sum() > 0


@pytest.mark.gpu
def test_relay_1m_properties_and_parity(sim):
    """1M peers: parity with the oracle and the size-independent invariants
    (every direct copy arrives exactly once; arrivals = copies delivered)."""
    n, k, ttl = 1_000_000, 20_000, 3
    case = make_case(n, k, 31, dead_frac=0.05)
    (grows, gdv, gfr), (orows, odv, ofr) = _both(sim, case, ttl)
    assert grows == orows and np.array_equal(gdv, odv) and np.array_equal(gfr, ofr)
    assert sum(r["direct"] for r in grows) == sum(r["arrived"] for r in grows) == int(gdv.sum())
    assert all(r["arrived"] == 0 for r in grows[:1])
    assert (gfr[gdv > 0] < len(grows)).all() and (gfr[gdv == 0] == NEVER).all()
