"""Every node heartbeats: the forest, a handle created
with psim_config.max_roots > 16 that keeps every root's eager / lazy sets
(partisan_plumtree_broadcast.erl:1240-1248, 1278-1282) and the backend's
timestamps for every origin (partisan_plumtree_backend.erl:400-417) for good,
and runs all roots' rounds in one launch.

The reference heartbeats from every node on a timer (backend :341-368,
:421-428); an interval here = every root's heartbeat at once
(psim_plumtree_broadcast_many), then rounds to quiescence.  Checked against
the oracle (oracle/plumtree.c keeps a Root -> ordset map per vertex, as the
reference does): per-round message counts summed over the roots, and for
every root its eager / lazy sets, delivered set and accepted Round; the
outstanding rows and in-flight messages over all roots.
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import pyoracle as O  # noqa: E402

KINDS = ("broadcast", "prune", "i_have", "ignored_i_have", "graft")


def _forest(n, seed, max_roots, L=1, deg=5):
    import partisan_amd as pa
    rp, col = pa.overlay.random_regular(n, deg, seed)
    sim = pa.Simulator(lazy_tick_rounds=L, max_roots=max_roots)
    sim.load_overlay(rp, col)
    orc = O.Plumtree(rp, col, lazy_tick_rounds=L)
    return pa, sim, orc


def _compare_roots(sim, orc, monos, roots):
    """Every listed root's per-root state equals the oracle's; the rows over
    all roots equal the oracle's rows (one ETS table per node)."""
    rp, cl = sim.slot_row_ptr, sim.slot_col
    ost_all = np.zeros(sim.n, np.uint32)
    for root in roots:
        sim.focus(root)
        e, l_, o, rr = sim.plumtree_state()
        oe, ol, oo, orr = orc.dump_state(root, monos[root], rp, cl)
        assert np.array_equal(e, oe), ("eager", root, np.flatnonzero(e != oe)[:5])
        assert np.array_equal(l_, ol), ("lazy", root, np.flatnonzero(l_ != ol)[:5])
        assert np.array_equal(rr, orr), ("Round", root, np.flatnonzero(rr != orr)[:5])
        assert np.array_equal(sim.delivered(), orc.delivered(root, monos[root])), ("delivered", root)
        ost_all |= o
    oo = orc.dump_state(roots[0], monos[roots[0]], rp, cl)[2]
    return ost_all, oo


def _lockstep_interval(sim, orc, monos, roots, full_every=4, max_rounds=60):
    rounds = 0
    while rounds < max_rounds:
        gs, os_ = sim.step(1)[0], orc.step(1)[0]
        rounds += 1
        for k in KINDS:
            assert gs[k] == os_[k], (rounds, k, gs, os_)
        assert gs["delivered_new"] == os_["delivered_new"], rounds
        if rounds % full_every == 0:
            ost_all, oo = _compare_roots(sim, orc, monos, roots)
            assert np.array_equal(ost_all, oo), ("rows", rounds)
            inflight = []
            for root in roots:
                sim.focus(root)
                inflight += sim.decode_inflight()
            want = [(s_, d, t, r if t in (1, 3) else 0) for (s_, d, t, r) in orc.pending()]
            assert sorted(inflight) == sorted(want), rounds
        if sum(gs[k] for k in KINDS) == 0 and os_["outstanding_live"] == 0:
            break
    return rounds


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed,L", [(600, 3, 1), (400, 4, 2)])
def test_all_roots_two_intervals_lockstep(n, seed, L):
    """Every vertex heartbeats, twice: the first interval floods n trees,
    the second travels each root's pruned tree (i_have / ignored_i_have on
    the lazy links), then one root heartbeats a third time on its own -- its
    tree kept through the other n - 1 roots' traffic ("revisited after
    eviction pressure": nothing is evicted)."""
    pa, sim, orc = _forest(n, seed, max_roots=n, L=L)
    roots = list(range(n))
    monos = {}
    for interval in range(2):
        got = sim.broadcast_many(roots)
        for r in roots:
            monos[r] = orc.heartbeat(r)
            assert got[r] == monos[r]
        _lockstep_interval(sim, orc, monos, roots)
        ost_all, oo = _compare_roots(sim, orc, monos, roots)
        assert np.array_equal(ost_all, oo)
        for r in roots[:: max(1, n // 20)]:
            sim.focus(r)
            assert sim.delivered().all(), (interval, r)
    monos[7] = int(sim.broadcast_many([7])[0])
    assert monos[7] == orc.heartbeat(7)
    _lockstep_interval(sim, orc, monos, [7], full_every=1)
    sim.close()


@pytest.mark.gpu
def test_forest_matches_lanes_for_few_roots():
    """The forest and the 16-lane handle give the same per-round counts and
    per-root sets for the same heartbeats (10 roots, overlapping floods)."""
    import partisan_amd as pa
    rp, col = pa.overlay.random_regular(3000, 5, 11)
    a = pa.Simulator()
    a.load_overlay(rp, col)
    b = pa.Simulator(max_roots=64)
    b.load_overlay(rp, col)
    sched = {0: [0, 1, 2], 3: [100, 200], 5: [2999, 1500, 7, 8, 9]}
    for rnd in range(40):
        for r in sched.get(rnd, []):
            assert a.broadcast(r) == b.broadcast(r)
        sa, sb = a.step(1)[0], b.step(1)[0]
        for k in KINDS + ("delivered_new", "active", "senders", "words_stored"):
            assert sa[k] == sb[k], (rnd, k)
    for r in (0, 2, 200, 2999, 9):
        a.focus(r)
        b.focus(r)
        for x, y in zip(a.plumtree_state(), b.plumtree_state()):
            assert np.array_equal(x, y), r
        assert a.trace_hash() == b.trace_hash(), r
    a.close()
    b.close()


@pytest.mark.gpu
def test_forest_capacity_busy_and_errors():
    """max_roots is a hard limit (PSIM_ENOSPC, nothing changed); a root whose
    heartbeat is in flight is PSIM_EBUSY (a forest keeps one heartbeat per
    root); duplicates in one call are PSIM_EINVAL; getters before any
    heartbeat are PSIM_ESTATE."""
    pa, sim, orc = _forest(500, 21, max_roots=20)
    with pytest.raises(pa.PsimError) as ei:
        sim.delivered()
    assert ei.value.name == "PSIM_ESTATE"
    with pytest.raises(pa.PsimError) as ei:
        sim.broadcast_many(list(range(21)))
    assert ei.value.name == "PSIM_ENOSPC"
    with pytest.raises(pa.PsimError) as ei:
        sim.broadcast_many([3, 4, 3])
    assert ei.value.name == "PSIM_EINVAL"
    monos = {r: int(m) for r, m in zip(range(20), sim.broadcast_many(list(range(20))))}
    for r in range(20):
        assert monos[r] == orc.heartbeat(r)
    sim.step(2)
    orc.step(2)
    with pytest.raises(pa.PsimError) as ei:
        sim.broadcast(5)
    assert ei.value.name == "PSIM_EBUSY"
    with pytest.raises(pa.PsimError) as ei:
        sim.broadcast(20)
    assert ei.value.name == "PSIM_ENOSPC"
    _, gr = sim.run()
    _, orr = orc.run()
    assert gr == orr
    monos[5] = sim.broadcast(5)
    assert monos[5] == orc.heartbeat(5)
    _lockstep_interval(sim, orc, monos, list(range(20)), full_every=1)
    sim.close()


@pytest.mark.gpu
def test_forest_faults_reset_and_restart():
    """Omission faults on every root's traffic, a reset_peers (every root's
    sets dropped), a backend restart (the node forgets every origin) -- each
    against the oracle."""
    pa, sim, orc = _forest(300, 31, max_roots=300)
    roots = list(range(0, 300, 3))
    rng = np.random.default_rng(2)
    src = np.repeat(np.arange(sim.n), np.diff(sim.slot_row_ptr.astype(np.int64)))
    pick = rng.random(len(src)) < 0.08
    pairs = np.stack([src[pick], sim.slot_col[pick]], axis=1)
    sim.set_omissions(pairs)
    orc.set_omissions(pairs)
    monos = {}
    got = sim.broadcast_many(roots)
    for r, m in zip(roots, got):
        monos[r] = orc.heartbeat(r)
        assert m == monos[r]
    _lockstep_interval(sim, orc, monos, roots, full_every=2, max_rounds=12)
    sim.set_omissions([])
    orc.set_omissions([])
    _lockstep_interval(sim, orc, monos, roots, full_every=3)      # the lazy ticks repair every tree
    sim.reset_trees()
    orc.reset_peers_all()
    sim.restart_backend(12)
    orc.restart_backend(12)
    got = sim.broadcast_many(roots)
    for r, m in zip(roots, got):
        monos[r] = orc.heartbeat(r)
        assert m == monos[r]
    _lockstep_interval(sim, orc, monos, roots, full_every=2)
    sim.close()


@pytest.mark.gpu
def test_c2_all_roots_interval_properties():
    """The C2 overlay (10k HyParView peers) with all 10k roots heartbeating
    at once: every root's flood reaches every vertex and leaves a spanning
    tree of eager links (2(n-1) directed eager entries per root), and the
    second interval is pure tree traffic (every i_have answered by an
    ignored_i_have, no graft).  Size-independent properties: the oracle
    would take minutes here."""
    import partisan_amd as pa
    from partisan_amd.overlay import random_regular
    n = 10_000
    rp, col = random_regular(n, 5, 0x5EED0002)
    sim = pa.Simulator(max_roots=n)
    sim.load_overlay(rp, col)
    for interval in range(2):
        sim.broadcast_many(np.arange(n))
        st, rounds = sim.run()
        tot = {k: sum(s[k] for s in st) for k in KINDS + ("delivered_new",)}
        assert tot["delivered_new"] == n * (n - 1), (interval, tot)
        assert tot["i_have"] == tot["ignored_i_have"] + tot["graft"], tot   # every i_have answered once
        if interval == 1:
            # the trees carry the second heartbeat: n - 1 eager pushes per root
            # (the origins' own <= 5 are counted by broadcast_many, not the
            # rounds), plus the re-sends of the (rare) grafts
            assert n * (n - 1) - 5 * n <= tot["broadcast"] - tot["graft"] <= n * (n - 1), tot
        for r in range(0, n, 997):
            sim.focus(r)
            eager, lazy, outst, rr = sim.plumtree_state()
            assert sim.delivered().all()
            assert not outst.any()
            if interval == 0:     # a flood from fresh sets leaves a spanning tree of eager links
                assert int(np.bitwise_count(eager).sum()) == 2 * (n - 1), (interval, r)
    sim.close()


def test_forest_config_field_in_abi():
    """psim_config carries max_roots (ABI 3) and PSIM_ENOSPC is a named code."""
    from partisan_amd import _lib
    assert [f for f, _ in _lib.Config._fields_][5] == "max_roots"
    assert _lib.ERRORS[-9] == "PSIM_ENOSPC"
    assert _lib.PSIM_ABI_VERSION == 3


@pytest.mark.gpu
@pytest.mark.parametrize("L,dmax", [(1, 5), (2, 14)])
def test_forest_delay_faults_lockstep(L, dmax):
    """Delay faults on a forest (partisan_peer_service_client
    egress / ingress delay, :148-176): 25 % of the directed edges deliver
    1..dmax rounds late while 100 roots heartbeat at once; every lane's inbox
    is a ring of kRing buffers.  Round by round against the oracle
    (orc_pt_set_delays): counts by kind summed over roots every round, per-root
    sets / delivered / Round, the rows over all roots and the next round's
    in-flight messages every 3 rounds, until nothing is pending; then the
    roots heartbeat again over their pruned trees.  A root whose messages may
    still be on the wire cannot heartbeat again (PSIM_EBUSY)."""
    pa, sim, orc = _forest(700, 31 + L, max_roots=128, L=L)
    rng = np.random.default_rng(5 + L)
    src = np.repeat(np.arange(sim.n), np.diff(sim.slot_row_ptr.astype(np.int64)))
    pick = rng.random(len(src)) < 0.25
    pairs = np.stack([src[pick], sim.slot_col[pick]], axis=1)
    d = rng.integers(1, dmax + 1, len(pairs)).astype(np.uint8)
    sim.set_delays(pairs, d)
    orc.set_delays(pairs, d)
    roots = sorted(rng.choice(sim.n, 100, replace=False).tolist())
    monos = {}
    for interval in range(2):
        got = sim.broadcast_many(roots)
        for r, m in zip(roots, got):
            monos[r] = orc.heartbeat(r)
            assert m == monos[r]
        if interval == 0:
            sim.step(1)
            orc.step(1)
            with pytest.raises(pa.PsimError) as ei:
                sim.broadcast_many([roots[0]])
            assert ei.value.name == "PSIM_EBUSY"
        rounds = 0
        while True:
            gs, os_ = sim.step(1)[0], orc.step(1)[0]
            rounds += 1
            for k in KINDS:
                assert gs[k] == os_[k], (interval, rounds, k, gs, os_)
            assert gs["delivered_new"] == os_["delivered_new"], (interval, rounds)
            if rounds % 3 == 0:
                ost_all, oo = _compare_roots(sim, orc, monos, roots)
                assert np.array_equal(ost_all, oo), ("rows", rounds)
                inflight = []
                for root in roots:
                    sim.focus(root)
                    inflight += sim.decode_inflight()
                want = [(s_, d_, t, r if t in (1, 3) else 0) for (s_, d_, t, r) in orc.pending()]
                assert sorted(inflight) == sorted(want), (interval, rounds)
            if orc.inflight() == 0 and os_["outstanding_live"] == 0:
                break
            assert rounds < 400
        ost_all, oo = _compare_roots(sim, orc, monos, roots)
        assert np.array_equal(ost_all, oo)
        for r in roots:
            sim.focus(r)
            assert sim.delivered().all(), (interval, r)
    # healed while quiescent: next-round delivery again, psim_run to quiescence
    sim.set_delays([], [])
    orc.set_delays([], [])
    got = sim.broadcast_many(roots[:10])
    for r, m in zip(roots[:10], got):
        monos[r] = orc.heartbeat(r)
        assert m == monos[r]
    gst, gr = sim.run()
    ost, orr = orc.run()
    assert gr == orr
    for a, b in zip(gst, ost):
        for k in KINDS:
            assert a[k] == b[k], (k, a, b)
    _compare_roots(sim, orc, monos, roots[:10])
    sim.close()
