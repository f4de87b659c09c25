"""Parked roots: a forest that keeps
every root's per-root records -- the reference's eager_sets / lazy_sets
entries, kept for good (partisan_plumtree_broadcast.erl:1240-1248,
1278-1282), and the backend's delivered ids (partisan_plumtree_backend.erl:
400-417) -- in 16 B per vertex and root, while only `forest_lanes` roots at
a time hold the ~40 B per vertex a heartbeat in flight needs (inbox words,
flags, rows, counts).  A heartbeat takes the lane of a root whose own is done
(psim_forest_set_lanes).

Checked three ways: round by round against the oracle (every root
heartbeating in batches through 16 lanes, twice -- the second interval
travels each root's pruned tree after its lane went to other roots); equal,
round by round and root by root, to a forest with one lane per root on the
same schedule; and at 4M peers x 2,000 roots, where one lane per root does
not fit in HBM (PSIM_ENOMEM) and the parked forest does.
"""
import numpy as np
import pytest

from test_forest import KINDS, _compare_roots, _lockstep_interval


def _parked(n, seed, lanes, L=1, deg=5, max_roots=None):
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import pyoracle as O
    import partisan_amd as pa
    rp, col = pa.overlay.random_regular(n, deg, seed)
    sim = pa.Simulator(lazy_tick_rounds=L, max_roots=max_roots or n, forest_lanes=lanes)
    sim.load_overlay(rp, col)
    orc = O.Plumtree(rp, col, lazy_tick_rounds=L)
    return pa, sim, orc


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed,L", [(600, 3, 1), (400, 4, 2)])
def test_parked_roots_lockstep(n, seed, L):
    """Every vertex heartbeats through 16 lanes, 16 roots at a time, each
    batch in lockstep with the oracle to quiescence; then every root's
    records (most of them parked) equal the oracle's.  A second interval in
    another order: each root's heartbeat travels its pruned tree (i_have /
    ignored_i_have on the lazy links) from records it kept while parked."""
    pa, sim, orc = _parked(n, seed, 16, L=L)
    roots = list(range(n))
    monos = {}
    for interval in range(2):
        order = roots if interval == 0 else roots[::-1]
        for b in range(0, n, 16):
            batch = order[b:b + 16]
            got = sim.broadcast_many(batch)
            for r, m in zip(batch, got):
                monos[r] = orc.heartbeat(r)
                assert m == monos[r], (interval, r)
            _lockstep_interval(sim, orc, monos, batch, full_every=5)
        ost_all, oo = _compare_roots(sim, orc, monos, roots)
        assert np.array_equal(ost_all, oo), interval
        for r in roots[:: max(1, n // 25)]:
            sim.focus(r)
            assert sim.delivered().all(), (interval, r)
            assert sim.decode_inflight() == [], (interval, r)   # a parked root has nothing in flight
    sim.close()


@pytest.mark.gpu
def test_parked_lanes_busy_and_errors():
    """Lanes are handed out to heartbeats in flight: more at once than lanes
    is PSIM_ENOSPC (nothing changed, the call can be repeated once a lane's
    root is done); a root in flight is PSIM_EBUSY; roots beyond max_roots
    are PSIM_ENOSPC; psim_forest_set_lanes only before the overlay, only on a
    forest, at most max_roots."""
    import partisan_amd as pa
    with pytest.raises(pa.PsimError) as ei:
        pa.Simulator(max_roots=8, forest_lanes=4)          # 8 roots: lanes, not a forest
    assert ei.value.name == "PSIM_ESTATE"
    with pytest.raises(pa.PsimError) as ei:
        pa.Simulator(max_roots=40, forest_lanes=41)
    assert ei.value.name == "PSIM_EINVAL"
    pa, sim, orc = _parked(500, 21, 8, max_roots=40)
    from partisan_amd._lib import lib
    rc = lib().psim_forest_set_lanes(sim._h, 4)
    assert pa._lib.ERRORS[rc] == "PSIM_ESTATE"
    monos = {}
    got = sim.broadcast_many(list(range(6)))
    for r, m in zip(range(6), got):
        monos[r] = orc.heartbeat(r)
        assert m == monos[r]
    sim.step(2)
    orc.step(2)
    with pytest.raises(pa.PsimError) as ei:
        sim.broadcast_many([10, 11, 12])                   # 6 lanes busy, 2 free
    assert ei.value.name == "PSIM_ENOSPC"
    with pytest.raises(pa.PsimError) as ei:
        sim.broadcast(3)
    assert ei.value.name == "PSIM_EBUSY"
    got = sim.broadcast_many([10, 11])                     # the 2 free lanes
    for r, m in zip((10, 11), got):
        monos[r] = orc.heartbeat(r)
        assert m == monos[r]
    _lockstep_interval(sim, orc, monos, list(range(6)) + [10, 11], full_every=2)
    got = sim.broadcast_many([12, 13, 14, 15, 16, 17, 18, 19])   # every lane's root is done: 8 reused
    for r, m in zip(range(12, 20), got):
        monos[r] = orc.heartbeat(r)
        assert m == monos[r]
    _lockstep_interval(sim, orc, monos, list(range(12, 20)), full_every=3)
    with pytest.raises(pa.PsimError) as ei:
        sim.broadcast_many(list(range(20, 45)))            # 16 + 25 roots > max_roots = 40
    assert ei.value.name == "PSIM_ENOSPC"
    got = sim.broadcast_many([0, 5, 39])                   # parked roots take lanes back
    for r, m in zip((0, 5, 39), got):
        monos[r] = orc.heartbeat(r)
        assert m == monos[r]
    _lockstep_interval(sim, orc, monos, [0, 5, 39], full_every=1)
    ost_all, oo = _compare_roots(sim, orc, monos, list(range(6)) + list(range(10, 20)) + [39])
    assert np.array_equal(ost_all, oo)
    sim.close()


def _schedule(sims, n_roots, batch, rng, check):
    """The same heartbeats on every handle: batches of `batch` roots, the next
    batch started 3 rounds into the last one (overlapping floods, within the
    lanes), every round's counters equal across the handles."""
    order = rng.permutation(n_roots).tolist()
    live = []
    for b in range(0, n_roots, batch):
        roots = order[b:b + batch]
        monos = [list(s.broadcast_many(roots)) for s in sims]
        assert all(m == monos[0] for m in monos), roots
        live.append(roots)
        for _ in range(3):
            st = [s.step(1)[0] for s in sims]
            for k in KINDS + ("delivered_new", "active", "senders", "words_stored"):
                assert all(x[k] == st[0][k] for x in st), k
        if len(live) == 2:                                  # the older batch runs out
            while True:
                st = [s.step(1)[0] for s in sims]
                for k in KINDS + ("delivered_new", "active", "senders", "words_stored"):
                    assert all(x[k] == st[0][k] for x in st), k
                if sum(st[0][k] for k in KINDS) == 0 and st[0]["outstanding_vertices"] == 0:
                    break
            live = []
    for s in sims:
        s.run()
    for r in check:
        ref = None
        for s in sims:
            s.focus(r)
            got = [*s.plumtree_state(), s.delivered(), s.trace_hash()]
            if ref is None:
                ref = got
            else:
                for x, y in zip(got, ref):
                    assert np.array_equal(x, y), r


@pytest.mark.gpu
def test_parked_equals_one_lane_per_root_100k():
    """100k peers, 1,000 roots, two intervals of overlapping batches of 8:
    the parked forest (16 lanes) and the forest with one lane per root give
    the same counters every round and the same records for every checked
    root."""
    import partisan_amd as pa
    rp, col = pa.overlay.random_regular(100_000, 5, 0x5EED0011)
    a = pa.Simulator(max_roots=1000, forest_lanes=16)
    b = pa.Simulator(max_roots=1000)
    for s in (a, b):
        s.load_overlay(rp, col)
    rng = np.random.default_rng(7)
    for interval in range(2):
        _schedule([a, b], 1000, 8, rng, check=range(0, 1000, 97))
    a.close()
    b.close()


@pytest.mark.gpu
def test_parked_forest_fits_where_one_lane_per_root_does_not():
    """4M peers x 2,000 roots: one lane per root would take ~470 GB (the
    handle refuses it, PSIM_ENOMEM, nothing allocated); the parked forest
    keeps the 2,000 roots' records (128 GB) with 8 lanes (~1.4 GB) and runs
    heartbeats through them (80 roots, batches of 8): every flood reaches
    every vertex and a parked root's records survive the other roots'
    heartbeats bit for bit."""
    import partisan_amd as pa
    n = 4_000_000
    rp, col = pa.overlay.random_regular(n, 5, 0x5EED0012)
    dense = pa.Simulator(max_roots=2000)
    with pytest.raises(pa.PsimError) as ei:
        dense.load_overlay(rp, col)
    assert ei.value.name == "PSIM_ENOMEM"
    dense.close()
    sim = pa.Simulator(max_roots=2000, forest_lanes=8)
    sim.load_overlay(rp, col)
    first = list(range(0, 16_000, 1000))                  # 16 roots, two batches of 8
    hashes = {}
    for b in range(0, 16, 8):
        sim.broadcast_many(first[b:b + 8])
        st, rounds = sim.run()
        assert sum(s["delivered_new"] for s in st) == 8 * (n - 1), b
    for r in first:
        sim.focus(r)
        assert sim.delivered().all(), r
        hashes[r] = sim.trace_hash()[:3]                       # (records, live words, delivered)
    others = list(range(1_000_000, 1_000_000 + 64 * 7, 7))     # 64 more roots, 8 batches through the lanes
    for b in range(0, 64, 8):
        sim.broadcast_many(others[b:b + 8])
        st, _ = sim.run()
        assert sum(s["delivered_new"] for s in st) == 8 * (n - 1), b
    for r in first:
        sim.focus(r)
        assert sim.trace_hash()[:3] == hashes[r], r             # parked: untouched
    sim.close()
