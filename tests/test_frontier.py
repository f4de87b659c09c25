"""Frontier kernel parity (plumtree.hip pt_frontier_kernel).

One workgroup runs the leading sparse rounds of a chunk back to back; the
round kernels take over after any round (the flags, worklist, counts and
holder ring it leaves are a round kernel's) and return at once for the rounds
it ran.  Right after a broadcast the host leaves the first rounds to it alone
(a bound on the frontier, psim_host.hip fr_plan), so a wrong bound or a wrong
hand-off loses rounds -- these tests compare the HIP path with the ORACLE:

* whole heartbeats through psim_run (16-round chunks), a flood and two
  heartbeats over the tree (the origin holds rows: its tick visits come from
  the kernel's holder list), at L = 1 and 2, with the frontier threshold
  (PSIM_FR_THR) at its default and at values that hand off after round 2-3 or
  4-5: per-round counters, then every vertex's eager / lazy / outstanding
  sets, Round, delivery and every in-flight word after each heartbeat;
* single rounds (psim_step(1), a frontier launch per round while no row is
  held) with 10 % omission faults (the kernel's fault instance);
* the same heartbeats with the kernel switched off give the same trace hash.
The kernel is opt-in (PSIM_FRONTIER=1) until it measures faster.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
KINDS = ("broadcast", "prune", "i_have", "ignored_i_have", "graft")
SEED = 0x5EED0300
ROOT_V = 777


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    return O


@pytest.mark.gpu
@pytest.mark.parametrize("thr", [None, "64", "900"])
@pytest.mark.parametrize("L", [1, 2])
def test_frontier_run_parity_200k(thr, L, monkeypatch):
    from test_worklist_parity import check_vertices, sorted_layout
    O = _oracle()
    import partisan_amd as pa
    monkeypatch.setenv("PSIM_FRONTIER", "1")
    if thr is not None:
        monkeypatch.setenv("PSIM_FR_THR", thr)
    n = 200_000
    rp, col = pa.overlay.random_regular(n, 5, SEED)
    srp, scol = sorted_layout(rp, col)
    sim = pa.Simulator(lazy_tick_rounds=L)
    sim.load_overlay(rp, col)
    orc = O.Plumtree(rp, col, L)
    for hb in range(3):
        mono = sim.broadcast(ROOT_V)
        assert mono == orc.heartbeat(ROOT_V)
        gs, gr = sim.run()
        os_, orr = orc.run()
        assert gr == orr, (thr, L, hb, gr, orr)
        for r, (g, o) in enumerate(zip(gs, os_)):
            for k in KINDS + ("delivered_new",):
                assert g[k] == o[k], (thr, L, hb, r, k, g, o)
        check_vertices(sim, orc, ROOT_V, mono, srp, scol, 0, n, (thr, L, hb))
        assert sim.delivered().all()
    rounds, launches = sim.frontier_stats()
    assert rounds >= 3 * 2 and launches >= 3, (rounds, launches)
    sim.close()
    orc.close()


@pytest.mark.gpu
def test_frontier_single_rounds_with_omissions(monkeypatch):
    from test_worklist_parity import check_vertices, sorted_layout
    monkeypatch.setenv("PSIM_FRONTIER", "1")
    O = _oracle()
    import partisan_amd as pa
    n = 50_000
    rp, col = pa.overlay.random_regular(n, 5, SEED + 1)
    srp, scol = sorted_layout(rp, col)
    rng = np.random.default_rng(7)
    src = np.repeat(np.arange(n, dtype=np.uint32), np.diff(np.asarray(rp, np.int64)))
    dst = np.asarray(col, np.uint32)
    pick = rng.random(len(dst)) < 0.10
    sim = pa.Simulator(lazy_tick_rounds=1)
    sim.load_overlay(rp, col)
    pairs = np.stack([src[pick], dst[pick]], axis=1)
    sim.set_omissions(pairs)
    orc = O.Plumtree(rp, col, 1)
    orc.set_omissions(pairs)
    mono = sim.broadcast(ROOT_V)
    assert mono == orc.heartbeat(ROOT_V)
    for rnd in range(1, 200):
        g, o = sim.step(1)[0], orc.step(1)[0]
        for k in KINDS + ("delivered_new",):
            assert g[k] == o[k], (rnd, k, g, o)
        if rnd % 3 == 0:
            check_vertices(sim, orc, ROOT_V, mono, srp, scol, 0, n, rnd)
        if sum(o[k] for k in KINDS) == 0 and o["outstanding_live"] == 0:
            break
    check_vertices(sim, orc, ROOT_V, mono, srp, scol, 0, n, "end")
    assert sim.frontier_stats()[0] > 0
    sim.close()
    orc.close()


def _hashes(pa, rp, col, L):
    sim = pa.Simulator(lazy_tick_rounds=L)
    sim.load_overlay(rp, col)
    out = []
    for _ in range(3):
        sim.broadcast(ROOT_V)
        _, r = sim.run()
        out.append((r,) + sim.trace_hash())
    fr = sim.frontier_stats()[0]
    sim.close()
    return out, fr


@pytest.mark.gpu
def test_frontier_off_same_trace_1m(monkeypatch):
    import partisan_amd as pa
    rp, col = pa.overlay.random_regular(1_000_000, 5, SEED + 2)
    monkeypatch.setenv("PSIM_FRONTIER", "1")
    on, fr_on = _hashes(pa, rp, col, 1)
    monkeypatch.setenv("PSIM_FRONTIER", "0")
    off, fr_off = _hashes(pa, rp, col, 1)
    assert fr_on > 0 and fr_off == 0
    assert on == off
