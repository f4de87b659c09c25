"""Committed Plumtree traces (tests/golden/plumtree_traces.json, written by
tests/golden/make_plumtree_traces.py from oracle/plumtree.c) replayed
round by round: against the oracle on CPU (it cannot drift without this
test failing), and against libpsim (both Plumtree engines) on the GPU.

Parity status: the reference holds no Plumtree trace (SURVEY 8(c)
"Unpinned") and cannot run here (no erts), so these pin the oracle and the
HIP path to each other and to this file -- parity against the reference
itself stays unpinned for Plumtree; the topologies come from the KAT-pinned
build_tree/3 restatement (src/partisan_plumtree_util.erl:43-58).
"""
import json
import os

import numpy as np
import pytest

import pyoracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KINDS = ("broadcast", "prune", "i_have", "ignored_i_have", "graft")
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "plumtree_traces.json")))
CASES = {c["name"]: c for c in GOLD["cases"]}


def csr(case):
    return np.asarray(case["row_ptr"], np.uint64), np.asarray(case["col"], np.uint32)


def test_build_tree_topologies_match_kat_generator():
    """The trace topologies are build_tree/3 outputs of the KAT-pinned oracle."""
    for c in GOLD["cases"]:
        if "build_tree" not in c:
            continue
        arity = int(c["name"].split("_a")[1][0])
        cyc = c["name"].endswith("_cycles")
        assert O.build_tree(arity, list(range(c["n"])), cyc) == c["build_tree"]


def _norm(pending):
    return [[s, d, t, r if t in (1, 3) else 0] for (s, d, t, r) in pending]


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_replays_golden_trace(name):
    c = CASES[name]
    rp, col = csr(c)
    orc = O.Plumtree(rp, col, c["lazy_tick_rounds"])
    n = c["n"]
    for ev in c["events"]:
        if "alive" in ev:
            orc.set_alive(np.asarray(ev["alive"], np.uint8))
            continue
        if "omit" in ev:
            orc.set_omissions(ev["omit"])
            continue
        if "heartbeat" in ev:
            assert orc.heartbeat(ev["heartbeat"]) == ev["mono"]
            assert _norm(orc.pending()) == ev["origin_msgs"]
        root = ev.get("heartbeat", ev.get("continue"))
        for i, r in enumerate(ev["rounds"]):
            st = orc.step(1)[0]
            assert [st[k] for k in KINDS] + [st["delivered_new"]] == r["stats"], (name, i)
            assert _norm(orc.pending()) == r["msgs"], (name, i)
        f = ev["final"]
        for v in range(n):
            e, lz = orc.peers(v, root)
            assert e == f["eager"][v] and lz == f["lazy"][v], (name, v)
            assert sorted([p, rr] for p, rr, _ in orc.outstanding(v)) == f["outstanding"][v], (name, v)
        assert orc.delivered(root, ev["mono"]).astype(int).tolist() == f["delivered"]
        assert [int(x) for x in orc.recv_round(root, ev["mono"])] == f["recv_round"]
    orc.close()


ENGINES = {"slot_scatter": {}, "slot_scatter_csr": {"csr": True}, "binned": {"binned": True}}


@pytest.mark.gpu
@pytest.mark.parametrize("engine", sorted(ENGINES))
@pytest.mark.parametrize("name", sorted(CASES))
def test_hip_replays_golden_trace(name, engine):
    import partisan_amd as pa
    c = CASES[name]
    rp, col = csr(c)
    sim = pa.Simulator(lazy_tick_rounds=c["lazy_tick_rounds"], device=0, **ENGINES[engine])
    sim.load_overlay(rp, col)
    n = c["n"]
    for ev in c["events"]:
        if "alive" in ev:
            sim.set_alive(np.asarray(ev["alive"], np.uint8))
            continue
        if "omit" in ev:
            sim.set_omissions(ev["omit"])
            continue
        if "heartbeat" in ev:
            assert sim.broadcast(ev["heartbeat"]) == ev["mono"]
            assert [list(m) for m in sim.decode_inflight()] == ev["origin_msgs"]
        root = ev.get("heartbeat", ev.get("continue"))
        for i, r in enumerate(ev["rounds"]):
            st = sim.step(1)[0]
            assert [st[k] for k in KINDS] + [st["delivered_new"]] == r["stats"], (name, i)
            assert [list(m) for m in sim.decode_inflight()] == r["msgs"], (name, i)
        f = ev["final"]
        eager, lazy, outst, rr = sim.plumtree_state()
        for v in range(n):
            assert sim.mask_to_peers(v, eager[v]) == f["eager"][v], (name, v)
            assert sim.mask_to_peers(v, lazy[v]) == f["lazy"][v], (name, v)
            rows = f["outstanding"][v]
            assert sim.mask_to_peers(v, outst[v]) == sorted({p for p, _ in rows}), (name, v)
            want = f["recv_round"][v]
            assert int(rr[v]) == (0xFFFF if want == 0xFFFFFFFF else 0xFFFE if want == 0xFFFFFFFE else want), v
            if rows:
                my = 0 if rr[v] == 0xFFFE else int(rr[v]) + 1
                assert {r_ for _, r_ in rows} == {my}, (name, v)
        assert sim.delivered().astype(int).tolist() == f["delivered"]
    sim.close()
