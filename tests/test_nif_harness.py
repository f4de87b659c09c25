"""The Erlang NIF shim (erl/c_src/partisan_gpu_sim_nif.c), linked with
libpsim.so and a functional mock of erts (tests/nif_mock/mock_erts.c), driven
through its ErlNifFunc table by tests/nif_mock/nif_harness.c -- the calls an
Erlang host makes (SURVEY 8(b) "What calls it"; 8(f) row 3), minus the BEAM,
which this image does not have.

CPU: the harness builds and links.  GPU: it runs a small C2 (HyParView
sequential joins, shuffle periods, a Plumtree heartbeat over the active
views), Demers, SCAMP v2, full membership, C3, causal delivery, vclock and
the world-1 sharded run over the library's own RCCL communicator through the
shim, and its C2 result is bit-identical (rounds, broadcasts, trace digest)
to the same scenario driven from Python over the same ABI.
"""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MOCK = os.path.join(ROOT, "tests", "nif_mock")
SRCS = [os.path.join(ROOT, "erl", "c_src", "partisan_gpu_sim_nif.c"), os.path.join(MOCK, "mock_erts.c"),
        os.path.join(MOCK, "nif_harness.c")]
BIN = os.path.join(MOCK, "nif_harness")


def build_harness(out=BIN):
    """gcc the shim + mock erts + harness against libpsim.so (rpath: the in-tree library)."""
    cmd = ["gcc", "-O1", "-std=gnu11", "-Wall", "-Wextra", "-Wno-unused-parameter", "-Werror",
           "-I", MOCK, "-I", os.path.join(ROOT, "include")] + SRCS + \
          ["-L", os.path.join(ROOT, "partisan_amd"), "-lpsim", "-Wl,-rpath," + os.path.join(ROOT, "partisan_amd"),
           "-lpthread", "-o", out]
    subprocess.check_call(cmd)
    return out


def test_harness_builds_and_links(tmp_path):
    build_harness(str(tmp_path / "nif_harness"))
    assert os.path.getsize(tmp_path / "nif_harness") > 0


def _lcg(s):
    s = (s * 6364136223846793005 + 1442695040888963407) & ((1 << 64) - 1)
    return s, s >> 33


def _check_fm_wire(w):
    """SURVEY 8(f) row 3, full membership: the {Src, Dst, Seq, Known, Removed}
    records the shim renders (what the cluster module turns into
    {membership_strategy, {Spec, #full_v1{}}}) equal, round by round, the
    oracle's messages in flight (src, dst, token bitmaps of the state) in
    handling order; a node's messages taken off (fm_take) and put back
    (fm_put), and a state put from a node outside the cluster, leave every
    node's state equal to the oracle's after the same operations."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    n = w["n"]
    orc = O.FullMembership(n, periodic_rounds=3)
    for i in range(1, n):
        orc.join(i, i - 1)

    def bits(rows):
        k = r = 0
        for _, t, act in rows:
            k |= 1 << t
            if not act:
                r |= 1 << t
        return k, r

    for r, got in enumerate(w["rounds"]):
        orc.step(1)
        ms = orc.messages()
        assert [[s, d, *bits(rows)] for s, d, _q, rows in ms] == got, r
        if r == 3 and ms:
            orc.put(orc.take(ms[0][1]))
        if r == 5:
            orc.put([(n, 4, 0, orc.payload(2))])
    assert w["taken"] > 0
    for v in range(n):
        assert list(bits(orc.payload(v))) == [w["known"][v], w["removed"][v]], v


def _check_scamp_wire(w):
    """the {membership_strategy, Msg} terms the shim renders
    for a SCAMP v2 run, round by round, equal the oracle's messages in
    flight (type, src, dst, emission seq, node ids) in handling order; one
    node's messages taken off the wire (scamp_take) and put back
    (scamp_put, as its manager's handle_message/2 would) change nothing: the
    views after 12 more rounds equal the oracle's, which never took them."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    n = w["n"]
    orc = O.Scamp(n, version=2, c=5, periodic_rounds=10, seed=0x5EED0004)
    s, k = 11, 1
    while k < n:
        hi = min(2 * k, n)
        for i in range(k, hi):
            s, r = _lcg(s)
            orc.join(i, r % k)
        orc.step(3)
        k *= 2
    assert w["taken"] > 0
    for r, got in enumerate(w["rounds"]):
        assert [tuple(m) for m in got] == orc.pending(), r
        orc.step(1)
    for v in range(n):
        assert w["views"][v] == orc.view(v), v


@pytest.mark.gpu
def test_nif_harness_on_gpu(tmp_path):
    exe = build_harness()
    report = tmp_path / "report.json"
    out = subprocess.run([exe, str(report)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    rep = json.loads(report.read_text())
    n = rep["c2"]["n"]
    assert rep["c2"]["delivered"] == n                       # the reliable-broadcast postcondition
    assert rep["shard_rccl_world1"] == {"rounds": rep["c2"]["rounds"], "delivered": n, "step2": 2}
    assert rep["c2_getters"] == {"delivered_mono": n, "messages": 0, "rows0": 0, "is_delivered": n}
    assert rep["demers"]["complete"] == rep["demers"]["n"]
    # the sharded entry points with the exchange in the library (RCCL, world 1): the same epidemic
    assert rep["demers_shard_rccl_world1"] == {"rounds": rep["demers"]["rounds"], "complete": rep["demers"]["n"]}
    assert rep["fullmem"]["knows_all"] == rep["fullmem"]["n"]
    assert rep["fullmem"]["tokens_used"] == rep["fullmem"]["own_tokens"] == rep["fullmem"]["n"]
    assert rep["scamp"]["view_entries"] > rep["scamp"]["n"]
    _check_scamp_wire(rep["scamp_wire"])
    _check_fm_wire(rep["fm_wire"])
    assert 0 < rep["c3"]["delivered_live"] <= rep["c3"]["live"]
    assert rep["c3"]["run_rounds"] == 3 and rep["c3"]["run_live"] == rep["c3"]["n"]   # c3_run: crashed, then rejoined
    assert rep["causal"]["delivered"] > 0
    assert rep["causal_shard_rccl_world1"]["delivered"] == rep["causal"]["delivered"]
    assert rep["vclock_merge"] == [3, 1, 4]
    # the forest through the NIF: every root of the C2 overlay heartbeats, twice
    assert rep["forest"]["roots"] == n and rep["forest"]["delivered"] == n * (n - 1), rep["forest"]
    assert all(r > 0 for r in rep["forest"]["rounds"])
    # parked roots through the NIF (forest_lanes): every root's flood, 16 lanes at a time
    assert rep["parked"]["delivered"] == n * (n - 1) and rep["parked"]["enospc"] == 1, rep["parked"]

    # the same C2 through the Python binding of the same ABI: bit-identical
    import partisan_amd as pa
    sim = pa.Simulator(lazy_tick_rounds=1, device=0, seed=0x5EED0002)
    hv = pa.hyparview.HyParViewCluster(sim, n, shuffle_rounds=10, promotion_rounds=5)
    s = 2
    for i in range(1, n):
        s, r = _lcg(s)
        hv.join(i, r % i)
        hv.step(1)
    hv.step(100)
    act, na, _, _ = hv.views()
    rows = [[int(u) for u in act[v, :na[v]] if u != v] for v in range(n)]
    rp = np.zeros(n + 1, np.uint64)
    rp[1:] = np.cumsum([len(r) for r in rows])
    col = np.asarray([u for r in rows for u in r], np.uint32)
    assert int(rp[-1]) == rep["c2"]["edges"]
    sim.load_overlay(rp, col)
    assert sim.broadcast(0) == rep["c2"]["mono"]
    stats, rounds = sim.run(1000)
    assert rounds == rep["c2"]["rounds"]
    assert sum(x["broadcast"] for x in stats) == rep["c2"]["broadcasts"]
    assert [str(x) for x in sim.trace_hash()] == rep["c2"]["trace"]
    # root 0's second heartbeat: the NIF's broadcast_run = broadcast + run here
    assert sim.broadcast(0) == rep["c2_hb2"]["mono"]
    stats, rounds = sim.run(1000)
    assert rounds == rep["c2_hb2"]["rounds"]
    assert sum(x["broadcast"] for x in stats) == rep["c2_hb2"]["broadcasts"]
    assert [str(x) for x in sim.trace_hash()] == rep["c2_hb2"]["trace"]
    # three more over the tree in one NIF call (broadcast_run_n) = three broadcast + run here
    got, bsum, nrows = [], 0, 0
    for _ in range(3):
        m = sim.broadcast(0)
        stats, rounds = sim.run(1000)
        got.append([m, rounds])
        bsum += sum(x["broadcast"] for x in stats)
        nrows += len(stats)
    assert got == rep["c2_hb345"]["intervals"]
    assert nrows == rep["c2_hb345"]["rows"]
    assert bsum == rep["c2_hb345"]["broadcasts"]
    assert [str(x) for x in sim.trace_hash()] == rep["c2_hb345"]["trace"]
    sim.close()
