"""HyParView view maintenance: HIP path (csrc/hyparview.hip) vs the oracle
(oracle/hyparview.c), round by round, bit-exact: every vertex's active and
passive views, its rand draw count, its sent/recv id maps, and the per-round
message counts by kind.  Trajectories are parity unpinned by reference
vectors (no reference test fixes them); the view invariants the
reference checks in test/partisan_SUITE.erl:2331-2395 (active views
symmetric, overlay connected) are asserted on both paths.
"""
import collections

import numpy as np
import pytest

import pyoracle as O

SEED = 0x5EED0002


def contacts(n, seed=SEED):
    """Joiner i (1..n-1) contacts a uniform earlier vertex: Philox stream kind 1
    (workload), counter {i, 0, 1, 0}; mulhi of the low 64 bits by i."""
    key = [seed & 0xFFFFFFFF, seed >> 32]
    out = np.zeros(n, np.uint32)
    for i in range(1, n):
        r = O.philox([i, 0, 1, 0], key)
        out[i] = ((r[0] | (r[1] << 32)) * i) >> 64
    return out


def views_of_oracle(o, n):
    return [o.views(v) for v in range(n)]


def check_invariants(active, n, alive=None):
    """active[v] = active view of v including self (sorted list)."""
    up = np.ones(n, bool) if alive is None else np.asarray(alive, bool)
    adj = [set(a) - {v} for v, a in enumerate(active)]
    for v in range(n):
        if not up[v]:
            continue
        for p in adj[v]:
            if up[p]:
                assert v in adj[p], (v, p)       # symmetric between live peers
    start = next(v for v in range(n) if up[v])
    seen = {start}
    dq = collections.deque([start])
    while dq:
        v = dq.popleft()
        for p in adj[v]:
            if up[p] and p not in seen:
                seen.add(p)
                dq.append(p)
    assert len(seen) == int(up.sum()), "overlay of live peers is not connected"


# ------------------------------------------------------------------ CPU (oracle)
def test_oracle_sequential_joins_invariants():
    n = 1500
    c = contacts(n)
    o = O.HyParView(n, SEED)
    err = 0
    for i in range(1, n):
        o.join(i, int(c[i]))
        err |= o.step(1)[0]["error"]
    for s in o.step(60):
        err |= s["error"]
    assert err == 0
    act = [o.views(v)[0] for v in range(n)]
    check_invariants(act, n)
    deg = np.array([len(a) - 1 for a in act])
    assert deg.min() >= 1 and deg.max() <= O.HV_DEFAULTS["active_max_size"] - 1
    pas = np.array([len(o.views(v)[1]) for v in range(n)])
    assert pas.mean() > 20


def test_oracle_deterministic():
    def run():
        o = O.HyParView(300, 7)
        c = contacts(300, 7)
        for i in range(1, 300):
            o.join(i, int(c[i]))
            o.step(1)
        st = o.step(30)
        return [o.views(v) for v in range(300)], [o.draws(v) for v in range(300)], st
    assert run() == run()


# ------------------------------------------------------------------ GPU parity
def _pair(n, seed=SEED, **cfg):
    import partisan_amd as pa
    sim = pa.Simulator(seed=seed)
    g = pa.hyparview.HyParViewCluster(sim, n, **cfg)
    o = O.HyParView(n, seed, **cfg)
    return sim, g, o


def _compare(g, o, n, maps=True):
    act, na, pas, np_ = g.views()
    dr = g.draws()
    for v in range(n):
        oa, op = o.views(v)
        assert act[v, :na[v]].tolist() == oa, ("active", v)
        assert pas[v, :np_[v]].tolist() == op, ("passive", v)
        assert int(dr[v]) == o.draws(v), ("draws", v)
        if maps:
            for which in (0, 1):
                assert sorted(g.idmap(v, which)) == sorted(o.idmap(v, which)), ("idmap", which, v)
    assert g.inflight() == o.inflight()


def _same_stats(gs, os_):
    assert len(gs) == len(os_)
    for r, (a, b) in enumerate(zip(gs, os_)):
        assert a["sent"] == b["sent"], (r, a["sent"], b["sent"])
        assert a["draws"] == b["draws"], (r, a["draws"], b["draws"])
        assert (a["error"] & 12 != 0) == (b["error"] != 0), r
        assert a["error"] & 3 == 0


@pytest.mark.gpu
def test_lockstep_sequential_joins_small():
    n = 200
    sim, g, o = _pair(n)
    c = contacts(n)
    for i in range(1, n):
        g.join(i, int(c[i]))
        o.join(i, int(c[i]))
        _same_stats(g.step(1), o.step(1))
        if i % 25 == 0:
            _compare(g, o, n)
    for _ in range(6):
        _same_stats(g.step(5), o.step(5))
        _compare(g, o, n)
    check_invariants([g.active_view(v) for v in range(n)], n)
    sim.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,cfg", [(3000, {}), (2000, dict(active_max_size=5, passive_max_size=12,
                                                            shuffle_rounds=4, promotion_rounds=3))])
def test_mass_join_then_shuffles(n, cfg):
    """Every vertex joins a Philox-drawn earlier vertex in the same gap between
    rounds, then 80 rounds of message handling, promotions and shuffles."""
    sim, g, o = _pair(n, **cfg)
    c = contacts(n)
    vs = np.arange(1, n, dtype=np.uint32)
    g.join_many(vs, c[1:])
    for v in vs.tolist():
        o.join(v, int(c[v]))
    for _ in range(8):
        _same_stats(g.step(10), o.step(10))
    _compare(g, o, n)
    sim.close()


@pytest.mark.gpu
def test_failures_disconnect_and_promotion():
    """10% of the vertices die after the overlay settles: messages to them are
    lost, promotions refill active views from the passive views."""
    n = 2500
    sim, g, o = _pair(n)
    c = contacts(n)
    vs = np.arange(1, n, dtype=np.uint32)
    g.join_many(vs, c[1:])
    for v in vs.tolist():
        o.join(v, int(c[v]))
    _same_stats(g.step(40), o.step(40))
    alive = np.ones(n, np.uint8)
    alive[np.random.default_rng(3).choice(n, n // 10, replace=False)] = 0
    g.set_alive(alive)
    o.set_alive(alive)
    for _ in range(6):
        _same_stats(g.step(10), o.step(10))
    _compare(g, o, n)
    # the live overlay keeps working: new joins through live contacts
    live = np.nonzero(alive)[0]
    rng = np.random.default_rng(4)
    joiners = rng.choice(live, 50, replace=False).astype(np.uint32)
    cont = rng.choice(live, 50).astype(np.uint32)
    g.join_many(joiners, cont)
    for v, k in zip(joiners.tolist(), cont.tolist()):
        o.join(v, k)
    _same_stats(g.step(20), o.step(20))
    _compare(g, o, n)
    sim.close()


@pytest.mark.gpu
def test_c2_sequential_10k_final_state():
    """SURVEY 8 config C2's overlay: 10k sequential joins (one per round), then
    100 rounds; final views, draws and counters equal the oracle's."""
    n = 10000
    sim, g, o = _pair(n)
    c = contacts(n)
    gt, ot = np.zeros(9, np.int64), np.zeros(9, np.int64)
    for i in range(1, n):
        g.join(i, int(c[i]))
        o.join(i, int(c[i]))
        gt += np.array(g.step(1)[0]["sent"])
        ot += np.array(o.step(1)[0]["sent"])
    assert gt.tolist() == ot.tolist()
    _same_stats(g.step(100), o.step(100))
    _compare(g, o, n, maps=False)
    act, na, _, _ = g.views()
    check_invariants([act[v, :na[v]].tolist() for v in range(n)], n)
    sim.close()


@pytest.mark.gpu
def test_large_mass_join_properties():
    """200k vertices (oracle-free): symmetric, connected active views after
    the joins settle and two shuffle periods; queue and id maps in bounds."""
    import partisan_amd as pa
    n = 200_000
    sim = pa.Simulator(seed=SEED)
    g = pa.hyparview.HyParViewCluster(sim, n)
    rng = np.random.default_rng(9)
    vs = np.arange(1, n, dtype=np.uint32)
    g.join_many(vs, (rng.random(n - 1) * vs).astype(np.uint32))
    st = g.step(60)
    assert all(s["error"] == 0 for s in st)
    act, na, _, np_ = g.views()
    check_invariants([act[v, :na[v]].tolist() for v in range(n)], n)
    assert na.max() <= 6 and np_.max() <= 30
    rp, col = g.overlay()
    assert int(rp[-1]) == int(na.sum()) - n
    sim.close()
