"""HyParView view maintenance: HIP path (csrc/hyparview.hip) vs the oracle
(oracle/hyparview.c), round by round, bit-exact: every vertex's active and
passive views, its rand draw count, its sent/recv id maps, and the per-round
message counts by kind.  Trajectories are parity unpinned by reference
vectors (no reference test fixes them); the view invariants the
reference checks in test/partisan_SUITE.erl:2331-2395 (active views
symmetric, overlay connected) are asserted on both paths.
"""
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


def check_invariants(active, n, alive=None, min_giant=1.0):
    """active[v] = active view of v including self (sorted list): the active
    views of live peers are symmetric and the live overlay is connected."""
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components
    up = np.ones(n, bool) if alive is None else np.asarray(alive, bool)
    src = np.repeat(np.arange(n), [len(a) for a in active])
    dst = np.fromiter((p for a in active for p in a), np.int64, len(src))
    keep = (src != dst) & up[src] & up[dst]
    src, dst = src[keep], dst[keep]
    A = coo_matrix((np.ones(len(src), np.int8), (src, dst)), shape=(n, n)).tocsr()
    assert (A != A.T).nnz == 0, "active views are not symmetric"
    live = np.nonzero(up)[0]
    k, lab = connected_components(A[live][:, live], directed=False)
    giant = np.bincount(lab).max() / len(live)
    assert giant >= min_giant, f"overlay of live peers has {k} components (largest {giant:.5f})"


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
@pytest.mark.parametrize("rounds", [0, 1, 3, 20])
def test_join_seq_equals_join_and_step(rounds):
    """psim_hv_join_seq = psim_hv_join + psim_hv_step(rounds) per joiner:
    per-round stats, views, draws and id maps (rounds 20: the plain calls)."""
    import partisan_amd as pa
    n = 600
    c = contacts(n)
    out = []
    for seq in (False, True):
        sim = pa.Simulator(seed=SEED)
        g = pa.hyparview.HyParViewCluster(sim, n, shuffle_rounds=4, promotion_rounds=3)
        if seq:
            st = g.join_seq(np.arange(1, n, dtype=np.uint32), c[1:], rounds=rounds)
        else:
            st = []
            for i in range(1, n):
                g.join(i, int(c[i]))
                if rounds:
                    st += g.step(rounds)
        st += g.step(7)
        act, na, pas, np_ = g.views()
        out.append(([{k: x[k] for k in ("sent", "draws", "error", "processed", "active")} for x in st],
                    act.tolist(), na.tolist(), pas.tolist(), np_.tolist(), g.draws().tolist(),
                    [sorted(g.idmap(v, w)) for v in range(0, n, 37) for w in (0, 1)], g.inflight()))
        sim.close()
    assert out[0] == out[1]


@pytest.mark.gpu
def test_join_seq_mixed_rounds_one_handle():
    """join_seq calls with rounds 16, then 1, then 0, then 5 on the SAME handle
    (the row buffers are sized once: rounds = 1 needs the most rows)
    equal the plain join + step calls."""
    import partisan_amd as pa
    n = 400
    c = contacts(n)
    plan = [(1, 40, 16), (40, 140, 1), (140, 200, 0), (200, n, 5)]
    out = []
    for seq in (False, True):
        sim = pa.Simulator(seed=SEED)
        g = pa.hyparview.HyParViewCluster(sim, n, shuffle_rounds=4, promotion_rounds=3)
        st = []
        for lo, hi, rounds in plan:
            if seq:
                st += g.join_seq(np.arange(lo, hi, dtype=np.uint32), c[lo:hi], rounds=rounds)
            else:
                for i in range(lo, hi):
                    g.join(i, int(c[i]))
                    if rounds:
                        st += g.step(rounds)
        st += g.step(6)
        act, na, pas, np_ = g.views()
        out.append(([{k: x[k] for k in ("sent", "draws", "error", "processed", "active")} for x in st],
                    act.tolist(), na.tolist(), pas.tolist(), np_.tolist(), g.draws().tolist(), g.inflight()))
        sim.close()
    assert out[0] == out[1]


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
def test_c2_hyparview_overlay_then_plumtree():
    """10k sequential joins (one per round), S = 10
    shuffle periods (100 rounds), then one Plumtree broadcast from vertex 0
    over the resulting active views; every stage equals the oracle's."""
    n = 10000
    sim, g, o = _pair(n)
    c = contacts(n)
    # the device's joins in one call (psim_hv_join_seq: the same schedule as
    # a join + step(1) per vertex), round by round against the oracle's loop
    gs = g.join_seq(np.arange(1, n, dtype=np.uint32), c[1:], rounds=1)
    os_ = []
    for i in range(1, n):
        o.join(i, int(c[i]))
        os_ += o.step(1)
    _same_stats(gs, os_)
    _same_stats(g.step(100), o.step(100))
    _compare(g, o, n, maps=False)
    act, na, _, _ = g.views()
    check_invariants([act[v, :na[v]].tolist() for v in range(n)], n)
    # ... then one Plumtree broadcast from vertex 0 over the active views:
    # per-round counters and the final tree equal the oracle's
    rp, col = g.overlay()
    sim.load_overlay(rp, col)
    pt = O.Plumtree(rp, col, 1)
    assert sim.broadcast(0) == pt.heartbeat(0)
    gst, gr = sim.run()
    ost, orr = pt.run()
    assert gr == orr
    for a, b in zip(gst, ost):
        for k in ("broadcast", "prune", "i_have", "ignored_i_have", "graft"):
            assert a[k] == b[k], (k, a, b)
    assert sim.delivered().all()
    eager, lazy, _, _ = sim.plumtree_state()
    for v in range(0, n, 97):
        oe, ol = pt.peers(v, 0)
        assert sim.mask_to_peers(v, eager[v]) == oe and sim.mask_to_peers(v, lazy[v]) == ol, v
    sim.close()


def _join_waves(n, wave, seed=9):
    """Vertex i joins in round (i-1) // wave, contacting a uniform earlier
    vertex (a simultaneous mass join can leave islands; so can the reference)."""
    rng = np.random.default_rng(seed)
    vs = np.arange(1, n, dtype=np.uint32)
    return [(vs[lo:lo + wave], (rng.random(len(vs[lo:lo + wave])) * vs[lo:lo + wave]).astype(np.uint32))
            for lo in range(0, n - 1, wave)]


@pytest.mark.gpu
def test_join_waves_200k_parity():
    """200k vertices joining in waves of 1000 per round, then 40 rounds:
    views, draws and counters equal the oracle's; the overlay is symmetric
    and connected."""
    n = 200_000
    sim, g, o = _pair(n)
    gs, os_ = [], []
    for vs, cs in _join_waves(n, 1000):
        g.join_many(vs, cs)
        for v, k in zip(vs.tolist(), cs.tolist()):
            o.join(v, k)
        gs += g.step(1)
        os_ += o.step(1)
    gs += g.step(40)
    os_ += o.step(40)
    _same_stats(gs, os_)
    act, na, pas, np_ = g.views()
    dr = g.draws()
    for v in range(n):
        oa, op = o.views(v)
        assert act[v, :na[v]].tolist() == oa and pas[v, :np_[v]].tolist() == op, v
        assert int(dr[v]) == o.draws(v), v
    check_invariants([act[v, :na[v]].tolist() for v in range(n)], n)
    sim.close()


@pytest.mark.gpu
def test_join_waves_2m_properties():
    """2M vertices (oracle-free): symmetric active views, a giant component
    holding >= 99.9% of the vertices (joins this fast can strand a few small
    islands, as the oracle shows at smaller n), queue and id maps in bounds;
    the exported membership CSR matches the views."""
    import partisan_amd as pa
    n = 2_000_000
    sim = pa.Simulator(seed=SEED)
    g = pa.hyparview.HyParViewCluster(sim, n)
    st = []
    for vs, cs in _join_waves(n, 10_000):
        g.join_many(vs, cs)
        st += g.step(1)
    st += g.step(40)
    assert all(s["error"] == 0 for s in st)
    act, na, _, np_ = g.views()
    check_invariants([act[v, :na[v]].tolist() for v in range(n)], n, min_giant=0.999)
    assert na.max() <= 6 and np_.max() <= 30
    rp, col = g.overlay()
    assert int(rp[-1]) == int(na.sum()) - n
    sim.close()
