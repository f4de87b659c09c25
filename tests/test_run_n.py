"""psim_plumtree_broadcast_run_n: `count` heartbeat intervals in one call must
equal psim_plumtree_reset_trees + psim_plumtree_broadcast_run in a loop --
the same per-round counts of every interval, rounds, heartbeat ids and final
state -- including intervals that run past one chunk of rounds (ring
lattice), lazy ticks every 2-3 rounds, dead vertices (rows that wait on a
dead peer) and heartbeats over the pruned tree (no reset).  The loop itself
is the path the oracle lockstep tests pin (tests/test_plumtree_gpu.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIELDS = ("sent", "delivered_new", "active", "senders", "sender_degree_sum", "outstanding_vertices", "algo_bytes",
          "words_stored")


def _pair(overlay, L, alive=None):
    import partisan_amd as pa
    rp, col = overlay
    sims = []
    for _ in range(2):
        s = pa.Simulator(lazy_tick_rounds=L, chunk_timing=True)
        s.load_overlay(rp, col)
        if alive is not None:
            s.set_alive(alive)
        sims.append(s)
    return sims


def _loop(sim, root, count, reset):
    monos, rows, rounds = [], [], []
    for _ in range(count):
        if reset:
            sim.reset_trees()
        m, st, r = sim.broadcast_run(root, as_dicts=False)
        monos.append(m)
        rows.append(st)
        rounds.append(r)
    return np.array(monos, np.uint32), np.concatenate(rows), np.array(rounds, np.uint32)


def _check(overlay, root, count, reset, L=1, alive=None, warm=0):
    a, b = _pair(overlay, L, alive)
    for s in (a, b):
        for _ in range(warm):
            s.broadcast_run(root, as_dicts=False)
    m1, s1, r1 = _loop(a, root, count, reset)
    m2, s2, r2 = b.broadcast_run_n(root, count, reset_trees=reset, cap=4096 * count)
    assert r1.tolist() == r2.tolist()
    assert m1.tolist() == m2.tolist()
    assert len(s1) == len(s2) == int(r1.sum())
    for f in FIELDS:
        assert np.array_equal(s1[f], s2[f]), f
    for x, y in zip(a.plumtree_state(), b.plumtree_state()):
        assert np.array_equal(x, y)
    assert np.array_equal(a.delivered(), b.delivered())
    a.close()
    b.close()
    return r1


@pytest.mark.parametrize("reset", [True, False])
def test_run_n_random_overlay(reset):
    import partisan_amd as pa
    r = _check(pa.overlay.random_regular(200_000, 5, 3), 0, 6, reset)
    assert (r > 0).all()


@pytest.mark.parametrize("L,reset", [(2, True), (3, True), (3, False)])
def test_run_n_lazy_ticks(L, reset):
    """The tick phase moves from interval to interval, so interval lengths
    differ by a round or two: the pipelined prediction misses both ways
    (the abandoned interval is undone, the short one finished by the plain
    driver)."""
    import partisan_amd as pa
    _check(pa.overlay.random_regular(50_000, 5, 4), 7, 6, reset, L=L, warm=1)


def test_run_n_long_floods_past_a_chunk():
    import partisan_amd as pa
    r = _check(pa.overlay.ring_lattice(3000, 2), 0, 3, True, L=2)
    assert (r > 16).all()          # every interval ran several chunks


def test_run_n_dead_vertices():
    import partisan_amd as pa
    n = 20_000
    alive = np.ones(n, np.uint8)
    alive[np.random.default_rng(5).choice(n, n // 10, replace=False)] = 0
    alive[11] = 1
    _check(pa.overlay.random_regular(n, 5, 6), 11, 4, True, alive=alive)
    _check(pa.overlay.random_regular(n, 5, 6), 11, 4, False, alive=alive)
