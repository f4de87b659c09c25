"""Demers rumor mongering + anti-entropy: HIP path (csrc/demers.hip) vs the
oracle (oracle/demers.c), round by round, bit-exact (every vertex's store and
the message counters).  Trajectories are parity unpinned by reference
vectors; the convergence postcondition of
test/prop_partisan_reliable_broadcast.erl:127-172 is checked too.
Also: the Philox4x32-10 restatement against the Random123 known answers."""
import numpy as np
import pytest

import pyoracle as O

KEYS = ("rm_sent", "push_sent", "pull_sent", "delivered_new", "complete")


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32 R=10
    assert O.philox([0, 0, 0, 0], [0, 0]) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    f = 0xFFFFFFFF
    assert O.philox([f, f, f, f], [f, f]) == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert O.philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0]) == \
        [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


@pytest.mark.parametrize("n", [7, 5000])
def test_select2_is_uniform_pair(n):
    """Faithful (n <= 1024: the two smallest of n sort keys) and scaled (2 draws)
    select_random_sublist(.., 2): a uniform ordered pair of distinct members,
    each call at its own draw index of the process's stream."""
    dpc = O.draws_per_call(n)
    assert dpc == (n if n <= 1024 else 2)
    bins = n if n == 7 else 10
    ha, hb = np.zeros(bins), np.zeros(bins)
    for call in range(20000):
        a, b = O.select2(123, 5, 2, n, call * dpc)
        assert a != b and 0 <= a < n and 0 <= b < n
        ha[a * bins // n] += 1
        hb[b * bins // n] += 1
    for h in (ha, hb):
        assert h.min() > 0.8 * h.mean() and h.max() < 1.2 * h.mean()


def test_select2_faithful_is_the_sorted_shuffle():
    """shuffle/1 (demers_rumor_mongering.erl:185-186): sort {uniform(), N};
    the first two = the members with the two smallest 53-bit keys."""
    n, j = 300, 1234
    keys = []
    for i in range(n):
        r = O.philox([5, (j + i) & 0xFFFFFFFF, 2, (j + i) >> 32], [123 & 0xFFFFFFFF, 0])
        keys.append(((r[0] | (r[1] << 32)) >> 11, i))
    keys.sort()
    assert O.select2(123, 5, 2, n, j) == [keys[0][1], keys[1][1]]


@pytest.mark.parametrize("rm,ae", [(True, 2), (True, 0), (False, 2), (True, 3), ("direct_mail", 0)])
def test_oracle_modes_converge_or_residue(rm, ae):
    d = O.Demers(3000, 64, 0x5EED0004, ae_period=ae, rm_on=rm)
    d.broadcast_all()
    st, r = d.run(300)
    if rm == "direct_mail":                         # one hop to every member
        assert r == 1 and st[0]["complete"] == 3000 and st[0]["rm_sent"] == 0
        assert st[0]["delivered_new"] == 64 * 2999      # each rumor reaches the n - 1 others
    elif ae:
        assert st[-1]["complete"] == 3000          # anti-entropy guarantees delivery
    else:
        assert r == 300 and st[-1]["complete"] < 3000   # rumor mongering leaves a residue


def lockstep(pa, n, m, seed, ae, rm, max_rounds=200):
    sim = pa.Simulator(seed=seed)
    dm = pa.demers.DemersEpidemic(sim, n, m, ae, rm)
    orc = O.Demers(n, m, seed, ae_period=ae, rm_on=rm)
    assert dm.origins().tolist() == orc.origins()
    dm.broadcast()
    orc.broadcast_all()
    assert np.array_equal(dm.seen(), orc.seen())
    for r in range(max_rounds):
        g = dm.step(1)[0]
        o = orc.step(1)[0]
        for k in KEYS:
            assert g[k] == o[k], (r, k, g, o)
        assert np.array_equal(dm.seen(), orc.seen()), r
        if o["complete"] == n:
            break
    sim.close()
    return r


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,ae,rm,seed", [
    (500, 64, 2, True, 1), (3000, 64, 2, True, 2), (2000, 17, 3, True, 3),
    (1500, 64, 2, False, 4), (800, 64, 0, True, 5), (20000, 64, 2, True, 0x5EED0004),
    (3000, 64, 0, "direct_mail", 6), (2500, 64, 2, "direct_mail", 7)])
def test_lockstep(n, m, ae, rm, seed):
    import partisan_amd as pa
    lockstep(pa, n, m, seed, ae, rm, max_rounds=60 if ae == 0 else 200)


@pytest.mark.gpu
def test_run_matches_oracle_and_converges():
    import partisan_amd as pa
    n = 200_000
    sim = pa.Simulator(seed=0x5EED0004)
    dm = pa.demers.DemersEpidemic(sim, n, 64, 2, True)
    orc = O.Demers(n, 64, 0x5EED0004, ae_period=2, rm_on=True)
    dm.broadcast()
    orc.broadcast_all()
    gst, gr = dm.run()
    ost, orr = orc.run()
    assert gr == orr
    assert [tuple(g[k] for k in KEYS) for g in gst] == [tuple(o[k] for k in KEYS) for o in ost]
    assert np.array_equal(dm.seen(), orc.seen())
    assert gst[-1]["complete"] == n


@pytest.mark.gpu
def test_large_converges():
    """C4 scale property: 4M peers, 64 rumors -> every vertex stores all."""
    import partisan_amd as pa
    n = 4_000_000
    sim = pa.Simulator(seed=0x5EED0004)
    dm = pa.demers.DemersEpidemic(sim, n, 64, 2, True)
    dm.broadcast()
    st, r = dm.run(200)
    assert st[-1]["complete"] == n
    seen = dm.seen()
    assert (seen == np.uint64(0xFFFFFFFFFFFFFFFF)).all()
    assert sum(s["delivered_new"] for s in st) == n * 64 - 64   # each rumor starts at its origin
