"""The partisan_membership_strategy behaviour mirror (partisan_amd/membership.py).

CPU: the behaviour's callbacks (src/partisan_membership_strategy.erl:55-77)
with their return shapes, compare/2's {Joiners, Leavers}, and the periodic
interval barrier (partisan_gpu_sim_cluster:periodic/1: the last live node's
call runs the interval) over a stand-in engine.

GPU: a cluster driven only through the strategy callbacks, as the pluggable
manager drives a strategy module, gives the members the oracle restatement
gives for the same joins and intervals (SCAMP v2 and full membership).
"""
import numpy as np
import pytest

import pyoracle as O
from partisan_amd.membership import GpuMembershipCluster, GpuMembershipStrategy, MembershipStrategy

CALLBACKS = ("init", "join", "leave", "periodic", "handle_message", "compare", "prune")


class _Engine:
    """Stand-in for ScampCluster / FullMembershipCluster: records the calls."""

    def __init__(self, n):
        self.n = n
        self.calls = []
        self.mem = {v: [v] for v in range(n)}

    def join(self, v, peer):
        self.calls.append(("join", v, peer))
        self.mem[v] = sorted(set(self.mem[v]) | {peer})

    def leave(self, v, node):
        self.calls.append(("leave", v, node))
        self.mem[v] = [x for x in self.mem[v] if x != node]

    def step(self, rounds):
        self.calls.append(("step", rounds))
        return [{"round": i} for i in range(rounds)]

    def members(self, v):
        return self.mem[v]


def _cluster(n, periodic_rounds=7, live=None):
    c = GpuMembershipCluster.__new__(GpuMembershipCluster)
    c.n, c.strategy, c.periodic_rounds = n, "scamp_v2", periodic_rounds
    c.engine = _Engine(n)
    c.live = n if live is None else live
    c._calls, c.intervals, c.last_stats = 0, 0, []
    return c


def test_behaviour_callbacks():
    for name in CALLBACKS:
        assert callable(getattr(MembershipStrategy, name)), name
        with pytest.raises(NotImplementedError):
            args = {"init": 1, "compare": 2, "prune": 2, "leave": 2, "handle_message": 2, "join": 3,
                    "periodic": 1}[name]
            getattr(MembershipStrategy(), name)(*([None] * args))


def test_return_shapes_and_queueing():
    c = _cluster(4)
    s = GpuMembershipStrategy(c, 2)
    ok, members, st = s.init("actor-2")
    assert ok == "ok" and members == [2] and st == {"vertex": 2, "actor": "actor-2"}
    ok, members, out, st2 = s.join(3, None, st)
    assert (ok, members, out, st2) == ("ok", [2, 3], [], st)
    assert c.engine.calls == [("join", 2, 3)]
    ok, members, out, _ = s.handle_message(("membership", "from-outside"), st)
    assert (ok, members, out) == ("ok", [2, 3], [])
    assert s.compare([1, 2], st) == ([1], [3])
    ok, members, out, _ = s.leave(3, st)
    assert (ok, members, out) == ("ok", [2], [])
    ok, members, _ = s.prune([2], st)
    assert ok == "ok" and members == []


def test_periodic_barrier_runs_one_interval_per_live_round_of_calls():
    c = _cluster(5, periodic_rounds=7, live=3)
    strategies = [GpuMembershipStrategy(c, v) for v in range(5)]
    states = [s.init(v)[2] for v, s in enumerate(strategies)]
    for k in range(2):
        for v in range(3):
            assert c.intervals == k
            strategies[v].periodic(states[v])
    assert c.intervals == 2
    assert [x for x in c.engine.calls if x[0] == "step"] == [("step", 7), ("step", 7)]


def test_unknown_strategy_rejected():
    with pytest.raises(ValueError):
        GpuMembershipCluster(4, strategy="hyparview_as_strategy")


# ------------------------------------------------------------------ GPU
SEED = 0x5EED0003


@pytest.mark.gpu
def test_gpu_scamp_v2_through_strategy_callbacks():
    """Join waves issued as join/3 callbacks, each interval closed by every
    node's periodic/1: the members equal the oracle's partial views."""
    from partisan_amd.overlay import philox_uniform
    n, periodic = 1000, 4
    c = GpuMembershipCluster(n, "scamp_v2", periodic_rounds=periodic, seed=SEED, device=0)
    s = O.Scamp(n, 2, 5, periodic, SEED)
    strat = [c.strategy_for(v) for v in range(n)]
    states = [strat[v].init(("actor", v))[2] for v in range(n)]
    k = 1
    while k < n:
        v = np.arange(k, min(2 * k, n), dtype=np.uint32)
        con = philox_uniform(SEED, v, 0x5CA0, k)
        for a, b in zip(v.tolist(), con.tolist()):
            strat[a].join(b, None, states[a])
            s.join(a, b)
        for u in range(n):
            strat[u].periodic(states[u])
        s.step(periodic)
        k *= 2
    assert c.intervals > 0
    for u in range(0, n, 7):
        ok, members, out, _ = strat[u].handle_message(None, states[u])
        assert ok == "ok" and out == []
        assert members == sorted(set(s.view(u))), u
    c.close()


@pytest.mark.gpu
def test_gpu_full_membership_c1_through_strategy_callbacks():
    """C1's 16-node cluster: every node joins every other through join/3,
    three intervals of periodic/1 barriers; members = the oracle's, all n."""
    n, periodic = 16, 5
    c = GpuMembershipCluster(n, "full", periodic_rounds=periodic, device=0)
    f = O.FullMembership(n, periodic_rounds=periodic)
    strat = [c.strategy_for(v) for v in range(n)]
    states = [strat[v].init(v)[2] for v in range(n)]
    for v in range(n):
        for u in range(n):
            if u != v:
                strat[v].join(u, None, states[v])
                f.join(v, u)
    for _ in range(3):
        for v in range(n):
            strat[v].periodic(states[v])
        f.step(periodic)
    for v in range(n):
        assert c.members(v) == f.members(v) == list(range(n))
    assert strat[0].compare(list(range(n)), states[0]) == ([], [])
    c.close()
