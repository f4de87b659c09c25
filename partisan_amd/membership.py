"""Host mirror of the ``partisan_membership_strategy`` behaviour
(src/partisan_membership_strategy.erl:55-77) over the simulator's device.

The pluggable peer service manager calls a strategy module with
``init/1``, ``join/3``, ``leave/2``, ``periodic/1``, ``handle_message/2``,
``compare/2`` and ``prune/2`` (src/partisan_pluggable_peer_service_manager.erl
:1386-1419 periodic, :1532-1597 join, :1739-1808 handle_message, :2059-2109
leave).  ``MembershipStrategy`` is that behaviour with the same callback
names and return shapes; ``GpuMembershipStrategy`` implements it for one node
of a simulated cluster (``GpuMembershipCluster``) whose SCAMP v1/v2 or full
membership runs on the GPU (``ScampCluster`` / ``FullMembershipCluster``,
parity-checked against the oracle restatements).  It is the Python twin of
``erl/src/partisan_gpu_sim_membership_strategy.erl`` over
``partisan_gpu_sim_cluster.erl``:

* the simulated nodes' membership messages travel on the device, so every
  callback returns no outgoing messages (``[]``) and the members are read
  back from the device;
* a join / leave is queued on the device and handled by the next round;
* ``periodic/1`` is a barrier: when every live node of the cluster has called
  it for the interval, the last call runs the interval (``periodic_rounds``
  device rounds, which contain each node's own periodic timer).

Members are node ids (ints) in term order (node names are
zero-padded, so term order is id order).
"""
from .fullmem import FullMembershipCluster
from .scamp import ScampCluster
from .sim import Simulator


class MembershipStrategy:
    """partisan_membership_strategy behaviour (:55-77).

    init(identity)                     -> ("ok", members, state)
    join(node, peer_state, state)      -> ("ok", members, outgoing, state)
    leave(node, state)                 -> ("ok", members, outgoing, state)
    periodic(state)                    -> ("ok", members, outgoing, state)
    handle_message(message, state)     -> ("ok", members, outgoing, state)
    compare(members, state)            -> (joiners, leavers)
    prune(nodes, state)                -> ("ok", members, state)
    """

    def init(self, identity):
        raise NotImplementedError

    def join(self, node, peer_state, state):
        raise NotImplementedError

    def leave(self, node, state):
        raise NotImplementedError

    def periodic(self, state):
        raise NotImplementedError

    def handle_message(self, message, state):
        raise NotImplementedError

    def compare(self, members, state):
        raise NotImplementedError

    def prune(self, nodes, state):
        raise NotImplementedError


STRATEGIES = ("scamp_v2", "scamp_v1", "full")


class GpuMembershipCluster:
    """One simulated cluster of n nodes (partisan_gpu_sim_cluster.erl).

    strategy: "scamp_v2" | "scamp_v1" | "full"; periodic_rounds: device rounds
    per periodic interval (each node's periodic/1 timer fires inside them)."""

    def __init__(self, n, strategy="scamp_v2", periodic_rounds=10, seed=0, device=0, scamp_c=5,
                 max_tokens=None, live=None):
        if strategy not in STRATEGIES:
            raise ValueError(f"strategy {strategy!r}: one of {STRATEGIES}")
        self.n, self.strategy, self.periodic_rounds = n, strategy, periodic_rounds
        self.sim = Simulator(seed=seed, device=device)
        if strategy == "full":
            self.engine = FullMembershipCluster(self.sim, n, periodic_rounds=periodic_rounds,
                                                max_tokens=max_tokens if max_tokens is not None else 2 * n)
        else:
            self.engine = ScampCluster(self.sim, n, version=1 if strategy == "scamp_v1" else 2, c=scamp_c,
                                       periodic_rounds=periodic_rounds)
        self.live = n if live is None else live   # nodes whose periodic/1 closes an interval
        self._calls = 0
        self.intervals = 0
        self.last_stats = []

    # -- queued on the device (handled by the next round) --------------------
    def join(self, v, peer):
        self.engine.join(v, peer)

    def leave(self, v, node):
        self.engine.leave(v, node)

    # -- the interval barrier (partisan_gpu_sim_cluster:periodic/1) ----------
    def periodic(self, v):
        del v
        self._calls += 1
        if self._calls >= self.live:
            self._calls = 0
            self.run_interval()

    def run_interval(self):
        self.last_stats = self.engine.step(self.periodic_rounds)
        self.intervals += 1
        return self.last_stats

    def members(self, v):
        """The members node v's strategy holds, sorted (term order)."""
        return sorted(set(self.engine.members(v)))

    def strategy_for(self, v):
        return GpuMembershipStrategy(self, v)

    def close(self):
        self.sim.close()


class GpuMembershipStrategy(MembershipStrategy):
    """partisan_membership_strategy for node `vertex` of a GpuMembershipCluster
    (erl/src/partisan_gpu_sim_membership_strategy.erl).  The state is
    ``{"vertex": v, "actor": identity}``."""

    def __init__(self, cluster, vertex):
        self.cluster, self.vertex = cluster, vertex

    def _members(self, state):
        return self.cluster.members(state["vertex"])

    # init/1 (scamp_v2 :75-85, full :70-74)
    def init(self, identity):
        state = {"vertex": self.vertex, "actor": identity}
        return "ok", self._members(state), state

    # {connected, Node, ...} -> join/3 (pluggable :1532-1597)
    def join(self, node, peer_state, state):
        del peer_state
        self.cluster.join(state["vertex"], int(node))
        return "ok", self._members(state), [], state

    # internal_leave (pluggable :2059-2109) -> leave/2
    def leave(self, node, state):
        self.cluster.leave(state["vertex"], int(node))
        return "ok", self._members(state), [], state

    # handle_info(periodic) (pluggable :1386-1419)
    def periodic(self, state):
        self.cluster.periodic(state["vertex"])
        return "ok", self._members(state), [], state

    # {membership_strategy, Msg} (pluggable :1739-1808): the simulated nodes'
    # messages are delivered on the device; one from outside the simulation
    # leaves the state unchanged
    def handle_message(self, message, state):
        del message
        return "ok", self._members(state), [], state

    # {Joiners, Leavers}: the given members that are not ours, ours that are not given
    def compare(self, members, state):
        cur = self._members(state)
        given = [int(m) for m in members]
        return [m for m in given if m not in cur], [m for m in cur if m not in given]

    def prune(self, nodes, state):
        for x in nodes:
            self.cluster.leave(state["vertex"], int(x))
        return "ok", self._members(state), state
