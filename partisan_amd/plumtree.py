"""Host mirror of Partisan's Plumtree API over the simulator.

Mirrors the reference's operator/plugin interface for the hot path:

* ``PlumtreeBroadcastHandler`` -- the ``partisan_plumtree_broadcast_handler``
  behaviour (src/partisan_plumtree_broadcast_handler.erl:47-78): callbacks
  broadcast_data/1, merge/2, is_stale/1, graft/1, exchange/1 and the optional
  broadcast_channel/0.
* ``PlumtreeBackend`` -- the default handler, partisan_plumtree_backend
  (heartbeats; src/partisan_plumtree_backend.erl:180-417).  Its callbacks are
  executed by the HIP round kernel on device; the Python class carries the
  same names and returns the same shapes for host-side calls.
* ``PlumtreeBroadcast`` -- the partisan_plumtree_broadcast server API
  (src/partisan_plumtree_broadcast.erl:234-476): broadcast/2, update/1,
  get_peers/1, get_eager_peers/1, get_lazy_peers/1, broadcast_members/0,
  exchanges/0, cancel_exchanges/1, broadcast_channel/1 -- addressed per
  simulated node.

Only handlers whose callbacks the device implements can drive the device
path; registering any other module raises (no silent CPU fallback).
"""
import numpy as np

from .sim import Simulator

MEMBERSHIP_CHANNEL = "partisan_membership"   # include/partisan.hrl:120


class PlumtreeBroadcastHandler:
    """partisan_plumtree_broadcast_handler behaviour (:47-78)."""

    def broadcast_data(self, broadcast):                 # -> (MessageId, Payload)
        raise NotImplementedError

    def broadcast_channel(self):                         # optional callback
        return None

    def merge(self, message_id, payload):                # -> bool
        raise NotImplementedError

    def is_stale(self, message_id):                      # -> bool
        raise NotImplementedError

    def graft(self, message_id):                         # -> "stale" | ("ok", M) | ("error", R)
        raise NotImplementedError

    def exchange(self, peer):                            # -> ("ok", pid) | ("error", R) | "ignore"
        raise NotImplementedError


class PlumtreeBackend(PlumtreeBroadcastHandler):
    """partisan_plumtree_backend: heartbeat ids {Node, Epoch, Monotonic}.

    Bound to one simulated node of a PlumtreeBroadcast; merge/is_stale/graft
    query the device state of that node for the current heartbeat.
    """

    device_native = True

    def __init__(self, cluster=None, node=None):
        self.cluster = cluster
        self.node = node

    def broadcast_channel(self):                          # backend :180-181
        return MEMBERSHIP_CHANNEL

    def broadcast_data(self, broadcast):                  # backend :192-195
        ts = broadcast["timestamp"]
        return ts, ts

    def is_stale(self, message_id):                       # backend :229-244
        """Monotonic in this node's interval set for the origin: the latest
        heartbeat's delivery is read from the device, an earlier one's from the
        delivered set recorded when the origin heartbeated again (a heartbeat
        runs to quiescence before its origin's next one: PSIM_EBUSY)."""
        origin, _epoch, mono = message_id
        c = self.cluster
        cur = c.ids.get(origin)
        if cur is None or mono > cur[2]:
            return False
        if mono == cur[2]:
            if origin in c._state:                # this round's state is cached: no device call
                return bool(c._delivered(origin)[self.node])
            c.sim.focus(origin)                   # one vertex: psim_get_delivered_range, O(1)
            return c.sim.delivered_at(self.node)
        past = c._hist.get(origin, {}).get(mono)   # recorded when the origin heartbeated again
        return bool(past is not None and past[self.node])

    def merge(self, message_id, payload):                 # backend :205-215 (read-only view)
        return not self.is_stale(message_id)

    def graft(self, message_id):                          # backend :254-280
        if self.is_stale(message_id):
            return ("ok", message_id)
        return ("error", ("not_found", message_id))

    def exchange(self, peer):                             # backend :292-293
        return "ignore"


class PlumtreeBroadcast:
    """The Plumtree servers of every node of a simulated cluster."""

    def __init__(self, row_ptr, col, mods=None, lazy_tick_rounds=1, exchange_tick_rounds=10, device=-1):
        mods = list(mods) if mods is not None else [PlumtreeBackend]
        for m in mods:
            if not getattr(m, "device_native", False):
                raise NotImplementedError(
                    f"handler {getattr(m, '__name__', m)!r} has no device implementation; "
                    "only partisan_plumtree_backend (heartbeats) runs on the GPU path")
        self.sim = Simulator(lazy_tick_rounds=lazy_tick_rounds, exchange_tick_rounds=exchange_tick_rounds,
                             device=device)
        self.sim.load_overlay(row_ptr, col)
        self.members_row_ptr = np.asarray(row_ptr, dtype=np.uint64)
        self.members_col = np.asarray(col, dtype=np.uint32)
        self.mods = mods
        self.current_id = None            # {Node, Epoch, Monotonic} of the latest heartbeat
        self.ids = {}                     # origin -> its latest heartbeat id
        self._hist = {}                   # origin -> {Monotonic: delivered set} of its earlier heartbeats
        self._state = {}                  # root -> device state of its lane (cached until the next round)
        # roots whose per-root sets the device keeps: every root on one GPU
        # (heartbeat lanes); only the latest on a binned / sharded handle
        self._one_lane = bool(getattr(self.sim, "binned", False)) or self.sim.world > 1

    # -- partisan_plumtree_broadcast API ------------------------------------
    def broadcast(self, node, mod=PlumtreeBackend):
        """Heartbeat at `node` (backend handle_info(heartbeat) :341-368 ->
        broadcast/2 :324-326).  Returns the message id."""
        prev = self.ids.get(node)
        if prev is not None:
            self._hist.setdefault(node, {})[prev[2]] = self._delivered(node).astype(bool)
        mono = self.sim.broadcast(node)
        if self._one_lane:
            self.ids = {r: i for r, i in self.ids.items() if r == node}
        self.current_id = (node, 0, mono)
        self.ids[node] = self.current_id
        self._state = {}
        return self.current_id

    def run(self, max_rounds=100000):
        stats, rounds = self.sim.run(max_rounds)
        self._state = {}
        return stats, rounds

    def step(self, rounds=1):
        st = self.sim.step(rounds)
        self._state = {}
        return st

    def update(self, members_added=True):
        """Membership update with new members at every node: reset_peers/4
        drops per-root sets (:607-639, :1320-1328)."""
        if members_added:
            self.sim.reset_trees()
        self._state = {}

    def _st(self, root):
        if root not in self._state:
            self.sim.focus(root)
            self._state[root] = (self.sim.plumtree_state(), self.sim.delivered())
        return self._state[root]

    def _delivered(self, root):
        return self._st(root)[1]

    def get_peers(self, node, root):                       # :516-536
        """all_peers(Root, eager_sets, common_eagers) / (.., lazy_sets, common_lazys)
        (:1278-1282): the root's map entries when the device holds a tree for
        that root, else the common sets (members minus self, and [])."""
        if root not in self.ids:
            return [p for p in self.broadcast_members(node) if p != node], []
        (eager, lazy, _, _), _ = self._st(root)
        return self.sim.mask_to_peers(node, eager[node]), self.sim.mask_to_peers(node, lazy[node])

    def get_eager_peers(self, node, root):                 # :538-542
        return self.get_peers(node, root)[0]

    def get_lazy_peers(self, node, root):                  # :544-548
        return self.get_peers(node, root)[1]

    def broadcast_members(self, node):                     # :550-551 (all_members incl. self)
        lo, hi = int(self.members_row_ptr[node]), int(self.members_row_ptr[node + 1])
        return sorted(set(self.members_col[lo:hi].tolist()) | {node})

    def exchanges(self, node):                             # :553-554: backend exchange/1 -> ignore
        return []

    def cancel_exchanges(self, node, which):               # :556-558
        return []

    def broadcast_channel(self, mod=PlumtreeBackend):      # :340-346
        return mod().broadcast_channel() or None

    def handler(self, node):
        return PlumtreeBackend(self, node)

    def close(self):
        self.sim.close()
