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
from ._lib import PsimError

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
        """{Origin, Epoch, Monotonic} against this node's table row for the
        origin: same epoch -> Monotonic in the row's interval set; otherwise
        stale iff the row holds a newer epoch.  A heartbeat lane that keeps
        every id (window lane) answers for any id on device; a static lane
        holds the newest id only, and earlier ones are read from the delivered
        set recorded when the origin heartbeated again (the lane was static,
        so that heartbeat had finished)."""
        return self._row_has(message_id)[0]

    def merge(self, message_id, payload):                 # backend :205-215 (read-only view)
        return not self.is_stale(message_id)

    def graft(self, message_id):                          # backend :254-280
        stale, newer = self._row_has(message_id, want_epoch=True)
        if not stale:
            return ("error", ("not_found", message_id))
        return "stale" if newer else ("ok", message_id)

    def _row_has(self, message_id, want_epoch=False):
        """(is_stale(id), the row holds a newer epoch than id's)."""
        origin, epoch, mono = message_id
        c = self.cluster
        cur = c.ids.get(origin)
        if cur is None:
            return False, False
        pid = (epoch << 24) | mono
        cid = (cur[1] << 24) | cur[2]
        if pid > cid:                                     # not started yet: no row holds it
            return False, False
        if pid == cid:                            # the newest id: no row holds a newer epoch
            if origin in c._state:                # this round's state is cached: no device call
                return bool(c._delivered(origin)[self.node]), False
            c.sim.focus(origin)                   # one vertex: psim_get_delivered_range, O(1)
            return c.sim.delivered_at(self.node), False
        c.sim.focus(origin)
        try:                                      # a window lane's table rows answer any id
            st = c.sim.delivered_at(self.node, pid)
            # Monotonic 2^24-1 is never an id: stale for it <=> the row's epoch is newer
            newer = want_epoch and st and c.sim.delivered_at(self.node, (epoch << 24) | 0xFFFFFF)
            return st, bool(newer)
        except PsimError:                         # a static lane: the newest id only
            pass
        return c._row_from_history(self.node, origin, pid)

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
        self._hist = {}                   # origin -> [(seq, id, delivered set)] of its earlier heartbeats
        self._seq = 0                     # heartbeats started
        self._restart = {}                # node -> heartbeats started before its backend last restarted
        self._latest_seq = {}             # origin -> seq of its newest heartbeat
        self._state = {}                  # root -> device state of its lane (cached until the next round)
        # roots whose per-root sets the device keeps: every root on one GPU
        # (heartbeat lanes); only the latest on a binned / sharded handle
        self._one_lane = bool(getattr(self.sim, "binned", False)) or self.sim.world > 1

    # -- partisan_plumtree_broadcast API ------------------------------------
    def broadcast(self, node, mod=PlumtreeBackend):
        """Heartbeat at `node` (backend handle_info(heartbeat) :341-368 ->
        broadcast/2 :324-326).  Returns the message id."""
        self._snapshot(node)
        pid = self.sim.broadcast(node)
        if self._one_lane:
            self.ids = {r: i for r, i in self.ids.items() if r == node}
        self._seq += 1
        self.current_id = (node, pid >> 24, pid & 0xFFFFFF)
        self.ids[node] = self.current_id
        self._latest_seq[node] = self._seq
        self._state = {}
        return self.current_id

    def restart_backend(self, node):
        """`node`'s heartbeat backend crashes and its supervisor starts it again
        (backend init/1 :316-329): a newer epoch, Monotonic 0 and an empty
        timestamp table (psim_plumtree_restart_backend).  The broadcast
        server's state (trees, outstanding i_haves) is kept."""
        for origin in list(self.ids):
            self._snapshot(origin, keep_latest=True)
        self.sim.restart_backend(node)
        self._restart[node] = self._seq
        self._state = {}

    def _snapshot(self, origin, keep_latest=False):
        """Record the delivered set of origin's newest heartbeat (its lane may
        be static, keeping the newest id only)."""
        prev = self.ids.get(origin)
        if prev is None:
            return
        d = self._delivered(origin).astype(bool)
        h = self._hist.setdefault(origin, [])
        s = self._latest_seq[origin]
        h[:] = [x for x in h if x[0] != s]
        h.append((s, (prev[1] << 24) | prev[2], d))

    def _row_from_history(self, node, origin, pid):
        """is_stale / newer-epoch from the recorded sets: node's row holds the
        ids it delivered since its backend last restarted, of the newest
        epoch among them (add_timestamp/1 :400-417)."""
        since = self._restart.get(node, 0)
        got = [(s, i) for s, i, d in self._hist.get(origin, []) if s > since and d[node]]
        ls = self._latest_seq.get(origin)
        if ls is not None and ls > since and not any(s == ls for s, _ in got):
            self.sim.focus(origin)
            if self.sim.delivered_at(node):
                cur = self.ids[origin]
                got.append((ls, (cur[1] << 24) | cur[2]))
        if not got:
            return False, False
        e = max(got)[1] >> 24
        if e == pid >> 24:
            return any(i == pid for _, i in got), False
        return e > pid >> 24, e > pid >> 24

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
