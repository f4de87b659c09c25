"""SCAMP membership (src/partisan_scamp_v2_membership_strategy.erl and
src/partisan_scamp_v1_membership_strategy.erl) on the simulator's device.

Host mirror of the pluggable peer service manager driving the
`partisan_membership_strategy` behaviour (src/partisan_membership_strategy.erl
:55-77) with a SCAMP strategy, for n nodes at once:

  * ``join(v, contact)``  -- partisan_peer_service:join at v -> {connected, ...}
                             -> Strategy:join/3 (pluggable :1532-1597)
  * ``leave(v, node)``    -- partisan_peer_service:leave -> Strategy:leave/2
  * ``crash(v)``          -- the node's BEAM dies and restarts (init/1 state)
  * ``step(rounds)``      -- handle_message/2 deliveries (:1739-1808) and the
                             periodic/1 timer (:1386-1419)
  * ``views()``           -- each node's partial view (its `members`) and in-view
  * ``messages()`` / ``take(v)`` / ``put(msgs)`` -- the membership messages on
                             the wire, {membership_strategy, Msg} in the
                             strategy's term shapes (pluggable :1396-1407, :1739-1808)
"""
import ctypes as C

import numpy as np

from ._lib import ScampMsg, ScampStats, check, lib

_P = C.POINTER
PV_CAP = 128
IV_CAP = 64


class ScampCluster:
    def __init__(self, sim, n, version=2, c=5, periodic_rounds=10):
        self.sim, self.n, self.version = sim, n, version
        check(lib().psim_scamp_setup(sim._h, n, version, c, periodic_rounds), sim._h)

    def _c(self, rc):
        return check(rc, self.sim._h)

    @staticmethod
    def _u32(x):
        a = np.ascontiguousarray(np.atleast_1d(x), dtype=np.uint32)
        return a, a.ctypes.data_as(_P(C.c_uint32))

    def join(self, v, contact):
        a, pa = self._u32(v)
        b, pb = self._u32(contact)
        self._c(lib().psim_scamp_join(self.sim._h, pa, pb, len(a)))

    def leave(self, v, node):
        a, pa = self._u32(v)
        b, pb = self._u32(node)
        self._c(lib().psim_scamp_leave(self.sim._h, pa, pb, len(a)))

    def crash(self, v):
        a, pa = self._u32(v)
        self._c(lib().psim_scamp_crash(self.sim._h, pa, len(a)))

    def set_alive(self, alive):
        a = np.ascontiguousarray(alive, dtype=np.uint8)
        self._c(lib().psim_scamp_set_alive(self.sim._h, a.ctypes.data_as(_P(C.c_uint8)), len(a)))

    def step(self, rounds=1):
        st = (ScampStats * rounds)()
        self._c(lib().psim_scamp_step(self.sim._h, rounds, st, rounds))
        return [s.as_dict() for s in st]

    def views(self):
        """(pv[n, PV_CAP], npv[n], iv[n, IV_CAP], niv[n]) in the reference's list order."""
        pv = np.zeros((self.n, PV_CAP), np.uint32)
        iv = np.zeros((self.n, IV_CAP), np.uint32)
        npv = np.zeros(self.n, np.uint32)
        niv = np.zeros(self.n, np.uint32)
        self._c(lib().psim_scamp_get_views(self.sim._h, pv.ctypes.data_as(_P(C.c_uint32)),
                                           npv.ctypes.data_as(_P(C.c_uint32)), iv.ctypes.data_as(_P(C.c_uint32)),
                                           niv.ctypes.data_as(_P(C.c_uint32)), self.n))
        return pv, npv, iv, niv

    def members(self, v):
        pv, npv, _, _ = self.views()
        return [int(x) for x in pv[v, :npv[v]]]

    def nodes(self):
        """(draws[n], last_ping[n], alive[n])"""
        d = np.zeros(self.n, np.uint64)
        lp = np.zeros(self.n, np.int32)
        al = np.zeros(self.n, np.uint8)
        self._c(lib().psim_scamp_get_nodes(self.sim._h, d.ctypes.data_as(_P(C.c_uint64)),
                                           lp.ctypes.data_as(_P(C.c_int32)), al.ctypes.data_as(_P(C.c_uint8)),
                                           self.n))
        return d, lp, al

    def inflight(self):
        x = C.c_uint64()
        self._c(lib().psim_scamp_inflight(self.sim._h, C.byref(x)))
        return x.value

    # ---- the wire -------------------------------------
    KINDS = {1: "forward_subscription", 2: "keep_subscription", 3: "ping", 4: "remove_subscription",
             5: "replace_subscription", 6: "bootstrap_remove_subscription"}

    @staticmethod
    def term(m):
        """(src, dst, seq, ('membership_strategy', Msg)) with Msg the reference's
        tuple, e.g. ('forward_subscription', A) or ('replace_subscription', A, B)."""
        t, src, dst, seq, a, b = m
        body = (ScampCluster.KINDS[t], a, b) if t == 5 else (ScampCluster.KINDS[t], a)
        return (src, dst, seq, ("membership_strategy", body))

    @staticmethod
    def parse(term):
        src, dst, seq, (tag, body) = term
        if tag != "membership_strategy":
            raise ValueError(term)
        kind = {v: k for k, v in ScampCluster.KINDS.items()}[body[0]]
        return (kind, src, dst, seq, body[1], body[2] if kind == 5 else 0)

    def messages(self):
        """The messages the next round delivers as (type, src, dst, seq, a, b), handling order."""
        k = C.c_size_t()
        self._c(lib().psim_scamp_messages(self.sim._h, None, 0, C.byref(k)))
        buf = (ScampMsg * max(1, k.value))()
        self._c(lib().psim_scamp_messages(self.sim._h, buf, k.value, C.byref(k)))
        return [(m.type, m.src, m.dst, m.seq, m.a, m.b) for m in buf[:k.value]]

    def take(self, v):
        """Takes vertex v's messages off the wire (the next round will not deliver them)."""
        cap = max(1, len(self.messages()))
        buf = (ScampMsg * cap)()
        k = C.c_size_t()
        self._c(lib().psim_scamp_take(self.sim._h, v, buf, cap, C.byref(k)))
        return [(m.type, m.src, m.dst, m.seq, m.a, m.b) for m in buf[:k.value]]

    def put(self, msgs):
        """Puts (type, src, dst, seq, a, b) messages on the wire for the next round."""
        buf = (ScampMsg * max(1, len(msgs)))(*[ScampMsg(*m) for m in msgs])
        self._c(lib().psim_scamp_put(self.sim._h, buf, len(msgs)))


def join_waves(n, seed):
    """C3 overlay construction: vertices [k, 2k) join a contact drawn uniformly
    from [0, k) (Philox workload stream), k = 1, 2, 4, ...; returns a list of
    (joiners, contacts) batches, one per wave."""
    from .overlay import philox_uniform
    waves, k = [], 1
    while k < n:
        v = np.arange(k, min(2 * k, n), dtype=np.uint32)
        c = philox_uniform(seed, v, 0x5CA0, k)
        waves.append((v, c))
        k *= 2
    return waves


def churn_batch(n, seed, rnd, frac=0.05):
    """C3 churn of round `rnd`: ~frac*n distinct vertices crash and rejoin a
    contact drawn uniformly among the other vertices (Philox workload stream)."""
    from .overlay import philox_uniform
    k = max(1, int(n * frac))
    cand = philox_uniform(seed, np.arange(k, dtype=np.uint32) + np.uint32((rnd * 7919) & 0xFFFFFFFF), 0xC4A5, n)
    v = np.unique(cand).astype(np.uint32)
    c = philox_uniform(seed, v, 0xC0A0 + (rnd & 0xFFF), n - 1)
    c = np.where(c >= v, c + 1, c).astype(np.uint32)
    return v, c
