"""Causal delivery (src/partisan_causality_backend.erl) on the simulator's
device: m <= 64 emitters broadcasting causal messages (emit/4 to every other
vertex) that land after Philox-drawn delays; every vertex runs
receive_message/2 per arrival and the redelivery timer (see include/psim.h).

Host mirror of the backend's observable state: ``clock(v)`` (local_clock as
(actor, counter) pairs), ``buffered(v)`` (buffered_messages as
(emitter index, emission round)), ``delivered()`` counts.
"""
import ctypes as C

import numpy as np

from ._lib import CausalStats, check, lib

_u32p = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint32))  # noqa: E731


class CausalCluster:
    def __init__(self, sim, n, m=64, period=1, dmax=4, redeliver=1):
        self.sim, self.n, self.m = sim, n, m
        check(lib().psim_causal_setup(sim._h, n, m, period, dmax, redeliver), sim._h)
        self.emitters = np.zeros(m, np.uint32)
        self._c(lib().psim_causal_emitters(sim._h, _u32p(self.emitters), m))

    def _c(self, rc):
        return check(rc, self.sim._h)

    def step(self, rounds=1):
        st = (CausalStats * max(1, rounds))()
        self._c(lib().psim_causal_step(self.sim._h, rounds, st, rounds))
        return [s.as_dict() for s in st[:rounds]]

    def clocks(self):
        """(lanes[n, 64], self[n]) dense clocks."""
        lanes = np.zeros((self.n, 64), np.uint32)
        slf = np.zeros(self.n, np.uint32)
        self._c(lib().psim_causal_get_clocks(self.sim._h, _u32p(lanes), _u32p(slf), self.n))
        return lanes, slf

    def clock(self, v, lanes=None, slf=None):
        """local_clock of v as sorted (actor, counter) pairs."""
        if lanes is None:
            lanes, slf = self.clocks()
        out = [(int(self.emitters[k]), int(lanes[v, k])) for k in range(self.m) if lanes[v, k]]
        if slf[v]:
            out.append((v, int(slf[v])))
        return sorted(out)

    def buffered(self, v, cap=512):
        k = np.zeros(cap, np.uint32)
        r = np.zeros(cap, np.uint32)
        ln = C.c_size_t()
        self._c(lib().psim_causal_get_buffered(self.sim._h, v, _u32p(k), _u32p(r), cap, C.byref(ln)))
        return [(int(k[i]), int(r[i])) for i in range(min(ln.value, cap))]

    def delivered(self):
        out = np.zeros(self.n, np.uint64)
        self._c(lib().psim_causal_get_delivered(self.sim._h, out.ctypes.data_as(C.POINTER(C.c_uint64)), self.n))
        return out
