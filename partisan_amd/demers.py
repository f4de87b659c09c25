"""Demers epidemics (protocols/demers_rumor_mongering.erl,
protocols/demers_anti_entropy.erl) on the simulator's device.

Host mirror of the two gen_servers' API: ``broadcast`` (all rumors at their
Philox-drawn origins), ``step``/``run`` rounds, and the per-vertex store
(``seen``: bit i = rumor i; see include/psim.h for Q20's id reuse).
"""
import ctypes as C

import numpy as np

from ._lib import DemersStats, check, lib


class DemersEpidemic:
    def __init__(self, sim, n, m=64, ae_period=2, rumor_mongering=True):
        self.sim, self.n, self.m = sim, n, m
        check(lib().psim_demers_setup(sim._h, n, m, ae_period, 1 if rumor_mongering else 0), sim._h)

    def _c(self, rc):
        return check(rc, self.sim._h)

    def origins(self):
        out = np.zeros(self.m, np.uint32)
        self._c(lib().psim_demers_origins(self.sim._h, out.ctypes.data_as(C.POINTER(C.c_uint32)), self.m))
        return out

    def broadcast(self):
        self._c(lib().psim_demers_broadcast_all(self.sim._h))

    def step(self, rounds=1):
        st = (DemersStats * rounds)()
        self._c(lib().psim_demers_step(self.sim._h, rounds, st, rounds))
        return [s.as_dict() for s in st]

    def run(self, max_rounds=10000, cap=4096):
        st = (DemersStats * cap)()
        ran = C.c_uint32()
        self._c(lib().psim_demers_run(self.sim._h, max_rounds, st, cap, C.byref(ran)))
        return [s.as_dict() for s in st[: min(ran.value, cap)]], ran.value

    def seen(self):
        out = np.zeros(self.n, np.uint64)
        self._c(lib().psim_demers_get_seen(self.sim._h, out.ctypes.data_as(C.POINTER(C.c_uint64)), self.n))
        return out
