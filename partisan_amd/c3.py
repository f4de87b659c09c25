"""Configuration C3: Plumtree broadcast repaired by graft/prune
over churning SCAMP v2 membership, on the simulator's device (ptdyn.hip).

Host mirror of a cluster running the pluggable peer service manager with the
SCAMP v2 strategy and the Plumtree server fed by its {update, Members} casts:
``join``/``crash`` drive membership (crash = node restart), ``heartbeat``
is the backend's heartbeat at a root, ``step`` runs rounds; ``plumtree(v)``
returns a vertex's all_eager_peers / all_lazy_peers / outstanding rows, and
``scamp`` is the membership side (ScampCluster view of the same handle).
"""
import ctypes as C

import numpy as np

from ._lib import C3Stats, check, lib
from .scamp import ScampCluster

_P = C.POINTER


class C3Cluster:
    def __init__(self, sim, n, c=5, periodic_rounds=10):
        self.sim, self.n = sim, n
        check(lib().psim_c3_setup(sim._h, n, c, periodic_rounds), sim._h)
        self.scamp = ScampCluster.__new__(ScampCluster)
        self.scamp.sim, self.scamp.n, self.scamp.version = sim, n, 2

    def _c(self, rc):
        return check(rc, self.sim._h)

    def join(self, v, contact):
        a = np.ascontiguousarray(np.atleast_1d(v), dtype=np.uint32)
        b = np.ascontiguousarray(np.atleast_1d(contact), dtype=np.uint32)
        self._c(lib().psim_c3_join(self.sim._h, a.ctypes.data_as(_P(C.c_uint32)), b.ctypes.data_as(_P(C.c_uint32)),
                                   len(a)))

    def crash(self, v):
        a = np.ascontiguousarray(np.atleast_1d(v), dtype=np.uint32)
        self._c(lib().psim_c3_crash(self.sim._h, a.ctypes.data_as(_P(C.c_uint32)), len(a)))

    def heartbeat(self, root):
        mono = C.c_uint32()
        self._c(lib().psim_c3_heartbeat(self.sim._h, root, C.byref(mono)))
        return mono.value

    def step(self, rounds=1):
        st = (C3Stats * rounds)()
        self._c(lib().psim_c3_step(self.sim._h, rounds, st, rounds))
        return [s.as_dict() for s in st]

    @staticmethod
    def plan(crashes, joins):
        """Flat arrays for run(): (crash_off, crash_v, join_off, join_v,
        join_c) from one crash list and one (vertices, contacts) join list per
        round."""
        rounds = len(crashes)
        if len(joins) != rounds:
            raise ValueError("one crash list and one join list per round")

        def flat(parts):
            parts = [np.atleast_1d(x).astype(np.uint32, copy=False) for x in parts]
            off = np.zeros(rounds + 1, np.uint32)
            off[1:] = np.cumsum([len(x) for x in parts])
            v = np.concatenate(parts) if parts else np.zeros(0, np.uint32)
            return off, np.ascontiguousarray(v, dtype=np.uint32)

        co, cv = flat(crashes)
        jo, jv = flat([j[0] for j in joins])
        _, jc = flat([j[1] for j in joins])
        return co, cv, jo, jv, jc

    def run(self, crashes=None, joins=None, heartbeat_every=0, root=0, plan=None):
        """Rounds of churn in one call (psim_c3_run): round i = heartbeat at
        `root` when heartbeat_every and i % heartbeat_every == 0, crash of
        crashes[i], join of joins[i] = (vertices, contacts), one step -- the
        same as those calls one by one, with no host wait between rounds.
        `plan` (from C3Cluster.plan) replaces crashes / joins."""
        co, cv, jo, jv, jc = plan if plan is not None else self.plan(crashes, joins)
        rounds = len(co) - 1
        u32 = _P(C.c_uint32)
        st = (C3Stats * max(rounds, 1))()
        self._c(lib().psim_c3_run(self.sim._h, rounds, co.ctypes.data_as(u32), cv.ctypes.data_as(u32),
                                  jo.ctypes.data_as(u32), jv.ctypes.data_as(u32), jc.ctypes.data_as(u32),
                                  heartbeat_every, root, st, rounds))
        return [s.as_dict() for s in st[:rounds]]

    def plumtree(self, v, cap=128):
        """(eager, lazy, outstanding) sorted ids, delivered heartbeat serial, pushed Round."""
        e, l_, o = (C.c_uint32 * cap)(), (C.c_uint32 * cap)(), (C.c_uint32 * cap)()
        ne, nl, no = C.c_size_t(), C.c_size_t(), C.c_size_t()
        mono, rnd = C.c_uint32(), C.c_uint32()
        self._c(lib().psim_c3_get_plumtree(self.sim._h, v, e, C.byref(ne), l_, C.byref(nl), o, C.byref(no), cap,
                                           C.byref(mono), C.byref(rnd)))
        return list(e[:ne.value]), list(l_[:nl.value]), list(o[:no.value]), mono.value, rnd.value
