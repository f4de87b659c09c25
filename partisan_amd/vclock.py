"""partisan_vclock on dense lanes (host mirror; kernels in csrc/vclock.hip).

A clock is PSIM_VC_LANES u32 lanes over a fixed actor table (lane i = the
i-th actor in term order); lane value 0 = absent, c + 1 = counter c.
``to_dense`` / ``to_sparse`` convert from / to the reference's
``[{Actor, Counter}]`` lists (keysorted, the form ``merge/1`` of >= 2 clocks
returns; compare with ``equal/2`` semantics, Q23).
"""
import ctypes as C

import numpy as np

from ._lib import check, lib

LANES = 64


def to_dense(clocks, actors):
    """clocks: list of [[actor, ctr], ...]; actors: sorted actor ids (<= 64)."""
    idx = {a: i for i, a in enumerate(actors)}
    if len(actors) > LANES:
        raise ValueError("more than 64 actors")
    out = np.zeros((len(clocks), LANES), dtype=np.uint32)
    for k, clk in enumerate(clocks):
        for a, c in clk:
            if c < 0 or c >= 0xFFFFFFFF:
                raise ValueError("counter out of u32 range")
            out[k, idx[a]] = c + 1
    return out


def to_sparse(dense, actors):
    res = []
    for row in np.asarray(dense):
        res.append([[actors[i], int(v) - 1] for i, v in enumerate(row[: len(actors)]) if v])
    return res


def _u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


class VClockOps:
    """Batched vclock kernels on the simulator's device."""

    def __init__(self, sim):
        self.sim = sim

    def _pair(self, a, b):
        a, b = _u32(a), _u32(b)
        if a.shape != b.shape or a.ndim != 2 or a.shape[1] != LANES:
            raise ValueError("clock arrays must be (n, 64)")
        return a, b

    def descends(self, a, b):
        a, b = self._pair(a, b)
        out = np.zeros(len(a), np.uint8)
        P = C.POINTER
        check(lib().psim_vclock_descends(self.sim._h, a.ctypes.data_as(P(C.c_uint32)),
                                         b.ctypes.data_as(P(C.c_uint32)), out.ctypes.data_as(P(C.c_uint8)),
                                         len(a)), self.sim._h)
        return out.astype(bool)

    def dominates(self, a, b):
        a, b = self._pair(a, b)
        out = np.zeros(len(a), np.uint8)
        P = C.POINTER
        check(lib().psim_vclock_dominates(self.sim._h, a.ctypes.data_as(P(C.c_uint32)),
                                          b.ctypes.data_as(P(C.c_uint32)), out.ctypes.data_as(P(C.c_uint8)),
                                          len(a)), self.sim._h)
        return out.astype(bool)

    def merge(self, a, b):
        a, b = self._pair(a, b)
        out = np.zeros_like(a)
        P = C.POINTER
        check(lib().psim_vclock_merge(self.sim._h, a.ctypes.data_as(P(C.c_uint32)), b.ctypes.data_as(P(C.c_uint32)),
                                      out.ctypes.data_as(P(C.c_uint32)), len(a)), self.sim._h)
        return out

    def _bool(self, fn, a, b):
        a, b = self._pair(a, b)
        out = np.zeros(len(a), np.uint8)
        P = C.POINTER
        check(fn(self.sim._h, a.ctypes.data_as(P(C.c_uint32)), b.ctypes.data_as(P(C.c_uint32)),
                 out.ctypes.data_as(P(C.c_uint8)), len(a)), self.sim._h)
        return out.astype(bool)

    def _clock(self, fn, a, b):
        a, b = self._pair(a, b)
        out = np.zeros_like(a)
        P = C.POINTER
        check(fn(self.sim._h, a.ctypes.data_as(P(C.c_uint32)), b.ctypes.data_as(P(C.c_uint32)),
                 out.ctypes.data_as(P(C.c_uint32)), len(a)), self.sim._h)
        return out

    def equal(self, a, b):
        """equal/2 (:163-164)."""
        return self._bool(lib().psim_vclock_equal, a, b)

    def glb(self, a, b):
        """glb/2 (:183-198): lane-wise min."""
        return self._clock(lib().psim_vclock_glb, a, b)

    def subtract_dots(self, dots, clock):
        """subtract_dots(DotList, VClock) (:85-99)."""
        return self._clock(lib().psim_vclock_subtract_dots, dots, clock)

    def get_counter(self, a, actor_lanes):
        """get_counter(Actor, VClock) (:132-137), one actor lane per clock."""
        a = _u32(a)
        act = _u32(actor_lanes)
        if act.shape != (len(a),):
            raise ValueError("one actor lane per clock")
        out = np.zeros(len(a), np.uint32)
        P = C.POINTER
        check(lib().psim_vclock_get_counter(self.sim._h, a.ctypes.data_as(P(C.c_uint32)),
                                            act.ctypes.data_as(P(C.c_uint32)), out.ctypes.data_as(P(C.c_uint32)),
                                            len(a)), self.sim._h)
        return out

    def increment(self, a, actor_lanes):
        a = _u32(a)
        act = _u32(actor_lanes)
        out = np.zeros_like(a)
        P = C.POINTER
        check(lib().psim_vclock_increment(self.sim._h, a.ctypes.data_as(P(C.c_uint32)),
                                          act.ctypes.data_as(P(C.c_uint32)), out.ctypes.data_as(P(C.c_uint32)),
                                          len(a)), self.sim._h)
        return out
