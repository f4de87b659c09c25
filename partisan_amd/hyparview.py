"""HyParView view maintenance (src/partisan_hyparview_peer_service_manager.erl)
on the simulator's device.

Host mirror of the peer service manager's surface for this path: ``join``
(handle_cast({join, Peer}) :999-1016), rounds of message handling and the two
timers (``step``), and the state getters (``active_view`` / ``passive_view``
= the ``active``/``passive`` of the #state record, ``members`` =
members_for_orchestration/0 :2159-2168, i.e. the active view).  ``overlay``
exports the active views as the membership CSR that the Plumtree engine loads
(the peer service feeding partisan_plumtree_broadcast).
"""
import ctypes as C

import numpy as np

from ._lib import HV_MSG_KINDS, HvConfig, HvStats, check, lib

# partisan.hrl defaults; the periods are the ms timers mapped to rounds
# (passive_view_shuffle_period 10000 ms, random_promotion_interval 5000 ms,
# 1 round = 1000 ms, DESIGN.md "Schedule").
DEFAULTS = dict(active_max_size=6, active_min_size=3, active_rwl=6, passive_max_size=30, passive_rwl=6,
                shuffle_k_active=3, shuffle_k_passive=4, shuffle_rounds=10, promotion_rounds=5)

_u8p = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint8))    # noqa: E731
_u32p = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint32))  # noqa: E731
_u64p = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint64))  # noqa: E731


class HyParViewCluster:
    """n HyParView peer service managers, one vertex each."""

    def __init__(self, sim, n, **cfg):
        c = dict(DEFAULTS)
        c.update(cfg)
        self.sim, self.n, self.cfg = sim, n, c
        check(lib().psim_hv_setup(sim._h, n, C.byref(HvConfig(**c))), sim._h)

    def _c(self, rc):
        return check(rc, self.sim._h)

    def set_alive(self, alive):
        a = np.ascontiguousarray(alive, dtype=np.uint8)
        self._c(lib().psim_hv_set_alive(self.sim._h, _u8p(a), len(a)))

    def join(self, v, contact):
        """One join cast; see join_many for a batch made between two rounds."""
        self.join_many([v], [contact])

    def join_many(self, vs, contacts):
        v = np.ascontiguousarray(vs, dtype=np.uint32)
        c = np.ascontiguousarray(contacts, dtype=np.uint32)
        if v.shape != c.shape:
            raise ValueError("vs and contacts differ in length")
        self._c(lib().psim_hv_join(self.sim._h, _u32p(v), _u32p(c), len(v)))

    def join_seq(self, vs, contacts, rounds=1):
        """Sequential joins (C2's schedule) in one call (psim_hv_join_seq):
        vs[i] joins contacts[i], then `rounds` rounds -- the same as
        join(vs[i], contacts[i]) + step(rounds) per i.  Returns the rounds'
        stats (len(vs) * rounds dicts)."""
        v = np.ascontiguousarray(vs, dtype=np.uint32)
        c = np.ascontiguousarray(contacts, dtype=np.uint32)
        if v.shape != c.shape:
            raise ValueError("vs and contacts differ in length")
        k = len(v) * rounds
        st = (HvStats * max(1, k))()
        self._c(lib().psim_hv_join_seq(self.sim._h, _u32p(v), _u32p(c), len(v), rounds, st, k))
        return [s.as_dict() for s in st[:k]]

    def step(self, rounds=1):
        st = (HvStats * max(1, rounds))()
        self._c(lib().psim_hv_step(self.sim._h, rounds, st, rounds))
        return [s.as_dict() for s in st[:rounds]]

    def views(self):
        """(act[n,8], na[n], pas[n,32], np[n]); rows padded with 0xFFFFFFFF."""
        act = np.zeros((self.n, 8), np.uint32)
        pas = np.zeros((self.n, 32), np.uint32)
        na = np.zeros(self.n, np.uint8)
        np_ = np.zeros(self.n, np.uint8)
        self._c(lib().psim_hv_get_views(self.sim._h, _u32p(act), _u8p(na), _u32p(pas), _u8p(np_), self.n))
        return act, na, pas, np_

    def active_view(self, v):
        act, na, _, _ = self.views()
        return act[v, :na[v]].tolist()

    def passive_view(self, v):
        _, _, pas, np_ = self.views()
        return pas[v, :np_[v]].tolist()

    def draws(self):
        out = np.zeros(self.n, np.uint64)
        self._c(lib().psim_hv_get_draws(self.sim._h, _u64p(out), self.n))
        return out

    def idmap(self, v, which, cap=256):
        """which 0 = sent_message_map, 1 = recv_message_map: [(peer, epoch, cnt)]."""
        p, e, c = (np.zeros(cap, np.uint32) for _ in range(3))
        ln = C.c_size_t()
        self._c(lib().psim_hv_get_idmap(self.sim._h, v, which, _u32p(p), _u32p(e), _u32p(c), cap, C.byref(ln)))
        return [(int(p[i]), int(e[i]), int(c[i])) for i in range(min(ln.value, cap))]

    def inflight(self):
        m = C.c_uint64()
        self._c(lib().psim_hv_inflight(self.sim._h, C.byref(m)))
        return m.value

    def overlay(self):
        """Active views minus self as a membership CSR (row_ptr uint64, col uint32)."""
        act, na, _, _ = self.views()
        mask = (np.arange(8)[None, :] < na[:, None]) & (act != np.arange(self.n, dtype=np.uint32)[:, None])
        deg = mask.sum(1)
        rp = np.zeros(self.n + 1, np.uint64)
        np.cumsum(deg, out=rp[1:])
        return rp, act[mask].astype(np.uint32)


def kind_counts(stats):
    """Sum per-kind message counts over a list of step() dicts."""
    tot = {k: 0 for k in HV_MSG_KINDS.values()}
    for s in stats:
        for i, k in HV_MSG_KINDS.items():
            tot[k] += s["sent"][i - 1]
    return tot
