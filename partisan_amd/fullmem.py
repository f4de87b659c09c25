"""Full-membership strategy (src/partisan_full_membership_strategy.erl) on the
simulator's device, for a cluster of n nodes.

Host mirror of what the pluggable peer service manager does with the
`partisan_membership_strategy` behaviour (src/partisan_membership_strategy.erl
:55-77) when the strategy is full membership:

  * ``join(v, peer)``   -- partisan_peer_service:join at v: {connected, ...}
                           -> Strategy:join/3 (pluggable :1532-1597)
  * ``leave(v, who)``   -- partisan_peer_service:leave at v -> Strategy:leave/2
                           (pluggable :2059-2109)
  * ``step(rounds)``    -- deliveries to handle_message/2 (:1739-1808) and the
                           periodic/1 timer (:1386-1419)
  * ``members(v)``      -- the manager's `members` (partisan_membership_set:to_list)
  * ``messages()`` / ``take(v)`` / ``put(msgs)`` -- the gossip on the wire,
                           {membership_strategy, {NodeSpec, #full_v1{}}}
                           (gossip_messages/2 :247-267, handle_message/2
                           :135-166): what the manager sends, what node v's
                           manager receives, what it hands back to the device

Each node's membership is a state_orset (partisan_membership_set) held on the
device as two token bitmaps (known / removed); see fullmem.hip.
"""
import ctypes as C

import numpy as np

from ._lib import FmMsg, FmStats, check, lib

_P = C.POINTER


class FullMembershipCluster:
    def __init__(self, sim, n, periodic_rounds=10, max_tokens=None):
        self.sim, self.n = sim, n
        self.max_tokens = max_tokens if max_tokens is not None else n + 64
        self.words = (self.max_tokens + 63) // 64
        check(lib().psim_fm_setup(sim._h, n, periodic_rounds, self.max_tokens), sim._h)

    def _c(self, rc):
        return check(rc, self.sim._h)

    @staticmethod
    def _u32(x):
        a = np.ascontiguousarray(np.atleast_1d(x), dtype=np.uint32)
        return a, a.ctypes.data_as(_P(C.c_uint32))

    def join(self, v, peer):
        a, pa = self._u32(v)
        b, pb = self._u32(peer)
        self._c(lib().psim_fm_join(self.sim._h, pa, pb, len(a)))

    def leave(self, v, leaving):
        a, pa = self._u32(v)
        b, pb = self._u32(leaving)
        self._c(lib().psim_fm_leave(self.sim._h, pa, pb, len(a)))

    def set_alive(self, alive):
        a = np.ascontiguousarray(alive, dtype=np.uint8)
        self._c(lib().psim_fm_set_alive(self.sim._h, a.ctypes.data_as(_P(C.c_uint8)), len(a)))

    def step(self, rounds=1):
        st = (FmStats * rounds)()
        self._c(lib().psim_fm_step(self.sim._h, rounds, st, rounds))
        return [s.as_dict() for s in st]

    def state(self):
        """(known[n, words], removed[n, words], alive[n]): the state_orset payloads."""
        K = np.zeros((self.n, self.words), np.uint64)
        R = np.zeros((self.n, self.words), np.uint64)
        al = np.zeros(self.n, np.uint8)
        self._c(lib().psim_fm_get_state(self.sim._h, K.ctypes.data_as(_P(C.c_uint64)),
                                        R.ctypes.data_as(_P(C.c_uint64)), al.ctypes.data_as(_P(C.c_uint8)),
                                        self.n, self.words))
        return K, R, al

    def token_nodes(self):
        out = np.zeros(64 * self.words, np.uint32)
        used = C.c_uint32()
        self._c(lib().psim_fm_tokens(self.sim._h, out.ctypes.data_as(_P(C.c_uint32)), len(out), C.byref(used)))
        return out[:used.value]

    def members(self, v):
        """partisan_membership_set:to_list/1 of node v (sorted node ids)."""
        K, R, _ = self.state()
        tok = self.token_nodes()
        act = [t for t in range(len(tok)) if (int(K[v, t >> 6]) >> (t & 63)) & 1 and
               not (int(R[v, t >> 6]) >> (t & 63)) & 1]
        return sorted({int(tok[t]) for t in act})

    def inflight(self):
        x = C.c_uint64()
        self._c(lib().psim_fm_inflight(self.sim._h, C.byref(x)))
        return x.value

    # ---------------------------------------------------------------- wire
    def _unpack(self, m, K, R, k):
        return [(int(m[i].src), int(m[i].dst), int(m[i].seq), K[i].copy(), R[i].copy()) for i in range(k)]

    def messages(self):
        """[(src, dst, seq, known[words], removed[words])] the next round delivers, in handling order."""
        k = C.c_size_t()
        self._c(lib().psim_fm_messages(self.sim._h, None, None, None, 0, self.words, C.byref(k)))
        n = k.value
        m = (FmMsg * max(1, n))()
        K = np.zeros((max(1, n), self.words), np.uint64)
        R = np.zeros((max(1, n), self.words), np.uint64)
        self._c(lib().psim_fm_messages(self.sim._h, m, K.ctypes.data_as(_P(C.c_uint64)),
                                       R.ctypes.data_as(_P(C.c_uint64)), n, self.words, C.byref(k)))
        return self._unpack(m, K, R, min(n, k.value))

    def take(self, v):
        """Node v's messages off the wire (its manager receives them), in handling order."""
        cap = max(1, self.inflight())
        k = C.c_size_t()
        m = (FmMsg * cap)()
        K = np.zeros((cap, self.words), np.uint64)
        R = np.zeros((cap, self.words), np.uint64)
        self._c(lib().psim_fm_take(self.sim._h, v, m, K.ctypes.data_as(_P(C.c_uint64)),
                                   R.ctypes.data_as(_P(C.c_uint64)), cap, self.words, C.byref(k)))
        return self._unpack(m, K, R, k.value)

    def put(self, msgs):
        """[(src, dst, seq, known, removed)] onto the wire for the next round."""
        k = len(msgs)
        if not k:
            return
        m = (FmMsg * k)()
        K = np.zeros((k, self.words), np.uint64)
        R = np.zeros((k, self.words), np.uint64)
        for i, (src, dst, seq, kn, rm) in enumerate(msgs):
            m[i].src, m[i].dst, m[i].seq = src, dst, seq
            K[i], R[i] = kn, rm
        self._c(lib().psim_fm_put(self.sim._h, m, K.ctypes.data_as(_P(C.c_uint64)),
                                  R.ctypes.data_as(_P(C.c_uint64)), k, self.words))
