"""Simulator: one libpsim handle = one simulated cluster on one GPU.

Thin numpy-facing wrapper over include/psim.h; every method is one ABI
call (the HIP kernels do the protocol work).
"""
import ctypes as C

import numpy as np

from ._lib import (PSIM_ABI_VERSION, PSIM_CFG_BINNED, PSIM_CFG_CHUNK_TIMING, PSIM_CFG_CSR, Config, RoundStats, check,
                   lib)

_u8p = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint8))    # noqa: E731
_u16p = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint16))  # noqa: E731
_u32p = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint32))  # noqa: E731
_u64p = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint64))  # noqa: E731


_ROUND_DTYPE = np.dtype([("sent", np.uint64, 6), ("delivered_new", np.uint64), ("active", np.uint64),
                         ("senders", np.uint64), ("sender_degree_sum", np.uint64),
                         ("outstanding_vertices", np.uint64), ("algo_bytes", np.uint64), ("kernel_ms", np.float64),
                         ("words_stored", np.uint64)])
assert _ROUND_DTYPE.itemsize == C.sizeof(RoundStats)


class Simulator:
    """Round-synchronous simulator of Partisan's gossip hot path."""

    def __init__(self, lazy_tick_rounds=1, exchange_tick_rounds=10, device=-1, seed=0, rank=0, world=1,
                 binned=False, csr=False, chunk_timing=False, max_roots=0, forest_lanes=0):
        """binned: route Plumtree messages through receiver bins on a single
        GPU instead of scattering receiver-slot words (PSIM_CFG_BINNED; same
        results).  csr: keep CSR slot rows in the slot-scatter
        engine instead of fixed-width ELL rows (PSIM_CFG_CSR; same results).
        chunk_timing: one hipEvent pair per chunk of rounds (PSIM_CFG_CHUNK_TIMING;
        kernel_ms of a round = the chunk's device time / its rounds).
        max_roots: heartbeat roots whose per-root trees the handle keeps
        (psim_config.max_roots; 0 = 16 lanes).  Above 16 the roots live in one
        forest launched together; a root beyond max_roots is
        PSIM_ENOSPC.  forest_lanes (< max_roots): lanes for heartbeats in
        flight; every root's records are kept, a done root's lane is reused
        (psim_forest_set_lanes; 0 = one lane per root)."""
        flags = ((PSIM_CFG_BINNED if binned else 0) | (PSIM_CFG_CSR if csr else 0)
                 | (PSIM_CFG_CHUNK_TIMING if chunk_timing else 0))
        cfg = Config(abi_version=PSIM_ABI_VERSION, device=device, lazy_tick_rounds=lazy_tick_rounds,
                     exchange_tick_rounds=exchange_tick_rounds, flags=flags, max_roots=max_roots, seed=seed)
        h = C.c_void_p()
        check(lib().psim_create(C.byref(cfg), C.byref(h)))
        self._h = h
        self.n = 0
        self.binned = binned
        self.lazy_tick_rounds = lazy_tick_rounds
        self.rank, self.world = rank, world
        if forest_lanes:
            check(lib().psim_forest_set_lanes(h, forest_lanes), h)
        if world > 1:
            check(lib().psim_shard_init(h, rank, world), h)

    # ---------------------------------------------------------------- lifecycle
    def close(self):
        if getattr(self, "_h", None):
            lib().psim_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _c(self, rc):
        return check(rc, self._h)

    def device_info(self):
        buf = C.create_string_buffer(256)
        self._c(lib().psim_device_info(self._h, buf, 256))
        return buf.value.decode()

    # ---------------------------------------------------------------- overlay
    def load_overlay(self, row_ptr, col):
        """Membership lists (members minus self) as CSR; see psim_load_csr."""
        rp = np.ascontiguousarray(row_ptr, dtype=np.uint64)
        cc = np.ascontiguousarray(col, dtype=np.uint32)
        if len(rp) < 1 or rp[0] != 0 or int(rp[-1]) != len(cc):
            raise ValueError(f"CSR shape: row_ptr[0]={int(rp[0]) if len(rp) else None}, "
                             f"row_ptr[n]={int(rp[-1]) if len(rp) else None}, len(col)={len(cc)}")
        self._c(lib().psim_load_csr(self._h, len(rp) - 1, _u64p(rp), _u32p(cc) if len(cc) else None, len(cc)))
        v_lo, n_local, n_global = C.c_uint32(), C.c_uint32(), C.c_uint32()
        slot_base = C.c_uint64()
        self._c(lib().psim_shard_info(self._h, C.byref(v_lo), C.byref(n_local), C.byref(slot_base),
                                      C.byref(n_global)))
        self.v_lo, self.n_global, self.slot_base = v_lo.value, n_global.value, slot_base.value
        n = self.n = n_local.value
        E = C.c_uint64()
        self._c(lib().psim_num_slots(self._h, C.byref(E)))
        self.slot_row_ptr = np.zeros(n + 1, dtype=np.uint64)
        self.slot_col = np.zeros(max(1, E.value), dtype=np.uint32)
        self._c(lib().psim_get_slots(self._h, _u64p(self.slot_row_ptr), _u32p(self.slot_col)))
        self.slot_col = self.slot_col[: E.value]
        self.num_slots = E.value

    def set_alive(self, alive):
        a = np.ascontiguousarray(alive, dtype=np.uint8)
        self._c(lib().psim_set_alive(self._h, _u8p(a), len(a)))

    # ---------------------------------------------------------------- plumtree
    def reset_trees(self):
        self._c(lib().psim_plumtree_reset_trees(self._h))

    def broadcast(self, root):
        mono = C.c_uint32()
        self._c(lib().psim_plumtree_broadcast(self._h, root, C.byref(mono)))
        return mono.value

    def broadcast_many(self, roots):
        """Heartbeats from every root in `roots` at once (psim_plumtree_broadcast_many):
        the backend's timer firing at each node.  Returns their ids."""
        r = np.ascontiguousarray(np.asarray(roots, dtype=np.uint32).reshape(-1))
        monos = np.zeros(len(r), np.uint32)
        self._c(lib().psim_plumtree_broadcast_many(self._h, _u32p(r), len(r), _u32p(monos)))
        return monos

    def step(self, rounds=1):
        st = (RoundStats * max(1, rounds))()
        self._c(lib().psim_step(self._h, rounds, st, rounds))
        return [s.as_dict() for s in st[:rounds]]

    def run(self, max_rounds=100000, cap=4096, as_dicts=True):
        """Rounds to quiescence (psim_run): (per-round stats, rounds).  as_dicts=False
        returns the stats as a numpy structured array (fields of psim_round_stats)
        instead of one dict per round -- no per-round Python objects."""
        st = getattr(self, "_run_buf", None)          # reused: a 4096-row ctypes array costs ~0.1 ms to zero
        if st is None or len(st) < cap:
            st = self._run_buf = (RoundStats * cap)()
        ran = C.c_uint32()
        self._c(lib().psim_run(self._h, max_rounds, st, cap, C.byref(ran)))
        k = min(ran.value, cap)
        if not as_dicts:
            return np.frombuffer(st, dtype=_ROUND_DTYPE, count=k).copy(), ran.value
        return [s.as_dict() for s in st[:k]], ran.value

    def broadcast_run(self, root, max_rounds=100000, cap=4096, as_dicts=True):
        """broadcast(root) then run() in one call (psim_plumtree_broadcast_run):
        the origin's counters come back with the first chunk of rounds.
        Returns (id, per-round stats, rounds)."""
        st = getattr(self, "_run_buf", None)
        if st is None or len(st) < cap:
            st = self._run_buf = (RoundStats * cap)()
        mono, ran = C.c_uint32(), C.c_uint32()
        self._c(lib().psim_plumtree_broadcast_run(self._h, root, C.byref(mono), max_rounds, st, cap, C.byref(ran)))
        k = min(ran.value, cap)
        if not as_dicts:
            return mono.value, np.frombuffer(st, dtype=_ROUND_DTYPE, count=k).copy(), ran.value
        return mono.value, [s.as_dict() for s in st[:k]], ran.value

    def broadcast_run_n(self, root, count, reset_trees=True, max_rounds=100000, cap=None):
        """`count` heartbeat intervals of `root` back to back in one call
        (psim_plumtree_broadcast_run_n): each reset_trees() (when asked) then
        broadcast_run(root).  Returns (ids, per-round stats of every interval
        as one numpy record array, rounds per interval)."""
        cap = cap if cap is not None else 64 * max(1, count)
        st = getattr(self, "_runn_buf", None)
        if st is None or len(st) < cap:
            st = self._runn_buf = (RoundStats * cap)()
        rounds = np.zeros(count, np.uint32)
        monos = np.zeros(count, np.uint32)
        done = C.c_uint32()
        self._c(lib().psim_plumtree_broadcast_run_n(self._h, root, count, 1 if reset_trees else 0, max_rounds, st, cap,
                                                    _u32p(rounds), _u32p(monos), C.byref(done)))
        k = min(int(rounds.astype(np.int64).sum()), cap)
        return monos, np.frombuffer(st, dtype=_ROUND_DTYPE, count=k).copy(), rounds

    def plumtree_state(self):
        n = self.n
        eager = np.zeros(n, np.uint32)
        lazy = np.zeros(n, np.uint32)
        outst = np.zeros(n, np.uint32)
        rr = np.zeros(n, np.uint16)
        self._c(lib().psim_get_plumtree(self._h, _u32p(eager), _u32p(lazy), _u32p(outst), _u16p(rr), n))
        return eager, lazy, outst, rr

    def delivered(self):
        out = np.zeros(self.n, np.uint8)
        self._c(lib().psim_get_delivered(self._h, _u8p(out), self.n))
        return out

    def max_degree(self):
        """Widest peer row of this handle's vertices (rows of <= 8 slots load as ELL rows)."""
        d = np.diff(np.asarray(self.slot_row_ptr, dtype=np.int64))
        return int(d.max()) if len(d) else 0

    def restart_backend(self, v):
        """v's heartbeat backend restarts (psim_plumtree_restart_backend): newer
        epoch, Monotonic 0, v forgets every origin's heartbeats.  Ids are then
        reported as epoch << 24 | Monotonic."""
        self._c(lib().psim_plumtree_restart_backend(self._h, v))

    def delivered_at(self, v, mono=0):
        """Mod:is_stale at ONE local vertex (psim_get_delivered_range): mono 0 =
        the focused root's newest heartbeat.  No copy of the whole set."""
        out = np.zeros(1, np.uint8)
        self._c(lib().psim_get_delivered_range(self._h, mono, v, 1, _u8p(out)))
        return bool(out[0])

    def delivered_mono(self, mono):
        """Mod:is_stale({root, epoch, mono}) per vertex (psim_get_delivered_mono)."""
        out = np.zeros(self.n, np.uint8)
        self._c(lib().psim_get_delivered_mono(self._h, mono, _u8p(out), self.n))
        return out

    def messages(self):
        """Messages the next round delivers, in handling order: a list of
        (src, dst, kind, Round, Monotonic) (psim_get_messages)."""
        k = C.c_size_t(0)
        self._c(lib().psim_get_messages(self._h, None, None, None, None, None, 0, C.byref(k)))
        a = [np.zeros(max(1, k.value), np.uint32) for _ in range(5)]
        self._c(lib().psim_get_messages(self._h, *[_u32p(x) for x in a], k.value, C.byref(k)))
        return list(zip(*[x[:k.value].tolist() for x in a]))

    def rows(self, v):
        """Vertex v's outstanding i_have rows in insertion order: (peer, Round, Monotonic)."""
        k = C.c_size_t(0)
        self._c(lib().psim_get_rows(self._h, v, None, None, None, 0, C.byref(k)))
        a = [np.zeros(max(1, k.value), np.uint32) for _ in range(3)]
        self._c(lib().psim_get_rows(self._h, v, *[_u32p(x) for x in a], k.value, C.byref(k)))
        return list(zip(*[x[:k.value].tolist() for x in a]))

    def inflight(self):
        w = np.zeros(max(1, self.num_slots), np.uint32)
        self._c(lib().psim_get_inflight(self._h, _u32p(w), self.num_slots))
        return w[: self.num_slots]

    def focus(self, root):
        """Point the per-vertex getters at heartbeat root `root`'s lane (psim_plumtree_focus)."""
        self._c(lib().psim_plumtree_focus(self._h, root))

    def set_omissions(self, pairs):
        """Omission faults on directed (src, dst) pairs (psim_set_omissions); [] heals."""
        p = np.ascontiguousarray(np.asarray(pairs, dtype=np.uint32).reshape(-1, 2))
        s, d = np.ascontiguousarray(p[:, 0]), np.ascontiguousarray(p[:, 1])
        self._c(lib().psim_set_omissions(self._h, s.ctypes.data_as(C.POINTER(C.c_uint32)),
                                         d.ctypes.data_as(C.POINTER(C.c_uint32)), len(p)))

    def set_delays(self, pairs, rounds):
        """Delay faults (psim_set_delays): messages over directed (src, dst)
        pairs arrive rounds[i] rounds late; [] removes them.  Raises with
        PSIM_EBUSY while messages are in flight."""
        p = np.ascontiguousarray(np.asarray(pairs, dtype=np.uint32).reshape(-1, 2))
        s, d = np.ascontiguousarray(p[:, 0]), np.ascontiguousarray(p[:, 1])
        r = np.ascontiguousarray(np.asarray(rounds, dtype=np.uint8).reshape(-1))
        if len(r) != len(p):
            raise ValueError("one delay per pair")
        self._c(lib().psim_set_delays(self._h, s.ctypes.data_as(C.POINTER(C.c_uint32)),
                                      d.ctypes.data_as(C.POINTER(C.c_uint32)),
                                      r.ctypes.data_as(C.POINTER(C.c_uint8)), len(p)))

    def egress_delay(self, v, rounds):
        """partisan's egress_delay for node v: every out-edge of v delayed."""
        rp = np.asarray(self.slot_row_ptr, dtype=np.int64)
        col = np.asarray(self.slot_col, dtype=np.uint32)[rp[v]:rp[v + 1]]
        return np.stack([np.full(len(col), v, np.uint32), col], axis=1), np.full(len(col), rounds, np.uint8)

    def partition_pairs(self, group):
        """Directed overlay edges (of this handle's vertices) whose ends lie in
        different groups: group[v] = partition of global vertex v."""
        group = np.asarray(group)
        rp = np.asarray(self.slot_row_ptr, dtype=np.int64)
        col = np.asarray(self.slot_col, dtype=np.int64)
        src = np.repeat(np.arange(len(rp) - 1, dtype=np.int64) + self.v_lo, np.diff(rp))
        cut = group[src] != group[col]
        return np.stack([src[cut], col[cut]], axis=1)

    def inject_partition(self, group):
        """partisan's inject_partition: messages across groups are lost."""
        self.set_omissions(self.partition_pairs(group))

    def resolve_partition(self):
        self.set_omissions(np.zeros((0, 2), np.uint32))

    def trace_hash(self):
        """psim_trace_hash: (state digest, in-flight digest, delivered, rounds)."""
        out = (C.c_uint64 * 4)()
        self._c(lib().psim_trace_hash(self._h, out))
        return tuple(int(x) for x in out)

    def set_chunk_timing(self, chunk):
        """psim_set_chunk_timing: one event pair per chunk (True) or per round kernel."""
        self._c(lib().psim_set_chunk_timing(self._h, 1 if chunk else 0))

    def timing(self):
        ms = C.c_double()
        r = C.c_uint64()
        self._c(lib().psim_get_timing(self._h, C.byref(ms), C.byref(r)))
        return ms.value, r.value

    def mask_to_peers(self, v, mask):
        """Decode a per-vertex slot mask into the sorted list of peer ids."""
        lo = int(self.slot_row_ptr[v])
        hi = int(self.slot_row_ptr[v + 1])
        return [int(self.slot_col[lo + s]) for s in range(hi - lo) if (int(mask) >> s) & 1]

    def decode_inflight(self, words=None):
        """In-flight messages as sorted (src, dst, kind, round) tuples (global
        ids; dst = a local vertex); the Round is reported for broadcast /
        i_have only (the others carry an echo or nothing).  Order within a
        (src, dst) pair is FIFO order."""
        if words is None:
            words = self.inflight()
        out = []
        rp = self.slot_row_ptr
        nz = np.nonzero(words)[0]
        dst_of = np.searchsorted(rp, nz, side="right") - 1
        for e, dst in zip(nz.tolist(), dst_of.tolist()):
            w = int(words[e])
            src = int(self.slot_col[e])
            f, rnd = w & 0xFFFF, w >> 16
            while f:
                t = f & 0xF
                f >>= 4
                out.append((src, int(dst) + self.v_lo, t, rnd if t in (1, 3) else 0))
        out.sort(key=lambda m: (m[1], m[0]))
        return out
