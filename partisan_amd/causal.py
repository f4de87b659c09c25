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


class ShardedCausal:
    """Causal delivery vertex-sharded over `world` processes, one GPU each
    (SURVEY 8(e), config C5).  Receivers enumerate their own arrivals, so the
    only exchange per round is the 64 x 64 clock slab of the emitters that
    broadcast: sum-all-reduced.

    transport: "rccl" (default with backend "nccl") / "callback" (default
    with "gloo"): inside libpsim on the handle's transport
    (psim_causal_shard_step -- what an Erlang host drives through the NIF);
    "torch": the split-phase entry points with the all-reduce issued from
    Python."""

    def __init__(self, n, rank, world, m=64, period=1, dmax=4, redeliver=1, device=0, backend="nccl", seed=0,
                 transport=None):
        import torch

        from .sim import Simulator
        self.torch, self.n, self.m, self.rank, self.world, self.backend = torch, n, m, rank, world, backend
        self.transport = transport or ("rccl" if backend == "nccl" else "callback")
        self.dev = torch.device("cuda", device)
        if backend == "nccl":
            torch.cuda.set_device(self.dev)
        self.sim = Simulator(device=device, seed=seed)
        self._h = self.sim._h
        if self.transport == "rccl":
            import torch.distributed as dist

            from ._lib import PSIM_RCCL_ID_BYTES
            uid = (C.c_uint8 * PSIM_RCCL_ID_BYTES)()
            if rank == 0:
                check(lib().psim_rccl_unique_id(uid))
            if world > 1:
                box = [bytes(uid)]
                dist.broadcast_object_list(box, src=0)
                uid = (C.c_uint8 * PSIM_RCCL_ID_BYTES).from_buffer_copy(box[0])
            check(lib().psim_shard_init_rccl(self._h, rank, world, uid), self._h)
        elif self.transport == "callback":
            from .shard import gloo_transport
            self._tp, self._keep = gloo_transport()
            check(lib().psim_shard_set_transport(self._h, C.byref(self._tp)), self._h)
        check(lib().psim_causal_shard_setup(self._h, n, m, period, dmax, redeliver, rank, world), self._h)
        lo, nl = C.c_uint32(), C.c_uint32()
        check(lib().psim_causal_shard_info(self._h, C.byref(lo), C.byref(nl)), self._h)
        self.v_lo, self.n_local = lo.value, nl.value
        self.emitters = np.zeros(m, np.uint32)
        check(lib().psim_causal_emitters(self._h, _u32p(self.emitters), m), self._h)
        self.slab = torch.zeros(64 * 64, dtype=torch.int32, device=self.dev)
        self.local_kernel_ms = 0.0

    def _allreduce(self, vals):
        import torch.distributed as dist
        t = self.torch.tensor(vals, dtype=self.torch.int64, device=self.dev if self.backend == "nccl" else "cpu")
        dist.all_reduce(t)
        return t.tolist()

    def step(self, rounds=1):
        """Rounds; per-round GLOBAL stats (summed over shards)."""
        if self.transport != "torch":
            st = (CausalStats * max(1, rounds))()
            check(lib().psim_causal_shard_step(self._h, rounds, st, rounds), self._h)
            out = [s_.as_dict() for s_ in st[:rounds]]
            for d in out:
                self.local_kernel_ms += d["kernel_ms"]
            return out
        import torch.distributed as dist
        out = []
        keys = ["emitted", "received", "delivered", "checks", "buffered", "algo_bytes"]
        for _ in range(rounds):
            st = CausalStats()
            check(lib().psim_causal_shard_round(self._h, C.c_void_p(self.slab.data_ptr()), C.byref(st)), self._h)
            if self.backend == "nccl":
                dist.all_reduce(self.slab)
                self.torch.cuda.synchronize(self.dev)
            else:
                h = self.slab.cpu()
                dist.all_reduce(h)
                self.slab.copy_(h.to(self.dev))
                self.torch.cuda.synchronize(self.dev)
            check(lib().psim_causal_shard_ingest(self._h, C.c_void_p(self.slab.data_ptr())), self._h)
            d = st.as_dict()
            self.local_kernel_ms += d["kernel_ms"]
            g = dict(zip(keys, self._allreduce([d[k] for k in keys])))
            g["kernel_ms"] = d["kernel_ms"]
            out.append(g)
        return out

    def clocks(self):
        lanes = np.zeros((max(1, self.n_local), 64), np.uint32)
        slf = np.zeros(max(1, self.n_local), np.uint32)
        check(lib().psim_causal_get_clocks(self._h, _u32p(lanes), _u32p(slf), self.n_local), self._h)
        return lanes, slf

    def clock(self, lv, lanes, slf):
        """local_clock of global vertex v_lo + lv as sorted (actor, counter) pairs."""
        out = [(int(self.emitters[k]), int(lanes[lv, k])) for k in range(self.m) if lanes[lv, k]]
        if slf[lv]:
            out.append((self.v_lo + lv, int(slf[lv])))
        return sorted(out)

    def buffered(self, lv, cap=512):
        k = np.zeros(cap, np.uint32)
        r = np.zeros(cap, np.uint32)
        ln = C.c_size_t()
        check(lib().psim_causal_get_buffered(self._h, lv, _u32p(k), _u32p(r), cap, C.byref(ln)), self._h)
        return [(int(k[i]), int(r[i])) for i in range(min(ln.value, cap))]

    def delivered(self):
        out = np.zeros(max(1, self.n_local), np.uint64)
        check(lib().psim_causal_get_delivered(self._h, out.ctypes.data_as(C.POINTER(C.c_uint64)), self.n_local),
              self._h)
        return out[:self.n_local]

    def close(self):
        self.sim.close()
