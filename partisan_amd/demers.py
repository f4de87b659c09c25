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
        """rumor_mongering: True (demers_rumor_mongering), False (anti-entropy
        alone) or "direct_mail" (demers_direct_mail, the baseline)."""
        self.sim, self.n, self.m = sim, n, m
        mode = 2 if rumor_mongering == "direct_mail" else (1 if rumor_mongering else 0)
        check(lib().psim_demers_setup(sim._h, n, m, ae_period, mode), sim._h)

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


class ShardedDemers:
    """Demers epidemic vertex-sharded over `world` processes, one GPU each
    (SURVEY 8(e)); include/psim.h "vertex-sharded Demers".  The exchange per
    round: all-to-all of the RM count-plane slices (summed, saturating, by the
    receiver), reduce-scatter of the pull slots, all-gather of every RM
    process's call records (rumors called, calls before the round), all-gather
    of the AE snapshots after a tick.

    transport: "rccl" (default with backend "nccl") / "callback" (default with
    "gloo"): the exchange runs inside libpsim on the handle's transport
    (psim_demers_shard_step: RCCL all-to-all-v / all-gather over xGMI on the
    library's stream, or gloo callbacks) -- what an Erlang host drives through
    the NIF; "torch": the split-phase entry points with the collectives issued
    from Python (the round-1 path, kept for A/B)."""

    def __init__(self, n, m, rank, world, device=0, backend="nccl", ae_period=2, rumor_mongering=True, seed=0,
                 transport=None):
        import torch

        from .sim import Simulator
        self.torch = torch
        self.n, self.m, self.rank, self.world, self.backend = n, m, rank, world, backend
        self.transport = transport or ("rccl" if backend == "nccl" else "callback")
        self.dev = torch.device("cuda", device)
        if backend == "nccl":
            torch.cuda.set_device(self.dev)
        self.sim = Simulator(device=device, seed=seed)
        self._h = self.sim._h
        if self.transport == "rccl":
            from ._lib import PSIM_RCCL_ID_BYTES
            uid = (C.c_uint8 * PSIM_RCCL_ID_BYTES)()
            if rank == 0:
                check(lib().psim_rccl_unique_id(uid))
            if world > 1:
                box = [bytes(uid)]
                self._dist().broadcast_object_list(box, src=0)
                uid = (C.c_uint8 * PSIM_RCCL_ID_BYTES).from_buffer_copy(box[0])
            check(lib().psim_shard_init_rccl(self._h, rank, world, uid), self._h)
        elif self.transport == "callback":
            from .shard import gloo_transport
            self._tp, self._keep = gloo_transport()
            check(lib().psim_shard_set_transport(self._h, C.byref(self._tp)), self._h)
        chunk = C.c_uint64()
        check(lib().psim_demers_shard_setup(self._h, n, m, ae_period, 1 if rumor_mongering else 0, rank, world,
                                            C.byref(chunk)), self._h)
        self.chunk = Cn = chunk.value
        vlo, nl = C.c_uint32(), C.c_uint32()
        check(lib().psim_demers_shard_info(self._h, C.byref(vlo), C.byref(nl), None), self._h)
        self.v_lo, self.n_local = vlo.value, nl.value
        G = world
        if self.transport == "torch":    # the caller-side buffers of the split-phase entry points
            z = lambda *shape: torch.zeros(*shape, dtype=torch.int64, device=self.dev)  # noqa: E731
            self.rm_shadow, self.rm_recv = z(3, G * Cn), z(3, G * Cn)
            self.pull_shadow, self.pull_recv = z(2 * G * Cn), z(2 * Cn)
            self.snap_all = z(G * Cn)
            # RM call records: [G C] u64 rumors called, then [G C] u32 calls before the round
            self.rmx_all = torch.zeros(3 * G * Cn, dtype=torch.int32, device=self.dev)
        self.local_kernel_ms = 0.0
        self.local_algo_bytes = 0

    @staticmethod
    def _p(t):
        return C.c_void_p(t.data_ptr())

    def set_exchange(self, mode):
        """In-library exchange form of the RM planes and call records: "auto"
        (records below n/8 slots), "dense" or "records" (psim.h
        psim_demers_shard_set_exchange); every shard must pass the same."""
        check(lib().psim_demers_shard_set_exchange(self._h, {"auto": 0, "dense": 1, "records": 2}[mode]), self._h)

    def exchange_stats(self):
        """(bytes this shard sent to other shards, exchanges, exchanges that
        sent RM records, exchanges that sent call records)."""
        b, n, s1, s2 = C.c_uint64(), C.c_uint32(), C.c_uint32(), C.c_uint32()
        check(lib().psim_demers_shard_exchange_stats(self._h, C.byref(b), C.byref(n), C.byref(s1), C.byref(s2)),
              self._h)
        return b.value, n.value, s1.value, s2.value

    # -------------------------------------------------------------- exchange
    def _exchange(self, tick):
        dist, torch = self._dist(), self.torch
        G, Cn, r = self.world, self.chunk, self.rank
        if self.backend == "nccl":
            for k in range(3):
                dist.all_to_all_single(self.rm_recv[k], self.rm_shadow[k])
            dist.reduce_scatter_tensor(self.pull_recv, self.pull_shadow, op=dist.ReduceOp.SUM)
            for plane in self._rmx_planes():
                mine = plane[r * plane.numel() // G:(r + 1) * plane.numel() // G].clone()
                dist.all_gather_into_tensor(plane, mine)
            if tick:
                mine = self.snap_all[r * Cn:(r + 1) * Cn].clone()
                dist.all_gather_into_tensor(self.snap_all, mine)
            torch.cuda.synchronize(self.dev)
        else:   # gloo: host-staged all-gather of the shadows, each rank keeps its slices
            rm = self.rm_shadow.cpu()
            pull = self.pull_shadow.cpu()
            rm_all = [torch.zeros_like(rm) for _ in range(G)]
            pull_all = [torch.zeros_like(pull) for _ in range(G)]
            dist.all_gather(rm_all, rm)
            dist.all_gather(pull_all, pull)
            recv = torch.stack([x[:, r * Cn:(r + 1) * Cn] for x in rm_all], dim=1).reshape(3, G * Cn)
            self.rm_recv.copy_(recv.to(self.dev))
            ps = torch.zeros(2 * Cn, dtype=torch.int64)
            for x in pull_all:
                ps += x[2 * r * Cn:2 * (r + 1) * Cn]
            self.pull_recv.copy_(ps.to(self.dev))
            for plane in self._rmx_planes():
                k = plane.numel() // G
                host = plane.cpu()
                parts = [torch.zeros_like(host) for _ in range(G)]
                dist.all_gather(parts, host)
                plane.copy_(torch.cat([parts[g][g * k:(g + 1) * k] for g in range(G)]).to(self.dev))
            if tick:
                snap = self.snap_all.cpu()
                snap_all = [torch.zeros_like(snap) for _ in range(G)]
                dist.all_gather(snap_all, snap)
                full = torch.cat([snap_all[g][g * Cn:(g + 1) * Cn] for g in range(G)])
                self.snap_all.copy_(full.to(self.dev))
            torch.cuda.synchronize(self.dev)
        self.rm_shadow.zero_()
        self.pull_shadow.zero_()
        check(lib().psim_demers_shard_ingest(self._h, self._p(self.rm_recv), self._p(self.pull_recv),
                                             self._p(self.rmx_all), 1 if tick else 0), self._h)

    def _rmx_planes(self):
        """The two rmx_all planes as separate views: [G C] int64, [G C] int32."""
        n = self.world * self.chunk
        return [self.rmx_all[:2 * n].view(self.torch.int64), self.rmx_all[2 * n:3 * n]]

    @staticmethod
    def _dist():
        import torch.distributed as dist
        return dist

    def _allreduce(self, vals):
        t = self.torch.tensor(vals, dtype=self.torch.int64, device=self.dev if self.backend == "nccl" else "cpu")
        self._dist().all_reduce(t)
        return t.tolist()

    # -------------------------------------------------------------- protocol
    def broadcast(self):
        if self.transport != "torch":
            check(lib().psim_demers_shard_broadcast_x(self._h), self._h)
            return
        check(lib().psim_demers_shard_broadcast_all(self._h, self._p(self.rm_shadow), self._p(self.rmx_all)), self._h)
        self._exchange(False)

    def step(self, rounds=1):
        """Rounds; returns per-round GLOBAL stats (summed over shards)."""
        if self.transport != "torch":
            st = (DemersStats * max(1, rounds))()
            check(lib().psim_demers_shard_step(self._h, rounds, st, rounds), self._h)
            out = [s_.as_dict() for s_ in st[:rounds]]
            for d in out:
                self.local_kernel_ms += d["kernel_ms"]
            return out
        out = []
        for _ in range(rounds):
            st = DemersStats()
            tick = C.c_uint32()
            check(lib().psim_demers_shard_round(self._h, self._p(self.rm_shadow), self._p(self.pull_shadow),
                                                self._p(self.snap_all), self._p(self.rmx_all), C.byref(st),
                                                C.byref(tick)), self._h)
            d = st.as_dict()
            self.local_kernel_ms += d["kernel_ms"]
            self.local_algo_bytes += d["algo_bytes"]
            self._exchange(bool(tick.value))
            keys = ["rm_sent", "push_sent", "pull_sent", "delivered_new", "complete", "algo_bytes"]
            g = dict(zip(keys, self._allreduce([d[k] for k in keys])))
            g["kernel_ms"] = d["kernel_ms"]
            out.append(g)
        return out

    def run(self, max_rounds=10000):
        if self.transport != "torch":
            st = (DemersStats * min(max_rounds, 4096))()
            ran = C.c_uint32()
            check(lib().psim_demers_shard_run(self._h, max_rounds, st, len(st), C.byref(ran)), self._h)
            out = [s_.as_dict() for s_ in st[:min(ran.value, len(st))]]
            for d in out:
                self.local_kernel_ms += d["kernel_ms"]
            return out, ran.value
        out = []
        while len(out) < max_rounds:
            out += self.step(1)
            if out[-1]["complete"] == self.n:
                break
        return out, len(out)

    def seen(self):
        """This shard's stores, global ids [v_lo, v_lo + n_local)."""
        out = np.zeros(self.n_local, np.uint64)
        check(lib().psim_demers_shard_get_seen(self._h, out.ctypes.data_as(C.POINTER(C.c_uint64)), self.n_local),
              self._h)
        return out

    def close(self):
        self.sim.close()
