"""Vertex-sharded Plumtree over several GPUs, one process per GPU
(SURVEY 8(e)).

The library runs each round split-phase (include/psim.h, "vertex
sharding"); this driver moves the cross-shard records with
torch.distributed -- backend "nccl" (RCCL over xGMI, device tensors) on a
node, or "gloo" (host-staged) in tests -- and stops at GLOBAL quiescence
(all-reduced emitted messages and live outstanding rows), so the round
count equals the single-GPU engine's and the oracle's.
"""
import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

from ._lib import RoundStats, check, lib
from .sim import Simulator


class ShardedPlumtree:
    def __init__(self, row_ptr, col, rank, world, device=0, backend="nccl", lazy_tick_rounds=1):
        self.rank, self.world, self.backend = rank, world, backend
        self.dev = torch.device("cuda", device)
        self.sim = Simulator(lazy_tick_rounds=lazy_tick_rounds, device=device, rank=rank, world=world)
        self.sim.load_overlay(row_ptr, col)
        self._h = self.sim._h
        base = (C.c_uint64 * (world + 1))()
        check(lib().psim_shard_layout(self._h, base, world), self._h)
        self.base = [int(x) for x in base]
        cap = max(1, self.base[world])
        self.send = torch.zeros(cap, dtype=torch.int64, device=self.dev)   # uint2 records {slot, word}
        self.recv = torch.zeros(cap, dtype=torch.int64, device=self.dev)
        self.cap = cap
        self.counts = (C.c_uint64 * world)()
        self.local_algo_bytes = 0      # this GPU's SURVEY 8(d) bytes over the rounds run
        self.local_kernel_ms = 0.0     # this GPU's pt_round_kernel time (hipEvent)

    # -------------------------------------------------------------- exchange
    def _allreduce(self, vals):
        t = torch.tensor(vals, dtype=torch.int64, device=self.dev if self.backend == "nccl" else "cpu")
        dist.all_reduce(t)
        return t.tolist()

    def _exchange(self):
        W, r = self.world, self.rank
        counts = [int(self.counts[d]) for d in range(W)]
        cdev = self.dev if self.backend == "nccl" else "cpu"
        mine = torch.tensor(counts, dtype=torch.int64, device=cdev)
        allc = [torch.zeros(W, dtype=torch.int64, device=cdev) for _ in range(W)]
        dist.all_gather(allc, mine)
        rcv = [int(allc[s][r]) for s in range(W)]
        # receive regions laid out by source, sized by what each source sends
        offs = np.concatenate([[0], np.cumsum(rcv)]).astype(np.int64)
        if int(offs[-1]) > self.recv.numel():
            self.recv = torch.zeros(int(offs[-1]), dtype=torch.int64, device=self.dev)
        ins = [self.send[self.base[d]:self.base[d] + counts[d]] for d in range(W)]
        outs = [self.recv[int(offs[s]):int(offs[s + 1])] for s in range(W)]
        if self.backend == "nccl":
            dist.all_to_all(outs, ins)
            torch.cuda.synchronize(self.dev)
        else:
            reqs = []
            host_out = [torch.zeros(rcv[s], dtype=torch.int64) for s in range(W)]
            for d in range(W):
                if d != r and counts[d]:
                    reqs.append(dist.isend(ins[d].cpu(), d))
            for s in range(W):
                if s != r and rcv[s]:
                    reqs.append(dist.irecv(host_out[s], s))
            for q in reqs:
                q.wait()
            for s in range(W):
                if rcv[s]:
                    outs[s].copy_(host_out[s].to(self.dev))
            torch.cuda.synchronize(self.dev)
        total = int(offs[-1])
        if total:
            check(lib().psim_shard_ingest(self._h, C.c_void_p(self.recv.data_ptr()), total), self._h)

    # -------------------------------------------------------------- protocol
    def reset_trees(self):
        self.sim.reset_trees()

    def set_alive(self, alive):
        self.sim.set_alive(alive)

    def broadcast(self, root):
        mono = C.c_uint32()
        live = C.c_int64()
        check(lib().psim_shard_broadcast(self._h, root, C.byref(mono), C.c_void_p(self.send.data_ptr()), self.cap,
                                         self.counts, C.byref(live)), self._h)
        self._exchange()
        return mono.value

    def run(self, max_rounds=100000):
        """Rounds until global quiescence; returns (per-round GLOBAL stats, rounds)."""
        out, rounds = [], 0
        st = RoundStats()
        live = C.c_int64()
        while rounds < max_rounds:
            check(lib().psim_shard_round(self._h, C.c_void_p(self.send.data_ptr()), self.cap, self.counts,
                                         C.byref(st), C.byref(live)), self._h)
            self._exchange()
            d = st.as_dict()
            self.local_algo_bytes += d["algo_bytes"]
            self.local_kernel_ms += d["kernel_ms"]
            keys = ["broadcast", "prune", "i_have", "ignored_i_have", "graft", "delivered_new", "senders",
                    "sender_degree_sum", "algo_bytes"]
            g = self._allreduce([d[k] for k in keys] + [int(live.value)])
            gd = dict(zip(keys, g[:-1]))
            gd["kernel_ms"] = d["kernel_ms"]
            gd["live_rows"] = g[-1]
            out.append(gd)
            rounds += 1
            if sum(gd[k] for k in keys[:5]) == 0 and g[-1] == 0:
                break
        return out, rounds

    def close(self):
        self.sim.close()
