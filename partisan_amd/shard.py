"""Vertex-sharded Plumtree over several GPUs, one process per GPU
(SURVEY 8(e)).

Transports (``transport=``):

* ``"rccl"`` (default with backend "nccl"): the exchange lives in libpsim --
  ``psim_shard_init_rccl`` gives the handle its own RCCL communicator (the
  unique id is shipped once over torch.distributed), and ``psim_shard_run``
  runs a whole heartbeat: round kernel -> pack -> grouped ncclSend/ncclRecv
  -> ingest on the handle's stream, counters all-reduced every 4 rounds,
  stop at GLOBAL quiescence;
* ``"callback"`` (default with backend "gloo", tests): the same in-library
  run loop, the words moved by Python callbacks (``psim_shard_set_transport``)
  over gloo, host-staged;
* ``"torch"``: the split-phase ABI driven from Python with torch.distributed
  collectives (the round-1 path, kept for A/B).

All stop at global quiescence, so the round count equals the single-GPU
engine's and the oracle's.
"""
import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

from ._lib import (ALLREDUCE_FN, ALLTOALLV_FN, PSIM_RCCL_ID_BYTES, ExchangeStats, RoundStats, Transport, check,
                   lib)
from .sim import Simulator


def gloo_transport():
    """psim_transport callbacks over the default torch.distributed group
    (host buffers).  Returns (Transport struct, keep-alive refs)."""
    def a2a(_ctx, send, soff, recv, roff, world):
        try:
            so = [int(soff[i]) for i in range(world + 1)]
            ro = [int(roff[i]) for i in range(world + 1)]
            sb = np.ctypeslib.as_array(send, shape=(max(so[-1], 1),))[:so[-1]].view(np.int32)
            rb = np.ctypeslib.as_array(recv, shape=(max(ro[-1], 1),))[:ro[-1]].view(np.int32)
            tr = torch.from_numpy(rb)
            dist.all_to_all_single(tr, torch.from_numpy(sb.copy()), [ro[i + 1] - ro[i] for i in range(world)],
                                   [so[i + 1] - so[i] for i in range(world)])
            return 0
        except Exception as e:  # noqa: BLE001 -- must not unwind through C
            print("psim gloo transport alltoallv:", repr(e), flush=True)
            return 1

    def ared(_ctx, vals, n):
        try:
            v = np.ctypeslib.as_array(vals, shape=(max(n, 1),))[:n]
            t = torch.from_numpy(v)
            dist.all_reduce(t)
            return 0
        except Exception as e:  # noqa: BLE001
            print("psim gloo transport allreduce:", repr(e), flush=True)
            return 1

    fa, fr = ALLTOALLV_FN(a2a), ALLREDUCE_FN(ared)
    return Transport(None, fa, fr), (fa, fr)


class ShardedPlumtree:
    def __init__(self, row_ptr, col, rank, world, device=0, backend="nccl", lazy_tick_rounds=1, transport=None,
                 csr=False, chunk_timing=False, max_roots=0, forest_lanes=0):
        """csr: keep CSR slot rows (PSIM_CFG_CSR) instead of the ELL rows every
        shard uses when the overlay's widest row has <= 8 slots.  chunk_timing:
        psim_shard_run times each 4-round chunk with one event pair and puts no
        marker between its kernels (PSIM_CFG_CHUNK_TIMING; kernel_ms then
        includes the exchange).  max_roots > 16: a sharded forest (every
        root's trees kept; broadcast_many heartbeats many roots at once,
        DESIGN.md 5.10)."""
        self.rank, self.world, self.backend = rank, world, backend
        self.transport = transport or ("rccl" if backend == "nccl" else "callback")
        self.dev = torch.device("cuda", device)
        # torch's HIP runtime first: brought up after libpsim's RCCL communicator
        # it finds no device (torch ships its own libamdhip64)
        torch.cuda.set_device(self.dev)
        self.sim = Simulator(lazy_tick_rounds=lazy_tick_rounds, device=device, rank=rank, world=world, csr=csr,
                             chunk_timing=chunk_timing, max_roots=max_roots, forest_lanes=forest_lanes)
        self._h = self.sim._h
        self.last_exchange = {}
        self.exchange_total = {}      # psim_exchange_stats summed over runs (this rank)
        if self.transport == "rccl":
            uid = (C.c_uint8 * PSIM_RCCL_ID_BYTES)()
            if rank == 0:
                check(lib().psim_rccl_unique_id(uid))
            if world > 1:
                box = [bytes(uid)]
                dist.broadcast_object_list(box, src=0)
                uid = (C.c_uint8 * PSIM_RCCL_ID_BYTES).from_buffer_copy(box[0])
            check(lib().psim_shard_init_rccl(self._h, rank, world, uid), self._h)
        elif self.transport == "callback":
            self._tp, self._keep = gloo_transport()
            check(lib().psim_shard_set_transport(self._h, C.byref(self._tp)), self._h)
        self.sim.load_overlay(row_ptr, col)
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
        # dense exchange: fixed word positions per remote slot, static split sizes
        rb = (C.c_uint64 * (world + 1))()
        check(lib().psim_shard_recv_layout(self._h, rb, world), self._h)
        self.rbase = [int(x) for x in rb]
        self.in_splits = [self.base[d + 1] - self.base[d] for d in range(world)]
        self.out_splits = [self.rbase[s + 1] - self.rbase[s] for s in range(world)]
        self.send_w = torch.zeros(max(1, self.base[world]), dtype=torch.int32, device=self.dev)
        self.recv_w = torch.zeros(max(1, self.rbase[world]), dtype=torch.int32, device=self.dev)
        self.chunk_rounds = 4
        if backend == "nccl" and self.transport == "torch":   # kernels and RCCL on torch's stream: no host sync per round
            check(lib().psim_set_stream(self._h, C.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)),
                  self._h)

    def transport_info(self):
        """{"kind", "world", "rank"} of the handle's exchange as the library
        reports it; for RCCL world / rank come from the communicator itself."""
        kind, w, r = C.c_int(), C.c_int(), C.c_int()
        check(lib().psim_shard_transport_info(self._h, C.byref(kind), C.byref(w), C.byref(r)), self._h)
        return {"kind": {0: "none", 1: "rccl", 2: "callback"}[kind.value], "world": w.value, "rank": r.value}

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

    def _exchange_dense(self):
        W = self.world
        if W == 1:
            return
        if self.backend == "nccl":
            dist.all_to_all_single(self.recv_w[:self.rbase[W]], self.send_w[:self.base[W]],
                                   self.out_splits, self.in_splits)
        else:
            torch.cuda.synchronize(self.dev)
            hs = self.send_w[:self.base[W]].cpu()
            hr = torch.zeros(self.rbase[W], dtype=torch.int32)
            dist.all_to_all_single(hr, hs, self.out_splits, self.in_splits)
            self.recv_w[:self.rbase[W]].copy_(hr.to(self.dev))
            torch.cuda.synchronize(self.dev)
        check(lib().psim_shard_ingest_dense(self._h, C.c_void_p(self.recv_w.data_ptr())), self._h)

    # -------------------------------------------------------------- protocol
    def reset_trees(self):
        self.sim.reset_trees()

    def set_alive(self, alive):
        self.sim.set_alive(alive)

    def set_delays(self, pairs, rounds):
        """Delay faults (psim_set_delays, collective: every rank passes the same
        global pairs; each installs its own senders').  Needs the in-library
        exchange: its stop rule waits for the delayed messages."""
        if self.transport == "torch":
            raise ValueError("delay faults need the in-library exchange (transport 'rccl' or 'callback')")
        self.sim.set_delays(pairs, rounds)

    def set_omissions(self, pairs):
        self.sim.set_omissions(pairs)

    def broadcast(self, root):
        mono = C.c_uint32()
        if self.transport != "torch":
            check(lib().psim_shard_broadcast_x(self._h, root, C.byref(mono)), self._h)
            return mono.value
        check(lib().psim_shard_broadcast_dense(self._h, root, C.byref(mono), C.c_void_p(self.send_w.data_ptr())),
              self._h)
        self._exchange_dense()
        return mono.value

    def broadcast_many(self, roots):
        """Heartbeats from many roots at once on a sharded forest (collective:
        every rank passes the same global roots); returns their ids."""
        return self.sim.broadcast_many(roots)

    def focus(self, root):
        """Point the getters at root's lane (this rank's vertex range)."""
        self.sim.focus(root)

    KEYS = ["broadcast", "prune", "i_have", "ignored_i_have", "graft", "delivered_new", "senders",
            "sender_degree_sum", "algo_bytes"]

    def run(self, max_rounds=100000):
        """Rounds until global quiescence; returns (per-round GLOBAL stats, rounds).

        Rounds are enqueued in chunks of `chunk_rounds` (kernel -> all-to-all ->
        ingest, stream-ordered) and their counters collected with one sync and
        one all-reduce per chunk; rounds after the first globally quiescent one
        changed nothing and are not counted (as in psim_run)."""
        if self.transport != "torch":
            return self._run_in_library(max_rounds)
        out, rounds = [], 0
        K = self.chunk_rounds
        keys = self.KEYS
        while rounds < max_rounds:
            k = min(K, max_rounds - rounds)
            for _ in range(k):
                check(lib().psim_shard_round_async(self._h, C.c_void_p(self.send_w.data_ptr())), self._h)
                self._exchange_dense()
            st = (RoundStats * k)()
            live = (C.c_int64 * k)()
            got = C.c_uint32()
            check(lib().psim_shard_collect(self._h, st, k, C.byref(got), live), self._h)
            loc = [s.as_dict() for s in st[:got.value]]
            flat = []
            for d, lv in zip(loc, live):
                flat += [d[x] for x in keys] + [int(lv)]
            g = self._allreduce(flat)
            done = False
            for i, d in enumerate(loc):
                row = g[i * (len(keys) + 1):(i + 1) * (len(keys) + 1)]
                gd = dict(zip(keys, row[:-1]))
                gd["kernel_ms"] = d["kernel_ms"]
                gd["live_rows"] = row[-1]
                out.append(gd)
                rounds += 1
                self.local_algo_bytes += d["algo_bytes"]
                self.local_kernel_ms += d["kernel_ms"]
                if sum(gd[x] for x in keys[:5]) == 0 and row[-1] == 0:
                    done = True
                    extra = len(loc) - (i + 1)
                    if extra:
                        check(lib().psim_shard_uncount(self._h, extra), self._h)
                    break
            if done:
                break
        return out, rounds

    def step(self, rounds=1):
        """Exactly `rounds` rounds (psim_shard_step, collective): GLOBAL per-round stats."""
        if self.transport == "torch":
            raise ValueError("step() needs the in-library exchange (transport 'rccl' or 'callback')")
        st = (RoundStats * max(1, rounds))()
        xs = ExchangeStats()
        check(lib().psim_shard_step(self._h, rounds, st, rounds, C.byref(xs)), self._h)
        return [s_.as_dict() for s_ in st[:rounds]]

    def _run_in_library(self, max_rounds, cap=4096):
        st = (RoundStats * cap)()
        ran = C.c_uint32()
        xs = ExchangeStats()
        check(lib().psim_shard_run(self._h, max_rounds, st, cap, C.byref(ran), C.byref(xs)), self._h)
        out = []
        for s_ in st[:min(ran.value, cap)]:
            d = s_.as_dict()
            self.local_algo_bytes += d["algo_bytes"]
            self.local_kernel_ms += d["kernel_ms"]
            out.append(d)
        self.last_exchange = xs.as_dict()
        for k, v in self.last_exchange.items():
            self.exchange_total[k] = self.exchange_total.get(k, 0) + v
        return out, ran.value

    def close(self):
        self.sim.close()
