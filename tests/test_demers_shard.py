"""Vertex-sharded Demers epidemic (SURVEY 8(e), config C4's exchange).

GPU: world = 2, 3 and 4 processes on ONE GPU, and world = 1 over RCCL (the
nccl code path).  The exchange runs inside libpsim on the handle's transport
(psim_demers_shard_step: gloo callbacks / the library's RCCL communicator)
or, for A/B, from Python (transport "torch"); every rank checks its vertex range of the
stores against the oracle (oracle/demers.c) after every round, and the
per-round message counters summed over ranks against the oracle's.

CPU: world = 2 gloo processes drive ShardedDemers' exchange with the library
mocked out: RM slices are routed to their owner and OR-merged, pull slots
reduce-scattered, snapshots all-gathered.
"""
import os
import sys

import numpy as np
import pytest

from test_shard import free_port, run_world  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("rm_sent", "push_sent", "pull_sent", "delivered_new", "complete")


def _gpu_worker(rank, world, port, n, m, ae, rm, backend, transport, *rest):
    q, xmode = rest[-1], (rest[0] if len(rest) > 1 else "auto")      # run_world appends the queue
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import torch
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        if backend == "nccl":
            torch.cuda.set_device(0)
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        from partisan_amd.demers import ShardedDemers
        import pyoracle as O
        seed = 0x5EED0004
        sd = ShardedDemers(n, m, rank, world, device=0, backend=backend, ae_period=ae, rumor_mongering=rm, seed=seed,
                           transport=transport)
        if transport != "torch":
            sd.set_exchange(xmode)
        orc = O.Demers(n, m, seed, ae_period=ae, rm_on=rm)
        lo, hi = sd.v_lo, sd.v_lo + sd.n_local
        sd.broadcast()
        orc.broadcast_all()
        assert np.array_equal(sd.seen(), orc.seen()[lo:hi])
        for r in range(200):
            g = sd.step(1)[0]
            o = orc.step(1)[0]
            for k in KEYS:
                assert g[k] == o[k], (r, k, g, o)
            assert np.array_equal(sd.seen(), orc.seen()[lo:hi]), r
            if o["complete"] == n:
                break
        if transport != "torch" and world > 1:
            nbytes, ex, sp_rm, sp_calls = sd.exchange_stats()
            assert ex == r + 2 and nbytes > 0, (ex, r, nbytes)      # the broadcast's exchange + one per round
            if xmode == "records":
                assert sp_rm == ex and sp_calls == ex, (ex, sp_rm, sp_calls)
            elif xmode == "dense" or not rm:
                assert sp_rm == 0 and sp_calls == 0, (sp_rm, sp_calls)
            else:     # auto: the first and last rounds reach few slots, the middle ones most
                assert 0 < sp_rm < ex and 0 < sp_calls < ex, (ex, sp_rm, sp_calls)
        sd.close()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "FAIL " + repr(e) + "\n" + traceback.format_exc()))


@pytest.mark.gpu
@pytest.mark.parametrize("world,n,m,ae,rm,transport", [(2, 3000, 64, 2, True, "callback"),
                                                        (4, 5001, 64, 2, True, "callback"),
                                                        (3, 2000, 17, 3, False, "callback"),
                                                        (2, 2500, 64, 0, True, "callback"),
                                                        (2, 3000, 64, 2, True, "torch"),
                                                        (3, 2000, 17, 3, False, "torch")])
def test_sharded_demers_matches_oracle(world, n, m, ae, rm, transport):
    res = run_world(_gpu_worker, world, n, m, ae, rm, "gloo", transport)
    for r in range(world):
        assert res[r] == "ok", res[r]


# the same rounds with the RM planes and call records always as records, and
# always dense: both equal the oracle (auto, above, mixes the two)
@pytest.mark.gpu
@pytest.mark.parametrize("world,xmode", [(2, "records"), (3, "records"), (2, "dense")])
def test_sharded_demers_exchange_forms(world, xmode):
    res = run_world(_gpu_worker, world, 3000, 64, 2, True, "gloo", "callback", xmode)
    for r in range(world):
        assert res[r] == "ok", res[r]


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["rccl", "torch"])
def test_sharded_demers_nccl_world1(transport):
    res = run_world(_gpu_worker, 1, 4000, 64, 2, True, "nccl", transport)
    assert res[0] == "ok", res[0]


# ------------------------------------------------------------------ CPU gloo
def _cpu_worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        import torch
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from partisan_amd import demers

        seen = {}

        class FakeLib:
            def psim_demers_shard_ingest(self, h, rm_ptr, pull_ptr, rmx_ptr, tick):
                seen["tick"] = tick
                return 0

        G, Cn = world, 5
        sd = demers.ShardedDemers.__new__(demers.ShardedDemers)
        sd.torch, sd.rank, sd.world, sd.backend, sd.chunk = torch, rank, world, "gloo", Cn
        sd.dev, sd._h = torch.device("cpu"), None
        z = lambda *s: torch.zeros(*s, dtype=torch.int64)  # noqa: E731
        sd.rm_shadow, sd.rm_recv = z(3, G * Cn), z(3, G * Cn)
        sd.pull_shadow, sd.pull_recv, sd.snap_all = z(2 * G * Cn), z(2 * Cn), z(G * Cn)
        sd.rmx_all = torch.zeros(3 * G * Cn, dtype=torch.int32)
        rmx64, rmx32 = sd._rmx_planes()
        rmx64[rank * Cn:(rank + 1) * Cn] = (1 << 40) + rank      # this shard's call records, both planes
        rmx32[rank * Cn:(rank + 1) * Cn] = 50 + rank
        # rank r sets bit r of every RM entry and writes pull slot values r+1
        # into the slots of vertex 2*rank+1 of every shard; snapshot of its own slice
        for k in range(3):
            sd.rm_shadow[k] = 1 << (rank + 4 * k)
        for g in range(G):
            sd.pull_shadow[2 * (g * Cn + rank)] = 100 * (rank + 1) + g
        sd.snap_all[rank * Cn:(rank + 1) * Cn] = 7 + rank
        orig_lib, orig_sync = demers.lib, torch.cuda.synchronize
        demers.lib = lambda: FakeLib()
        torch.cuda.synchronize = lambda *a, **k: None
        try:
            sd._exchange(True)
        finally:
            demers.lib = orig_lib
            torch.cuda.synchronize = orig_sync
        for k in range(3):
            want = sum(1 << (s + 4 * k) for s in range(G))
            # slice g came from shard g and holds that shard's bit; their OR is the inbox
            got = 0
            for g in range(G):
                sl = sd.rm_recv[k, g * Cn:(g + 1) * Cn]
                assert (sl == (1 << (g + 4 * k))).all()
                got |= int(sl[0])
            assert got == want
        for s in range(G):
            assert int(sd.pull_recv[2 * s]) == 100 * (s + 1) + rank
        for g in range(G):
            assert (sd.snap_all[g * Cn:(g + 1) * Cn] == 7 + g).all()
            assert (rmx64[g * Cn:(g + 1) * Cn] == (1 << 40) + g).all()     # all-gathered in slices of C
            assert (rmx32[g * Cn:(g + 1) * Cn] == 50 + g).all()
        assert int(sd.rm_shadow.abs().sum()) == 0 and int(sd.pull_shadow.abs().sum()) == 0
        assert seen["tick"] == 1
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "FAIL " + repr(e) + "\n" + traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
def test_demers_exchange_routing_gloo_cpu(world):
    res = run_world(_cpu_worker, world, timeout=120)
    for r in range(world):
        assert res[r] == "ok", res[r]


def _overflow_worker(rank, world, port, q):
    """Only rank 1 lowers the anti-entropy push cap (PSIM_DM_PUSHCAP=1: any
    vertex pushed to twice in a tick overflows), so only its shard fails the
    round; every rank must leave psim_demers_shard_step with PSIM_EOVERFLOW
    instead of waiting in the exchange's collectives."""
    try:
        sys.path.insert(0, ROOT)
        if rank == 1:
            os.environ["PSIM_DM_PUSHCAP"] = "1"
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import partisan_amd as pa
        from partisan_amd.demers import ShardedDemers
        sd = ShardedDemers(3000, 64, rank, world, device=0, backend="gloo", ae_period=2, rumor_mongering=True,
                           seed=0x5EED0004, transport="callback")
        sd.broadcast()
        try:
            sd.step(8)
            q.put((rank, "no error"))
        except pa.PsimError as e:
            q.put((rank, e.name))
        sd.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "FAIL " + repr(e) + "\n" + traceback.format_exc()))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_demers_one_shard_overflows(world):
    res = run_world(_overflow_worker, world, timeout=240)
    assert all(res[r] == "PSIM_EOVERFLOW" for r in range(world)), res
