"""Vertex-sharded causal delivery (SURVEY 8(e), config C5's exchange).

GPU: world = 2 and 4 processes on ONE GPU (gloo) and world = 1 over RCCL;
every rank checks its range's clocks, buffers and delivery counts against
the oracle (oracle/causality.c) after every few rounds, and the per-round
counters summed over ranks against the oracle's.
"""
import os
import sys

import pytest

from test_shard import run_world

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("emitted", "received", "delivered", "checks", "buffered")


def _worker(rank, world, port, n, m, period, dmax, redeliver, backend, transport, q):
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
        from partisan_amd.causal import ShardedCausal
        import pyoracle as O
        seed = 0x5EED0005
        g = ShardedCausal(n, rank, world, m=m, period=period, dmax=dmax, redeliver=redeliver, device=0,
                          backend=backend, seed=seed, transport=transport)
        o = O.Causal(n, m, period=period, dmax=dmax, redeliver=redeliver, seed=seed)
        assert g.emitters.tolist() == [o.emitter(k) for k in range(m)]
        for _ in range(5):
            gs, os_ = g.step(4), o.step(4)
            for a, b in zip(gs, os_):
                for k in KEYS:
                    assert a[k] == b[k], (k, a, b)
            lanes, slf = g.clocks()
            dl = g.delivered()
            for lv in range(g.n_local):
                v = g.v_lo + lv
                assert g.clock(lv, lanes, slf) == sorted(o.clock(v)), v
                assert g.buffered(lv) == o.buffered(v), v
                assert int(dl[lv]) == o.delivered(v), v
        g.close()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "FAIL " + repr(e) + "\n" + traceback.format_exc()))


@pytest.mark.gpu
@pytest.mark.parametrize("world,n,m,period,dmax,redeliver,transport", [(2, 600, 16, 1, 4, 1, "callback"),
                                                                        (4, 1001, 64, 2, 5, 2, "callback"),
                                                                        (3, 500, 7, 3, 6, 1, "callback"),
                                                                        (2, 600, 16, 1, 4, 1, "torch")])
def test_sharded_causal_matches_oracle(world, n, m, period, dmax, redeliver, transport):
    """psim_causal_shard_step's exchange inside the library (gloo callbacks)
    and, for A/B, the split-phase entry points driven from Python."""
    res = run_world(_worker, world, n, m, period, dmax, redeliver, "gloo", transport)
    for r in range(world):
        assert res[r] == "ok", res[r]


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["rccl", "torch"])
def test_sharded_causal_nccl_world1(transport):
    res = run_world(_worker, 1, 800, 64, 1, 4, 1, "nccl", transport)
    assert res[0] == "ok", res[0]


def _overflow_worker(rank, world, port, q):
    """Only rank 1 lowers its buffer cap (PSIM_CS_BUFCAP, read when a round's
    arguments are built), so only its shard overflows; both ranks must leave
    psim_causal_shard_step with PSIM_EOVERFLOW (the failing shard
    used to return before the all-reduce, leaving rank 0 in it forever)."""
    try:
        sys.path.insert(0, ROOT)
        if rank == 1:
            os.environ["PSIM_CS_BUFCAP"] = "1"
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import partisan_amd as pa
        from partisan_amd.causal import ShardedCausal
        g = ShardedCausal(600, rank, world, m=16, period=1, dmax=4, redeliver=1, device=0, backend="gloo",
                          seed=0x5EED0005, transport="callback")
        try:
            g.step(12)
            q.put((rank, "no error"))
        except pa.PsimError as e:
            q.put((rank, e.name))
        g.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "FAIL " + repr(e) + "\n" + traceback.format_exc()))


@pytest.mark.gpu
def test_sharded_causal_one_shard_overflows():
    res = run_world(_overflow_worker, 2, timeout=240)
    assert res[0] == "PSIM_EOVERFLOW" and res[1] == "PSIM_EOVERFLOW", res
