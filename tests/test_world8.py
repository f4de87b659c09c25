"""The configs' own 8-way splits, rehearsed on ONE GPU before the driver's
8-GPU run: eight rank processes, every one on device 0, the
exchanges inside libpsim over the gloo callback transport (the same
psim_transport hook RCCL replaces on an 8-GPU node).

* the bench overlay (10M peers, Plumtree flood + a heartbeat over the tree)
  at world 8 against the plain single-GPU handle: per-round global counts by
  kind and the summed trace hash (every shard's vertex states and in-flight
  words, keyed by global ids, add up to the plain handle's digest);
* C4 (10M peers, 64 rumors, Demers rumor mongering + anti-entropy) at world 8
  against the single-GPU run: the stores' digest, rounds and per-round new
  deliveries -- anti-entropy partners are uniform
  (protocols/demers_anti_entropy.erl:118-141), so 7/8 of the exchange crosses
  shards here;
* C5 (1M peers, 64 emitters, causal delivery) at world 8 against the
  single-GPU run: per-round counters and a digest of every clock and delivery
  count (src/partisan_causality_backend.erl:172-220).
"""
import os
import sys

import numpy as np
import pytest

from test_configs_at_scale import _demers_shard_worker, _digest
from test_shard import run_world

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KINDS = ("broadcast", "prune", "i_have", "ignored_i_have", "graft")
M64 = (1 << 64) - 1


def _split_sum(dist, torch, vals):
    """sum mod 2^64 of u64 values over the ranks (int64 all-reduce of 31-bit halves)."""
    t = torch.tensor([v & 0x7FFFFFFF for v in vals] + [v >> 31 for v in vals], dtype=torch.int64)
    dist.all_reduce(t)
    k = len(vals)
    return [(int(t[i]) + (int(t[k + i]) << 31)) & M64 for i in range(k)]


def _plumtree_worker(rank, world, port, n, q):
    try:
        sys.path.insert(0, ROOT)
        import torch
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        torch.empty(1, device="cuda:0")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import partisan_amd as pa
        from partisan_amd.shard import ShardedPlumtree
        rp, col = pa.overlay.random_regular(n, 5, 0x5EED0001)
        print(f"[world8 plumtree rank {rank}] overlay built", flush=True)
        sp = ShardedPlumtree(rp, col, rank, world, device=0, backend="gloo", transport="callback", chunk_timing=True)
        del rp, col
        print(f"[world8 plumtree rank {rank}] shard loaded", flush=True)
        rows = []
        hashes = []
        for hb in range(2):
            if hb == 0:
                sp.reset_trees()
            m = sp.broadcast(0)
            st, rounds = sp.run()
            rows.append((m, rounds, [[int(x[k]) for k in KINDS + ("delivered_new", "senders")] for x in st]))
            th = sp.sim.trace_hash()
            hashes.append(_split_sum(dist, torch, [int(th[0]), int(th[1]), int(th[2])]))
            print(f"[world8 plumtree rank {rank}] heartbeat {hb}: {rounds} rounds", flush=True)
        info = sp.transport_info()
        sp.close()
        dist.destroy_process_group()
        q.put((rank, {"rows": rows, "hashes": hashes, "world": info["world"]}))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "FAIL " + repr(e) + "\n" + traceback.format_exc()))


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_bench_overlay_world8_matches_plain_handle():
    import partisan_amd as pa
    n = 10_000_000
    rp, col = pa.overlay.random_regular(n, 5, 0x5EED0001)
    plain = pa.Simulator(device=0)
    plain.load_overlay(rp, col)
    del rp, col
    want_rows, want_hash = [], []
    for hb in range(2):
        if hb == 0:
            plain.reset_trees()
        m = plain.broadcast(0)
        st, rounds = plain.run()
        want_rows.append((m, rounds, [[int(x[k]) for k in KINDS + ("delivered_new", "senders")] for x in st]))
        want_hash.append([int(x) for x in plain.trace_hash()[:3]])
    plain.close()
    res = run_world(_plumtree_worker, 8, n, timeout=900)
    for r in range(8):
        assert not isinstance(res[r], str), res[r]
        assert res[r]["rows"] == want_rows, (r, res[r]["rows"][0][:2], want_rows[0][:2])
        assert res[r]["hashes"] == want_hash, (r, res[r]["hashes"], want_hash)


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_c4_10m_world8_matches_single_gpu():
    import partisan_amd as pa
    n, m = 10_000_000, 64
    sim = pa.Simulator(seed=0x5EED0004, device=0)
    dm = pa.demers.DemersEpidemic(sim, n, m, 2, True)
    dm.broadcast()
    st, rounds = dm.run(200)
    want = _digest(dm.seen(), 0)
    want_new = [s["delivered_new"] for s in st]
    sim.close()
    res = run_world(_demers_shard_worker, 8, n, m, timeout=900)
    for r in range(8):
        assert not isinstance(res[r], str), res[r]
    assert sum(res[r][0] for r in range(8)) % (1 << 64) == want
    for r in range(8):
        assert res[r][1] == rounds
        assert res[r][2] == want_new
        assert res[r][3] == n


def _clock_digest(lanes, slf, dl, v_lo):
    """sum over vertices of a mix of (global id, dense clock, own counter, deliveries)."""
    with np.errstate(over="ignore"):
        k = np.arange(lanes.shape[1], dtype=np.uint64)
        h = (lanes.astype(np.uint64) * (k * np.uint64(0x9E3779B97F4A7C15) + np.uint64(1))).sum(axis=1, dtype=np.uint64)
        z = (np.arange(len(slf), dtype=np.uint64) + np.uint64(v_lo)) * np.uint64(0xBF58476D1CE4E5B9)
        z ^= h ^ (slf.astype(np.uint64) << np.uint64(32)) ^ (dl.astype(np.uint64) * np.uint64(0x94D049BB133111EB))
        z = (z ^ (z >> np.uint64(29))) * np.uint64(0xBF58476D1CE4E5B9)
        z ^= z >> np.uint64(32)
        return int(z.sum(dtype=np.uint64))


C5 = dict(m=64, period=1, dmax=4, redeliver=1)
C5_ROUNDS = 12
C5_KEYS = ("emitted", "received", "delivered", "checks", "buffered")


def _causal_worker(rank, world, port, n, q):
    try:
        sys.path.insert(0, ROOT)
        import torch
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        torch.empty(1, device="cuda:0")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from partisan_amd.causal import ShardedCausal
        g = ShardedCausal(n, rank, world, device=0, backend="gloo", seed=0x5EED0005, transport="callback", **C5)
        st = []
        for i in range(C5_ROUNDS):
            st += g.step(1)
            print(f"[world8 causal rank {rank}] round {i + 1}", flush=True)
        lanes, slf = g.clocks()
        d = _clock_digest(lanes[:g.n_local], slf[:g.n_local], g.delivered(), g.v_lo)
        g.close()
        dist.destroy_process_group()
        q.put((rank, ([[int(x[k]) for k in C5_KEYS] for x in st], d)))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "FAIL " + repr(e) + "\n" + traceback.format_exc()))


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_c5_1m_world8_matches_single_gpu():
    import partisan_amd as pa
    from partisan_amd.causal import CausalCluster
    n = 1_000_000
    sim = pa.Simulator(seed=0x5EED0005, device=0)
    c = CausalCluster(sim, n, **C5)
    st = c.step(C5_ROUNDS)
    want_rows = [[int(x[k]) for k in C5_KEYS] for x in st]
    lanes, slf = c.clocks()
    want = _clock_digest(lanes, slf, c.delivered(), 0)
    sim.close()
    assert want_rows[-1][2] > 0                     # deliveries happened
    res = run_world(_causal_worker, 8, n, timeout=900)
    for r in range(8):
        assert not isinstance(res[r], str), res[r]
        assert res[r][0] == want_rows, (r, res[r][0][-1], want_rows[-1])
    assert sum(res[r][1] for r in range(8)) % (1 << 64) == want
