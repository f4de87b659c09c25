"""Sparse-round worklist parity at a size where list mode engages.

Round 2 disagreed once between a plain handle and two shards by one i_have
after a heartbeat over the tree: a workgroup that read the running row-holder
count after another workgroup of the same launch had flushed took the group
flags while the others read the worklist, and visited a listed vertex that had
just gained rows a second time as "due".  The round mode is now decided from
a per-round holder ring written by earlier launches (psim_internal.h
kMcntHold).  These tests compare the HIP path with the oracle -- not with
another GPU path -- over a flood and two heartbeats over the tree, at L = 1
and 2, on 200k peers (ng / 8 = 1562 messages: the first and last rounds of
every heartbeat run in list mode):

* the plain handle, every round: per-kind counters, delivered set, accepted
  Round, eager / lazy / outstanding sets of every vertex and every in-flight
  word (oracle bulk views orc_pt_dump_state / orc_pt_inflight_words);
* the same with PSIM_WL_THR above every count (every round lists; tick rounds
  whose holders appear mid-round are the case that raced);
* two shards (gloo, the in-library loop psim_shard_step with seeded counts fed
  by the ingests), in 3-round calls so that the 2nd and 3rd rounds of each
  call read lists: per-round global counters every round, each shard's
  vertices and in-flight words at every call's end.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KINDS = ("broadcast", "prune", "i_have", "ignored_i_have", "graft")
N = 200_000
SEED = 0x5EED0200
ROOT_V = 4242


def sorted_layout(rp, col):
    """The handle's slot layout: each CSR row sorted by peer id."""
    rp = np.asarray(rp, dtype=np.int64)
    col = np.asarray(col, dtype=np.uint32)
    row = np.repeat(np.arange(len(rp) - 1), np.diff(rp))
    order = np.lexsort((col, row))
    return rp.astype(np.uint64), col[order]


def check_vertices(sim, orc, root, mono, srp, scol, lo, hi, tag):
    import pyoracle as O
    eager, lazy, outst, rr = sim.plumtree_state()
    oe, ol, oo, orr = orc.dump_state(root, mono, srp, scol, lo, hi)
    for name, g, o in (("eager", eager, oe), ("lazy", lazy, ol), ("outstanding", outst, oo), ("Round", rr, orr)):
        bad = np.nonzero(g != o)[0]
        assert len(bad) == 0, (tag, name, [(int(lo + v), int(g[v]), int(o[v])) for v in bad[:5]])
    assert np.array_equal(sim.delivered(), orc.delivered(root, mono)[lo:hi]), (tag, "delivered")
    gw = O.inflight_protocol_words(sim.inflight())
    ow = orc.inflight_words(srp, scol, lo, hi)
    bad = np.nonzero(gw != ow)[0]
    assert len(bad) == 0, (tag, "in-flight words", [(int(e), hex(int(gw[e])), hex(int(ow[e]))) for e in bad[:5]])


@pytest.mark.gpu
@pytest.mark.parametrize("force_list", [False, True])
def test_plain_handle_lockstep_200k(force_list, monkeypatch):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O

    import partisan_amd as pa
    if force_list:
        monkeypatch.setenv("PSIM_WL_THR", "100000000")
    rp, col = pa.overlay.random_regular(N, 5, SEED)
    srp, scol = sorted_layout(rp, col)
    listed = 0
    for L in (1, 2):
        sim = pa.Simulator(lazy_tick_rounds=L)
        sim.load_overlay(rp, col)
        assert np.array_equal(np.asarray(sim.slot_col, np.uint32), scol)
        orc = O.Plumtree(rp, col, L)
        for hb in range(3):
            mono = sim.broadcast(ROOT_V)
            assert mono == orc.heartbeat(ROOT_V)
            check_vertices(sim, orc, ROOT_V, mono, srp, scol, 0, N, (L, hb, 0))
            for rnd in range(1, 400):
                g, o = sim.step(1)[0], orc.step(1)[0]
                for k in KINDS + ("delivered_new",):
                    assert g[k] == o[k], (L, hb, rnd, k, g, o)
                check_vertices(sim, orc, ROOT_V, mono, srp, scol, 0, N, (L, hb, rnd))
                sent = sum(o[k] for k in KINDS)
                listed += 0 < sent < N // 16 // 8
                if sent == 0 and o["outstanding_live"] == 0:
                    break
            assert sim.delivered().all()
        sim.close()
        orc.close()
    assert listed > 10          # rounds the next round read as a list


def _shard_worker(rank, world, port, L, q):
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import pyoracle as O

        import partisan_amd as pa
        from partisan_amd.shard import ShardedPlumtree
        rp, col = pa.overlay.random_regular(N, 5, SEED)
        srp, scol = sorted_layout(rp, col)
        sp = ShardedPlumtree(rp, col, rank, world, device=0, backend="gloo", lazy_tick_rounds=L,
                             transport="callback", chunk_timing=True)
        sim = sp.sim
        lo, hi = sim.v_lo, sim.v_lo + sim.n
        orc = O.Plumtree(rp, col, L)
        for hb in range(3):
            mono = sp.broadcast(ROOT_V)
            assert mono == orc.heartbeat(ROOT_V)
            done = False
            call = 0
            while not done:
                call += 1
                gs = sp.step(3)
                os_ = orc.step(3)
                for i, (g, o) in enumerate(zip(gs, os_)):
                    for k in KINDS + ("delivered_new",):
                        assert g[k] == o[k], (L, hb, call, i, k, g, o)
                    if sum(o[k] for k in KINDS) == 0 and o["outstanding_live"] == 0:
                        done = True
                check_vertices(sim, orc, ROOT_V, mono, srp, scol, lo, hi, (rank, L, hb, call))
                assert call < 200
            assert sim.delivered().all()
        sp.close()
        orc.close()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "FAIL " + repr(e) + "\n" + traceback.format_exc()))


@pytest.mark.gpu
@pytest.mark.parametrize("L", [1, 2])
def test_two_shards_lockstep_200k(L):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_shard import run_world
    res = run_world(_shard_worker, 2, L, timeout=900)
    for r in range(2):
        assert res[r] == "ok", res[r]
