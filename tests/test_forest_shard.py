"""Every node heartbeats on a SHARDED overlay (SURVEY 8(f) row 1 x 8(e);
VERDICT r5 "What's missing" 1): a forest handle (max_roots > 16) whose
vertices are split over several ranks.  One launch per round runs every
root's lane on each shard; every lane's cross-shard words move in ONE
all-to-all-v per round (lane after lane inside each destination's region);
counters are all-reduced per chunk.

GPU: world 2 and 3 gloo processes on one GPU, n = 600 with every vertex a
root, two intervals, lockstep against the oracle -- per-round message
counts by kind summed over roots AND ranks every round; every 4 rounds and
at the end of each interval, for every root this rank's slice of the eager
/ lazy sets, accepted Round and delivered set, the outstanding rows over
all roots, and the in-flight messages to this rank's vertices as a
multiset; then one root heartbeats a third time on its own -- as
tests/test_forest.py does on one GPU.  Plus a world-8 run of the C2-size
all-roots interval on one GPU (10k peers, 2k roots) whose per-round counts
and per-root state hashes equal the single-GPU forest's.
"""
import os
import sys

import numpy as np
import pytest

from test_shard import ROOT, _init, run_world

KINDS = ("broadcast", "prune", "i_have", "ignored_i_have", "graft")


def _forest_worker(rank, world, port, n, seed, L, q, lanes=0):
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        dist = _init(rank, world, port)
        import partisan_amd as pa
        from partisan_amd.shard import ShardedPlumtree
        import pyoracle as O
        rp, col = pa.overlay.random_regular(n, 5, seed)
        sp = ShardedPlumtree(rp, col, rank, world, device=0, backend="gloo", lazy_tick_rounds=L,
                             transport="callback", max_roots=n, forest_lanes=lanes)
        sim = sp.sim
        lo, hi = sim.v_lo, sim.v_lo + sim.n
        g = pa.Simulator(lazy_tick_rounds=L, device=0)      # the global slot layout (rows sorted by id)
        g.load_overlay(rp, col)
        grp, gcl = g.slot_row_ptr, g.slot_col
        g.close()
        orc = O.Plumtree(rp, col, L)

        def compare(monos, roots, inflight=True):
            ost_all = np.zeros(sim.n, np.uint32)
            for root in roots:
                sp.focus(root)
                e, l_, o, rr = sim.plumtree_state()
                oe, ol, oo, orr = orc.dump_state(root, monos[root], grp, gcl)
                assert np.array_equal(e, oe[lo:hi]), ("eager", rank, root)
                assert np.array_equal(l_, ol[lo:hi]), ("lazy", rank, root)
                assert np.array_equal(rr, orr[lo:hi]), ("Round", rank, root)
                assert np.array_equal(sim.delivered(), orc.delivered(root, monos[root])[lo:hi]), ("delivered", root)
                ost_all |= o
            oo = orc.dump_state(roots[0], monos[roots[0]], grp, gcl)[2]
            assert np.array_equal(ost_all, oo[lo:hi]), ("rows", rank)
            if inflight:
                got = []
                for root in roots:
                    sp.focus(root)
                    got += sim.decode_inflight()
                want = [(s_, d, t, r if t in (1, 3) else 0) for (s_, d, t, r) in orc.pending() if lo <= d < hi]
                assert sorted(got) == sorted(want), ("inflight", rank)

        def lockstep(monos, roots, full_every=4, max_rounds=60):
            rounds = 0
            while rounds < max_rounds:
                gs, os_ = sp.step(1)[0], orc.step(1)[0]
                rounds += 1
                for k in KINDS:
                    assert gs[k] == os_[k], (rank, rounds, k, gs, os_)
                assert gs["delivered_new"] == os_["delivered_new"], (rank, rounds)
                if rounds % full_every == 0:
                    compare(monos, roots)
                if sum(gs[k] for k in KINDS) == 0 and os_["outstanding_live"] == 0:
                    break
            return rounds

        with pytest.raises(pa.PsimError) as ei:           # delay faults: one GPU only
            sim.set_delays([(lo, int(sim.slot_col[0]))], [2])
        assert ei.value.name == "PSIM_ENOTSUP"
        roots = list(range(n))
        monos = {}
        if lanes:
            # parked roots (psim_forest_set_lanes): every root through `lanes`
            # lanes, a batch at a time, twice (the second interval in reverse
            # order, from the records each root kept while parked)
            for interval in range(2):
                order = roots if interval == 0 else roots[::-1]
                for b in range(0, n, lanes):
                    batch = order[b:b + lanes]
                    got = sp.broadcast_many(batch)
                    for r, m in zip(batch, got):
                        monos[r] = orc.heartbeat(r)
                        assert m == monos[r]
                    lockstep(monos, batch, full_every=6)
                compare(monos, roots)
            sp.close()
            dist.destroy_process_group()
            q.put((rank, "ok"))
            return
        for interval in range(2):
            got = sp.broadcast_many(roots)
            for r in roots:
                monos[r] = orc.heartbeat(r)
                assert got[r] == monos[r]
            lockstep(monos, roots)
            compare(monos, roots)
            for r in roots[:: max(1, n // 20)]:
                sp.focus(r)
                assert sim.delivered().all(), (interval, r)
        monos[7] = int(sp.broadcast_many([7])[0])
        assert monos[7] == orc.heartbeat(7)
        lockstep(monos, [7], full_every=1)
        # a run to quiescence through psim_shard_run: every root again
        got = sp.broadcast_many(roots)
        for r in roots:
            monos[r] = orc.heartbeat(r)
            assert got[r] == monos[r]
        gst, gr = sp.run()
        ost, orr = orc.run()
        assert gr == orr, (gr, orr)
        for a, b in zip(gst, ost):
            for k in KINDS:
                assert a[k] == b[k], (k, a, b)
        compare(monos, roots, inflight=False)
        sp.close()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "FAIL " + repr(e) + "\n" + traceback.format_exc()))


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("world,n,seed,L", [(2, 600, 3, 1), (3, 400, 4, 2)])
def test_sharded_forest_all_roots_lockstep(world, n, seed, L):
    res = run_world(_forest_worker, world, n, seed, L)
    for r in range(world):
        assert res[r] == "ok", res[r]


def _parked_worker(rank, world, port, n, seed, L, q):
    _forest_worker(rank, world, port, n, seed, L, q, lanes=16)


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_sharded_parked_forest_lockstep():
    """Parked roots on a sharded forest (world 2, n = 600, 16 lanes): the
    lanes' busy test and reuse agree on every rank (one all-reduce), and the
    result is the oracle's round by round."""
    res = run_world(_parked_worker, 2, 600, 3, 1)
    for r in range(2):
        assert res[r] == "ok", res[r]


def _c2all_worker(rank, world, port, n, k, q):
    try:
        sys.path.insert(0, ROOT)
        dist = _init(rank, world, port)
        import partisan_amd as pa
        from partisan_amd.shard import ShardedPlumtree
        rp, col = pa.overlay.random_regular(n, 5, 0xC2)
        sp = ShardedPlumtree(rp, col, rank, world, device=0, backend="gloo", transport="callback", max_roots=k)
        roots = list(range(0, n, n // k))[:k]
        sp.broadcast_many(roots)
        st, rounds = sp.run()
        counts = [[d[x] for x in KINDS + ("delivered_new",)] for d in st]
        hashes = []
        for r in roots[:: max(1, k // 50)]:
            sp.focus(r)
            hashes.append(list(sp.sim.trace_hash()[:3]))
        sp.close()
        dist.destroy_process_group()
        q.put((rank, {"rounds": rounds, "counts": counts, "hashes": hashes}))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "FAIL " + repr(e) + "\n" + traceback.format_exc()))


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_sharded_forest_world8_matches_one_gpu():
    """C2-size overlay (10k peers), 2,000 roots heartbeating at once: the
    world-8 sharded forest's rounds, global per-round counts and per-root
    state hashes (shards' sums) equal the single-GPU forest's."""
    import partisan_amd as pa
    n, k, world = 10_000, 2_000, 8
    res = run_world(_c2all_worker, world, n, k)
    for r in range(world):
        assert isinstance(res[r], dict), res[r]
    rp, col = pa.overlay.random_regular(n, 5, 0xC2)
    one = pa.Simulator(max_roots=k)
    one.load_overlay(rp, col)
    roots = list(range(0, n, n // k))[:k]
    one.broadcast_many(roots)
    st, rounds = one.run()
    assert res[0]["rounds"] == rounds
    assert res[0]["counts"] == [[d[x] for x in KINDS + ("delivered_new",)] for d in st]
    want = []
    for r in roots[:: max(1, k // 50)]:
        one.focus(r)
        want.append(list(one.trace_hash()[:3]))
    got = [[sum(res[q]["hashes"][i][j] for q in range(world)) % (1 << 64) for j in range(3)] for i in range(len(want))]
    assert got == want
    one.close()
