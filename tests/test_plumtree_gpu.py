"""Parity of the HIP Plumtree path (libpsim.so via the C ABI) with the CPU
oracle (oracle/plumtree.c), round by round, bit-exact.

Compared after every round: delivered set, Round of the accepted broadcast,
eager and lazy peer sets of every vertex for the root, outstanding i_have
rows (peer and Round), the full set of messages in flight (src, dst, kind,
Round) in FIFO order, and the per-kind message counters.  Plumtree traces
are not pinned by any reference test (SURVEY 8(c) "Unpinned"): the oracle is
the reference restatement these are checked against.
"""
import numpy as np
import pytest

import pyoracle as O

pytestmark = pytest.mark.gpu

KINDS = ("broadcast", "prune", "i_have", "ignored_i_have", "graft")


@pytest.fixture(scope="module", params=["slot_scatter", "slot_scatter_csr", "binned"])
def psim(request):
    """partisan_amd with Simulator bound to one Plumtree engine: the
    slot-scatter engine (the default: ELL rows when every degree is <= 8),
    the same with CSR rows (PSIM_CFG_CSR; what sharded handles run) and the
    binned one (PSIM_CFG_BINNED) must all match the oracle."""
    import functools
    import types

    import partisan_amd
    ns = types.SimpleNamespace(**{k: getattr(partisan_amd, k) for k in dir(partisan_amd) if not k.startswith("__")})
    kw = {"slot_scatter": {}, "slot_scatter_csr": {"csr": True}, "binned": {"binned": True}}
    ns.Simulator = functools.partial(partisan_amd.Simulator, **kw[request.param])
    ns.engine = request.param
    return ns


def make(psim, rp, col, L=1):
    sim = psim.Simulator(lazy_tick_rounds=L)
    sim.load_overlay(rp, col)
    orc = O.Plumtree(rp, col, lazy_tick_rounds=L)
    return sim, orc


def compare(sim, orc, root, mono):
    n = sim.n
    eager, lazy, outst, rr = sim.plumtree_state()
    assert np.array_equal(sim.delivered(), orc.delivered(root, mono)), "delivered sets differ"
    orr = orc.recv_round(root, mono)
    for v in range(n):
        oe, ol = orc.peers(v, root)
        assert sim.mask_to_peers(v, eager[v]) == oe, f"eager set of {v}"
        assert sim.mask_to_peers(v, lazy[v]) == ol, f"lazy set of {v}"
        rows = orc.outstanding(v)
        assert sim.mask_to_peers(v, outst[v]) == sorted({p for p, _, _ in rows}), f"outstanding of {v}"
        if orr[v] == 0xFFFFFFFF:
            assert rr[v] == 0xFFFF, v
        elif orr[v] == 0xFFFFFFFE:
            assert rr[v] == 0xFFFE, v
        else:
            assert rr[v] == orr[v], v
        if rows:
            my_round = 0 if rr[v] == 0xFFFE else int(rr[v]) + 1
            assert {r for _, r, _ in rows} == {my_round}, v
            assert {m for _, _, m in rows} == {mono}, v
    want = [(s, d, t, r if t in (1, 3) else 0) for (s, d, t, r) in orc.pending()]
    assert sim.decode_inflight() == want, "in-flight messages differ"


def lockstep(sim, orc, root, mono, max_rounds=200):
    rounds = 0
    while rounds < max_rounds:
        gs = sim.step(1)[0]
        os_ = orc.step(1)[0]
        rounds += 1
        for k in KINDS:
            assert gs[k] == os_[k], (rounds, k, gs, os_)
        assert gs["delivered_new"] == os_["delivered_new"]
        compare(sim, orc, root, mono)
        if sum(gs[k] for k in KINDS) == 0 and os_["outstanding_live"] == 0:
            break
    return rounds


@pytest.mark.parametrize("n,seed,L", [(40, 1, 1), (300, 2, 1), (300, 3, 2), (1500, 4, 3), (1000, 5, 1)])
def test_flood_then_tree_lockstep(psim, n, seed, L):
    rp, col = psim.overlay.random_regular(n, 5, seed)
    sim, orc = make(psim, rp, col, L)
    root = seed % n
    for _ in range(3):          # flood, then two heartbeats over the pruned tree
        mono_g = sim.broadcast(root)
        mono_o = orc.heartbeat(root)
        assert mono_g == mono_o
        compare(sim, orc, root, mono_o)
        lockstep(sim, orc, root, mono_o)


def test_dead_vertices_lockstep(psim):
    n = 800
    rp, col = psim.overlay.random_regular(n, 5, 11)
    sim, orc = make(psim, rp, col, 1)
    root = 3
    m = sim.broadcast(root)
    orc.heartbeat(root)
    lockstep(sim, orc, root, m)
    rng = np.random.default_rng(7)
    alive = np.ones(n, np.uint8)
    alive[rng.choice(n, n // 10, replace=False)] = 0
    alive[root] = 1
    sim.set_alive(alive)
    orc.set_alive(alive)
    m = sim.broadcast(root)
    assert m == orc.heartbeat(root)
    lockstep(sim, orc, root, m)


def test_ring_lattice_long_rounds(psim):
    rp, col = psim.overlay.ring_lattice(600, 2)
    sim, orc = make(psim, rp, col, 2)
    for _ in range(2):
        m = sim.broadcast(0)
        orc.heartbeat(0)
        lockstep(sim, orc, 0, m, max_rounds=1000)


def test_complete_graph_c1(psim):
    # config C1: 16 nodes, full membership (degree 15)
    rp, col = psim.overlay.complete(16)
    sim, orc = make(psim, rp, col, 1)
    for _ in range(3):
        m = sim.broadcast(0)
        orc.heartbeat(0)
        lockstep(sim, orc, 0, m)


def test_reset_trees_and_root_change(psim):
    rp, col = psim.overlay.random_regular(500, 5, 21)
    sim, orc = make(psim, rp, col, 1)
    for root, reset in [(7, False), (7, True), (9, False), (9, False)]:
        if reset:
            sim.reset_trees()
            orc.reset_peers_all()
        if root != getattr(sim, "_last_root", root) and psim.engine == "binned":
            orc.reset_peers_all()      # one lane: a new root drops the old root's sets
        sim._last_root = root
        m = sim.broadcast(root)
        assert m == orc.heartbeat(root)
        lockstep(sim, orc, root, m)


def test_run_matches_oracle_round_count(psim):
    rp, col = psim.overlay.random_regular(5000, 5, 31)
    for L in (1, 3):
        sim, orc = make(psim, rp, col, L)
        for _ in range(3):
            sim.broadcast(17)
            m = orc.heartbeat(17)
            gst, gr = sim.run()
            ost, orr = orc.run()
            assert gr == orr
            for g, o in zip(gst, ost):
                for k in KINDS:
                    assert g[k] == o[k]
            compare(sim, orc, 17, m)


def test_busy_until_quiescent(psim):
    """A root heartbeating while its last heartbeat is in flight: the binned
    engine keeps one heartbeat per root (PSIM_EBUSY until quiescent); the
    slot-scatter engine turns the lane into a window lane and both floods
    complete."""
    rp, col = psim.overlay.random_regular(200, 5, 41)
    sim = psim.Simulator()
    sim.load_overlay(rp, col)
    m1 = sim.broadcast(0)
    if psim.engine == "binned":
        with pytest.raises(psim.PsimError) as ei:
            sim.broadcast(0)
        assert ei.value.name == "PSIM_EBUSY"
        sim.run()
        sim.broadcast(0)
        return
    m2 = sim.broadcast(0)
    sim.run()
    assert sim.delivered_mono(m1).all() and sim.delivered_mono(m2).all()
    with pytest.raises(psim.PsimError):
        sim.inflight()                  # a window lane has no per-slot word view: psim_get_messages


def test_facade_mirrors_reference_api(psim):
    rp, col = psim.overlay.random_regular(300, 5, 51)
    pt = psim.PlumtreeBroadcast(rp, col)
    orc = O.Plumtree(rp, col, 1)
    msg_id = pt.broadcast(4)
    orc.heartbeat(4)
    pt.run()
    orc.run()
    for v in (0, 4, 100, 299):
        assert pt.get_peers(v, 4) == orc.peers(v, 4)
        assert pt.get_eager_peers(v, 4) == orc.peers(v, 4)[0]
        assert pt.handler(v).is_stale(msg_id)
        assert pt.handler(v).graft(msg_id) == ("ok", msg_id)
        assert pt.exchanges(v) == []
    assert pt.broadcast_channel() == "partisan_membership"
    with pytest.raises(NotImplementedError):
        psim.PlumtreeBroadcast(rp, col, mods=[object])


@pytest.mark.parametrize("n", [100_000])
def test_large_final_state_parity(psim, n):
    rp, col = psim.overlay.random_regular(n, 5, 61)
    sim, orc = make(psim, rp, col, 1)
    for _ in range(2):
        sim.broadcast(0)
        m = orc.heartbeat(0)
        _, gr = sim.run()
        _, orr = orc.run()
        assert gr == orr
    eager, lazy, outst, rr = sim.plumtree_state()
    assert np.array_equal(sim.delivered(), orc.delivered(0, m))
    orr = orc.recv_round(0, m)
    got = np.where(rr == 0xFFFF, 0xFFFFFFFF, np.where(rr == 0xFFFE, 0xFFFFFFFE, rr.astype(np.int64)))
    assert np.array_equal(got.astype(np.uint64), orr.astype(np.uint64))
    rng = np.random.default_rng(0)
    for v in rng.choice(n, 2000, replace=False).tolist():
        oe, ol = orc.peers(v, 0)
        assert sim.mask_to_peers(v, eager[v]) == oe
        assert sim.mask_to_peers(v, lazy[v]) == ol


def popcount32(x):
    x = x.astype(np.uint64)
    c = np.zeros_like(x)
    for i in range(32):
        c += (x >> np.uint64(i)) & np.uint64(1)
    return c


@pytest.mark.parametrize("n", [2_000_000])
def test_large_flood_properties(psim, n):
    """Size-independent properties at scale: after a flood from a fresh state
    every vertex delivered, no row is outstanding, and the eager graph is a
    spanning tree (2(n-1) directed eager edges, each vertex's Round = its
    parent's + 1)."""
    rp, col = psim.overlay.random_regular(n, 5, 71)
    sim = psim.Simulator()
    sim.load_overlay(rp, col)
    sim.broadcast(0)
    stats, rounds = sim.run()
    assert sim.delivered().all()
    eager, lazy, outst, rr = sim.plumtree_state()
    assert not outst.any()
    assert int(popcount32(eager).sum()) == 2 * (n - 1)
    assert sum(s["delivered_new"] for s in stats) == n - 1
    assert stats[-1]["broadcast"] == 0


M64 = (1 << 64) - 1


def _mix(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def trace_hash_ref(sim):
    """psim_trace_hash recomputed on the host from the getters (include/psim.h)."""
    eager, lazy, outst, rr = sim.plumtree_state()
    h0 = 0
    for v in range(sim.n):
        g = v + sim.v_lo
        h0 = (h0 + _mix(_mix(_mix(int(outst[v])) ^ (int(eager[v]) << 32 | int(lazy[v]))) ^ (g << 32 | int(rr[v])))) & M64
    words = sim.inflight()
    h1 = 0
    for e in np.nonzero(words)[0].tolist():
        h1 = (h1 + _mix(((e + sim.slot_base) << 32) | int(words[e]))) & M64
    return h0, h1, int(sim.delivered().sum())


def test_trace_hash_matches_getters(psim):
    rp, col = psim.overlay.random_regular(3000, 5, 81)
    sim, orc = make(psim, rp, col, 1)
    sim.broadcast(7)
    for _ in range(12):
        sim.step(1)
        th = sim.trace_hash()
        assert th[:3] == trace_hash_ref(sim)


def test_trace_hash_engines_agree_at_scale():
    """The engines at 2M peers, round by round, compared by digest only."""
    import partisan_amd
    rp, col = partisan_amd.overlay.random_regular(2_000_000, 5, 91)
    sims = [partisan_amd.Simulator(), partisan_amd.Simulator(csr=True), partisan_amd.Simulator(binned=True)]
    for s in sims:
        s.load_overlay(rp, col)
    for root in (0, 12345):
        for s in sims:
            s.reset_trees()
            s.broadcast(root)
        for _ in range(40):
            st = [s.step(1)[0] for s in sims]
            for k in KINDS + ("delivered_new", "active", "senders"):
                assert len({x[k] for x in st}) == 1, k
            th = [s.trace_hash() for s in sims]
            assert all(t == th[0] for t in th), th
            if sum(st[0][k] for k in KINDS) == 0:
                break
    for s in sims:
        s.close()


def _omit_step(sim, orc, root, mono, rounds):
    for r in range(rounds):
        gs, os_ = sim.step(1)[0], orc.step(1)[0]
        for k in KINDS:
            assert gs[k] == os_[k], (r, k, gs, os_)
        assert gs["delivered_new"] == os_["delivered_new"], r
        compare(sim, orc, root, mono)


def test_omission_faults_lockstep(psim):
    """Send/receive omission faults (prop_partisan_crash_fault_model.erl
    :117-196) on 10 % of the directed edges during a flood, then healed: the
    omitted messages are counted as sent and lost, round by round as in the
    oracle; after the heal the lazy ticks' i_have/graft repair the tree."""
    rp, col = psim.overlay.random_regular(1500, 5, 101)
    sim, orc = make(psim, rp, col, 1)
    rng = np.random.default_rng(5)
    src = np.repeat(np.arange(sim.n), np.diff(sim.slot_row_ptr.astype(np.int64)))
    pick = rng.random(len(src)) < 0.10
    pairs = np.stack([src[pick], sim.slot_col[pick]], axis=1)
    sim.set_omissions(pairs)
    orc.set_omissions(pairs)
    sim.broadcast(3)
    mono = orc.heartbeat(3)
    _omit_step(sim, orc, 3, mono, 14)
    assert orc.omitted() > 0
    sim.set_omissions([])
    orc.set_omissions([])
    lockstep(sim, orc, 3, mono)
    assert sim.delivered().all()


def test_partition_then_heal(psim):
    """inject_partition: a flood from vertex 0 stays on its side while the
    partition holds (same delivered sets as the oracle).  Eager pushes lost on
    the cut leave no outstanding row (only lazy peers get rows), so after the
    heal only i_have over lazy links crosses -- as in the oracle; the next
    heartbeat then reaches every vertex (the reliable-broadcast postcondition,
    prop_partisan_reliable_broadcast.erl:127-172, holds from there)."""
    rp, col = psim.overlay.random_regular(2000, 5, 111)
    sim, orc = make(psim, rp, col, 1)
    group = (np.arange(2000) >= 1000).astype(np.int64)
    pairs = sim.partition_pairs(group)
    sim.inject_partition(group)
    orc.set_omissions(pairs)
    sim.broadcast(0)
    mono = orc.heartbeat(0)
    _omit_step(sim, orc, 0, mono, 20)
    d = sim.delivered()
    assert not d[1000:].any() and d[:1000].sum() > 900   # side 0 minus vertices cut off inside it
    sim.resolve_partition()
    orc.set_omissions([])
    lockstep(sim, orc, 0, mono)
    sim.broadcast(0)
    mono = orc.heartbeat(0)
    lockstep(sim, orc, 0, mono)
    assert sim.delivered().all()


def _multi_compare(sim, orc, monos):
    """Per root: delivered set, Round, eager / lazy sets; all roots together:
    outstanding peers per vertex and the in-flight messages (as a multiset:
    lanes keep no FIFO order across roots, which no per-root state depends on)."""
    n = sim.n
    outst_all = [set() for _ in range(n)]
    inflight = []
    for root, mono in monos.items():
        sim.focus(root)
        eager, lazy, outst, rr = sim.plumtree_state()
        assert np.array_equal(sim.delivered(), orc.delivered(root, mono)), root
        orr = orc.recv_round(root, mono)
        got = np.where(rr == 0xFFFF, 0xFFFFFFFF, np.where(rr == 0xFFFE, 0xFFFFFFFE, rr.astype(np.int64)))
        assert np.array_equal(got.astype(np.uint64), orr.astype(np.uint64)), root
        for v in range(n):
            oe, ol = orc.peers(v, root)
            assert sim.mask_to_peers(v, eager[v]) == oe, (root, v)
            assert sim.mask_to_peers(v, lazy[v]) == ol, (root, v)
            outst_all[v] |= set(sim.mask_to_peers(v, outst[v]))
        inflight += sim.decode_inflight()
    for v in range(n):
        assert outst_all[v] == {p for p, _, _ in orc.outstanding(v)}, v
    want = [(s_, d, t, r if t in (1, 3) else 0) for (s_, d, t, r) in orc.pending()]
    assert sorted(inflight) == sorted(want)


def test_multi_root_heartbeats_lockstep():
    """heartbeats of several roots in flight at once (and
    a root heartbeating again while others are in flight), each root's tree
    kept -- round by round against the oracle, whose state is per root."""
    import partisan_amd as pa
    rp, col = pa.overlay.random_regular(1200, 5, 121)
    sim = pa.Simulator()
    sim.load_overlay(rp, col)
    orc = O.Plumtree(rp, col, lazy_tick_rounds=1)
    monos = {}
    schedule = {0: [0, 7], 2: [500], 5: [1100], 12: [7]}   # round -> roots heartbeating before it
    for rnd in range(40):
        for root in schedule.get(rnd, []):
            m = sim.broadcast(root)
            assert m == orc.heartbeat(root)
            monos[root] = m
        gs, os_ = sim.step(1)[0], orc.step(1)[0]
        for k in KINDS:
            assert gs[k] == os_[k], (rnd, k, gs, os_)
        assert gs["delivered_new"] == os_["delivered_new"], rnd
        _multi_compare(sim, orc, monos)
    sim.focus(7)
    assert sim.delivered().all()
    with pytest.raises(pa.PsimError):
        sim.focus(3)                 # never heartbeated: no lane
    sim.close()


def test_multi_root_lanes_full_is_enospc():
    """More roots than lanes: a 17th root is PSIM_ENOSPC (VERDICT r4 -- the
    least recently used lane used to be reused silently, forgetting its root's
    trees); the 16 roots keep their trees and another heartbeat of any of
    them still runs on its own lane."""
    import partisan_amd as pa
    rp, col = pa.overlay.random_regular(400, 5, 131)
    sim = pa.Simulator()
    sim.load_overlay(rp, col)
    orc = O.Plumtree(rp, col, lazy_tick_rounds=1)
    monos = {}
    for root in range(16):
        monos[root] = sim.broadcast(root)
        assert monos[root] == orc.heartbeat(root)
        sim.run()
        orc.run()
        assert sim.delivered().all()
    with pytest.raises(pa.PsimError) as ei:
        sim.broadcast(16)
    assert ei.value.name == "PSIM_ENOSPC"
    monos[0] = sim.broadcast(0)            # root 0's pruned tree, not a fresh flood
    assert monos[0] == orc.heartbeat(0)
    lockstep(sim, orc, 0, monos[0])
    for root in (0, 7, 15):
        sim.focus(root)
        eager, lazy, _, _ = sim.plumtree_state()
        for v in range(0, 400, 13):
            assert sim.mask_to_peers(v, eager[v]) == orc.peers(v, root)[0], (root, v)
            assert sim.mask_to_peers(v, lazy[v]) == orc.peers(v, root)[1], (root, v)
    sim.close()


def test_graft_storm_counts_every_graft(psim):
    """One vertex answers >= 16 i_haves with grafts in one round (ADVICE r1:
    the per-thread kind counters once kept the graft count mod 16).  Complete
    graph of 33 nodes (32 peers each, the slot limit): after two heartbeats
    every non-root link is lazy; the third heartbeat's messages INTO vertex 17
    are omitted, then healed, so at the next lazy tick all 31 lazy peers'
    i_have reach 17 in the same round and it grafts each of them."""
    n, V = 33, 17
    rp, col = psim.overlay.complete(n)
    sim, orc = make(psim, rp, col, 1)
    for _ in range(2):
        m = sim.broadcast(0)
        orc.heartbeat(0)
        lockstep(sim, orc, 0, m)
    pairs = [(u, V) for u in range(n) if u != V]
    sim.set_omissions(pairs)
    orc.set_omissions(pairs)
    sim.broadcast(0)
    mono = orc.heartbeat(0)
    _omit_step(sim, orc, 0, mono, 3)
    sim.set_omissions([])
    orc.set_omissions([])
    grafts = []
    for _ in range(10):
        gs, os_ = sim.step(1)[0], orc.step(1)[0]
        for k in KINDS:
            assert gs[k] == os_[k], (k, gs, os_)
        compare(sim, orc, 0, mono)
        grafts.append(gs["graft"])
    assert max(grafts) >= 16, grafts
    assert sim.delivered().all()


def test_facade_get_peers_per_root():
    """PlumtreeBroadcast.get_peers(Node, Root) answers for Root's tree
    (all_peers/3 :1278-1282), not the last broadcast one; a root that never
    broadcast has no map entry: the common sets (members -- self, [])."""
    import partisan_amd as pa
    rp, col = pa.overlay.random_regular(400, 5, 141)
    pt = pa.PlumtreeBroadcast(rp, col)
    orc = O.Plumtree(rp, col, 1)
    ids = {}
    for root in (3, 250):
        ids[root] = pt.broadcast(root)
        orc.heartbeat(root)
        pt.run()
        orc.run()
    for root in (3, 250):
        for v in (0, 3, 99, 250, 399):
            assert pt.get_peers(v, root) == orc.peers(v, root), (root, v)
            assert pt.handler(v).is_stale(ids[root])
    for v in (0, 99):
        assert pt.get_peers(v, 7) == orc.peers(v, 7)       # never broadcast
    first = ids[3]
    ids[3] = pt.broadcast(3)
    orc.heartbeat(3)
    pt.run()
    orc.run()
    assert pt.handler(99).is_stale(first) and pt.handler(99).is_stale(ids[3])
    assert not pt.handler(99).is_stale((3, 0, ids[3][2] + 1))
    pt.close()


def test_round_tags_across_wrap(psim):
    """Consumed inbox words are left in place with their round tag (mod 256);
    hundreds of idle rounds between heartbeats (and a lane that sat idle)
    must not let an old word alias a new round's tag: lockstep after 600
    idle rounds, across several tag wraps and scrubs."""
    rp, col = psim.overlay.random_regular(700, 5, 151)
    sim, orc = make(psim, rp, col, 1)
    for gap in (0, 300, 257, 43):
        if gap:
            gs = sim.step(gap)
            os_ = orc.step(gap)
            assert all(sum(g[k] for k in KINDS) == 0 for g in gs)
            assert all(sum(o[k] for k in KINDS) == 0 for o in os_)
        m = sim.broadcast(5)
        assert m == orc.heartbeat(5)
        compare(sim, orc, 5, m)
        lockstep(sim, orc, 5, m)


def test_round_tags_one_round_steps_at_wrap(psim):
    """Single-round steps across the tag period, then two heartbeats in
    lockstep.  A scrub run at exactly round S + 256 keeps the words tagged for
    round S + 257 -- and any stale word written for round S + 1 carries the
    same tag; round 3 moved the scrub one round earlier (psim_host.hip
    scrub_if_needed).  That case needs a stale round-(S+1) word nobody
    overwrote, which this overlay does not produce (every origin word is
    overwritten by a prune); it did occur with a 64-round tag on a ring lattice
    (profiles/r03/experiments/ab_word16_round_profile.txt)."""
    rp, col = psim.overlay.random_regular(300, 5, 153)
    sim, orc = make(psim, rp, col, 1)
    m = sim.broadcast(3)
    assert m == orc.heartbeat(3)
    for r in range(256):
        gs, os_ = sim.step(1)[0], orc.step(1)[0]
        for k in KINDS:
            assert gs[k] == os_[k], (r, k)
    for _ in range(2):
        m = sim.broadcast(3)
        assert m == orc.heartbeat(3)
        compare(sim, orc, 3, m)
        lockstep(sim, orc, 3, m)


def _delay_pairs(sim, frac, dmax, seed):
    rng = np.random.default_rng(seed)
    src = np.repeat(np.arange(sim.n), np.diff(sim.slot_row_ptr.astype(np.int64)))
    pick = rng.random(len(src)) < frac
    pairs = np.stack([src[pick], sim.slot_col[pick]], axis=1)
    return pairs, rng.integers(1, dmax + 1, len(pairs)).astype(np.uint8)


def _delay_lockstep(sim, orc, root, mono, max_rounds=300):
    """lockstep() whose end also waits for the delayed messages."""
    for r in range(max_rounds):
        gs, os_ = sim.step(1)[0], orc.step(1)[0]
        for k in KINDS:
            assert gs[k] == os_[k], (r, k, gs, os_)
        assert gs["delivered_new"] == os_["delivered_new"], r
        compare(sim, orc, root, mono)
        if orc.inflight() == 0 and os_["outstanding_live"] == 0:
            return r + 1
    raise AssertionError("no quiescence")


@pytest.mark.parametrize("n,seed,L,dmax", [(600, 1, 1, 3), (1500, 2, 2, 14), (1000, 3, 1, 6)])
def test_delay_faults_lockstep(psim, n, seed, L, dmax):
    """Delay faults (partisan_SUITE with_egress_delay / with_ingress_delay):
    30 % of the directed edges deliver 1..dmax rounds late.  Round by round
    against the oracle -- every clause sees its messages in the same round and
    order, the late eager pushes turn into prunes, lazy i_haves race the
    delayed pushes -- over a flood and two tree heartbeats; psim_run's round
    count (it waits for the pending delayed messages) equals the oracle's."""
    rp, col = psim.overlay.random_regular(n, 5, 200 + seed)
    sim, orc = make(psim, rp, col, L)
    pairs, d = _delay_pairs(sim, 0.3, dmax, seed)
    if psim.engine == "binned":
        with pytest.raises(psim.PsimError) as ei:
            sim.set_delays(pairs, d)
        assert ei.value.name == "PSIM_ENOTSUP"       # an explicit capability gap
        return
    sim.set_delays(pairs, d)
    orc.set_delays(pairs, d)
    root = seed * 7 % n
    for _ in range(2):
        m = sim.broadcast(root)
        assert m == orc.heartbeat(root)
        compare(sim, orc, root, m)
        _delay_lockstep(sim, orc, root, m)
    assert sim.delivered().all()
    m = sim.broadcast(root)
    assert m == orc.heartbeat(root)
    gst, gr = sim.run(1000)
    ost, orr = orc.run(1000)
    assert gr == orr
    assert [x["broadcast"] for x in gst] == [x["broadcast"] for x in ost]
    assert sim.delivered().all()


def test_delay_faults_egress_and_busy(psim):
    """A node's egress delay (all its out-edges) on the heartbeat root, with
    omission faults on other edges at the same time; changing delays while
    messages are in flight is refused (PSIM_EBUSY), as it could reorder a
    pair; removing them (k = 0) while quiescent restores next-round delivery."""
    if psim.engine == "binned":
        return
    rp, col = psim.overlay.random_regular(800, 5, 211)
    sim, orc = make(psim, rp, col, 1)
    root = 5
    pairs, d = sim.egress_delay(root, 4)
    sim.set_delays(pairs, d)
    orc.set_delays(pairs, d)
    op, _ = _delay_pairs(sim, 0.05, 1, 9)
    op = op[op[:, 0] != root]
    sim.set_omissions(op)
    orc.set_omissions(op)
    m = sim.broadcast(root)
    assert m == orc.heartbeat(root)
    gs, os_ = sim.step(3), orc.step(3)
    assert sum(g["delivered_new"] for g in gs) == 0 == sum(o["delivered_new"] for o in os_)
    with pytest.raises(psim.PsimError):
        sim.set_delays([], [])                     # the root's pushes are still on the wire
    with pytest.raises(RuntimeError):
        orc.set_delays([], [])
    _delay_lockstep(sim, orc, root, m)
    sim.set_omissions([])
    orc.set_omissions([])
    sim.set_delays([], [])
    orc.set_delays([], [])
    m = sim.broadcast(root)
    assert m == orc.heartbeat(root)
    _delay_lockstep(sim, orc, root, m)
    assert sim.delivered().all()


def test_delay_faults_multi_root():
    """Delays with several heartbeat lanes in flight (each lane gets its own
    ring), checked per root against the oracle."""
    import partisan_amd as pa
    rp, col = pa.overlay.random_regular(900, 5, 221)
    sim = pa.Simulator()
    sim.load_overlay(rp, col)
    orc = O.Plumtree(rp, col, lazy_tick_rounds=1)
    pairs, d = _delay_pairs(sim, 0.25, 5, 4)
    sim.set_delays(pairs, d)
    orc.set_delays(pairs, d)
    monos = {}
    schedule = {0: [0, 7], 3: [450]}
    for rnd in range(45):
        for root in schedule.get(rnd, []):
            m = sim.broadcast(root)
            assert m == orc.heartbeat(root)
            monos[root] = m
        gs, os_ = sim.step(1)[0], orc.step(1)[0]
        for k in KINDS:
            assert gs[k] == os_[k], (rnd, k, gs, os_)
        assert gs["delivered_new"] == os_["delivered_new"], rnd
        _multi_compare(sim, orc, monos)
    for root in monos:
        sim.focus(root)
        assert sim.delivered().all()
    sim.close()


def test_delay_faults_across_tag_wrap(psim):
    """The delay ring's words carry their arrival round's tag: idle gaps of
    hundreds of rounds (tag wraps, ring scrubs keeping the next 15 rounds)
    between heartbeats whose messages are up to 14 rounds late."""
    if psim.engine == "binned":
        return
    rp, col = psim.overlay.random_regular(500, 5, 231)
    sim, orc = make(psim, rp, col, 1)
    pairs, d = _delay_pairs(sim, 0.4, 14, 12)
    sim.set_delays(pairs, d)
    orc.set_delays(pairs, d)
    for gap in (0, 300, 257, 250):
        if gap:
            sim.step(gap)
            orc.step(gap)
        m = sim.broadcast(9)
        assert m == orc.heartbeat(9)
        _delay_lockstep(sim, orc, 9, m)
        sim.step(7)                                # part of the next gap with rows still acked late
        orc.step(7)
        compare(sim, orc, 9, m)


def _win_compare(sim, orc, root, monos):
    """Window lanes: every heartbeat in flight checked apart -- delivered
    per Monotonic, rows {peer, Round, Monotonic} in insertion order, the
    messages with their ids in handling order -- plus the shared eager /
    lazy sets and the newest heartbeat's Rounds."""
    for m in monos:
        assert np.array_equal(sim.delivered_mono(m), orc.delivered(root, m)), m
    eager, lazy, _, rr = sim.plumtree_state()
    orr = orc.recv_round(root, monos[-1])
    for v in range(sim.n):
        oe, ol = orc.peers(v, root)
        assert sim.mask_to_peers(v, eager[v]) == oe, f"eager set of {v}"
        assert sim.mask_to_peers(v, lazy[v]) == ol, f"lazy set of {v}"
        assert sim.rows(v) == orc.outstanding(v), f"rows of {v}"
        want = 0xFFFF if orr[v] == 0xFFFFFFFF else (0xFFFE if orr[v] == 0xFFFFFFFE else orr[v])
        assert rr[v] == want, v
    assert sim.messages() == orc.pending_full(), "in-flight messages differ"


def _win_step(sim, orc, root, monos):
    gs, os_ = sim.step(1)[0], orc.step(1)[0]
    for k in KINDS:
        assert gs[k] == os_[k], (k, gs, os_)
    assert gs["delivered_new"] == os_["delivered_new"]
    _win_compare(sim, orc, root, monos)
    return gs, os_


@pytest.mark.parametrize("n,seed,L", [(400, 1, 1), (1200, 2, 2), (800, 3, 1)])
def test_overlapping_heartbeats_lockstep(psim, n, seed, L):
    """SURVEY 8(f) row 1 / backend :341-368: the root heartbeats every 3
    rounds during its own flood.  Its lane turns into a window lane at the
    second heartbeat; round by round against the oracle, every heartbeat's
    deliveries, rows and messages are kept apart (the backend's interval set
    answers is_stale per Monotonic), over the shared per-root eager / lazy
    sets; the run ends quiescent with every heartbeat delivered everywhere."""
    rp, col = psim.overlay.random_regular(n, 5, 300 + seed)
    sim, orc = make(psim, rp, col, L)
    root = 11 * seed % n
    monos = []
    if psim.engine == "binned":
        sim.broadcast(root)
        sim.step(2)
        with pytest.raises(psim.PsimError):
            sim.broadcast(root)              # one heartbeat per root on the binned engine
        return
    for rnd in range(60):
        if rnd % 3 == 0 and rnd <= 12:
            m = sim.broadcast(root)
            assert m == orc.heartbeat(root)
            monos.append(m)
            _win_compare(sim, orc, root, monos)
        gs, os_ = _win_step(sim, orc, root, monos)
        if rnd > 12 and sum(gs[k] for k in KINDS) == 0 and os_["outstanding_live"] == 0:
            break
    for m in monos:
        assert sim.delivered_mono(m).all(), m
    stats, r = sim.run(100)
    assert r == 0 or all(sum(s[k] for k in KINDS) == 0 for s in stats)


def test_window_lane_with_faults_and_dead_peers(psim):
    """A window lane under omission faults and dead vertices: vertices die
    after the first flood, so the second leaves rows to dead lazy peers (a
    static lane would then hold rows of an older heartbeat: the next
    heartbeat switches the lane), omitted messages are counted and lost;
    lockstep with the oracle throughout, then every vertex revives."""
    if psim.engine == "binned":
        return
    n = 900
    rp, col = psim.overlay.random_regular(n, 5, 331)
    sim, orc = make(psim, rp, col, 1)
    root = 4
    m = sim.broadcast(root)
    assert m == orc.heartbeat(root)
    lockstep(sim, orc, root, m)
    rng = np.random.default_rng(3)
    alive = np.ones(n, np.uint8)
    alive[rng.choice(n, 60, replace=False)] = 0
    alive[root] = 1
    sim.set_alive(alive)
    orc.set_alive(alive)
    monos = [sim.broadcast(root)]
    assert monos[0] == orc.heartbeat(root)
    for _ in range(25):
        _win_step(sim, orc, root, monos)
    assert any(orc.outstanding(v) for v in range(n))          # rows to dead peers outlive the flood
    src = np.repeat(np.arange(n), np.diff(sim.slot_row_ptr.astype(np.int64)))
    pick = rng.random(len(src)) < 0.05
    pairs = np.stack([src[pick], sim.slot_col[pick]], axis=1)
    sim.set_omissions(pairs)
    orc.set_omissions(pairs)
    for rnd in range(40):
        if rnd in (0, 2, 7):
            m = sim.broadcast(root)
            assert m == orc.heartbeat(root)
            monos.append(m)
        if rnd == 20:
            sim.set_omissions([])
            orc.set_omissions([])
        _win_step(sim, orc, root, monos)
    sim.set_alive(np.ones(n, np.uint8))
    orc.set_alive(np.ones(n, np.uint8))
    m = sim.broadcast(root)
    assert m == orc.heartbeat(root)
    monos.append(m)
    for _ in range(30):
        _win_step(sim, orc, root, monos)
    assert sim.delivered_mono(m).all()


def _tree_csr(arity, n, cycles):
    """partisan_plumtree_util:build_tree/3 (the KAT-pinned oracle
    restatement) as a membership CSR: node k's members = its children
    (self dropped); the loader symmetrises them into peer slots."""
    t = dict((k, [c for c in ch if c != k]) for k, ch in O.build_tree(arity, list(range(n)), cycles))
    rows = [sorted(set(t.get(v, []))) for v in range(n)]
    rp = np.zeros(n + 1, np.uint64)
    rp[1:] = np.cumsum([len(r) for r in rows])
    return rp, np.asarray([u for r in rows for u in r], np.uint32)


@pytest.mark.parametrize("arity,n,cycles", [(1, 8, False), (2, 8, True), (3, 40, False), (2, 300, True),
                                             (3, 2000, True), (1, 64, True)])
def test_build_tree_overlays_lockstep(psim, arity, n, cycles):
    """SURVEY 8(a) build_tree row: the trees partisan_plumtree_util builds
    (arity 1-3, with and without cycles) as overlays -- paths, rings, k-ary
    trees, their cyclic closures -- flooded and re-flooded in lockstep with
    the oracle; a tree without cycles has no lazy link, so its second
    heartbeat sends no i_have."""
    rp, col = _tree_csr(arity, n, cycles)
    sim, orc = make(psim, rp, col, 1)
    for hb in range(3):
        m = sim.broadcast(0)
        assert m == orc.heartbeat(0)
        compare(sim, orc, 0, m)
        lockstep(sim, orc, 0, m)
        assert sim.delivered().all()


@pytest.mark.parametrize("cap,thr", [("1", None), ("2", "100000000"), (None, "100000000"), ("3", None)])
def test_worklist_overflow_and_forced_list_mode(psim, monkeypatch, cap, thr):
    """The sparse-round worklist is an optimisation over the
    group flags: with list shards of 1-3 entries every sparse round overflows
    and must fall back to the flags, and with the list threshold above any
    round's count every round lists its groups (dense ones too, overflowing
    or not).  Either way the rounds equal the oracle's, over a flood, tree
    heartbeats with i_have / graft (L = 2: tick rounds with rows read the
    flags) and dead vertices."""
    if psim.engine != "slot_scatter":
        pytest.skip("worklist: ELL rows on the slot-scatter engine")
    if cap:
        monkeypatch.setenv("PSIM_WL_CAP", cap)
    if thr:
        monkeypatch.setenv("PSIM_WL_THR", thr)
    n = 2500
    rp, col = psim.overlay.random_regular(n, 5, 91)
    for L in (1, 2):
        sim, orc = make(psim, rp, col, L)
        root = 17
        for hb in range(3):
            if hb == 2:
                alive = np.ones(n, np.uint8)
                alive[np.random.default_rng(3).choice(n, n // 15, replace=False)] = 0
                alive[root] = 1
                sim.set_alive(alive)
                orc.set_alive(alive)
            m = sim.broadcast(root)
            assert m == orc.heartbeat(root)
            lockstep(sim, orc, root, m)
        sim.close()


def _win_compare_ids(sim, orc, root, ids):
    """_win_compare with heartbeat ids in psim's packed form (epoch << 24 |
    Monotonic): a restarted origin's heartbeats of two epochs in flight."""
    for m in ids:
        assert np.array_equal(sim.delivered_mono(m), orc.delivered(root, m)), hex(m)
    eager, lazy, _, rr = sim.plumtree_state()
    orr = orc.recv_round(root, ids[-1])
    for v in range(sim.n):
        oe, ol = orc.peers(v, root)
        assert sim.mask_to_peers(v, eager[v]) == oe, f"eager set of {v}"
        assert sim.mask_to_peers(v, lazy[v]) == ol, f"lazy set of {v}"
        assert sim.rows(v) == orc.outstanding(v), f"rows of {v}"
        want = 0xFFFF if orr[v] == 0xFFFFFFFF else (0xFFFE if orr[v] == 0xFFFFFFFE else orr[v])
        assert rr[v] == want, v
    assert sim.messages() == orc.pending_full(packed=True), "in-flight messages differ"


def test_backend_restart_quiescent_lockstep(psim):
    """backend init/1 (:316-329) after a crash: a vertex's table forgets every
    origin, so the heartbeat it had delivered is no longer stale there (a
    later copy would be delivered again); the root's next heartbeat carries
    the newer epoch, {Root, 1, 1} = 1 << 24 | 1, and floods the pruned tree
    like any other -- lockstep with the oracle."""
    n = 400
    rp, col = psim.overlay.random_regular(n, 5, 77)
    sim, orc = make(psim, rp, col, 1)
    root, u = 7, 123
    m0 = sim.broadcast(root)
    assert m0 == orc.heartbeat(root) == 1
    lockstep(sim, orc, root, m0)
    if psim.engine == "binned":
        with pytest.raises(psim.PsimError):
            sim.restart_backend(u)          # the binned engine keeps one epoch per root
        return
    for v in (u, root):
        sim.restart_backend(v)
        orc.restart_backend(v)
    d = sim.delivered_mono(m0)
    assert np.array_equal(d, orc.delivered(root, m0))
    assert not d[u] and not d[root] and d.sum() == n - 2
    m1 = sim.broadcast(root)
    assert m1 == orc.heartbeat(root) == (1 << 24) | 1
    compare(sim, orc, root, m1)
    lockstep(sim, orc, root, m1)
    assert sim.delivered().all()
    m2 = sim.broadcast(root)                # the epoch's Monotonic counts on
    assert m2 == orc.heartbeat(root) == (1 << 24) | 2
    lockstep(sim, orc, root, m2)


def test_backend_restart_in_flight_lockstep(psim):
    """Restarts while a heartbeat floods: three vertices that delivered it
    forget it (each delivers the next copy again and holds a second row set
    for it -- the lane keeps every row: a window lane), then the root itself
    restarts and heartbeats at once, so heartbeats of two epochs are in
    flight together; a vertex holding the newer epoch treats the older one
    as stale (is_stale :237-238: Epoch0 > Epoch) and prunes its sender.
    Round by round against the oracle: deliveries per id, rows, messages."""
    if psim.engine == "binned":
        return                              # covered by the quiescent test's EBUSY/ESTATE check
    n = 600
    rp, col = psim.overlay.random_regular(n, 5, 78)
    sim, orc = make(psim, rp, col, 1)
    root = 31
    m0 = sim.broadcast(root)
    assert m0 == orc.heartbeat(root)
    ids = [m0]
    for _ in range(3):
        lockstep_one(sim, orc, root, m0)
    got = np.flatnonzero(sim.delivered())
    forget = [int(v) for v in got if v != root][:3]
    assert len(forget) == 3
    for v in forget:
        sim.restart_backend(v)
        orc.restart_backend(v)
    _win_compare_ids(sim, orc, root, ids)
    for _ in range(2):
        _win_step_ids(sim, orc, root, ids)
    sim.restart_backend(root)
    orc.restart_backend(root)
    m1 = sim.broadcast(root)
    assert m1 == orc.heartbeat(root) == (1 << 24) | 1
    ids.append(m1)
    _win_compare_ids(sim, orc, root, ids)
    for _ in range(200):
        gs, os_ = _win_step_ids(sim, orc, root, ids)
        if sum(gs[k] for k in KINDS) == 0 and os_["outstanding_live"] == 0:
            break
    else:
        raise AssertionError("no quiescence")
    assert sim.delivered_mono(m1).all()
    assert sim.delivered_mono(m0).all()     # stale everywhere: delivered, or the newer epoch is held


def lockstep_one(sim, orc, root, mono):
    gs, os_ = sim.step(1)[0], orc.step(1)[0]
    for k in KINDS:
        assert gs[k] == os_[k], (k, gs, os_)
    compare(sim, orc, root, mono)


def _win_step_ids(sim, orc, root, ids):
    gs, os_ = sim.step(1)[0], orc.step(1)[0]
    for k in KINDS:
        assert gs[k] == os_[k], (k, gs, os_)
    assert gs["delivered_new"] == os_["delivered_new"]
    _win_compare_ids(sim, orc, root, ids)
    return gs, os_


def _expect_graft(orc, root, v, mid):
    """backend graft/1 (:254-280) from the oracle's is_stale views: the id
    itself in v's row -> ok; a newer epoch in v's row -> stale."""
    pid = (mid[1] << 24) | mid[2]
    if not orc.delivered(root, pid)[v]:
        return ("error", ("not_found", mid))
    if orc.delivered(root, (mid[1] << 24) | 0xFFFFFF)[v]:
        return "stale"
    return ("ok", mid)


@pytest.mark.parametrize("in_flight", [False, True])
def test_facade_backend_restart_epochs(in_flight):
    """PlumtreeBackend.is_stale/graft with {Node, Epoch, Monotonic} ids across
    backend restarts, for every vertex and every id, against the oracle's
    table rows: quiescent heartbeats (static lanes: earlier ids from the
    recorded sets) and, with in_flight, a restart and a new-epoch heartbeat
    while the old one floods (a window lane answers on device)."""
    import partisan_amd as P
    n = 300
    rp, col = P.overlay.random_regular(n, 5, 91)
    pb = P.PlumtreeBroadcast(rp, col)
    orc = O.Plumtree(rp, col)
    root, u = 5, 77

    def advance():
        if in_flight:
            pb.step(2)
            orc.step(2)
        else:
            pb.run()
            orc.run(100000)

    id0 = pb.broadcast(root)
    assert id0 == (root, 0, 1) and orc.heartbeat(root) == 1
    advance()
    id0b = pb.broadcast(root)
    assert id0b == (root, 0, 2) and orc.heartbeat(root) == 2
    advance()
    for v in (u, root):
        pb.restart_backend(v)
        orc.restart_backend(v)
    advance()
    id1 = pb.broadcast(root)
    assert id1 == (root, 1, 1) and orc.heartbeat(root) == (1 << 24) | 1
    advance()
    pb.run()
    orc.run(100000)
    for mid in (id0, id0b, id1):
        want = orc.delivered(root, (mid[1] << 24) | mid[2])
        for v in range(n):
            h = pb.handler(v)
            assert h.is_stale(mid) == bool(want[v]), (mid, v)
            assert h.merge(mid, mid) == (not want[v])
        for v in (u, root, 0, 1, n - 1):
            assert pb.handler(v).graft(mid) == _expect_graft(orc, root, v, mid), (mid, v)
    assert pb.handler(3).graft(id0) == "stale"          # the row holds epoch 1 now
    assert pb.handler(3).graft(id1) == ("ok", id1)


def test_unsupported_combinations_are_enotsup():
    """combinations with no implementation answer
    PSIM_ENOTSUP (not a generic state error): delay faults on the binned
    engine and on a window lane (a root heartbeating during its own flood); a
    backend restart on a binned handle."""
    import partisan_amd as pa
    rp, col = pa.overlay.random_regular(300, 5, 241)
    b = pa.Simulator(binned=True)
    b.load_overlay(rp, col)
    pairs = [(0, int(b.slot_col[0]))]
    for call in (lambda: b.set_delays(pairs, [2]), lambda: b.restart_backend(3)):
        with pytest.raises(pa.PsimError) as ei:
            call()
        assert ei.value.name == "PSIM_ENOTSUP"
    b.close()
    s = pa.Simulator()
    s.load_overlay(rp, col)
    s.broadcast(0)
    s.step(2)
    s.broadcast(0)                            # the lane becomes a window lane
    s.run()
    with pytest.raises(pa.PsimError) as ei:
        s.set_delays([(0, int(s.slot_col[0]))], [2])
    assert ei.value.name == "PSIM_ENOTSUP"
    s.close()
    # (a forest takes delay faults since round 6: tests/test_forest.py; a
    # SHARDED forest refuses them: tests/test_forest_shard.py)


def _nt(st):
    """per-round stats without the timing field"""
    return [{k: v for k, v in x.items() if k != "kernel_ms"} for x in st]


def _same(a, b):
    for x, y in zip(a.plumtree_state(), b.plumtree_state()):
        assert np.array_equal(x, y)
    assert np.array_equal(a.delivered(), b.delivered())
    assert a.decode_inflight() == b.decode_inflight()
    assert a.trace_hash() == b.trace_hash()


def test_broadcast_run_matches_broadcast_then_run(psim):
    """psim_plumtree_broadcast_run (the origin's counters read back with the
    first chunk) = psim_plumtree_broadcast + psim_run: ids, per-round stats,
    round counts and every vertex's state -- floods, tree heartbeats, dead
    peers, a root change, a root with no peers (a quiet origin: zero rounds),
    a root whose every peer is dead, and a second root heartbeating while the first is in flight
    (several lanes, the pending origin on one of them)."""
    n = 2000
    rp, col = psim.overlay.random_regular(n - 1, 5, 77)
    rp = np.append(rp, rp[-1]).astype(rp.dtype)      # vertex n - 1 has no peers: its origin is quiet
    a = psim.Simulator()
    a.load_overlay(rp, col)
    b = psim.Simulator()
    b.load_overlay(rp, col)

    def both(root):
        ma = a.broadcast(root)
        sa, ra = a.run()
        mb, sb, rb = b.broadcast_run(root)
        assert (ma, ra) == (mb, rb)
        assert _nt(sa) == _nt(sb)
        _same(a, b)
        return ra

    assert both(5) > 3
    assert both(5) > 3
    dead = np.ones(n, np.uint8)
    dead[np.random.default_rng(1).choice(n, 100, replace=False)] = 0
    a.set_alive(dead)
    b.set_alive(dead)
    both(9)
    both(9)
    assert both(n - 1) == 0                   # nothing sent: zero rounds
    # a root whose every peer is dead: its pushes are lost on arrival
    r = 1234
    nb = col[rp[r]:rp[r + 1]]
    alive = np.ones(n, np.uint8)
    alive[nb] = 0
    a.set_alive(alive)
    b.set_alive(alive)
    both(r)
    a.set_alive(np.ones(n, np.uint8))
    b.set_alive(np.ones(n, np.uint8))
    both(r)
    # max_rounds 0: the origin alone (its counters are read without a chunk), then the rounds
    ma = a.broadcast(r)
    mb, sb0, rb0 = b.broadcast_run(r, max_rounds=0)
    assert (ma, rb0, sb0) == (mb, 0, [])
    sa, ra = a.run()
    sb, rb = b.run()
    assert (ra, _nt(sa)) == (rb, _nt(sb))
    _same(a, b)
    if psim.engine != "binned":       # binned handles keep one root
        a.broadcast(17)
        b.broadcast(17)
        a.step(2)
        b.step(2)
        ma = a.broadcast(400)
        sa, ra = a.run()
        mb, sb, rb = b.broadcast_run(400)
        assert (ma, ra, _nt(sa)) == (mb, rb, _nt(sb))
        for root in (17, 400):
            a.focus(root)
            b.focus(root)
            _same(a, b)
    a.close()
    b.close()


def test_broadcast_run_with_delays_matches():
    """Delay faults: the origin's words go to the due ring, so broadcast_run
    reads the origin first (as the two calls do); same results."""
    import partisan_amd as pa
    n = 1500
    rp, col = pa.overlay.random_regular(n, 5, 78)
    sims = []
    for _ in range(2):
        s = pa.Simulator()
        s.load_overlay(rp, col)
        src = np.repeat(np.arange(n), np.diff(rp.astype(np.int64)))
        pick = np.random.default_rng(3).random(len(src)) < 0.1
        s.set_delays(np.stack([src[pick], col[pick]], axis=1), np.full(int(pick.sum()), 2))
        sims.append(s)
    a, b = sims
    for _ in range(2):
        ma = a.broadcast(3)
        sa, ra = a.run()
        mb, sb, rb = b.broadcast_run(3)
        assert (ma, ra, _nt(sa)) == (mb, rb, _nt(sb))
        _same(a, b)
    a.close()
    b.close()
