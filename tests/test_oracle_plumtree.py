"""Properties of the Plumtree oracle (CPU).  The reference pins no Plumtree
trace; these pin the restatement to the protocol's documented
behaviour (partisan_plumtree_broadcast.erl) and to the reliable-broadcast
postcondition of test/prop_partisan_reliable_broadcast.erl:127-172 (every
message is received by every live member)."""
import numpy as np
import pytest

import pyoracle as O
from partisan_amd import overlay


def eager_edges(orc, n, root):
    tot = 0
    for v in range(n):
        e, _ = orc.peers(v, root)
        tot += len(e)
    return tot


@pytest.mark.parametrize("n,seed", [(50, 1), (400, 2), (2000, 3)])
def test_flood_builds_spanning_tree(n, seed):
    rp, col = overlay.random_regular(n, 5, seed)
    orc = O.Plumtree(rp, col, 1)
    m = orc.heartbeat(0)
    st, r = orc.run()
    assert orc.delivered(0, m).all()
    assert eager_edges(orc, n, 0) == 2 * (n - 1)
    assert st[-1]["outstanding"] == 0
    # Q1: the first broadcast is pure gossip: no lazy traffic at all
    assert sum(s["i_have"] + s["graft"] + s["ignored_i_have"] for s in st) == 0
    rr = orc.recv_round(0, m)
    # every vertex's Round = its eager parent's Round + 1
    for v in range(1, n):
        e, _ = orc.peers(v, 0)
        parents = [u for u in e if (rr[u] == 0xFFFFFFFE and rr[v] == 0) or
                   (rr[u] != 0xFFFFFFFE and rr[u] + 1 == rr[v])]
        assert parents, v


def test_second_heartbeat_uses_tree_and_lazy_links():
    n = 1000
    rp, col = overlay.random_regular(n, 5, 9)
    orc = O.Plumtree(rp, col, 1)
    orc.heartbeat(0)
    orc.run()
    m = orc.heartbeat(0)
    st, _ = orc.run()
    assert orc.delivered(0, m).all()
    # eager pushes travel the tree only: one per non-root vertex (the root's
    # own round-0 pushes are emitted by the heartbeat call, not by a round)
    assert sum(s["broadcast"] for s in st) + len(orc.peers(0, 0)[0]) == n - 1
    # every i_have is answered (ignored_i_have) because the tree already delivered
    assert sum(s["i_have"] for s in st) == sum(s["ignored_i_have"] for s in st) > 0
    assert sum(s["graft"] for s in st) == 0
    assert st[-1]["outstanding"] == 0


def test_graft_repairs_tree_after_failures():
    n = 1000
    rp, col = overlay.random_regular(n, 5, 13)
    orc = O.Plumtree(rp, col, 1)
    orc.heartbeat(0)
    orc.run()
    alive = np.ones(n, np.uint8)
    alive[np.random.default_rng(1).choice(np.arange(1, n), 50, replace=False)] = 0
    orc.set_alive(alive)
    m = orc.heartbeat(0)
    st, _ = orc.run()
    d = orc.delivered(0, m)
    assert sum(s["graft"] for s in st) > 0
    # reachable live vertices all deliver (graft repairs the broken tree)
    live = np.nonzero(alive)[0]
    assert d[live].mean() > 0.99
    assert not d[alive == 0].any()


def test_deterministic():
    rp, col = overlay.random_regular(500, 5, 17)
    runs = []
    for _ in range(2):
        orc = O.Plumtree(rp, col, 2)
        orc.heartbeat(3)
        st, r = orc.run()
        orc.heartbeat(3)
        st2, r2 = orc.run()
        runs.append((st, r, st2, r2, [orc.peers(v, 3) for v in range(500)]))
    assert runs[0] == runs[1]


def test_update_resets_per_root_sets():
    # Q2: an update with new members drops every per-root eager/lazy set
    rp, col = overlay.random_regular(200, 5, 19)
    orc = O.Plumtree(rp, col, 1)
    orc.heartbeat(0)
    orc.run()
    v = 5
    lo, hi = int(rp[v]), int(rp[v + 1])
    members = sorted(set(col[lo:hi].tolist()) | {v})
    e0, l0 = orc.peers(v, 0)
    assert l0, "some link must have been pruned"
    orc.update(v, members + [199] if 199 not in members else members + [198])
    e1, l1 = orc.peers(v, 0)
    assert l1 == [] and len(e1) == len(members)      # common_eagers U New, minus self
    # neighbors_down: removing a member removes it everywhere
    orc.update(v, members)
    e2, _ = orc.peers(v, 0)
    assert e2 == [u for u in members if u != v]


def test_bulk_views_match_per_vertex_getters():
    """orc_pt_dump_state / orc_pt_inflight_words (the whole-overlay lockstep
    views of tests/test_worklist_parity.py) agree with the per-vertex getters
    and the pending list, round by round, over a flood and a tree heartbeat
    with dead vertices (L = 2: outstanding rows over several rounds)."""
    n = 1200
    rp, col = overlay.random_regular(n, 5, 77)
    rp = np.asarray(rp, np.int64)
    row = np.repeat(np.arange(n), np.diff(rp))
    scol = np.asarray(col, np.uint32)[np.lexsort((col, row))]
    orc = O.Plumtree(rp, col, 2)
    for hb in range(2):
        if hb == 1:
            alive = np.ones(n, np.uint8)
            alive[np.random.default_rng(1).choice(n, 60, replace=False)] = 0
            alive[5] = 1
            orc.set_alive(alive)
        mono = orc.heartbeat(5)
        for _ in range(40):
            e, l_, o, rr = orc.dump_state(5, mono, rp, scol)
            orr = orc.recv_round(5, mono)
            assert np.array_equal(rr, np.where(orr == 0xFFFFFFFF, 0xFFFF, orr & 0xFFFF).astype(np.uint16))
            for v in range(0, n, 13):
                row_v = scol[rp[v]:rp[v + 1]].tolist()
                dec = lambda m: sorted(row_v[s] for s in range(len(row_v)) if (int(m) >> s) & 1)
                pe, pl = orc.peers(v, 5)
                assert dec(e[v]) == pe and dec(l_[v]) == pl
                assert dec(o[v]) == sorted({p for p, _, _ in orc.outstanding(v)})
            w = orc.inflight_words(rp, scol)
            msgs = []
            for s in np.nonzero(w)[0].tolist():
                dst = int(np.searchsorted(rp, s, side="right") - 1)
                f = int(w[s]) & 0xFFFF
                while f:
                    t = f & 0xF
                    f >>= 4
                    msgs.append((int(scol[s]), dst, t, int(w[s]) >> 16 if t in (1, 3) else 0))
            want = sorted((s_, d, t, r if t in (1, 3) else 0) for (s_, d, t, r) in orc.pending())
            assert sorted(msgs) == want
            st = orc.step(1)[0]
            if sum(st[k] for k in ("broadcast", "prune", "i_have", "ignored_i_have", "graft")) == 0 \
                    and st["outstanding_live"] == 0:
                break
    orc.close()
