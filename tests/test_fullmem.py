"""Full-membership strategy over the state_orset membership set.

Oracle (CPU): the OR-set restatement is pinned by every eunit test of
src/partisan_membership_set.erl:269-522 (tests/golden/membership_set_kat.json);
the strategy round simulation (oracle/fullmem.c) is checked for the
convergence the reference's connectivity_test expects
(test/partisan_SUITE.erl:1296-1341: every node ends up knowing every node).

GPU (-m gpu): csrc/fullmem.hip through the C ABI, bit-exact against the
oracle round by round: per-round counters, every node's known/removed token
bitmaps (= its state_orset payload) and liveness.
"""
import json
import os

import numpy as np
import pytest

import pyoracle as O


def _kat(golden_dir):
    with open(os.path.join(golden_dir, "membership_set_kat.json")) as f:
        return json.load(f)


def run_script(ops):
    env, tok = {}, [0]

    def fresh():
        tok[0] += 1
        return tok[0]

    for op in ops:
        k = op[0]
        if k == "new":
            env[op[1]] = O.ORSet()
        elif k == "alias":
            env[op[1]] = env[op[2]]
        elif k == "add":
            env[op[1]] = env[op[4]].add(op[2], fresh())
        elif k == "remove":
            env[op[1]] = env[op[4]].remove(op[2])
        elif k == "merge":
            env[op[1]] = env[op[2]].merge(env[op[3]])
        elif k == "to_list":
            if op[2] is not None:
                assert env[op[1]].to_list() == op[2], op
        elif k == "same_list":
            assert env[op[1]].to_list() == env[op[2]].to_list(), op
        elif k == "same_term":
            assert env[op[1]].dump() == env[op[2]].dump(), op
        elif k == "equal":
            assert env[op[2]].equal(env[op[3]]) is op[1], op
        elif k == "compare":
            lst, members = set(op[1]), set(env[op[2]].to_list())
            if lst:   # compare([], _) -> {[], []} (:151-152)
                joiners, leavers = sorted(lst - members), sorted(members - lst)
            else:
                joiners, leavers = [], []
            assert joiners == op[3] and leavers == op[4], op
        else:
            raise ValueError(op)
    return env


@pytest.mark.parametrize("name", sorted(json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                                                      "membership_set_kat.json")))["tests"]))
def test_membership_set_kat(golden_dir, name):
    run_script(_kat(golden_dir)["tests"][name])


def test_orset_remove_absent_is_precondition_error():
    with pytest.raises(KeyError):
        O.ORSet().remove(7)


def cluster_joins(f, n):
    """partisan_support:cluster/4: every node joins every other node."""
    for v in range(n):
        for u in range(n):
            if u != v:
                f.join(v, u)


def test_c1_full_membership_converges():
    n = 16
    f = O.FullMembership(n, periodic_rounds=10)
    cluster_joins(f, n)
    st = f.step(12)
    assert all(f.members(v) == list(range(n)) for v in range(n))
    assert st[-1]["member_sum"] == n * n
    # converged: after the join waves only periodic gossip remains, all equal
    assert st[3]["sent"] == 0 and st[9]["sent"] == n * (n - 1) and st[10]["merges"] == 0


def test_leave_removes_and_stops_the_leaver():
    n = 8
    f = O.FullMembership(n, periodic_rounds=0)
    cluster_joins(f, n)
    f.step(4)
    f.leave(0, 5)                    # node 0 removes node 5; 5 learns it and stops (:1791-1803)
    f.step(4)
    assert not f.alive(5)
    for v in range(n):
        if v != 5:
            assert f.members(v) == [u for u in range(n) if u != 5]


# ------------------------------------------------------------------ GPU parity
def oracle_bitmaps(f, n, words):
    K = np.zeros((n, words), np.uint64)
    R = np.zeros((n, words), np.uint64)
    for v in range(n):
        for _, t, act in f.payload(v):
            K[v, t >> 6] |= np.uint64(1 << (t & 63))
            if not act:
                R[v, t >> 6] |= np.uint64(1 << (t & 63))
    return K, R


def check_round(g, f, n):
    K, R, alive = g.state()
    oK, oR = oracle_bitmaps(f, n, g.words)
    assert np.array_equal(alive.astype(bool), np.array([f.alive(v) for v in range(n)]))
    assert np.array_equal(K, oK) and np.array_equal(R, oR)


def _drive(n, periodic, script, rounds):
    import partisan_amd as pa
    sim = pa.Simulator(device=0)
    g = pa.fullmem.FullMembershipCluster(sim, n, periodic_rounds=periodic, max_tokens=n + 64)
    f = O.FullMembership(n, periodic_rounds=periodic)
    for r in range(rounds):
        for kind, a, b in script.get(r, []):
            if kind == "join":
                g.join([a], [b]); f.join(a, b)
            elif kind == "leave":
                g.leave([a], [b]); f.leave(a, b)
            elif kind == "alive":
                g.set_alive(a); f.set_alive(a)
        gs = g.step(1)[0]
        os_ = f.step(1)[0]
        for k in os_:
            assert gs[k] == os_[k], (r, k, gs, os_)
        check_round(g, f, n)
    return g, f


@pytest.mark.gpu
def test_gpu_c1_parity():
    n = 16
    script = {0: [("join", v, u) for v in range(n) for u in range(n) if u != v]}
    g, f = _drive(n, 5, script, 14)
    assert all(g.members(v) == list(range(n)) for v in range(n))


@pytest.mark.gpu
def test_gpu_random_joins_leaves_failures_parity():
    """Concurrent random joins (the re-gossip storm of handle_message/2 on every
    differing state: up to ~3e5 messages a round at n=16), leaves, a
    self-leave (fresh token) and failures."""
    n = 16
    rng = np.random.default_rng(7)
    script = {}
    for r in range(30):
        ev = []
        for _ in range(rng.integers(0, 6)):
            ev.append(("join", int(rng.integers(n)), int(rng.integers(n))))
        if r in (12, 20):
            ev.append(("leave", int(rng.integers(n)), int(rng.integers(n))))
        if r == 16:
            v = int(rng.integers(n))
            ev.append(("leave", v, v))             # self-leave: new_state with a fresh token
        if r == 18:
            a = np.ones(n, np.uint8)
            a[rng.choice(n, 3, replace=False)] = 0
            ev.append(("alive", a, None))
        script[r] = ev
    _drive(n, 4, script, 34)


@pytest.mark.gpu
def test_gpu_two_words_of_nodes():
    """n > 64: node and token bitmaps span two words.  A chain of joins, one
    every 3 rounds, so each join's storm (~n^2 messages) settles first."""
    n = 70
    script = {3 * (v - 1): [("join", v, v - 1)] for v in range(1, n)}
    g, f = _drive(n, 7, script, 3 * n + 3)
    assert all(g.members(v) == list(range(n)) for v in range(n))


# ------------------------------------------------------------------ the wire
def _rows_to_bits(rows, words):
    K = np.zeros(words, np.uint64)
    R = np.zeros(words, np.uint64)
    for _, t, act in rows:
        K[t >> 6] |= np.uint64(1 << (t & 63))
        if not act:
            R[t >> 6] |= np.uint64(1 << (t & 63))
    return K, R


def _bits_to_rows(K, R, token_node):
    rows = []
    for t in range(64 * len(K)):
        if (int(K[t >> 6]) >> (t & 63)) & 1:
            rows.append((int(token_node[t]), t, not (int(R[t >> 6]) >> (t & 63)) & 1))
    return rows


def test_oracle_wire_take_put_round_trip():
    """A node's manager taking its messages off the wire and handing them
    back (handle_message/2) changes nothing; the listing is in handling order
    and each message carries the {NodeSpec, #full_v1{}} state its sender
    gossiped (gossip_messages/2 :247-267)."""
    n = 12
    a, b = O.FullMembership(n, periodic_rounds=3), O.FullMembership(n, periodic_rounds=3)
    for f in (a, b):
        cluster_joins(f, n)
    for r in range(8):
        for f in (a, b):
            f.step(1)
        ms = a.messages()
        assert ms == b.messages()
        assert [(d, s, q) for s, d, q, _ in ms] == sorted((d, s, q) for s, d, q, _ in ms)
        if ms:
            d = ms[len(ms) // 2][1]
            got = a.take(d)
            assert got == [m for m in ms if m[1] == d]
            assert all(m[1] != d for m in a.messages())
            a.put(got)
            assert a.messages() == ms
    for v in range(n):
        assert a.payload(v) == b.payload(v)


@pytest.mark.gpu
def test_gpu_wire_messages_take_put_parity():
    """psim_fm_messages / _take / _put against the oracle's wire: every round
    the messages the next round delivers -- (src, dst) in handling order and
    the #full_v1{} state each carries -- equal the oracle's; a manager's round
    trip (take a node's messages, hand them back) and a message from a node
    outside the simulated cluster (src = n) go onto both wires, and the states,
    counters and liveness stay bit-exact through joins, a leave and a failure."""
    import partisan_amd as pa
    n = 16
    sim = pa.Simulator(device=0)
    g = pa.fullmem.FullMembershipCluster(sim, n, periodic_rounds=4, max_tokens=n + 64)
    f = O.FullMembership(n, periodic_rounds=4)
    rng = np.random.default_rng(11)
    ext = 0
    took = 0
    for r in range(24):
        if r < 6:
            for _ in range(3):
                a_, b_ = int(rng.integers(n)), int(rng.integers(n))
                g.join([a_], [b_]); f.join(a_, b_)
        if r == 10:
            g.leave([3], [7]); f.leave(3, 7)
        if r == 14:
            al = np.ones(n, np.uint8)
            al[5] = 0
            g.set_alive(al); f.set_alive(al)
        gs, os_ = g.step(1)[0], f.step(1)[0]
        for k in os_:
            assert gs[k] == os_[k], (r, k, gs, os_)
        check_round(g, f, n)
        gm, om = g.messages(), f.messages()
        assert len(gm) == len(om), (r, len(gm), len(om))
        for (s1, d1, _q1, K1, R1), (s2, d2, _q2, rows) in zip(gm, om):
            K2, R2 = _rows_to_bits(rows, g.words)
            assert (s1, d1) == (s2, d2) and np.array_equal(K1, K2) and np.array_equal(R1, R2), r
        if gm and r % 3 == 1:              # a manager's round trip at one node
            d = gm[(7 * r) % len(gm)][1]
            gt, ot = g.take(d), f.take(d)
            assert [(m[0], m[1]) for m in gt] == [(m[0], m[1]) for m in ot]
            assert all(m[1] != d for m in g.messages())
            took += len(gt)
            g.put(gt)
            f.put(ot)
        if r % 4 == 2:                     # gossip from a node outside the cluster: node 2's state, to node 9
            K, R, _ = g.state()
            tok = g.token_nodes()
            g.put([(n, 9, ext, K[2], R[2])])
            f.put([(n, 9, ext, _bits_to_rows(K[2], R[2], tok))])
            ext += 1
    assert took > 0 and ext > 0
    assert all(g.members(v) == f.members(v) for v in range(n) if f.alive(v))


@pytest.mark.gpu
def test_gpu_wire_put_refuses_unknown_tokens():
    import partisan_amd as pa
    from partisan_amd._lib import PsimError
    n = 8
    sim = pa.Simulator(device=0)
    g = pa.fullmem.FullMembershipCluster(sim, n, periodic_rounds=4, max_tokens=n + 64)
    K = np.zeros(g.words, np.uint64)
    R = np.zeros(g.words, np.uint64)
    K[0] = np.uint64(1 << 20)                  # token 20: never allocated (8 nodes, no self-leave)
    with pytest.raises(PsimError):
        g.put([(n, 1, 0, K, R)])
    K[0] = np.uint64(1)
    R[0] = np.uint64(2)                        # removed but not known
    with pytest.raises(PsimError):
        g.put([(n, 1, 0, K, R)])
    assert g.messages() == []
