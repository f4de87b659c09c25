"""Delay faults in the Plumtree oracle (oracle/plumtree.c orc_pt_set_delays):
the CPU half of the delay-fault parity tests (the GPU half is in
test_plumtree_gpu.py).  partisan_SUITE's with_egress_delay /
with_ingress_delay groups hold no trace to pin against, so these check the
schedule's definition directly: a message emitted in round t over a pair
with delay d is delivered in round t + 1 + d, each pair stays FIFO."""
import numpy as np
import pytest

import pyoracle as O
from partisan_amd import overlay


def _path(n):
    rows = [[u for u in (v - 1, v + 1) if 0 <= u < n] for v in range(n)]
    rp = np.zeros(n + 1, np.uint64)
    rp[1:] = np.cumsum([len(r) for r in rows])
    return rp, np.asarray([u for r in rows for u in r], np.uint32)


def test_delay_moves_delivery_round():
    rp, col = _path(4)
    o = O.Plumtree(rp, col, 1)
    o.set_delays([(0, 1), (2, 3)], [3, 2])
    m = o.heartbeat(0)
    st, rounds = o.run(100)
    rr = o.recv_round(0, m)
    # 0 -> 1 arrives in round 4 (1 + 3), 1 -> 2 in round 5, 2 -> 3 in round 8 (6 + 2)
    assert [int(x) for x in rr[1:]] == [0, 1, 2]        # Round carried, not wall rounds
    newly = [s["delivered_new"] for s in st]
    assert [i + 1 for i, x in enumerate(newly) if x] == [4, 5, 8]
    assert rounds == 8 and o.inflight() == 0


def test_zero_delays_are_no_delays():
    rp, col = overlay.random_regular(300, 5, 3)
    a, b = O.Plumtree(rp, col, 1), O.Plumtree(rp, col, 1)
    src = np.repeat(np.arange(300), np.diff(rp.astype(np.int64)))
    b.set_delays(np.stack([src, col], axis=1), np.zeros(len(col), np.uint8))
    for _ in range(2):
        ma, mb = a.heartbeat(7), b.heartbeat(7)
        assert a.run(500) == b.run(500)
        assert np.array_equal(a.delivered(7, ma), b.delivered(7, mb))


def test_delays_conserve_messages_and_delivery():
    rp, col = overlay.random_regular(500, 5, 4)
    o = O.Plumtree(rp, col, 1)
    rng = np.random.default_rng(1)
    src = np.repeat(np.arange(500), np.diff(rp.astype(np.int64)))
    pick = rng.random(len(col)) < 0.5
    o.set_delays(np.stack([src[pick], col[pick]], axis=1), rng.integers(1, 15, pick.sum()).astype(np.uint8))
    m = o.heartbeat(0)
    st, rounds = o.run(1000)
    assert o.delivered(0, m).all()
    assert sum(s["delivered_new"] for s in st) == 499
    # every broadcast received (the origin's 5 pushes included) is a delivery or a prune
    assert sum(s["broadcast"] for s in st) + 5 == 499 + sum(s["prune"] for s in st)
    with pytest.raises(RuntimeError):
        o.heartbeat(0)
        o.set_delays([], [])
