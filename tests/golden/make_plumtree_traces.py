"""Generates tests/golden/plumtree_traces.json: per-round Plumtree traces of
the CPU oracle (oracle/plumtree.c, the line-by-line restatement of
src/partisan_plumtree_broadcast.erl:487-1328 with the heartbeat backend
src/partisan_plumtree_backend.erl:180-417).

The reference's own suites hold no Plumtree trace (SURVEY 8(c)
"Unpinned"), so these vectors pin the ORACLE against silent drift: a CPU
test replays them against oracle/plumtree.c, a GPU test against libpsim.
Topologies: partisan_plumtree_util:build_tree/3 outputs (arity 1-3, with and
without cycles, 8 nodes; the KAT-pinned generator of
src/partisan_plumtree_util.erl:43-58, eunit :102-261) used as membership
lists, random 5-peer overlays of 40 and 300 nodes, a 120-node overlay with
dead vertices, and a 40-node overlay with omission faults then a heal.

Recorded per heartbeat: every round's per-kind counters and the messages it
emitted as (src, dst, kind, Round) -- Round kept for broadcast / i_have only,
sorted by (dst, src) with FIFO order within a pair -- and after quiescence
every vertex's eager / lazy peers for the root, outstanding rows (peer,
Round), the delivered set and accepted Round.

Run from the repo root:  python tests/golden/make_plumtree_traces.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import pyoracle as O  # noqa: E402
from partisan_amd import overlay  # noqa: E402

KINDS = ("broadcast", "prune", "i_have", "ignored_i_have", "graft")


def tree_csr(arity, n, cycles):
    """build_tree(Arity, [0..n-1], Opts) as membership lists: v's members are
    its children (the simulator symmetrises links)."""
    t = O.build_tree(arity, list(range(n)), cycles)
    src, dst = [], []
    for node, children in t:
        for c in children:
            if c != node:
                src.append(node)
                dst.append(c)
    a, b = np.asarray(src, np.int64), np.asarray(dst, np.int64)
    return overlay._csr_from_directed(n, a, b), t


def norm_msgs(pending):
    return [[s, d, t, r if t in (1, 3) else 0] for (s, d, t, r) in pending]


def final_state(orc, n, root, mono):
    eager, lazy, rows = [], [], []
    for v in range(n):
        e, lz = orc.peers(v, root)
        eager.append(e)
        lazy.append(lz)
        rows.append(sorted([p, r] for p, r, _m in orc.outstanding(v)))
    rr = orc.recv_round(root, mono)
    return {"eager": eager, "lazy": lazy, "outstanding": rows,
            "delivered": orc.delivered(root, mono).astype(int).tolist(),
            "recv_round": [int(x) for x in rr]}


def record(name, rp, col, L, script, meta=None):
    """script items: ("heartbeat", root[, limit]) -- a heartbeat, then rounds
    until quiescence (or `limit` rounds); ("continue"[, limit]) -- more rounds
    of the last heartbeat; ("alive", bytes); ("omit", pairs); ("heal",)."""
    n = len(rp) - 1
    orc = O.Plumtree(rp, col, L)
    events = []
    root = mono = None
    for ev in script:
        if ev[0] == "alive":
            orc.set_alive(np.asarray(ev[1], np.uint8))
            events.append({"alive": [int(x) for x in ev[1]]})
            continue
        if ev[0] == "omit":
            orc.set_omissions(ev[1])
            events.append({"omit": [[int(s), int(d)] for s, d in ev[1]]})
            continue
        if ev[0] == "heal":
            orc.set_omissions([])
            events.append({"omit": []})
            continue
        if ev[0] == "heartbeat":
            root, limit = ev[1], (ev[2] if len(ev) > 2 else 10000)
            mono = orc.heartbeat(root)
            hb = {"heartbeat": root, "mono": mono, "origin_msgs": norm_msgs(orc.pending()), "rounds": []}
        else:
            limit = ev[1] if len(ev) > 1 else 10000
            hb = {"continue": root, "mono": mono, "rounds": []}
        for _ in range(limit):
            st = orc.step(1)[0]
            hb["rounds"].append({"stats": [st[k] for k in KINDS] + [st["delivered_new"]],
                                 "msgs": norm_msgs(orc.pending())})
            if sum(st[k] for k in KINDS) == 0 and st["outstanding_live"] == 0:
                break
        hb["final"] = final_state(orc, n, root, mono)
        events.append(hb)
    orc.close()
    case = {"name": name, "n": n, "row_ptr": [int(x) for x in rp], "col": [int(x) for x in col],
            "lazy_tick_rounds": L, "events": events}
    if meta:
        case.update(meta)
    return case


def main():
    cases = []
    for arity in (1, 2, 3):
        for cycles in (False, True):
            (rp, col), t = tree_csr(arity, 8, cycles)
            cases.append(record(f"build_tree_a{arity}_{'cycles' if cycles else 'nocycles'}", rp, col, 1,
                                [("heartbeat", 0), ("heartbeat", 0), ("heartbeat", 5)],
                                {"build_tree": t}))
    rp, col = overlay.random_regular(40, 5, 1)
    cases.append(record("random40", rp, col, 1, [("heartbeat", 0), ("heartbeat", 0), ("heartbeat", 0)]))
    rp, col = overlay.random_regular(300, 5, 2)
    cases.append(record("random300_L2", rp, col, 2, [("heartbeat", 17), ("heartbeat", 17)]))
    rp, col = overlay.random_regular(120, 5, 3)
    alive = np.ones(120, np.uint8)
    alive[np.random.default_rng(4).choice(120, 12, replace=False)] = 0
    alive[9] = 1
    cases.append(record("dead120", rp, col, 1, [("heartbeat", 9), ("alive", alive), ("heartbeat", 9)]))
    rp, col = overlay.random_regular(40, 5, 5)
    src = np.repeat(np.arange(40), np.diff(rp.astype(np.int64)))
    pick = np.random.default_rng(6).random(len(src)) < 0.15
    pairs = np.stack([src[pick], col[pick]], axis=1).tolist()
    cases.append(record("omit40", rp, col, 1, [("heartbeat", 2), ("omit", pairs), ("heartbeat", 2, 12), ("heal",),
                                                 ("continue",), ("heartbeat", 2)]))
    out = {"source": ("oracle/plumtree.c via oracle/pyoracle.py (tests/golden/make_plumtree_traces.py); "
                      "topologies from partisan_plumtree_util:build_tree/3 (src/partisan_plumtree_util.erl:43-58) "
                      "and seeded random overlays"),
           "kinds": list(KINDS), "cases": cases}
    path = os.path.join(ROOT, "tests", "golden", "plumtree_traces.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(path, os.path.getsize(path), "bytes,", len(cases), "cases")


if __name__ == "__main__":
    main()
