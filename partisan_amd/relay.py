"""Transitive relay over Plumtree out-links (kernels in
csrc/relay.hip).

Host mirror of the caller side of
``partisan_hyparview_peer_service_manager``: a batch of
``forward_message(Node, Message, #{transitive => true})`` sends, each handled
by ``do_send_message/3`` (:2220-2290) at its origin -- connected: sent;
otherwise ``do_tree_forward/4`` (:2796-2842) over the origin's out-links with
``relay_ttl`` -- and by ``handle_message({relay_message, Node, Message, TTL})``
(:1800-1832) at every relay.  ``out_links`` are each node's eager peers in its
own broadcast tree (``retrieve_outlinks/1`` :2846-2870); :func:`out_links_from`
reads them from a :class:`partisan_amd.Simulator` after its trees settled.
"""
import ctypes as C

import numpy as np

from ._lib import PsimError, RelayStats, lib

RELAY_TTL = 5   # ?RELAY_TTL (include/partisan.hrl)


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def relay_run(sim, act_ptr, act, ol_ptr, ol, alive, src, dst, relay_ttl=RELAY_TTL, max_copies=50_000_000,
              cap=256):
    """Run the batch to quiescence on the simulator's device.

    Returns ``(rows, delivered, first_round)``: per-round dicts (direct,
    relay, dropped, lost, arrived), copies of Message that reached ``dst[i]``,
    and the round the first one arrived (``0xFFFFFFFF`` = never).
    """
    ap = np.ascontiguousarray(act_ptr, dtype=np.uint64)
    ai = np.ascontiguousarray(act, dtype=np.uint32)
    op = np.ascontiguousarray(ol_ptr, dtype=np.uint64)
    oi = np.ascontiguousarray(ol, dtype=np.uint32)
    al = np.ascontiguousarray(alive, dtype=np.uint8)
    s = np.ascontiguousarray(src, dtype=np.uint32)
    d = np.ascontiguousarray(dst, dtype=np.uint32)
    n = len(ap) - 1
    if len(op) != n + 1 or len(al) != n or len(s) != len(d):
        raise ValueError("relay_run: shapes disagree")
    if ap[0] != 0 or int(ap[-1]) != len(ai) or op[0] != 0 or int(op[-1]) != len(oi):
        raise ValueError("relay_run: row pointers must start at 0 and end at the id array's length")
    k = len(s)
    dv = np.zeros(max(k, 1), dtype=np.uint64)
    fr = np.zeros(max(k, 1), dtype=np.uint32)
    st = (RelayStats * cap)()
    r = lib().psim_relay_run(sim._h, n, _p(ap, C.c_uint64), _p(ai, C.c_uint32), len(ai), _p(op, C.c_uint64),
                             _p(oi, C.c_uint32), len(oi), _p(al, C.c_uint8), k, _p(s, C.c_uint32), _p(d, C.c_uint32),
                             relay_ttl, _p(dv, C.c_uint64), _p(fr, C.c_uint32), st, cap, max_copies)
    if r < 0:
        raise PsimError(int(r), lib().psim_last_error(sim._h).decode())
    rows = [st[i].as_dict() for i in range(min(int(r), cap))]
    return rows, dv[:k], fr[:k]


def out_links_from(sim, row_ptr, col, roots=()):
    """CSR of every vertex's out_links (retrieve_outlinks/1 :2846-2870): its
    eager peers in its OWN tree.  A root in ``roots`` that broadcast through
    ``sim`` (a lane of the multi-root engine) reads them from that lane;
    every other vertex has no per-root entry for itself, so its out-links are
    the common eagers = its members (start_link/0 :253-254)."""
    rp = np.asarray(row_ptr, dtype=np.uint64)
    cl = np.asarray(col, dtype=np.uint32)
    n = len(rp) - 1
    rows = {}
    for r in roots:
        sim.focus(int(r))
        eager = sim.plumtree_state()[0]
        rows[int(r)] = [p for p in sim.mask_to_peers(int(r), eager[int(r)]) if p != int(r)]
    ptr = np.zeros(n + 1, dtype=np.uint64)
    ids = []
    for v in range(n):
        ids.extend(rows[v] if v in rows else cl[rp[v]:rp[v + 1]].tolist())
        ptr[v + 1] = len(ids)
    return ptr, np.asarray(ids, dtype=np.uint32)
