"""Configuration C3: Plumtree broadcast repaired by graft/prune over churning
SCAMP v2 membership (oracle/c3.c composes the two restatements; csrc/ptdyn.hip
+ csrc/scamp.hip on the device).

CPU: the composition's behaviour -- the flood prunes redundant links and
announces lazy rows (i_have); restarted vertices lose the heartbeat.
GPU: bit-exact against the oracle round by round (both protocols' counters,
SCAMP views, every vertex's eager / lazy / outstanding sets, delivery and
pushed Round) through join waves, a heartbeat and 5 % crash/rejoin churn;
and the 1M-peer C3 shape.
"""
import numpy as np
import pytest

import pyoracle as O
from test_scamp import churn, waves

SEED = 0x5EED0003


def build_oracle(n, periodic, warm):
    c = O.C3(n, 5, periodic, SEED)
    for v, cc in waves(n):
        for a, b in zip(v, cc):
            c.join(int(a), int(b))
        c.step(3)
    c.step(warm)
    return c


def test_c3_oracle_repair_and_churn():
    n = 2000
    c = build_oracle(n, 10, 5)
    st = []
    for _ in range(3):                  # later heartbeats find lazy links: i_have / graft repair
        mono = c.heartbeat(0)
        st.append(c.step(9))
    assert sum(x["pt"]["prune"] for x in st[0]) > 0
    assert sum(x["pt"]["i_have"] for x in st[2]) > 0
    assert sum(x["pt"]["graft"] for x in st[2]) > 0
    assert sum(x["pt"]["ignored_i_have"] for x in st[2]) > 0
    assert st[2][-1]["delivered_live"] > n // 2
    v, cc = churn(n, 3)
    keep = v != 0
    v, cc = v[keep], cc[keep]
    for a in v:
        c.crash(int(a))
    d = c.pt.delivered(0, mono)
    assert not any(d[int(a)] for a in v)     # the restarted nodes lost the heartbeat
    for a, b in zip(v, cc):
        c.join(int(a), int(b))
    c.step(3)


def test_c3_run_plan_layout():
    """C3Cluster.plan: per-round lists flattened into psim_c3_run's arrays --
    offsets of R + 1 entries from 0, lists concatenated in round order, join
    vertices and contacts aligned; empty rounds are empty ranges."""
    import partisan_amd as pa
    crashes = [np.array([4, 2], np.uint32), np.zeros(0, np.uint32), np.array([9], np.int64)]
    joins = [(np.array([4, 2]), np.array([1, 1])), (np.zeros(0), np.zeros(0)), (np.array([9]), np.array([3]))]
    co, cv, jo, jv, jc = pa.c3.C3Cluster.plan(crashes, joins)
    assert co.tolist() == [0, 2, 2, 3] and cv.tolist() == [4, 2, 9]
    assert jo.tolist() == [0, 2, 2, 3] and jv.tolist() == [4, 2, 9] and jc.tolist() == [1, 1, 3]
    assert all(x.dtype == np.uint32 and x.flags.c_contiguous for x in (co, cv, jo, jv, jc))
    with pytest.raises(ValueError):
        pa.c3.C3Cluster.plan(crashes, joins[:2])


def _compare(g, o, n, root, mono):
    pv, npv, iv, niv = g.scamp.views()
    od = o.pt.delivered(root, mono) if mono else np.zeros(n, np.uint8)
    orr = o.pt.recv_round(root, mono) if mono else None
    for v in range(n):
        assert list(pv[v, :npv[v]]) == o.scamp.view(v), v
        if not o.scamp.alive(v):
            continue
        ge, gl, go, gm, gr = g.plumtree(v)
        oe, ol = o.pt.peers(v, root)
        assert ge == oe and gl == ol, (v, ge, oe, gl, ol)
        assert go == sorted({p for p, _, _ in o.pt.outstanding(v)}), v
        assert (gm == mono and mono != 0) == bool(od[v]), v
        if mono and od[v]:
            want = 0 if orr[v] == 0xFFFFFFFE else int(orr[v]) + 1
            assert gr == want, (v, gr, want)


def _step(g, o, r):
    gs, os_ = g.step(1)[0], o.step(1)[0]
    for k in ("sent", "dropped", "processed", "draws", "stopped", "pv_sum", "inview_sum", "resub"):
        assert gs["scamp"][k] == os_["scamp"][k], (r, "scamp", k)
    for k in ("broadcast", "prune", "i_have", "ignored_i_have", "graft"):
        assert gs["pt_sent"][k] == os_["pt"][k], (r, k, gs["pt_sent"], os_["pt"])
    assert gs["pt_dropped"] == os_["pt_dropped"], r
    assert gs["delivered_new"] == os_["pt"]["delivered_new"], r
    assert gs["active"] == os_["pt"]["active"], r
    assert gs["delivered_live"] == os_["delivered_live"] and gs["live"] == os_["live"], r
    return gs


@pytest.mark.gpu
@pytest.mark.parametrize("n,periodic,warm,churn_rounds", [(1500, 2, 16, 14), (3000, 10, 5, 10)])
def test_gpu_c3_parity(n, periodic, warm, churn_rounds):
    import partisan_amd as pa
    sim = pa.Simulator(device=0, seed=SEED)
    g = pa.c3.C3Cluster(sim, n, c=5, periodic_rounds=periodic)
    o = O.C3(n, 5, periodic, SEED)
    r = 0
    seen = []
    for v, cc in waves(n):
        g.join(v, cc)
        for a, b in zip(v, cc):
            o.join(int(a), int(b))
        for _ in range(3):
            _step(g, o, r)
            r += 1
    for _ in range(warm):
        _step(g, o, r)
        r += 1
    _compare(g, o, n, 0, 0)
    for _ in range(2):                  # a settled tree first: the next heartbeats use lazy links
        mono = g.heartbeat(0)
        assert mono == o.heartbeat(0)
        for _ in range(8):
            seen.append(_step(g, o, r))
            r += 1
        _compare(g, o, n, 0, mono)
    for i in range(churn_rounds):
        if i % 5 == 0:
            mono = g.heartbeat(0)
            assert mono == o.heartbeat(0)
        v, cc = churn(n, i)
        keep = v != 0
        v, cc = v[keep], cc[keep]
        g.crash(v)
        g.join(v, cc)
        for a, b in zip(v, cc):
            o.crash(int(a))
            o.join(int(a), int(b))
        seen.append(_step(g, o, r))
        r += 1
        _compare(g, o, n, 0, mono)
    for k in ("prune", "i_have", "ignored_i_have", "graft"):    # the repair paths were exercised
        assert sum(x["pt_sent"][k] for x in seen) > 0, k
    assert sum(x["pt_dropped"] for x in seen) > 0


@pytest.mark.gpu
def test_gpu_c3_1m():
    """C3 at 1M peers: join waves, heartbeat, 5 % churn per round; sanity of
    the device counters (oracle parity is covered above)."""
    import partisan_amd as pa
    n = 1_000_000
    sim = pa.Simulator(device=0, seed=SEED)
    g = pa.c3.C3Cluster(sim, n, c=5, periodic_rounds=10)
    for v, cc in waves(n):
        g.join(v, cc)
        g.step(3)
    g.step(5)
    g.heartbeat(0)
    st = g.step(10)
    for i in range(10):
        v, cc = churn(n, i)
        keep = v != 0
        g.crash(v[keep])
        g.join(v[keep], cc[keep])
        st += g.step(1)
    assert st[5]["delivered_live"] > 0
    assert all(x["live"] > 0.99 * n for x in st)


def _strip(st):
    out = []
    for x in st:
        x = dict(x)
        x.pop("pt_kernel_ms")
        x["scamp"] = {k: v for k, v in x["scamp"].items() if k != "kernel_ms"}
        out.append(x)
    return out


@pytest.mark.gpu
def test_gpu_c3_run_equals_per_round_calls():
    """psim_c3_run (churn rounds enqueued with no host wait between them) is
    the same as psim_c3_heartbeat / crash / join / step one by one: every
    round's counters, then both protocols' state at every vertex.  Two run
    calls of different lengths (the pinned rows are reused and grown)."""
    import partisan_amd as pa
    n, periodic = 3000, 10
    gs = []
    for _ in range(2):
        sim = pa.Simulator(device=0, seed=SEED)
        g = pa.c3.C3Cluster(sim, n, c=5, periodic_rounds=periodic)
        for v, cc in waves(n):
            g.join(v, cc)
            g.step(3)
        g.step(5)
        gs.append((sim, g))
    plan = []
    for i in range(17):
        v, cc = churn(n, i)
        keep = v != 0
        plan.append((v[keep], v[keep], cc[keep]))
    (sa, a), (sb, b) = gs
    per_round = []
    for i, (cr, jv, jc) in enumerate(plan):
        if i % 5 == 0:
            a.heartbeat(7)
        a.crash(cr)
        a.join(jv, jc)
        per_round += a.step(1)

    def run(lo, hi, **kw):
        return b.run([p[0] for p in plan[lo:hi]], [(p[1], p[2]) for p in plan[lo:hi]], **kw)

    # heartbeats at rounds 0, 5 (first call), none in 6..9, 10 and 15 (offsets 0 and 5 of the third)
    out = run(0, 6, heartbeat_every=5, root=7) + run(6, 10) + run(10, 17, heartbeat_every=5, root=7)
    assert len(out) == 17
    assert _strip(out) == _strip(per_round)
    pva, npva, _, _ = a.scamp.views()
    pvb, npvb, _, _ = b.scamp.views()
    assert (npva == npvb).all() and (pva == pvb).all()
    for v in range(n):
        assert a.plumtree(v) == b.plumtree(v), v
    assert sum(x["pt_sent"]["graft"] + x["pt_sent"]["prune"] for x in out) > 0
    sa.close()
    sb.close()


@pytest.mark.gpu
def test_gpu_c3_run_rejects_bad_lists():
    """psim_c3_run checks a round's lists before it enqueues that round:
    offsets that go backwards and a crash list naming a vertex twice are
    PSIM_EINVAL with nothing of that round run, and the handle stays usable."""
    import partisan_amd as pa
    from partisan_amd._lib import PsimError
    n = 500
    sim = pa.Simulator(device=0, seed=SEED)
    g = pa.c3.C3Cluster(sim, n, c=5, periodic_rounds=10)
    for v, cc in waves(n):
        g.join(v, cc)
        g.step(3)
    co, cv, jo, jv, jc = g.plan([np.array([5, 6], np.uint32)], [(np.zeros(0, np.uint32), np.zeros(0, np.uint32))])
    with pytest.raises(PsimError) as ei:
        g.run(plan=(np.array([2, 1], np.uint32), cv, jo, jv, jc))
    assert ei.value.name == "PSIM_EINVAL"
    with pytest.raises(PsimError) as ei:
        g.run([np.array([7, 9, 7], np.uint32)], [(np.zeros(0, np.uint32), np.zeros(0, np.uint32))])
    assert ei.value.name == "PSIM_EINVAL"
    g.join(np.array([11], np.uint32), np.array([3], np.uint32))      # a join not yet stepped
    with pytest.raises(PsimError) as ei:
        g.run([np.zeros(0, np.uint32)], [(np.zeros(0, np.uint32), np.zeros(0, np.uint32))])
    assert ei.value.name == "PSIM_ESTATE"
    g.step(1)
    st = g.run([np.array([7, 9], np.uint32)], [(np.array([7, 9], np.uint32), np.array([1, 2], np.uint32))],
               heartbeat_every=1, root=0)
    assert len(st) == 1 and st[0]["live"] == n
    sim.close()


@pytest.mark.gpu
def test_gpu_large_crash_list_resets_every_vertex():
    """A crash list larger than any before grows the device list buffer; the
    upload must land after the buffer's zero fill (regression: the fill ran
    on the null stream, unordered with the handle's stream, and could wipe
    the list).  Every listed vertex must come back in its start_link state."""
    import partisan_amd as pa
    n = 1_000_000
    sim = pa.Simulator(device=0, seed=SEED)
    g = pa.c3.C3Cluster(sim, n, c=5, periodic_rounds=10)
    for v, cc in waves(n)[:12]:
        g.join(v, cc)
        g.step(3)
    pv0, npv0, _, _ = g.scamp.views()
    fresh = pa.Simulator(device=0, seed=SEED)
    f = pa.c3.C3Cluster(fresh, n, c=5, periodic_rounds=10)
    fpv, fnpv, _, _ = f.scamp.views()
    for k in (2_000, 60_000, 200_000):          # growing lists
        v, _ = churn(n, k, frac=k / n)
        v = v[v != 0]
        g.crash(v)
        pv, npv, _, _ = g.scamp.views()
        assert np.array_equal(npv[v], fnpv[v])
        assert all(pv[x, :npv[x]].tolist() == fpv[x, :fnpv[x]].tolist() for x in v[:2000])
    sim.close()
    fresh.close()


def _max_grafts_per_sender(o):
    """Largest number of grafts one vertex sent in the last round (the oracle's in-flight list)."""
    import collections
    c = collections.Counter(s for s, _d, t, _r in o.pt.pending() if t == 5)
    return max(c.values()) if c else 0


@pytest.mark.gpu
def test_gpu_c3_many_grafts_per_vertex_round():
    """the per-kind send counters of pd_process are packed 12 bits
    per kind into one u64; graft used to sit at bit 60 with 4 bits, so a vertex
    sending more than 15 grafts in one round lost counts.  A heartbeat every
    round with 20 % churn every second round makes vertices answer 16+ i_haves of
    distinct undelivered serials in one tick (the oracle's in-flight list
    proves the case is reached; up to ~200 outstanding rows per vertex, within
    kPdRows); counters and state must stay bit-exact."""
    import partisan_amd as pa
    n, periodic = 300, 2
    sim = pa.Simulator(device=0, seed=SEED)
    g = pa.c3.C3Cluster(sim, n, c=5, periodic_rounds=periodic)
    o = O.C3(n, 5, periodic, SEED)
    r = 0
    for v, cc in waves(n):
        g.join(v, cc)
        for a, b in zip(v, cc):
            o.join(int(a), int(b))
        for _ in range(3):
            _step(g, o, r)
            r += 1
    for _ in range(30):
        _step(g, o, r)
        r += 1
    most = 0
    mono = 0
    for i in range(40):
        if i < 30:
            mono = g.heartbeat(0)
            assert mono == o.heartbeat(0)
        _step(g, o, r)
        r += 1
        most = max(most, _max_grafts_per_sender(o))
        if i % 2 == 0:
            v, cc = churn(n, i, frac=0.2)
            keep = v != 0
            v, cc = v[keep], cc[keep]
            g.crash(v)
            g.join(v, cc)
            for a, b in zip(v, cc):
                o.crash(int(a))
                o.join(int(a), int(b))
    _compare(g, o, n, 0, mono)
    assert most > 15, most
