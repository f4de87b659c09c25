"""Per-round device time of the HyParView, causal and C3 engines at scale
(writes a summary line per engine; used for DESIGN.md / profiles)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np

import partisan_amd as pa


def hv(n, wave):
    sim = pa.Simulator(seed=0x5EED0002)
    g = pa.hyparview.HyParViewCluster(sim, n)
    rng = np.random.default_rng(9)
    vs = np.arange(1, n, dtype=np.uint32)
    st = []
    t0 = time.time()
    for lo in range(0, n - 1, wave):
        v = vs[lo:lo + wave]
        g.join_many(v, (rng.random(len(v)) * v).astype(np.uint32))
        st += g.step(1)
    st += g.step(40)
    wall = time.time() - t0
    ms = sum(s["kernel_ms"] for s in st)
    last = st[-40:]
    out = dict(engine="hyparview", n=n, rounds=len(st), wall_s=round(wall, 3), kernel_ms_total=round(ms, 3),
               steady_ms_per_round=round(sum(s["kernel_ms"] for s in last) / len(last), 4),
               steady_msgs_per_round=sum(s["processed"] for s in last) / len(last),
               steady_GBps=round(sum(s["algo_bytes"] for s in last) / 1e6 / sum(s["kernel_ms"] for s in last), 1))
    sim.close()
    return out


def causal(n, m, rounds):
    sim = pa.Simulator(seed=0x5EED0005)
    g = pa.causal.CausalCluster(sim, n, m=m, period=1, dmax=4, redeliver=1)
    st = g.step(rounds)
    last = st[4:]
    ms = sum(s["kernel_ms"] for s in last)
    out = dict(engine="causal", n=n, m=m, rounds=rounds, ms_per_round=round(ms / len(last), 4),
               deliveries_per_round=sum(s["delivered"] for s in last) / len(last),
               deliveries_per_s=sum(s["delivered"] for s in last) / (ms / 1e3),
               algo_GBps=round(sum(s["algo_bytes"] for s in last) / 1e6 / ms, 1))
    sim.close()
    return out


def c3(n, churn_rounds, hb_every=10, seed=0x5EED0003):
    """C3: 1M-peer SCAMP v2 + Plumtree repair, 5 % crash/rejoin churn per
    round, a heartbeat at vertex 0 every `hb_every` rounds."""
    from partisan_amd.scamp import churn_batch, join_waves
    sim = pa.Simulator(seed=seed)
    g = pa.c3.C3Cluster(sim, n, c=5, periodic_rounds=10)
    for v, cc in join_waves(n, seed):
        g.join(v, cc)
        g.step(3)
    g.step(5)
    st, host_s = [], 0.0
    t0 = time.time()
    for i in range(churn_rounds):
        if i % hb_every == 0:
            g.heartbeat(0)
        h0 = time.time()
        v, cc = churn_batch(n, seed, i)
        keep = v != 0
        host_s += time.time() - h0
        g.crash(v[keep])
        g.join(v[keep], cc[keep])
        st += g.step(1)
    wall = time.time() - t0
    sc_ms = sum(s["scamp"]["kernel_ms"] for s in st)
    pt_ms = sum(s["pt_kernel_ms"] for s in st)
    out = dict(engine="c3", n=n, churn_rounds=churn_rounds, churn_per_round=int(n * 0.05),
               wall_s_per_round=round((wall - host_s) / churn_rounds, 4),
               scamp_ms_per_round=round(sc_ms / churn_rounds, 4), plumtree_ms_per_round=round(pt_ms / churn_rounds, 4),
               peer_rounds_per_s_device=n * churn_rounds / ((sc_ms + pt_ms) / 1e3),
               scamp_msgs_per_round=sum(s["scamp"]["processed"] for s in st) / churn_rounds,
               plumtree_msgs_per_round=sum(sum(s["pt_sent"].values()) for s in st) / churn_rounds,
               graft_total=sum(s["pt_sent"]["graft"] for s in st),
               delivered_live_last=st[-1]["delivered_live"], live_last=st[-1]["live"],
               scamp_GBps=round(sum(s["scamp"]["algo_bytes"] for s in st) / 1e6 / sc_ms, 1),
               plumtree_GBps=round(sum(s["pt_algo_bytes"] for s in st) / 1e6 / pt_ms, 1))
    sim.close()
    return out


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "c3":
        print(json.dumps(c3(int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000, 30)), flush=True)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "hv":
        print(json.dumps(hv(int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000, 5000)), flush=True)
        sys.exit(0)
    res = [hv(int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000, 5000), causal(1_000_000, 64, 12)]
    for r in res:
        print(json.dumps(r), flush=True)
