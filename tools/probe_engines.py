"""Per-round device time of the HyParView and causal engines at scale
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


if __name__ == "__main__":
    res = [hv(int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000, 5000), causal(1_000_000, 64, 12)]
    for r in res:
        print(json.dumps(r), flush=True)
