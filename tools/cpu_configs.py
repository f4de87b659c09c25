"""CPU baselines for the SURVEY 8(d) configurations C2-C5 (BASELINE.md
section 3): the oracle restatements (oracle/*.c, single-threaded C) timed on
the host's cores on a bounded sample of each workload, as peer-rounds/s
(vertices x rounds / seconds of the timed rounds).  "1 thread" is one
process; "all cores" runs P independent replicas (different seeds) in P
processes at once and sums their rates -- the oracle is a sequential
restatement, so replicas are how it uses more cores.  TEST INFRASTRUCTURE
(the oracle is only ever the checker / baseline, never the product path).

    python tools/cpu_configs.py [--workers P] [C2 C3 C4 C5]  > profiles/rNN/cpu_configs.jsonl
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def c2(seed, n=4000):
    """C2 sample: n-peer HyParView, sequential joins (one per round) + 10
    shuffle periods, then one Plumtree broadcast over the active views."""
    import numpy as np
    import pyoracle as O
    from partisan_amd.overlay import philox_uniform
    hv = O.HyParView(n, seed)
    t0 = time.perf_counter()
    rounds = 0
    for v in range(1, n):
        c = int(philox_uniform(seed, np.array([v], np.uint32), 0xC200, v)[0])
        hv.join(v, c)
        hv.step(1)
        rounds += 1
    hv.step(100)
    rounds += 100
    rows = []
    for v in range(n):
        a, _ = hv.views(v)
        rows.append(sorted(u for u in a if u != v))
    rp = np.zeros(n + 1, np.uint64)
    rp[1:] = np.cumsum([len(r) for r in rows])
    col = np.asarray([u for r in rows for u in r], np.uint32)
    pt = O.Plumtree(rp, col, 1)
    pt.heartbeat(0)
    _, pr = pt.run(1000)
    rounds += pr
    dt = time.perf_counter() - t0
    return dict(n=n, rounds=rounds, seconds=dt, sample=f"{n}-peer C2 (HyParView joins + 100 rounds + broadcast)")


def c3(seed, n=200_000, churn_rounds=20):
    """C3 sample: n-peer SCAMP v2 + Plumtree, built by join waves, then
    churn_rounds rounds of 5 % crash/rejoin with a heartbeat at vertex 0;
    only the churn rounds are timed."""
    import pyoracle as O
    from partisan_amd.scamp import churn_batch, join_waves
    g = O.C3(n, 5, 10, seed)
    for v, cc in join_waves(n, seed):
        for a, b in zip(v.tolist(), cc.tolist()):
            g.join(a, b)
        g.step(3)
    g.step(5)
    g.heartbeat(0)
    t0 = time.perf_counter()
    for i in range(churn_rounds):
        v, cc = churn_batch(n, seed, i)
        for a, b in zip(v.tolist(), cc.tolist()):
            if a == 0:
                continue
            g.crash(a)
            g.join(a, b)
        g.step(1)
    dt = time.perf_counter() - t0
    return dict(n=n, rounds=churn_rounds, seconds=dt, sample=f"{n}-peer C3, {churn_rounds} churn rounds")


def c4(seed, n=1_000_000, m=64):
    """C4 sample: n-peer Demers, 64 rumors, rumor mongering + anti-entropy to completion."""
    import pyoracle as O
    d = O.Demers(n, m, seed, 2, True)
    d.broadcast_all()
    t0 = time.perf_counter()
    _, r = d.run(400)
    dt = time.perf_counter() - t0
    return dict(n=n, rounds=r, seconds=dt, sample=f"{n}-peer Demers, {m} rumors, to completion")


def c5(seed, n=2000, m=64, rounds=16):
    """C5 sample: n-peer causal broadcast, 64 emitters with 64-lane vclocks, 16 rounds."""
    import pyoracle as O
    g = O.Causal(n, m=m, period=1, dmax=4, redeliver=1, seed=seed)
    t0 = time.perf_counter()
    g.step(rounds)
    dt = time.perf_counter() - t0
    return dict(n=n, rounds=rounds, seconds=dt, sample=f"{n}-peer causal, {m} emitters, {rounds} rounds")


FNS = {"C2": (c2, 0x5EED0002), "C3": (c3, 0x5EED0003), "C4": (c4, 0x5EED0004), "C5": (c5, 0x5EED0005)}


def _one(args):
    name, rep = args
    fn, seed = FNS[name]
    return fn(seed + 0x1000 * rep)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workers", type=int, default=min(16, os.cpu_count() or 1))
    p.add_argument("configs", nargs="*", default=["C2", "C3", "C4", "C5"])
    a = p.parse_args()
    for name in a.configs:
        r1 = _one((name, 0))
        one = r1["n"] * r1["rounds"] / r1["seconds"]
        t0 = time.perf_counter()
        with mp.get_context("spawn").Pool(a.workers) as pool:
            rs = pool.map(_one, [(name, k) for k in range(a.workers)])
        wall = time.perf_counter() - t0
        allc = sum(r["n"] * r["rounds"] for r in rs) / max(r["seconds"] for r in rs)
        print(json.dumps(dict(config=name, sample=r1["sample"], rounds=r1["rounds"],
                              one_thread_peer_rounds_per_s=round(one), one_thread_seconds=round(r1["seconds"], 3),
                              all_cores_peer_rounds_per_s=round(allc), all_cores_processes=a.workers,
                              all_cores_wall_s=round(wall, 2))), flush=True)


if __name__ == "__main__":
    main()
