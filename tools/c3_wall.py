"""C3 wall-time split (diagnostic): per churn round, the host time of each
driver call (crash, join, step, heartbeat) against the device time of the
round's SCAMP and Plumtree kernels -- where a C3 round's wall time goes.

Churn rounds 0 .. R-1 run untimed, rounds R .. 2R-1 are timed.  With a third
argument "run" each R rounds go through one psim_c3_run call (C3Cluster.run:
no host wait between rounds; the churn is drawn beforehand and not timed,
the flat plan's build is reported apart).

usage: python tools/c3_wall.py [n] [rounds] [run]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import partisan_amd as pa  # noqa: E402
from partisan_amd.scamp import churn_batch, join_waves  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    seed = 0x5EED0003
    sim = pa.Simulator(seed=seed)
    g = pa.c3.C3Cluster(sim, n, c=5, periodic_rounds=10)
    for v, cc in join_waves(n, seed):
        g.join(v, cc)
        g.step(3)
    g.step(5)
    if len(sys.argv) > 3 and sys.argv[3] == "run":
        def draw(lo):
            plan = []
            for i in range(lo, lo + rounds):
                v, cc = churn_batch(n, seed, i)
                keep = v != 0
                plan.append((v[keep], cc[keep]))
            return plan
        # a first call of the same shape (churn rounds 0 .. rounds-1, untimed)
        # allocates the call's pinned and device buffers; the second call
        # (rounds .. 2 rounds - 1) is timed
        warm = draw(0)
        g.run([p[0] for p in warm], [(p[0], p[1]) for p in warm], heartbeat_every=10, root=0)
        plan = draw(rounds)
        t0 = time.perf_counter()
        fp = g.plan([p[0] for p in plan], [(p[0], p[1]) for p in plan])
        t1 = time.perf_counter()
        st = g.run(plan=fp, heartbeat_every=10, root=0)
        wall = time.perf_counter() - t1
        print(json.dumps({"mode": "psim_c3_run", "n": n, "rounds": rounds,
                          "wall_ms_per_round": round(1e3 * wall / rounds, 4),
                          "plan_ms_per_round": round(1e3 * (t1 - t0) / rounds, 4),
                          "scamp_kernel_ms": round(sum(s["scamp"]["kernel_ms"] for s in st) / rounds, 4),
                          "plumtree_kernel_ms": round(sum(s["pt_kernel_ms"] for s in st) / rounds, 4),
                          "delivered_live_last": st[-1]["delivered_live"], "live_last": st[-1]["live"]}),
              flush=True)
        sim.close()
        return
    for i in range(rounds):            # churn rounds 0 .. rounds-1 untimed, as the run mode's first call
        if i % 10 == 0:
            g.heartbeat(0)
        v, cc = churn_batch(n, seed, i)
        keep = v != 0
        g.crash(v[keep])
        g.join(v[keep], cc[keep])
        g.step(1)
    t = {"heartbeat": 0.0, "churn_draw": 0.0, "crash": 0.0, "join": 0.0, "step": 0.0}
    sc_ms = pt_ms = 0.0
    t0 = time.perf_counter()
    for i in range(rounds, 2 * rounds):
        a = time.perf_counter()
        if i % 10 == 0:
            g.heartbeat(0)
        b = time.perf_counter()
        v, cc = churn_batch(n, seed, i)
        keep = v != 0
        c = time.perf_counter()
        g.crash(v[keep])
        d = time.perf_counter()
        g.join(v[keep], cc[keep])
        e = time.perf_counter()
        st = g.step(1)
        f = time.perf_counter()
        t["heartbeat"] += b - a
        t["churn_draw"] += c - b
        t["crash"] += d - c
        t["join"] += e - d
        t["step"] += f - e
        sc_ms += st[0]["scamp"]["kernel_ms"]
        pt_ms += st[0]["pt_kernel_ms"]
    wall = time.perf_counter() - t0
    out = {k: round(1e3 * x / rounds, 4) for k, x in t.items()}
    out.update(n=n, rounds=rounds, wall_ms_per_round=round(1e3 * wall / rounds, 4),
               wall_ms_per_round_excl_draw=round(1e3 * (wall - t["churn_draw"]) / rounds, 4),
               scamp_kernel_ms=round(sc_ms / rounds, 4), plumtree_kernel_ms=round(pt_ms / rounds, 4))
    print(json.dumps(out), flush=True)
    sim.close()


if __name__ == "__main__":
    main()
