"""Multi-root heartbeats: R roots of a
10M-peer overlay heartbeat at once after a tree reset, run to quiescence of
every lane; prints device time per flood set and peer-rounds/s over all lanes.
usage: python tools/multiroot_bench.py [--n N] [--roots R] [--steps K]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import partisan_amd as pa  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=10_000_000)
p.add_argument("--roots", type=int, default=16)
p.add_argument("--steps", type=int, default=3)
a = p.parse_args()

rp, col = pa.overlay.random_regular(a.n, 5, 0x5EED0001)
sim = pa.Simulator(lazy_tick_rounds=1)
sim.load_overlay(rp, col)
roots = np.random.default_rng(7).choice(a.n, size=a.roots, replace=False).tolist()
res = []
for step in range(a.steps + 1):
    sim.reset_trees()
    for r in roots:
        sim.broadcast(int(r))
    ms0, _ = sim.timing()
    t0 = time.time()
    st, rounds = sim.run()
    wall = time.time() - t0
    ms = sim.timing()[0] - ms0
    if step:
        res.append((ms, wall, rounds))
ms = float(np.mean([x[0] for x in res]))
wall = float(np.mean([x[1] for x in res]))
rounds = res[-1][2]
print(json.dumps({"config": "MULTIROOT", "n": a.n, "roots": a.roots, "rounds": rounds, "kernel_ms": round(ms, 3),
                  "wall_ms": round(wall * 1e3, 3), "root_peer_rounds_per_s": a.roots * a.n * rounds / (wall),
                  "delivered_all": bool(sim.delivered().all()), "lib": os.environ.get("PSIM_LIB_PATH", "default")}))
