"""Per-round HyParView counters and kernel time after 1M-peer join waves
(which rounds cost what)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import partisan_amd as pa  # noqa: E402

n, wave = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000, 5000
sim = pa.Simulator(seed=0x5EED0002)
g = pa.hyparview.HyParViewCluster(sim, n)
rng = np.random.default_rng(9)
vs = np.arange(1, n, dtype=np.uint32)
for lo in range(0, n - 1, wave):
    v = vs[lo:lo + wave]
    g.join_many(v, (rng.random(len(v)) * v).astype(np.uint32))
    g.step(1)
for s in g.step(40):
    print(json.dumps({k: s[k] for k in ("sent", "processed", "active", "kernel_ms")}), flush=True)
