"""Per-round breakdown of one 10M-peer flood (diagnostic; prints a table)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import partisan_amd as pa  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=10_000_000)
p.add_argument("--peers", type=int, default=5)
p.add_argument("--steps", type=int, default=3)
p.add_argument("--binned", action="store_true")
a = p.parse_args()

rp, col = pa.overlay.random_regular(a.n, a.peers, 0x5EED0001)
sim = pa.Simulator(binned=a.binned)
sim.load_overlay(rp, col)
for step in range(a.steps):
    sim.reset_trees()
    sim.broadcast(0)
    st, r = sim.run()
    if step == a.steps - 1:
        print(f"n={a.n} rounds={r}")
        print(f"{'r':>3} {'ms':>8} {'bcast':>9} {'prune':>9} {'ihave':>7} {'deliv':>9} {'active':>9} "
              f"{'senders':>9} {'algoMB':>8} {'GB/s':>7}")
        for i, s in enumerate(st):
            gbs = s["algo_bytes"] / (s["kernel_ms"] * 1e-3) / 1e9
            print(f"{i+1:>3} {s['kernel_ms']:8.3f} {s['broadcast']:9d} {s['prune']:9d} {s['i_have']:7d} "
                  f"{s['delivered_new']:9d} {s['active']:9d} {s['senders']:9d} "
                  f"{s['algo_bytes']/1e6:8.1f} {gbs:7.0f}")
        tot = sum(s["kernel_ms"] for s in st)
        print(f"total kernel ms {tot:.3f}; algo GB {sum(s['algo_bytes'] for s in st)/1e9:.3f}")
