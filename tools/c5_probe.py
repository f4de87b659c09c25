"""C5 causal round kernel probe (diagnostic): 1M peers, 64 emitters, P=1,
D=4, R=1 -- a few rounds, for rocprofv3 --pmc passes on cs_round_kernel."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import partisan_amd as pa  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
sim = pa.Simulator(seed=0x5EED0005)
g = pa.causal.CausalCluster(sim, n, m=64, period=1, dmax=4, redeliver=1)
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 8
st = g.step(rounds)
print({k: st[-1][k] for k in ("received", "delivered", "checks", "buffered", "kernel_ms")})
ms = [s["kernel_ms"] for s in st[4:]]
print("kernel ms per round, rounds 5..%d: mean %.3f min %.3f max %.3f" % (rounds, sum(ms) / len(ms), min(ms), max(ms)))
sim.close()
