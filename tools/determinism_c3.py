"""Diagnostic: per-round signature of a C3 run (SCAMP counters, view sums,
Plumtree counters), written as JSON so that two processes can be compared."""
import json
import sys

sys.path.insert(0, "/root/repo")
import partisan_amd as pa  # noqa: E402
from partisan_amd.scamp import churn_batch, join_waves  # noqa: E402


def run(n, rounds, seed=0x5EED0003, hb=True):
    sim = pa.Simulator(seed=seed)
    g = pa.c3.C3Cluster(sim, n, c=5, periodic_rounds=10)
    sig = []

    def rec(s, tag):
        sig.append([tag, s["scamp"]["sent"], s["scamp"]["processed"], s["scamp"]["draws"], s["scamp"]["pv_sum"],
                    s["scamp"]["inview_sum"], s["scamp"]["resub"], s["scamp"]["stopped"], s["pt_sent"],
                    s["delivered_live"], s["updates"]])

    for w, (v, cc) in enumerate(join_waves(n, seed)):
        g.join(v, cc)
        for s in g.step(3):
            rec(s, "wave%d" % w)
    for s in g.step(5):
        rec(s, "warm")
    for i in range(rounds):
        if hb and i % 10 == 0:
            g.heartbeat(0)
        v, cc = churn_batch(n, seed, i)
        keep = v != 0
        g.crash(v[keep])
        g.join(v[keep], cc[keep])
        rec(g.step(1)[0], "churn%d" % i)
    sim.close()
    return sig


if __name__ == "__main__":
    n = int(sys.argv[1])
    json.dump(run(n, int(sys.argv[2])), open(sys.argv[3], "w"))
