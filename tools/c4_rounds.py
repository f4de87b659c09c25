import sys, os
sys.path.insert(0, os.getcwd())
import partisan_amd as pa
sim = pa.Simulator(seed=0x5EED0004)
dm = pa.demers.DemersEpidemic(sim, 10_000_000, 64, 2, True)
dm.broadcast()
st, r = dm.run(400)
for i, s in enumerate(st):
    print(i + 1, round(s["kernel_ms"], 3), s["rm_sent"], s["push_sent"], s["pull_sent"], s["delivered_new"], s["complete"])
