import sys, os
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/oracle'); sys.path.insert(0, '/root/repo/tests')
import numpy as np
import pyoracle as O
import partisan_amd as pa
from test_hyparview import contacts, SEED
n = 200
sim = pa.Simulator(seed=SEED)
g = pa.hyparview.HyParViewCluster(sim, n)
o = O.HyParView(n, SEED)
c = contacts(n)
prev_act = None
for i in range(1, n):
    act, na, pas, np_ = g.views()
    snap = [(act[v, :na[v]].tolist(), pas[v, :np_[v]].tolist(), o.views(v)) for v in range(n)]
    dr0 = g.draws().copy()
    od0 = [o.draws(v) for v in range(n)]
    g.join(i, int(c[i])); o.join(i, int(c[i]))
    gs = g.step(1)[0]; os_ = o.step(1)[0]
    dr = g.draws()
    bad = [v for v in range(n) if int(dr[v]) != o.draws(v)]
    act, na, pas, np_ = g.views()
    badv = [v for v in range(n) if act[v, :na[v]].tolist() != o.views(v)[0] or pas[v, :np_[v]].tolist() != o.views(v)[1]]
    if bad or badv or gs["sent"] != os_["sent"] or gs["draws"] != os_["draws"]:
        print("round", i, "stats", gs["sent"], os_["sent"], gs["draws"], os_["draws"])
        print("draw-diff vertices", bad[:10], "view-diff", badv[:10])
        for v in (bad + badv)[:4]:
            print(" v", v, "before gpu", snap[v][0], snap[v][1], "oracle", snap[v][2], "draws", int(dr0[v]), od0[v])
            print("   after gpu", act[v, :na[v]].tolist(), pas[v, :np_[v]].tolist(), int(dr[v]), "oracle", o.views(v), o.draws(v))
        break
else:
    print("no divergence")
