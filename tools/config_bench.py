"""Throughput of the SURVEY 8(d) configurations other than the headline one
(bench.py measures the 10M-peer Plumtree broadcast).  One JSON line per
config: device time from the engines' hipEvents, the 8(d) algorithmic bytes
and their fraction of the 8 TB/s HBM roofline.  Synthetic inputs; run on the
GPU box:  python tools/config_bench.py > profiles/rNN/configs.jsonl
  C2  10k-peer HyParView overlay (sequential joins, 10 shuffle periods) + one Plumtree broadcast
  C3  1M-peer SCAMP v2, 5 % churn per round + Plumtree repair (tools/probe_engines.py c3)
  C4  10M-peer Demers rumor mongering (fanout 2) + anti-entropy (fanout 2, every 2 rounds), 64 rumors, 1 GPU
  C5  1M-peer causal broadcast, 64 emitters with 64-lane vclocks, 1 GPU
  C2ALL  every node heartbeats: the C2 overlay (10k HyParView peers) with all
         10k roots heartbeating at once, two intervals, on a forest handle (max_roots = 10k)
  RELAY  10M-peer transitive relay: 100k random sends, relay_ttl 3,
         5-peer views, out-links = members (no per-root entry), 1 GPU
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import partisan_amd as pa  # noqa: E402

HBM = 8000.0   # GB/s, MI355X peak (MI355X_MICROARCH.md)


def line(cfg, **kw):
    print(json.dumps(dict(config=cfg, **kw)), flush=True)


def c2():
    n = 10_000
    sim = pa.Simulator(seed=0x5EED0002)
    hv = pa.hyparview.HyParViewCluster(sim, n)
    from partisan_amd.overlay import philox_uniform
    t0 = time.time()
    # vertex v joins a Philox contact in [0, v), one join per round: the whole
    # sequence in one call (psim_hv_join_seq = join + step(1) per vertex)
    vs = np.arange(1, n, dtype=np.uint32)
    st = hv.join_seq(vs, philox_uniform(0x5EED0002, vs, 0xC200, vs), rounds=1)
    st += hv.step(10 * 10)                       # 10 shuffle periods (shuffle every 10 rounds)
    wall = time.time() - t0
    rp, col = hv.overlay()
    sim.load_overlay(rp, col)
    sim.broadcast(0)
    pst, rounds = sim.run()
    hv_ms = sum(s["kernel_ms"] for s in st)
    pt_ms = sum(s["kernel_ms"] for s in pst)
    line("C2", n=n, hyparview_rounds=len(st), hyparview_kernel_ms=round(hv_ms, 3),
         hyparview_ms_per_round=round(hv_ms / len(st), 4), hyparview_wall_s=round(wall, 2),
         plumtree_rounds=rounds, plumtree_kernel_ms=round(pt_ms, 3), delivered=int(sim.delivered().sum()),
         note="latency-bound at 10k peers: one join per round, as the sequential-join schedule prescribes")
    sim.close()


def c2_overlay(n=10_000):
    sim = pa.Simulator(seed=0x5EED0002)
    hv = pa.hyparview.HyParViewCluster(sim, n)
    from partisan_amd.overlay import philox_uniform
    vs = np.arange(1, n, dtype=np.uint32)
    hv.join_seq(vs, philox_uniform(0x5EED0002, vs, 0xC200, vs), rounds=1)
    hv.step(10 * 10)
    rp, col = hv.overlay()
    sim.close()
    return rp, col


def c2_all_roots(n=10_000, intervals=2):
    """Every node's heartbeat tree at once: all n roots heartbeat, rounds to
    quiescence, twice (the second interval travels the pruned trees).
    root-peer-rounds/s = roots x peers x rounds / device time; bytes = the
    touched-state model of bench.py summed over every root's lane."""
    rp, col = c2_overlay(n)
    sim = pa.Simulator(seed=0x5EED0002, max_roots=n, chunk_timing=True)
    sim.load_overlay(rp, col)
    out = []
    for it in range(intervals):
        t0 = time.time()
        sim.broadcast_many(np.arange(n, dtype=np.uint32))
        bc_s = time.time() - t0
        st, rounds = sim.run()
        ms = sum(s["kernel_ms"] for s in st)
        msgs = sum(sum(s[k] for k in ("broadcast", "prune", "i_have", "ignored_i_have", "graft")) for s in st)
        tb = sum(16 * s["active"] + 8 * s["senders"] + 4 * s["sender_degree_sum"] +
                 32 * sum(s[k] for k in ("broadcast", "prune", "i_have", "ignored_i_have", "graft")) for s in st)
        words = sum(s["words_stored"] for s in st)
        out.append(dict(interval=it + 1, rounds=rounds, kernel_ms=round(ms, 3), broadcast_call_s=round(bc_s, 4),
                        messages=msgs, words=words, delivered_new=sum(s["delivered_new"] for s in st),
                        root_peer_rounds_per_s=n * n * rounds / (ms / 1e3),
                        touched_GBps=round(tb / 1e6 / ms, 1), hbm_frac=round(tb / 1e6 / ms / HBM, 4),
                        words_per_s=words / (ms / 1e3), random_frac=round(words / (ms / 1e3) / 54.7e9, 4),
                        per_round_ms=[round(s["kernel_ms"], 3) for s in st]))
    sim.close()
    line("C2ALL", n=n, roots=n, engine="forest (max_roots)", intervals=out)


def c4(n=10_000_000, m=64):
    sim = pa.Simulator(seed=0x5EED0004)
    dm = pa.demers.DemersEpidemic(sim, n, m, 2, True)
    dm.broadcast()
    t0 = time.time()
    st, r = dm.run(400)
    wall = time.time() - t0
    ms = sum(s["kernel_ms"] for s in st)
    b = sum(s["algo_bytes"] for s in st)
    gbs = b / 1e6 / ms
    # the round is a stream of random 8-byte accesses: an RM send is one
    # atomicOr (its cascade rarely goes further), an AE push an atomicAdd on
    # the target's count plus the list store, a pull reply a snapshot load plus
    # the reply store -- priced against the chip's random 4-byte scatter rate
    # into a 200 MB target (54.24 G ops/s, profiles/r01/microbench2.txt:3)
    rnd = sum(s["rm_sent"] + 2 * s["push_sent"] + 2 * s["pull_sent"] for s in st)
    line("C4", n=n, rumors=m, rounds=r, complete=int(st[-1]["complete"]), kernel_ms=round(ms, 3),
         ms_per_round=round(ms / r, 4), wall_s=round(wall, 3), peer_rounds_per_s=n * r / (ms / 1e3),
         algo_GBps=round(gbs, 1), hbm_frac=round(gbs / HBM, 4),
         messages=int(sum(s["rm_sent"] + s["push_sent"] + s["pull_sent"] for s in st)),
         random_ops=int(rnd), random_Gops=round(rnd / ms / 1e6, 2), random_frac=round(rnd / ms / 1e6 / 54.24, 3))
    sim.close()


def c5(n=1_000_000, m=64, rounds=16):
    sim = pa.Simulator(seed=0x5EED0005)
    g = pa.causal.CausalCluster(sim, n, m=m, period=1, dmax=4, redeliver=1)
    st = g.step(rounds)
    last = st[4:]
    ms = sum(s["kernel_ms"] for s in last)
    # no HBM fraction: the round kernel moves ~0.5 GB per round (clocks in and
    # out, buffers; two 256-byte base rows per check come from L2) and is bound by
    # instruction issue (the scalar and vector pipes of the per-arrival fold),
    # DESIGN.md "Causal delivery" gives the SQ_INSTS_SALU / VALU bound
    line("C5", n=n, emitters=m, rounds=rounds, ms_per_round=round(ms / len(last), 4),
         deliveries_per_round=sum(s["delivered"] for s in last) / len(last),
         checks_per_round=sum(s["checks"] for s in last) / len(last), buffered_end=int(last[-1]["buffered"]),
         deliveries_per_s=sum(s["delivered"] for s in last) / (ms / 1e3),
         bound="instruction issue (SALU/VALU), not HBM")
    sim.close()


def relay(n=10_000_000, k=100_000, ttl=3):
    rp, col = pa.overlay.random_regular(n, 5, 0x5EED0006)
    rng = np.random.default_rng(6)
    src = rng.integers(0, n, size=k).astype(np.uint32)
    dst = rng.integers(0, n - 1, size=k).astype(np.uint32)
    dst = np.where(dst >= src, dst + 1, dst).astype(np.uint32)
    alive = np.ones(n, np.uint8)
    sim = pa.Simulator(seed=0x5EED0006)
    out = []
    for rep in range(3):                         # the first run also allocates the handle's buffers
        ms0, _ = sim.timing()
        t0 = time.time()
        rows, dv, fr = pa.relay.relay_run(sim, rp, col, rp, col, alive, src, dst, relay_ttl=ttl)
        wall = time.time() - t0
        ms = sim.timing()[0] - ms0
        out.append((ms, wall))
    ms, wall = out[-1]
    copies = sum(r["relay"] + r["direct"] for r in rows) + k
    line("RELAY", n=n, sends=k, relay_ttl=ttl, rounds=len(rows), copies_handled=int(copies),
         kernel_ms=round(ms, 3), copies_per_s=copies / (ms / 1e3), wall_s_incl_host_setup=round(wall, 3),
         delivered_sends=int((dv > 0).sum()), per_round=rows)
    sim.close()


if __name__ == "__main__":
    which = sys.argv[1:] or ["C2", "C3", "C4", "C5"]
    for w in which:
        if w == "C2":
            c2()
        elif w == "C3":
            sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
            import probe_engines
            r = probe_engines.c3(1_000_000, 30)
            line("C3", **r)
        elif w == "C4":
            c4()
        elif w == "C5":
            c5()
        elif w == "RELAY":
            relay()
        elif w == "C2ALL":
            c2_all_roots()
