"""8-GPU projection of the sharded 10M-peer Plumtree flood, measured on ONE
GPU: the eight shard handles (rank r of world 8, 1.25M vertices
each) live in one process on one device; every round each handle's kernels
run alone (round kernel + dense pack, then a sync), the dense regions are
copied between the handles' device buffers exactly as the all-to-all would
move them, and each handle ingests.  Per round it records every shard's
kernel time (hipEvents on the handle's stream, psim_shard_collect) and the
bytes each shard would put on the fabric.  The projection of an 8-GPU step
is then sum over rounds of max over shards (kernel) plus the exchange priced
at the measured xGMI rate the caller gives (default 7 links x 153 GB/s per
GPU, MI355X_MICROARCH.md), next to the single-GPU flood.

    python tools/shard_projection.py [--n 10000000] [--world 8] > profiles/rNN/shard_projection.json
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import partisan_amd as pa  # noqa: E402
from partisan_amd._lib import RoundStats, check, lib  # noqa: E402


def rccl_latency(iters=2000):
    """Per-call cost of what psim_shard_run adds per round on top of the
    kernels, on a world-1 RCCL communicator: one grouped send/recv (to self,
    4 KB: a sparse round's records) and the 11-value counter all-reduce every
    4 rounds.  A floor for the latency term: at world 8 the calls also wait
    for the slowest peer."""
    import time
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29631")
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    sb = torch.zeros(1024, dtype=torch.int32, device=dev)
    rb = torch.zeros(1024, dtype=torch.int32, device=dev)
    cnt = torch.zeros(11, dtype=torch.int64, device=dev)

    def sendrecv():
        for q in dist.batch_isend_irecv([dist.P2POp(dist.isend, sb, 0), dist.P2POp(dist.irecv, rb, 0)]):
            q.wait()

    res = {}
    for name, fn in (("grouped_send_recv_us", sendrecv), ("allreduce_11_us", lambda: dist.all_reduce(cnt))):
        for _ in range(50):
            fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize(dev)
        res[name] = round((time.perf_counter() - t0) / iters * 1e6, 2)
    dist.destroy_process_group()
    res["per_round_us"] = round(res["grouped_send_recv_us"] + res["allreduce_11_us"] / 4, 2)
    res["method"] = ("torch.distributed nccl (RCCL) world 1 on one MI355X, back-to-back calls with a sync at the "
                     "ends; per round = one grouped send/recv + a quarter of the 4-round counter all-reduce")
    return res


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--world", type=int, default=8)
    p.add_argument("--peers", type=int, default=5)
    p.add_argument("--seed", type=int, default=0x5EED0001)
    p.add_argument("--xgmi-gbps", type=float, default=7 * 153.0)
    p.add_argument("--floods", type=int, default=3)
    p.add_argument("--csr", action="store_true", help="CSR slot rows instead of the ELL rows shards load by default")
    p.add_argument("--rccl-latency", action="store_true",
                   help="also time a world-1 RCCL communicator's grouped send/recv + counter all-reduce per round "
                        "(the latency floor of psim_shard_run's exchange; torch.distributed nccl, 127.0.0.1)")
    a = p.parse_args()
    W, n = a.world, a.n
    dev = torch.device("cuda", 0)
    rp, col = pa.overlay.random_regular(n, a.peers, a.seed)
    sims, base, rbase, send, recv = [], [], [], [], []
    for r in range(W):
        s = pa.Simulator(lazy_tick_rounds=1, device=0, rank=r, world=W, csr=a.csr)
        s.load_overlay(rp, col)
        b = (C.c_uint64 * (W + 1))()
        check(lib().psim_shard_layout(s._h, b, W), s._h)
        rb = (C.c_uint64 * (W + 1))()
        check(lib().psim_shard_recv_layout(s._h, rb, W), s._h)
        sims.append(s)
        base.append([int(x) for x in b])
        rbase.append([int(x) for x in rb])
        send.append(torch.zeros(max(1, base[-1][W]), dtype=torch.int32, device=dev))
        recv.append(torch.zeros(max(1, rbase[-1][W]), dtype=torch.int32, device=dev))
    del rp, col

    def exchange():
        torch.cuda.synchronize(dev)
        for d in range(W):
            for r in range(W):
                if r == d:
                    continue
                k = base[r][d + 1] - base[r][d]
                if k:
                    recv[d][rbase[d][r]:rbase[d][r] + k].copy_(send[r][base[r][d]:base[r][d + 1]])
        torch.cuda.synchronize(dev)
        for d in range(W):
            check(lib().psim_shard_ingest_dense(sims[d]._h, C.c_void_p(recv[d].data_ptr())), sims[d]._h)
        torch.cuda.synchronize(dev)

    fabric = [sum(base[r][d + 1] - base[r][d] for d in range(W) if d != r) * 4 for r in range(W)]
    floods = []
    for f in range(a.floods):
        for s in sims:
            s.reset_trees()
        mono = C.c_uint32()
        for r, s in enumerate(sims):
            check(lib().psim_shard_broadcast_dense(s._h, 0, C.byref(mono), C.c_void_p(send[r].data_ptr())), s._h)
            torch.cuda.synchronize(dev)
        exchange()
        per_round = []
        for rnd in range(200):
            ks = []
            tb = []
            tot = 0
            live = 0
            hold = 0
            for r, s in enumerate(sims):
                check(lib().psim_shard_round_async(s._h, C.c_void_p(send[r].data_ptr())), s._h)
                st = (RoundStats * 1)()
                lv = (C.c_int64 * 1)()
                got = C.c_uint32()
                check(lib().psim_shard_collect(s._h, st, 1, C.byref(got), lv), s._h)   # syncs: kernels run alone
                d = st[0].as_dict()
                ks.append(d["kernel_ms"])
                # touched-state bytes of this shard's round (bench.py shard_touched_bytes)
                tb.append(int(d["algo_bytes"]) - 16 * s.n + 16 * int(d["active"]))
                tot += sum(d[k] for k in ("broadcast", "prune", "i_have", "ignored_i_have", "graft"))
                live += int(lv[0])
                hold += d["outstanding_vertices"]
            exchange()
            per_round.append({"kernel_ms": ks, "touched": tb, "msgs": tot, "holders": hold})
            if tot == 0 and live == 0:
                break
        floods.append(per_round)
    last = floods[-1][:-1] if len(floods[-1]) > 1 else floods[-1]    # the final silent round changes nothing
    kmax = sum(max(r["kernel_ms"]) for r in last)
    ksum = [sum(r["kernel_ms"][i] for r in last) for i in range(W)]
    xms = len(last) * max(fabric) / (a.xgmi_gbps * 1e6)
    # the in-library driver's format per round (psim_host.hip shard_drive_fast):
    # records of K = D (M + H) per peer while K <= n D / (8 W^2), M / H chained
    # from the last 4-round collective (the origin's D words after a broadcast)
    D = max(s.max_degree() for s in sims)
    thr = max(64, n * D // (8 * W * W))
    rec_fabric, bM, bH = [], float(D), 0.0
    for i, r in enumerate(last):
        S = D * (bM + bH)
        bH += bM
        bM = S
        rec_fabric.append((W - 1) * max(1, int(S)) * 8 if S <= thr else max(fabric))
        if i % 4 == 3:                               # collective: actual counts
            bM, bH = float(r["msgs"]), float(r["holders"])
    xms_rec = sum(rec_fabric) / (a.xgmi_gbps * 1e6)
    # touched-state roofline per shard over the flood (bench.py's model, each
    # shard against its own GPU's 8 TB/s)
    tbs = [sum(r["touched"][i] for r in last) for i in range(W)]
    frac = [tbs[i] / (ksum[i] * 1e-3) / 1e9 / 8000.0 if ksum[i] > 0 else None for i in range(W)]
    lat = rccl_latency() if a.rccl_latency else None
    lat_ms = (len(last) * lat["per_round_us"] / 1e3) if lat else 0.0
    step_ms = kmax + xms_rec + lat_ms
    import hashlib
    from partisan_amd import _lib
    with open(_lib.LIB_PATH, "rb") as fh:
        sha = hashlib.sha256(fh.read()).hexdigest()
    out = {
        "n": n, "world": W, "rounds": len(last), "rows": "csr" if a.csr else "ell",
        "lib_sha256": sha,
        "per_round": [{"round": i + 1, "msgs_global": r["msgs"],
                       "kernel_us_each_shard": [round(1e3 * x, 1) for x in r["kernel_ms"]],
                       "format": "records" if rec_fabric[i] != max(fabric) else "dense",
                       "fabric_bytes_per_shard": rec_fabric[i]} for i, r in enumerate(last)],
        "touched_bytes_per_flood_each_shard": tbs,
        "touched_frac_each_shard": [round(x, 4) if x is not None else None for x in frac],
        "rccl_latency": lat,
        "projected_step_ms_with_records_and_latency": round(step_ms, 4),
        "projected_touched_frac_at_step": round(sum(tbs) / W / (step_ms * 1e-3) / 1e9 / 8000.0, 4),
        "per_shard_vertices": [s.n for s in sims],
        "kernel_ms_per_flood_max_over_shards": round(kmax, 4),
        "kernel_ms_per_flood_each_shard": [round(x, 4) for x in ksum],
        "per_round_max_kernel_us": [round(1e3 * max(r["kernel_ms"]), 1) for r in last],
        "fabric_bytes_per_round_per_shard": fabric,
        "exchange_ms_per_flood_at_xgmi": round(xms, 4),
        "xgmi_GBps_assumed": a.xgmi_gbps,
        "fabric_bytes_per_round_with_records": rec_fabric,
        "exchange_ms_per_flood_with_records": round(xms_rec, 4),
        "projected_step_ms_with_records": round(kmax + xms_rec, 4),
        "projected_step_ms": round(kmax + xms, 4),
        "projected_peer_rounds_per_s": n * len(last) / ((kmax + xms) / 1e3),
        "method": "8 shard handles in one process on one GPU, each round's kernels run alone (sync per shard), "
                  "dense regions copied between the handles as the all-to-all moves them; exchange priced at "
                  "fabric bytes / xGMI rate",
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
