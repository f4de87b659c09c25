"""Headline benchmark: simulated peer-rounds/s and HBM GB/s of a 10M-peer
Plumtree broadcast to convergence (BASELINE.json `metric`).

A step = one heartbeat broadcast from a fresh tree to quiescence:
  psim_plumtree_reset_trees (an update with new members, Q2)
  -> psim_plumtree_broadcast(root)  (origin eager push, round 0)
  -> psim_run                       (rounds until nothing is in flight and no
                                      outstanding i_have row to a live peer)
On one GPU the W warmup and the K timed steps are each one
psim_plumtree_broadcast_run_n call: the same heartbeats as K reset_trees +
broadcast_run calls (tests/test_run_n.py), without a return to Python between
them.
value = n_peers * rounds / step time, summed over ranks.  The overlay is
resident in HBM before the timed region; nothing crosses PCIe inside it
except the per-chunk 8 KB counter read-back the round driver needs.

Roofline: dominant kernel pt_round_ell_kernel, HBM-bound.  achieved = the
algorithmic bytes of the timed rounds / their summed hipEvent durations
(events on the library's own stream: one pair per 16-round chunk, so the
average launch includes the dispatch gaps between round kernels), with the
state bytes of the vertices each round TOUCHED (16 B per vertex that
processed a word or a tick) -- SURVEY 8(d)'s model charges 16 B for all N
vertices every round, which credits a sparse round with state it never
reads (1.4x peak in the shortest launch); that figure stays as
frac_dense_model.  roofline.random_access puts the stored inbox words (one
random 4-byte store each) against the chip's measured scatter rate, the roof
the dense rounds actually hit.  roofline.per_round: one more step, untimed,
with an event pair per round kernel -- each round's bytes, words and
fractions (and PMC bytes when profiles/pmc_traffic.json has them for this
build).  traffic = rocprofv3 PMC bytes per launch from
profiles/pmc_traffic.json, reported only when that profile was taken on the
very libpsim.so this run loaded (sha256).
cpu_baseline: the C oracle (a scalar port of the reference modules) running
one flood of the benchmark's own configuration single-threaded, rank 0 only
(plus the 1M-peer sample and the 16-process all-core figure beside it).

Multi-GPU (N > 1): the SAME 10M-peer overlay is vertex-sharded over the N
GPUs (strong scaling; N = 1 is its one-shard case); cross-shard
words move every round through libpsim's own RCCL communicator (grouped
ncclSend / ncclRecv over xGMI); --mode replicas runs N independent copies
instead (weak scaling).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "simulated peer-rounds/sec + HBM GB/s at 10M-peer plumtree broadcast, 1–8 GPUs"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# random 4-byte stores into a 200 MB inbox, the round-12 shape (27.0M words
# into 50M slots), measured on MI355X: profiles/r04/experiments/mb_transpose_range.txt
# ("direct scatter 494 us, 54.7 G words/s"; tools/mb_transpose.hip)
SCATTER_PEAK_WPS = 54.7e9


def touched_bytes(st):
    """Algorithmic bytes of one round (a numpy record of psim_run) with 16 B
    of state per vertex the round touched: 16 active + 8 senders + 4 deg-sum
    + 32 messages (SURVEY 8(d) with the 16 N term replaced)."""
    msgs = int(st["sent"][1:6].sum())
    return 16 * int(st["active"]) + 8 * int(st["senders"]) + 4 * int(st["sender_degree_sum"]) + 32 * msgs


def shard_touched_bytes(d, n_local):
    """touched_bytes for one shard's round (a psim_shard_run row, a dict):
    its algo_bytes are this shard's 16 n_local + 8 senders + 4 deg-sum + 32
    messages (psim_host.hip shard rows), so replacing 16 n_local by 16 B per
    vertex the shard touched gives the same model per GPU."""
    return int(d["algo_bytes"]) - 16 * int(n_local) + 16 * int(d["active"])


def gather_floats(pg, vals):
    """[rank][i] = vals[i] of every rank (all-gather; one rank: [vals])."""
    if pg is None:
        return [list(vals)]
    import torch
    dev = "cuda" if pg.get_backend() == "nccl" else "cpu"
    mine = torch.tensor(vals, dtype=torch.float64, device=dev)
    out = [torch.zeros_like(mine) for _ in range(pg.get_world_size())]
    pg.all_gather(out, mine)
    return [t.cpu().tolist() for t in out]


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs (= ranks, one process each).  Without a launcher (WORLD_SIZE unset) N > 1 spawns the N "
                        "rank processes itself; under torchrun it must equal WORLD_SIZE")
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--num-peers", dest="n", type=int, default=10_000_000)
    p.add_argument("--peers", type=int, default=5)
    p.add_argument("--seed", type=int, default=0x5EED0001)
    p.add_argument("--lazy-tick-rounds", type=int, default=1)
    p.add_argument("--cpu-sample-n", type=int, default=1_000_000)
    p.add_argument("--no-cpu-full", action="store_true",
                   help="skip the single-thread C-oracle flood of the full --num-peers config (~25 s at 10M)")
    p.add_argument("--cpu-sample-reps", type=int, default=3)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-parity", action="store_true",
                   help="skip parity_10m: the C oracle's flood of the same overlay against the last step's per-round "
                        "counts and final state (gathered from every shard at N > 1; ~30 s of rank-0 CPU at 10M)")
    p.add_argument("--cpu-workers", type=int, default=16,
                   help="processes for the all-core CPU baseline (the box's CPU share is 16 per GPU); 0 = skip")
    p.add_argument("--mode", choices=["sharded", "replicas"], default="sharded")
    p.add_argument("--force-sharded", action="store_true",
                   help="measurement aid: drive one GPU through the sharded engine (psim_shard_run, world 1)")
    p.add_argument("--csr", action="store_true", help="A/B: CSR slot rows instead of ELL rows (DESIGN.md 4)")
    p.add_argument("--round-events", action="store_true",
                   help="a hipEvent pair around every round kernel (the markers cost ~10 us between rounds); "
                        "default: one pair per 16-round chunk (PSIM_CFG_CHUNK_TIMING)")
    p.add_argument("--transport", choices=["nccl", "gloo"], default="nccl",
                   help="nccl = RCCL over xGMI (the real path); gloo = host-staged, for tests")
    p.add_argument("--all-on-device0", action="store_true",
                   help="test aid: put every rank on GPU 0 (needs --transport gloo)")
    p.add_argument("--sustain-s", type=float, default=3.0,
                   help="after the timed steps, keep flooding for this many seconds and report the sustained rate "
                        "(the timed region alone is ~40 ms: too short for an SMI sampler to see); 0 = skip")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                   help="per-launch HBM bytes measured by tools/pmc_traffic.py for this workload")
    return p.parse_args()


def _free_port():
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def launch_ranks(n):
    """`bench.py --gpus N` with no launcher around it: start the N rank
    processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rendezvous on
    127.0.0.1) as children of this process, which never imports torch or
    touches a GPU, and exit with the first failing rank's status (rank 0
    prints the JSON line).  A failing rank takes the others down."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:          # the collective peers of a dead rank would wait forever
                    q.terminate()
    for p in procs:
        p.wait()
    return rc


def check_world(args):
    """The rank layout this process runs in; refuses --gpus != WORLD_SIZE."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        return 1 if args.gpus is None else args.gpus, False
    world = int(env_world)
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a "
                         f"{world}-rank run as {args.gpus} GPUs")
    return world, True


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if args.all_on_device0:
        local = 0
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if args.transport == "nccl":
            dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo", init_method="env://")
        pg = dist
    return rank, local, world, pg


def barrier(pg):
    if pg is not None:
        pg.barrier()


def _reduce(pg, x, op):
    if pg is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device="cuda" if pg.get_backend() == "nccl" else "cpu")
    pg.all_reduce(t, op=op)
    return float(t.item())


def max_over_ranks(pg, x):
    return x if pg is None else _reduce(pg, x, pg.ReduceOp.MAX)


def sum_over_ranks(pg, x):
    return x if pg is None else _reduce(pg, x, pg.ReduceOp.SUM)


def one_step(sim, root):
    sim.reset_trees()
    # broadcast + run in one call (psim_plumtree_broadcast_run): the origin's
    # counters come back with the first chunk; a numpy record array, no
    # per-round Python dicts in the timed loop
    _, st, rounds = sim.broadcast_run(root, as_dicts=False)
    return st, rounds


def verify(sim, pg, n, rounds_per_step):
    """After the timed region (outside it): the last step converged.  Every
    vertex delivered the heartbeat (the reliable-broadcast postcondition,
    test/prop_partisan_reliable_broadcast.erl:127-172), no outstanding i_have
    row is left, and the eager links form a spanning tree: 2(n-1) directed
    eager entries over all shards.  Every step ran the same number of rounds."""
    import numpy as np
    eager, _lazy, outst, _rr = sim.plumtree_state()
    local = [int(sim.delivered().sum()), int(np.count_nonzero(outst)),
             int(np.bitwise_count(eager).sum(dtype=np.int64))]
    tot = [int(sum_over_ranks(pg, float(x))) for x in local]
    ok = {"delivered": tot[0] == n, "no_outstanding": tot[1] == 0, "spanning_tree": tot[2] == 2 * (n - 1),
          "same_rounds_every_step": len(set(rounds_per_step)) == 1}
    if not all(ok.values()):
        raise SystemExit(f"bench: the timed steps did not converge: {ok} (delivered {tot[0]} of {n}, "
                         f"outstanding vertices {tot[1]}, eager entries {tot[2]}, rounds {rounds_per_step})")
    return ok


KINDS = ("broadcast", "prune", "i_have", "ignored_i_have", "graft")


def local_state(sim):
    """This handle's final Plumtree state and slot layout (its own vertices)."""
    import numpy as np
    e, l, o, rr = sim.plumtree_state()
    return {"delivered": sim.delivered(), "eager": e, "lazy": l, "outstanding": o, "Round": rr,
            "slot_row_ptr": np.asarray(sim.slot_row_ptr, dtype=np.uint64), "slot_col": np.asarray(sim.slot_col)}


def gather_state(pg, sim):
    """Every shard's final state and slot rows (local_state) gathered in rank
    order, i.e. global vertex order (shards own contiguous ranges): the whole
    overlay's delivered set, eager / lazy / outstanding masks, accepted Round
    and slot layout, as one GPU's handle reports them.  Collective (every
    rank calls it); every rank gets the result, rank 0 uses it."""
    import numpy as np
    import torch
    st = local_state(sim)
    n_l, e_l = len(st["eager"]), len(st["slot_col"])
    sizes = gather_floats(pg, [float(n_l), float(e_l)])
    nmax, emax = int(max(x[0] for x in sizes)), int(max(x[1] for x in sizes))
    dev = "cuda" if pg.get_backend() == "nccl" else "cpu"
    per_v = np.zeros((6, nmax), np.int32)
    per_v[0, :n_l] = st["eager"].view(np.int32)
    per_v[1, :n_l] = st["lazy"].view(np.int32)
    per_v[2, :n_l] = st["outstanding"].view(np.int32)
    per_v[3, :n_l] = st["Round"]
    per_v[4, :n_l] = st["delivered"]
    per_v[5, :n_l] = np.diff(st["slot_row_ptr"].astype(np.int64))
    cols = np.zeros(max(1, emax), np.int32)
    cols[:e_l] = st["slot_col"].view(np.int32)
    out = {}
    for name, arr in (("v", per_v), ("c", cols)):
        mine = torch.from_numpy(arr).to(dev)
        got = [torch.zeros_like(mine) for _ in sizes]
        pg.all_gather(got, mine)
        out[name] = [g.cpu().numpy() for g in got]
        del mine, got
    v = np.concatenate([out["v"][r][:, :int(sizes[r][0])] for r in range(len(sizes))], axis=1)
    c = np.concatenate([out["c"][r][:int(sizes[r][1])] for r in range(len(sizes))]).view(np.uint32)
    return {"delivered": v[4].astype(np.uint8), "eager": v[0].view(np.uint32), "lazy": v[1].view(np.uint32),
            "outstanding": v[2].view(np.uint32), "Round": v[3].astype(np.uint16),
            "slot_row_ptr": np.concatenate([[0], np.cumsum(v[5].astype(np.int64))]).astype(np.uint64),
            "slot_col": c}


def _row_counts(g):
    """(messages by kind, new deliveries) of one round: a psim_run record
    (numpy) or a psim_shard_run row (dict; global counts)."""
    if isinstance(g, dict):
        return [int(g[k]) for k in KINDS], int(g["delivered_new"])
    return [int(g["sent"][i + 1]) for i in range(len(KINDS))], int(g["delivered_new"])


def oracle_parity(state, orc, root, gpu_stats, gpu_rounds, ost, orr, omono):
    """The GPU's last heartbeat against the C oracle's heartbeat of the same
    overlay (outside any timed region): round count, per-round message counts
    by kind and new deliveries, and at the end every vertex's delivered bit,
    eager / lazy / outstanding sets and accepted Round (orc_pt_dump_state over
    the handle's slot layout).  state: local_state / gather_state (the whole
    overlay); gpu_stats: psim_run's rows or psim_shard_run's GLOBAL rows.
    Returns {"ok": bool, ...} with the first mismatch named."""
    import numpy as np
    res = {"n_peers": int(len(state["eager"])), "rounds_gpu": int(gpu_rounds), "rounds_oracle": int(orr),
           "ok": False}
    if gpu_rounds != orr:
        res["mismatch"] = "round count"
        return res
    for r in range(orr):
        (gk, gd), o = _row_counts(gpu_stats[r]), ost[r]
        for i, k in enumerate(KINDS):
            if gk[i] != o[k]:
                res["mismatch"] = f"round {r + 1} {k}: gpu {gk[i]} oracle {o[k]}"
                return res
        if gd != o["delivered_new"]:
            res["mismatch"] = f"round {r + 1} delivered_new"
            return res
    if not np.array_equal(state["delivered"], orc.delivered(root, omono)):
        res["mismatch"] = "delivered set"
        return res
    ge, gl, go, grr = state["eager"], state["lazy"], state["outstanding"], state["Round"]
    oe, ol, oo, orrs = orc.dump_state(root, omono, state["slot_row_ptr"], state["slot_col"])
    for name, g, o in (("eager", ge, oe), ("lazy", gl, ol), ("outstanding", go, oo), ("Round", grr, orrs)):
        bad = np.flatnonzero(g != o)
        if len(bad):
            res["mismatch"] = f"{name} sets differ at {len(bad)} vertices (first {int(bad[0])})"
            return res
    res.update(ok=True, messages=int(sum(sum(o[k] for k in KINDS) for o in ost)),
               compared=("round count; per-round broadcast / prune / i_have / ignored_i_have / graft and new "
                         "deliveries; final delivered set, eager / lazy / outstanding masks and accepted Round "
                         "of every vertex"))
    return res


def cpu_baseline_full(args, state=None, gpu_stats=None, gpu_rounds=None):
    """One single-thread C-oracle flood of the benchmark's own configuration
    (the same --num-peers overlay, seed and root), timed from heartbeat to
    quiescence (the 10M config itself, beside the 1M sample).
    With the GPU's last step (sim, its psim_run rows and round count) the
    same flood is then the oracle parity check of the metric config
    (VERDICT r3): returned as the second value."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    from partisan_amd import overlay
    rp, col = overlay.random_regular(args.n, args.peers, args.seed)
    orc = O.Plumtree(rp, col, args.lazy_tick_rounds)
    del rp, col
    t0 = time.perf_counter()
    omono = orc.heartbeat(0)
    ost, rounds = orc.run()
    dt = time.perf_counter() - t0
    parity = None
    if state is not None:
        t1 = time.perf_counter()
        parity = oracle_parity(state, orc, 0, gpu_stats, gpu_rounds, ost, rounds, omono)
        parity["check_s"] = round(time.perf_counter() - t1, 1)
    orc.close()
    return {
        "value": args.n * rounds / dt, "unit": "peer-rounds/s", "cores": 1, "kind": "port",
        "sample": (f"C oracle (oracle/plumtree.c), one flood of the benchmark's own {args.n}-peer random "
                   f"{args.peers}-peer overlay from root 0 to quiescence ({rounds} rounds), single thread, "
                   f"{dt:.1f} s"),
    }, parity


def lib_fingerprint():
    """sha256 of the libpsim.so this process loaded: profiles/pmc_traffic.json
    is keyed to it, so a kernel change cannot leave a stale traffic figure."""
    import hashlib
    from partisan_amd import _lib
    h = hashlib.sha256()
    with open(_lib.LIB_PATH, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def cpu_baseline(args):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    from partisan_amd import overlay
    rp, col = overlay.random_regular(args.cpu_sample_n, args.peers, args.seed)
    tot_t, tot_pr = 0.0, 0
    rounds = 0
    for _ in range(args.cpu_sample_reps):
        orc = O.Plumtree(rp, col, args.lazy_tick_rounds)
        t0 = time.perf_counter()
        orc.heartbeat(0)
        _, rounds = orc.run()
        tot_t += time.perf_counter() - t0
        tot_pr += args.cpu_sample_n * rounds
        orc.close()
    return {
        "value": tot_pr / tot_t, "unit": "peer-rounds/s", "cores": 1, "kind": "port",
        "sample": (f"C oracle (oracle/plumtree.c), {args.cpu_sample_reps} floods of a "
                   f"{args.cpu_sample_n}-peer random {args.peers}-peer overlay to quiescence "
                   f"({rounds} rounds each), single thread, {tot_t:.1f} s"),
    }


def cpu_baseline_allcores(args):
    """W single-thread oracle floods at once, one child process each (a
    fresh interpreter started by subprocess: no fork of this GPU-initialised
    process, and no multiprocessing pool whose resource tracker outlives the
    bench); value = the sum of the workers' own rates (peer-rounds / time
    inside their floods, which overlap).  Every child is waited for before
    this returns."""
    import subprocess
    w = args.cpu_workers
    worker = os.path.join(ROOT, "oracle", "cpu_flood.py")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    t0 = time.perf_counter()
    procs = [subprocess.Popen([sys.executable, worker, str(args.cpu_sample_n), str(args.peers), str(args.seed + i),
                               str(args.cpu_sample_reps), str(args.lazy_tick_rounds)],
                              stdout=subprocess.PIPE, text=True, env=env) for i in range(w)]
    res = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=600)
            if p.returncode != 0:
                raise RuntimeError(f"cpu_flood worker exited with {p.returncode}")
            res.append(json.loads(out.strip().splitlines()[-1]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
    wall = time.perf_counter() - t0
    rate = sum(r[0] / r[1] for r in res)
    return {
        "value": rate, "unit": "peer-rounds/s", "cores": w, "kind": "port",
        "sample": (f"{w} processes at once, each the single-thread C oracle running {args.cpu_sample_reps} "
                   f"floods of its own {args.cpu_sample_n}-peer random {args.peers}-peer overlay "
                   f"({res[0][2]} rounds); sum of per-process rates, {wall:.1f} s wall incl. interpreter starts "
                   f"and overlay builds"),
    }


def main():
    args = parse()
    world, launched = check_world(args)
    if world > 1 and not launched:
        sys.exit(launch_ranks(world))
    rank, local, world, pg = dist_setup(args)
    import numpy as np  # noqa: F401

    sharded = (world > 1 or args.force_sharded) and args.mode == "sharded"
    if sharded:
        # the sharded engine allocates its exchange buffers with torch: bring
        # torch's HIP runtime up before libpsim is loaded (as the multi-GPU
        # launch does in dist_setup), so both share it
        import torch
        torch.cuda.set_device(local)
        torch.empty(1, device=torch.device("cuda", local))
    import partisan_amd as pa

    rp, col = pa.overlay.random_regular(args.n, args.peers, args.seed)
    if sharded:
        from partisan_amd.shard import ShardedPlumtree
        sp = ShardedPlumtree(rp, col, rank, world, device=local, backend=args.transport,
                             lazy_tick_rounds=args.lazy_tick_rounds, csr=args.csr,
                             chunk_timing=not args.round_events)
        sim = sp.sim
    else:
        sp = None
        sim = pa.Simulator(lazy_tick_rounds=args.lazy_tick_rounds, device=local, csr=args.csr,
                           chunk_timing=not args.round_events)
        sim.load_overlay(rp, col)
    del rp, col
    root = 0

    def step():
        if sp is not None:
            sp.reset_trees()
            sp.broadcast(root)
            return sp.run()
        return one_step(sim, root)

    def steps(k):
        """k steps; on one GPU in one call (psim_plumtree_broadcast_run_n: the
        same heartbeats as k reset_trees + broadcast_run calls, without a return
        to Python between them).  Returns [(round records, rounds)] per step."""
        if sp is not None or k == 0:
            return [step() for _ in range(k)]
        _, st, rounds = sim.broadcast_run_n(root, k, reset_trees=True)
        out, o = [], 0
        for r in rounds.tolist():
            out.append((st[o:o + r], r))
            o += r
        return out

    steps(args.warmup)

    algo_bytes = 0
    active_bytes = 0
    words = 0
    round_ms = 0.0
    rounds_per_step = []
    if sp is not None:
        sp.local_algo_bytes, sp.local_kernel_ms = 0, 0.0
        sp.exchange_total = {}
    barrier(pg)
    t0 = time.perf_counter()
    done = steps(args.steps)
    # psim_run / psim_shard_round return after hipStreamSynchronize on the library stream
    barrier(pg)
    t1 = time.perf_counter()
    step_stats = [st for st, _ in done]
    rounds_per_step = [r for _, r in done]
    # the per-step bookkeeping after the timed region (a Python pass over each
    # step's round records cost ~3 % of a step inside it)
    last_stats = step_stats[-1] if step_stats else None
    if sp is None:
        for stats in step_stats:
            algo_bytes += int(stats["algo_bytes"].sum())
            round_ms += float(stats["kernel_ms"].sum())
            # the same model crediting the state bytes of the vertices a round touched, not of all N
            active_bytes += sum(touched_bytes(x) for x in stats)
            words += int(stats["words_stored"].sum())
    if sp is not None:   # this GPU's own bytes and launch times
        algo_bytes, round_ms = sp.local_algo_bytes, sp.local_kernel_ms
        for stats in step_stats:
            active_bytes += sum(shard_touched_bytes(x, sim.n) for x in stats)

    verified = verify(sim, pg, args.n, rounds_per_step)
    per_round_stats = None
    if sp is None:
        # one more step, outside the timed region, with an event pair around
        # every round kernel: the per-round table of roofline.per_round
        sim.set_chunk_timing(False)
        per_round_stats, _ = one_step(sim, root)
        sim.set_chunk_timing(not args.round_events)
    exchange = None
    counted = sum(rounds_per_step)
    if sp is not None:   # the in-library exchange (psim_shard_run): fabric bytes and device time per step
        xt = sp.exchange_total
        chunk_ms = float(xt.get("kernel_ms", 0.0)) / args.steps
        timed_rounds = float(xt.get("rounds", 0)) / args.steps
        fabric = float(xt.get("fabric_bytes", 0))
        if not args.round_events:
            # the timed chunks carry one event pair each, so their time holds the
            # exchanges too: one more step (outside the timed region) with an event
            # pair around every round kernel and every exchange gives the kernel's
            # own launch time for the roofline and the exchange time
            sp.sim.set_chunk_timing(False)
            sp.local_algo_bytes, sp.local_kernel_ms, sp.exchange_total = 0, 0.0, {}
            inst_rows, r_inst = step()
            algo_bytes, round_ms, counted = sp.local_algo_bytes, sp.local_kernel_ms, r_inst
            active_bytes = sum(shard_touched_bytes(x, sim.n) for x in inst_rows[:r_inst])
            xi = sp.exchange_total
            kernel_ms_step, exchange_ms_step = float(xi.get("kernel_ms", 0.0)), float(xi.get("exchange_ms", 0.0))
            sp.sim.set_chunk_timing(True)
        else:
            kernel_ms_step = chunk_ms
            exchange_ms_step = float(xt.get("exchange_ms", 0.0)) / args.steps
        comm_world = sp.transport_info()["world"]
        if args.transport == "nccl" and comm_world != world:
            # the RCCL communicator inside libpsim must span exactly the launched ranks
            raise SystemExit(f"bench: libpsim's RCCL communicator has {comm_world} ranks but WORLD_SIZE={world}")
        exchange = {
            "transport": sp.transport,
            # the library's own view of the job (RCCL: ncclCommCount / ncclCommUserRank of its communicator)
            "world": sp.transport_info()["world"],
            "transport_info": sp.transport_info(),
            "fabric_bytes_per_step": sum_over_ranks(pg, fabric) / args.steps,
            "exchange_ms_per_step_max_rank": max_over_ranks(pg, exchange_ms_step),
            "kernel_ms_per_step_max_rank": max_over_ranks(pg, kernel_ms_step),
            "device_ms_per_step_max_rank": max_over_ranks(pg, chunk_ms if not args.round_events
                                                         else kernel_ms_step + exchange_ms_step),
            "rounds_enqueued_per_step": timed_rounds,
            "timing": ("kernel / exchange split from one extra step with an event pair per round kernel and "
                       "exchange; device time per step from the timed steps' chunk events"
                       if not args.round_events else "event pairs per round kernel and exchange"),
        }

    step_s = max_over_ranks(pg, (t1 - t0) / args.steps)
    n_units = args.n if sharded else args.n * world      # peers simulated by the whole job
    sustained = None
    if args.sustain_s > 0:
        # the same steps back to back for a few seconds (outside the timed region, after every
        # timed figure is taken)
        barrier(pg)
        k, s0, sus_rounds = 0, time.perf_counter(), []
        while time.perf_counter() - s0 < args.sustain_s:
            for _, r in steps(max(1, args.steps)):
                sus_rounds.append(r)
                k += 1
        barrier(pg)
        dt = max_over_ranks(pg, time.perf_counter() - s0)
        sustained = {"steps": k, "seconds": round(dt, 3), "ms_per_step": dt / k * 1e3,
                     "value": float(n_units) * sum(sus_rounds) / dt,
                     "same_rounds_as_timed": set(sus_rounds) == set(rounds_per_step)}
    peer_rounds = float(n_units) * sum(rounds_per_step) / args.steps
    value = peer_rounds / step_s
    # per-launch figures over the rounds up to quiescence (the no-op tail of a
    # step's last chunk is not counted): hipEvent durations of each launch
    avg_launch_ms = round_ms / max(1, counted)
    dense_gbs = (algo_bytes / max(1, counted)) / (avg_launch_ms * 1e-3) / 1e9
    per_rank = None
    rep_steps = 1 if (sp is not None and not args.round_events) else args.steps   # steps the bytes / ms cover
    if sp is None:
        touched_gbs = (active_bytes / max(1, counted)) / (avg_launch_ms * 1e-3) / 1e9
    else:
        # every shard's touched-state bytes over its own round-kernel time
        # (hipEvents on its stream): the mean per-GPU rate = all shards' bytes
        # over all shards' kernel time, each GPU against its own 8 TB/s
        rk = gather_floats(pg, [float(active_bytes), float(round_ms), float(sim.n)])
        per_rank = [{"rank": i, "n_local": int(x[2]), "touched_bytes_per_step": x[0] / rep_steps,
                     "kernel_ms_per_step": x[1] / rep_steps,
                     "frac": (x[0] / (x[1] * 1e-3) / 1e9 / HBM_PEAK_GBS) if x[1] > 0 else None}
                    for i, x in enumerate(rk)]
        tot_ms = sum(x[1] for x in rk)
        touched_gbs = sum(x[0] for x in rk) / (tot_ms * 1e-3) / 1e9 if tot_ms > 0 else 0.0

    # ELL rows (every degree of the whole overlay <= 8) run the sweep kernel
    max_deg = int(max_over_ranks(pg, float(sim.max_degree())))
    kernel = "pt_round_kernel" if (args.csr or max_deg > 8) else "pt_round_ell_kernel"
    # parity_10m: the final state of the last flood -- at N > 1
    # every shard's, gathered to rank 0 in global vertex order -- for the C
    # oracle's flood of the same overlay, after every timed figure
    gstate = None
    if not args.no_parity:
        if sp is not None and world > 1:
            gstate = gather_state(pg, sim)
            if rank != 0:
                gstate = None
        elif rank == 0:
            gstate = local_state(sim)
    if rank == 0:
        traffic = traffic_fetch = traffic_write = None
        tj = {}
        traffic_note = "no PMC profile for this workload"
        fp = lib_fingerprint()
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if not (tj.get("n") == args.n and tj.get("peers") == args.peers and tj.get("kernel") == kernel):
                traffic_note = "PMC profile is for another workload"
            elif tj.get("lib_sha256") != fp:
                traffic_note = (f"PMC profile taken on another libpsim build ({str(tj.get('lib_sha256'))[:12]} "
                                f"vs loaded {fp[:12]}): not reported")
            else:
                traffic_fetch = tj["fetch_bytes_per_launch"]
                traffic_write = tj["write_bytes_per_launch"]
                traffic = traffic_fetch + traffic_write
                traffic_note = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this libpsim build "
                                f"({tj.get('source', args.traffic_json)}), per launch")
        except (OSError, ValueError, KeyError):
            pass
        launch_s = avg_launch_ms * 1e-3
        per_round = None
        if per_round_stats is not None:
            pmc_rounds = None
            if traffic is not None:
                pmc_rounds = tj.get("per_round")
            per_round = []
            for i, x in enumerate(per_round_stats):
                ms = float(x["kernel_ms"])
                tb, db, w = touched_bytes(x), int(x["algo_bytes"]), int(x["words_stored"])
                row = {"round": i + 1, "us": round(ms * 1e3, 2), "messages": int(x["sent"][1:6].sum()),
                       "words": w, "active": int(x["active"]), "bytes_touched": tb, "bytes_dense_model": db,
                       "frac": tb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS if ms > 0 else None,
                       "frac_random_access": w / (ms * 1e-3) / SCATTER_PEAK_WPS if ms > 0 else None}
                if pmc_rounds and i < len(pmc_rounds):
                    pb = pmc_rounds[i]["fetch"] + pmc_rounds[i]["write"]
                    row["pmc_bytes"] = pb
                    row["frac_pmc"] = pb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS if ms > 0 else None
                per_round.append(row)
        words_s = (words / (round_ms * 1e-3)) if (sp is None and round_ms > 0) else None
        achieved_gbs = touched_gbs if touched_gbs is not None else dense_gbs
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "peer-rounds/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": step_s * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if args.mode == "replicas" else "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {
                "workload": (f"{args.n}-peer Plumtree broadcast to convergence: heartbeat from a fresh "
                             f"tree (reset_peers), flood + prune, lazy tick every "
                             f"{args.lazy_tick_rounds} round(s)"),
                "n_peers": args.n,
                "overlay": f"random symmetric, {args.peers} peers per vertex (HyParView active view)",
                "rounds_to_convergence": rounds_per_step[-1],
                "verified_after_timing": verified,
                "parallelism": (f"vertex-sharded x{world}, "
                                + ("RCCL grouped send/recv over xGMI inside libpsim" if args.transport == "nccl"
                                   else "gloo host-staged") + " exchange per round" if sharded
                                else ("replicas" if world > 1 else "single")),
                "device": sim.device_info(),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS,
                "model": ("bytes per launch = 16 B per vertex the round touched + (8 + 4 deg) per sender + "
                          "32 per message (SURVEY 8(d) with its 16 N term charged only for touched vertices)"
                          + ("" if sp is None else
                             "; per GPU: every shard's bytes over its own round-kernel time, summed over shards "
                             "(per_rank)")),
                "per_rank": per_rank,
                # SURVEY 8(d)'s 16 N-per-round model credits state a sparse round never
                # reads (above 1.0 of peak in rounds 2-5): a model, not evidence
                "achieved_dense_model": dense_gbs,
                "frac_dense_model": dense_gbs / HBM_PEAK_GBS,
                "dense_model_note": "SURVEY 8(d) 16 N per round: model, not evidence (credits unread state)",
                "random_access": ({"achieved": words_s, "peak": SCATTER_PEAK_WPS, "unit": "words/s",
                                   "frac": words_s / SCATTER_PEAK_WPS,
                                   "words_per_step": words / args.steps,
                                   "peak_source": "profiles/r04/experiments/mb_transpose_range.txt (direct "
                                                  "random 4-byte scatter, round-12 shape)"}
                                  if words_s is not None else None),
                "per_round": per_round,
                "max_round_frac": max((r["frac"] for r in per_round if r["frac"] is not None), default=None)
                                  if per_round else None,
                "traffic": traffic,
                "traffic_note": traffic_note,
                # the same launch time against the PMC-measured bytes (tools/pmc_traffic.py): what
                # actually crossed the memory side.  MI355X_MICROARCH.md: on gfx950 FETCH_SIZE counts
                # half the bytes of wide coalesced reads (the sweep's 16-B loads), so the read side is
                # doubled for frac_traffic (an upper bound: the scattered 4-B reads need no doubling);
                # frac_traffic_raw is the uncorrected figure
                "frac_traffic": ((2 * traffic_fetch + traffic_write) / launch_s / 1e9 / HBM_PEAK_GBS)
                                if traffic else None,
                "frac_traffic_raw": (traffic / launch_s / 1e9 / HBM_PEAK_GBS) if traffic else None,
                "kernel": kernel,
                "avg_launch_us": avg_launch_ms * 1e3,
                "algo_bytes_per_launch": algo_bytes / max(1, counted),
                "lib_sha256": fp,
            },
        }
        if exchange is not None:
            out["exchange"] = exchange
        if sustained is not None:
            out["sustained"] = sustained
        if not args.no_cpu_baseline and world == 1:
            if args.no_cpu_full:
                out["cpu_baseline"] = cpu_baseline(args)
            else:
                out["cpu_baseline"], out["parity_10m"] = cpu_baseline_full(
                    args, gstate, last_stats, rounds_per_step[-1])
                out["cpu_baseline_sample_1m"] = cpu_baseline(args)
            if args.cpu_workers > 1:
                out["cpu_baseline_allcores"] = cpu_baseline_allcores(args)
        if gstate is not None and "parity_10m" not in out:
            # the oracle flood only as the checker here (cpu_baseline is rank 0 at N = 1)
            _, out["parity_10m"] = cpu_baseline_full(args, gstate, last_stats, rounds_per_step[-1])
        if gstate is not None and out.get("parity_10m"):
            out["parity_10m"]["shards"] = world if sp is not None else 1
        print(json.dumps(out), flush=True)
    del gstate
    barrier(pg)          # the other ranks wait for rank 0's oracle check before tearing down
    sim.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
