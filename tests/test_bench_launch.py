"""bench.py's rank layout: `--gpus N` must run N ranks.

CPU: a WORLD_SIZE that disagrees with --gpus is refused before anything
touches a GPU (the process exits non-zero with the reason).
GPU: `bench.py --gpus 2` with no launcher spawns its two rank processes
itself (gloo exchange, both ranks on device 0, 200k peers) and reports
n_gpus 2, the sharded exchange's own world size, a converged flood, the
touched-state roofline per shard and parity_10m: the C oracle's flood of the
same overlay against the global per-round counts and every shard's final
state gathered to rank 0.
CPU: gather_state over gloo (world 2, stand-in handles) reassembles the
shards' arrays and slot rows in global vertex order.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=600):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert r.returncode != 0
    assert "--gpus 4 but WORLD_SIZE=2" in (r.stdout + r.stderr)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_gpus_2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--transport", "gloo", "--all-on-device0", "--num-peers", "200000",
              "--no-cpu-baseline", "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout        # rank 0 alone prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["exchange"]["transport_info"]["kind"] == "callback"
    assert all(out["config"]["verified_after_timing"].values())
    assert out["config"]["n_peers"] == 200000
    # the N > 1 line carries the touched-state roofline, per
    # shard, and the oracle check of the sharded flood (state gathered)
    rl = out["roofline"]
    assert rl["model"].startswith("bytes per launch = 16 B per vertex the round touched")
    assert len(rl["per_rank"]) == 2 and all(0 < r["frac"] < 1 for r in rl["per_rank"])
    assert sum(r["n_local"] for r in rl["per_rank"]) == 200000
    assert 0 < rl["frac"] < 1
    par = out["parity_10m"]
    assert par["ok"], par
    assert par["n_peers"] == 200000 and par["shards"] == 2
    assert "cpu_baseline" not in out        # the CPU baseline is rank 0 at N = 1 only


class _FakeShard:
    """The getters gather_state reads, for shard `rank` of a tiny overlay."""
    def __init__(self, rank):
        import numpy as np
        n = 3 + rank                       # uneven shards: padding is cut off again
        self.n = n
        self.v_lo = 0 if rank == 0 else 3
        ids = np.arange(n) + self.v_lo
        self._e = (ids * 7 + 0x80000001).astype(np.uint32)      # top bit set: u32 survives the int32 view
        self._l = (ids * 5).astype(np.uint32)
        self._o = (ids * 3).astype(np.uint32)
        self._r = (ids + 60000).astype(np.uint16)
        self._d = (ids % 2).astype(np.uint8)
        deg = (ids % 3) + 1
        self.slot_row_ptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.uint64)
        self.slot_col = (np.arange(int(deg.sum())) + 100 * (rank + 1)).astype(np.uint32)

    def plumtree_state(self):
        return self._e, self._l, self._o, self._r

    def delivered(self):
        return self._d


def _gather_worker(rank, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    sys.path.insert(0, ROOT)
    import bench
    st = bench.gather_state(dist, _FakeShard(rank))
    if rank == 0:
        q.put({k: v.tolist() for k, v in st.items()})
    dist.destroy_process_group()


def test_gather_state_world2_gloo():
    import multiprocessing as mp
    import socket

    import numpy as np
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gather_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=120)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    a, b = _FakeShard(0), _FakeShard(1)
    assert got["eager"] == np.concatenate([a._e, b._e]).tolist()
    assert got["lazy"] == np.concatenate([a._l, b._l]).tolist()
    assert got["outstanding"] == np.concatenate([a._o, b._o]).tolist()
    assert got["Round"] == np.concatenate([a._r, b._r]).tolist()
    assert got["delivered"] == np.concatenate([a._d, b._d]).tolist()
    deg = np.concatenate([np.diff(a.slot_row_ptr.astype(np.int64)), np.diff(b.slot_row_ptr.astype(np.int64))])
    assert got["slot_row_ptr"] == np.concatenate([[0], np.cumsum(deg)]).tolist()
    assert got["slot_col"] == np.concatenate([a.slot_col, b.slot_col]).tolist()
