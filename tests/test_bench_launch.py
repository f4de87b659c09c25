"""bench.py's rank layout: `--gpus N` must run N ranks.

CPU: a WORLD_SIZE that disagrees with --gpus is refused before anything
touches a GPU (the process exits non-zero with the reason).
GPU: `bench.py --gpus 2` with no launcher spawns its two rank processes
itself (gloo exchange, both ranks on device 0, 200k peers) and reports
n_gpus 2, the sharded exchange's own world size and a converged flood.
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
