#!/usr/bin/env bash
# GPU box: sharded engine after the chunk-mode change -- sharded / NIF GPU
# tests, then the one-GPU bench through psim_shard_run (world 1, RCCL) with
# and without per-round markers, next to the plain single-GPU bench.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local n=$1 s=$2; shift 2; echo "=== $n"; timeout -k 10 "$s" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; tail -2 "gpurun_out/$n.log" | cut -c1-300; [ $rc -eq 0 ] || { echo "=== $n rc=$rc"; exit $rc; }; }
line() { python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],round(d['ms_per_step'],3),round(d['roofline']['avg_launch_us'],1),round(d['roofline']['frac'],4),d.get('exchange'))" "$@"; }
step pytest_shard 600 python -u -m pytest tests/test_shard.py tests/test_nif_harness.py tests/test_configs_at_scale.py -m gpu -x -q --timeout 300 --timeout-method thread
step b_single 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
step b_sh_chunk 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --force-sharded
step b_sh_round 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --force-sharded --round-events
line gpurun_out/b_single.log single; line gpurun_out/b_sh_chunk.log sharded_chunk; line gpurun_out/b_sh_round.log sharded_round_events
echo "=== session done"
