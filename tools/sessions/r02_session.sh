#!/usr/bin/env bash
# GPU box: build_tree overlay tests, the 8-shard projection, PMC traffic of the
# round kernel at head, then bench with that traffic and a rocprof trace.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local n=$1 s=$2; shift 2; echo "=== $n"; timeout -k 10 "$s" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; tail -3 "gpurun_out/$n.log"; [ $rc -eq 0 ] || { echo "=== $n rc=$rc"; exit $rc; }; }
step pytest_tree 300 python -u -m pytest tests/test_plumtree_gpu.py -m gpu -x -q -k build_tree --timeout 200 --timeout-method thread
step shard_projection 600 python tools/shard_projection.py
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --n 10000000 --peers 5 --rounds-per-step 16 --steps 3 --out gpurun_out/pmc_traffic.json || exit 1
step bench 600 python bench.py --steps 5 --warmup 2 --traffic-json gpurun_out/pmc_traffic.json
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline
echo done
