#!/usr/bin/env bash
# GPU box: A/B of per-round vs per-chunk hipEvents around the round kernels
# (bench twice each, interleaved) and a kernel trace of the chunk-timed bench
# for the gaps between round kernels.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local n=$1 s=$2; shift 2; echo "=== $n"; timeout -k 10 "$s" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; tail -2 "gpurun_out/$n.log" | cut -c1-400; [ $rc -eq 0 ] || { echo "=== $n rc=$rc"; exit $rc; }; }
step t_plumtree 300 python -u -m pytest tests/test_plumtree_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread
step b_round1 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
step b_chunk1 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --chunk-timing
step b_round2 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
step b_chunk2 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --chunk-timing
step trace_chunk 300 rocprofv3 --kernel-trace -d gpurun_out/trace_chunk -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --chunk-timing
echo "=== session done"
