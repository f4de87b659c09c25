#!/usr/bin/env bash
# GPU box: the sparse-round worklist -- full -m gpu suite, then A/B of the
# 10M flood with and without it (bench + per-round profile).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local n=$1 s=$2; shift 2; echo "=== $n"; timeout -k 10 "$s" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; tail -3 "gpurun_out/$n.log"; [ $rc -eq 0 ] || { echo "=== $n rc=$rc"; exit $rc; }; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_wl 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
step prof_wl 300 python tools/round_profile.py
export PSIM_NO_WORKLIST=1
step bench_nowl 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
step prof_nowl 300 python tools/round_profile.py
unset PSIM_NO_WORKLIST
step bench_wl2 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
echo "=== session done"
