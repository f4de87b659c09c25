#!/usr/bin/env bash
# C3 (round 6): psim_c3_run (churn rounds with no host wait between them)
# against the per-round calls -- GPU parity (tests/test_c3.py) first, then
# the 1M wall per round both ways, interleaved (tools/c3_wall.py).
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "step $name failed: $?"; tail -30 "gpurun_out/$name.log"; exit 1; }; tail -1 "gpurun_out/$name.log"; }
export PYTHONUNBUFFERED=1
step pytest_c3 400 python -u -m pytest tests/test_c3.py -m gpu -x -v --timeout 300 --timeout-method thread
for rep in 1 2; do
  step c3_calls_$rep 300 python tools/c3_wall.py 1000000 30
  step c3_run_$rep 300 python tools/c3_wall.py 1000000 30 run
done
echo done
