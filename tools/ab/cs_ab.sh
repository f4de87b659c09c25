#!/usr/bin/env bash
# A/B (round 3): C5 causal round kernel, default build vs the previous one
# (exp_cs_prev).  Earlier rounds of this A/B (profiles/r03/experiments/
# ab_c5_*.txt): round 2's fold 34.4 ms, watches in LDS 13.65, registers 13.09;
# last: a fast path for folds whose only candidate is the new entry.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "step $name failed: $?"; exit 1; }; }
export PYTHONUNBUFFERED=1
P="python tools/c5_probe.py 1000000 12"
step pytest_cs 300 python -m pytest tests/test_causal.py -m gpu -x -q
for rep in 1 2; do
  step c5_new_$rep 200 $P
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_cs_prev.so step c5_prev_$rep 200 $P
done
echo done
