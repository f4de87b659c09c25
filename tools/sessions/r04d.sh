#!/usr/bin/env bash
# Round-4 session D: batched candidate loads (PT_BATCH=2, default build) vs
# PT_BATCH=1 (exp_b1.so) vs the committed head (exp_head.so); the 3-pass
# transport micro-benchmark; the rewritten causal round kernel (lockstep
# parity, then C5 against the committed head's kernel).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; [ $rc -le 1 ] || exit $rc; }
step t_wl 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_worklist_parity.py
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
for rep in 1 2; do
  step b_b2_$rep 300 $B
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_b1.so step b_b1_$rep 300 $B
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_head.so step b_head_$rep 300 $B
done
step rp_b2 300 python tools/round_profile.py --steps 2
PSIM_LIB_PATH=$PWD/partisan_amd/exp_head.so step rp_head 300 python tools/round_profile.py --steps 2
step t_causal 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_causal.py
step c5_new 200 python tools/config_bench.py C5
PSIM_LIB_PATH=$PWD/partisan_amd/exp_cs_noring.so step c5_noring 200 python tools/config_bench.py C5
PSIM_LIB_PATH=$PWD/partisan_amd/exp_head.so step c5_head 200 python tools/config_bench.py C5
step mbb2 120 tools/mb_binned
echo done
