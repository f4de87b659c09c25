#!/usr/bin/env bash
# C3 (round 6): Plumtree pushes test the connection rule on the member mask
# (PD_CONN_MASK, product) instead of scanning the partial view
# (partisan_amd/exp_pd_off.so, -DPD_CONN_MASK=0).  First the check build
# (exp_pd_chk.so, -DPD_CONN_CHECK: both tests on every push, a difference is
# PSIM_ESTATE) through the C3 GPU tests and a 1M churn run, then the product
# build's C3 tests, then the 1M wall / kernel times both ways, interleaved.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "step $name failed: $?"; tail -30 "gpurun_out/$name.log"; exit 1; }; tail -1 "gpurun_out/$name.log"; }
export PYTHONUNBUFFERED=1
T="python -u -m pytest tests/test_c3.py -m gpu -x -v --timeout 300 --timeout-method thread"
PSIM_LIB_PATH=$PWD/partisan_amd/exp_pd_chk.so step pytest_c3_chk 400 $T
PSIM_LIB_PATH=$PWD/partisan_amd/exp_pd_chk.so step c3_chk_1m 300 python tools/c3_wall.py 1000000 30 run
step pytest_c3_mask 400 $T
for rep in 1 2; do
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_pd_off.so step c3_off_$rep 300 python tools/c3_wall.py 1000000 30 run
  step c3_mask_$rep 300 python tools/c3_wall.py 1000000 30 run
done
echo done
