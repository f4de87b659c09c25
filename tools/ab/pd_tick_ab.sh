#!/usr/bin/env bash
# C3 (round 6): the lazy tick tests a row's connection on the member mask via
# a table index kept in the row, BEFORE loading the peer's alive byte
# (partisan_amd/exp_pdt_tick.so) vs the product (alive byte, then the
# partial-view scan); the check build (exp_pdt_chk.so, -DPD_CONN_CHECK)
# through the C3 GPU tests and a 1M run first.  1M, churn rounds 30..59.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "step $name failed: $?"; tail -30 "gpurun_out/$name.log"; exit 1; }; tail -1 "gpurun_out/$name.log"; }
export PYTHONUNBUFFERED=1
PSIM_LIB_PATH=$PWD/partisan_amd/exp_pdt_chk.so step pytest_c3_tchk 400 python -u -m pytest tests/test_c3.py -m gpu -x -q --timeout 300 --timeout-method thread
PSIM_LIB_PATH=$PWD/partisan_amd/exp_pdt_chk.so step c3_tchk_1m 300 python tools/c3_wall.py 1000000 30 run
for rep in 1 2; do
  step c3_prod_$rep 300 python tools/c3_wall.py 1000000 30 run
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_pdt_tick.so step c3_tick_$rep 300 python tools/c3_wall.py 1000000 30 run
done
echo done
