#!/usr/bin/env bash
# C5 cost split (timing only, results wrong by construction): no fold
# (arrivals enumerated, nothing buffered) and no arrivals (clock load/store).
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "step $name failed: $?"; exit 1; }; }
export PYTHONUNBUFFERED=1
P="python tools/c5_probe.py 1000000 12"
step c5_full 200 $P
PSIM_LIB_PATH=$PWD/partisan_amd/exp_cs_nofold.so step c5_nofold 200 $P
PSIM_LIB_PATH=$PWD/partisan_amd/exp_cs_noarr.so step c5_noarr 200 $P
echo done
