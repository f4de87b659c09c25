#!/usr/bin/env bash
# A/B (round 3): memb loaded with the state (default) vs after it (PT_MEMB_LAZY),
# each with and without the frontier kernel; stamped frontier profile.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "step $name failed: $?"; exit 1; }; }
export PYTHONUNBUFFERED=1
LAZY=$PWD/partisan_amd/exp_memblazy.so
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
PSIM_FRONTIER=1 PSIM_LIB_PATH=$PWD/partisan_amd/exp_frstamp.so PSIM_FR_PROFILE=1 step frstamp 300 python tools/round_profile.py --steps 2
for rep in 1 2; do
  PSIM_FRONTIER=1 step b_eager_fr_$rep 300 $B
  PSIM_FRONTIER=0 step b_eager_nofr_$rep 300 $B
  PSIM_FRONTIER=1 PSIM_LIB_PATH=$LAZY step b_lazy_fr_$rep 300 $B
  PSIM_LIB_PATH=$LAZY PSIM_FRONTIER=0 step b_lazy_nofr_$rep 300 $B
done
PSIM_FRONTIER=0 step rp_eager_nofr 300 python tools/round_profile.py --steps 2
echo done
