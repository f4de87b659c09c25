#!/usr/bin/env bash
# A/B of the sparse-round changes (round 3): listed groups spread over the
# grid (PSIM_WL_GPC=64 = the old 64 per chunk) and the frontier kernel
# (PSIM_FRONTIER=0 = off); per-round profiles.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "step $name failed: $?"; exit 1; }; }
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  PSIM_FRONTIER=0 PSIM_WL_GPC=64 step bench_old_$rep 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
  PSIM_FRONTIER=0 step bench_spread_$rep 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
  PSIM_FRONTIER=1 step bench_frontier_$rep 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
done
PSIM_FRONTIER=0 PSIM_WL_GPC=64 step rp_old 300 python tools/round_profile.py --steps 2
PSIM_FRONTIER=0 step rp_spread 300 python tools/round_profile.py --steps 2
PSIM_FRONTIER=1 PSIM_FR_PROFILE=1 step rp_frontier 300 python tools/round_profile.py --steps 2
echo done
