#!/usr/bin/env bash
# A/B (round 3): a vertex's mark-2 flag claims issued together (default) vs
# each claim's result used before the next word (PT_SERIAL_CLAIMS build).
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "step $name failed: $?"; exit 1; }; }
export PYTHONUNBUFFERED=1
OLD=$PWD/partisan_amd/exp_serialclaims.so
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
step pytest_wl 300 python -m pytest tests/test_worklist_parity.py -m gpu -x -q
for rep in 1 2 3; do
  step b_new_$rep 300 $B
  PSIM_LIB_PATH=$OLD step b_old_$rep 300 $B
done
step rp_new 300 python tools/round_profile.py --steps 2
PSIM_LIB_PATH=$OLD step rp_old 300 python tools/round_profile.py --steps 2
echo done
