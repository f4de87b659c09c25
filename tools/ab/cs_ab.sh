#!/usr/bin/env bash
# A/B (round 3): C5 causal round kernel -- watch fold, buffer in registers while <= 64 with an incrementally kept pending mask
# (default build) vs the watch fold in LDS (exp_cs_lds); the
# round-2 fold (exp_cs_old, every entry fully checked per fold) measured 34.4 ms.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "step $name failed: $?"; exit 1; }; }
export PYTHONUNBUFFERED=1
P="python tools/c5_probe.py 1000000 12"
step pytest_cs 300 python -m pytest tests/test_causal.py -m gpu -x -q
for rep in 1 2; do
  step c5_new_$rep 200 $P
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_cs_lds.so step c5_lds_$rep 200 $P
done
echo done
