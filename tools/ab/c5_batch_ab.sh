#!/usr/bin/env bash
# A/B (round 6): C5 causal round kernel, batched fast path at CS_BATCH = 2 / 4
# / 8 (partisan_amd/exp_cs_b<K>.so; 8 = libpsim.so when built with it) vs the
# per-arrival fast path (partisan_amd/exp_cs_prev.so, -DCS_BATCH=0),
# interleaved; lockstep parity of each first.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "step $name failed: $?"; tail -30 "gpurun_out/$name.log"; exit 1; }; tail -1 "gpurun_out/$name.log"; }
export PYTHONUNBUFFERED=1
P="python tools/c5_probe.py 1000000 12"
for v in ${VARIANTS:-b2 b4}; do
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_cs_$v.so step pytest_cs_$v 300 python -u -m pytest tests/test_causal.py -m gpu -x -q --timeout 240 --timeout-method thread -k lockstep
done
for rep in 1 2; do
  for v in prev ${VARIANTS:-b2 b4}; do
    PSIM_LIB_PATH=$PWD/partisan_amd/exp_cs_$v.so step c5_${v}_$rep 200 $P
  done
done
echo done
