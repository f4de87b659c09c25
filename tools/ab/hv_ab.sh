#!/usr/bin/env bash
# A/B of the HyParView round kernel variants (tools/ab/libpsim_*.so): 1M steady rounds
set -u
mkdir -p gpurun_out
for v in w4s32 w6s32 w8s32 w4s64 w6s64 w4s32; do
  PSIM_LIB_PATH=$PWD/tools/ab/libpsim_$v.so timeout -k 10 200 python tools/probe_engines.py hv > gpurun_out/hv_$v.log 2>&1 || exit $?
  echo "$v $(tail -1 gpurun_out/hv_$v.log)"
done
