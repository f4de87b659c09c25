#!/usr/bin/env bash
# A/B of Demers (C4, 10M) library variants: tools/config_bench.py C4 per variant
set -u
mkdir -p gpurun_out
for v in ${VARIANTS:-cur dmnt cur dmnt}; do
  PSIM_LIB_PATH=$PWD/tools/ab/libpsim_$v.so timeout -k 10 300 python tools/config_bench.py C4 > gpurun_out/c4ab.log 2>&1 || exit $?
  echo "$v $(grep '^{' gpurun_out/c4ab.log | tail -1)"
done
