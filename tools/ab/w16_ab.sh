#!/usr/bin/env bash
# A/B of round-profile runs over library variants (tools/ab/libpsim_<name>.so)
set -u
mkdir -p gpurun_out
for v in ${VARIANTS:-prev cur norf prev cur norf}; do
  echo "== $v"
  PSIM_LIB_PATH=$PWD/tools/ab/libpsim_$v.so timeout -k 10 200 python tools/round_profile.py --steps 4 || exit $?
done
