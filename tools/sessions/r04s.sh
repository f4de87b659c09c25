#!/usr/bin/env bash
# Round-4 session S: the partial-view membership test and the C3 peer-table lookup read as quads
# (row_has, row_find: SCAMP in_pv, C3 connected, tab_find) and sends to known members without
# the scan (working tree) against the head (exp_head.so): parity, C3 A/B,
# C3 kernel stats.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -h '^{' "gpurun_out/$name.log" | cut -c1-260; tail -1 "gpurun_out/$name.log" | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
step t_sc 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_scamp.py tests/test_c3.py
for rep in 1 2; do
  step c3_new_$rep 300 python tools/config_bench.py C3
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_head.so step c3_old_$rep 300 python tools/config_bench.py C3
done
step prof_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 tools/config_bench.py C3
echo done
