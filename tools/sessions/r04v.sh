#!/usr/bin/env bash
# Round-4 session V: C3 i_haves and SCAMP pings reserved once per lane (working tree)
# against one reservation per send (exp_head.so): parity, C3 A/B, C3 kernel stats.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -h '^{' "gpurun_out/$name.log" | cut -c1-260; tail -1 "gpurun_out/$name.log" | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
step t_sc 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_scamp.py tests/test_c3.py tests/test_nif_harness.py tests/test_membership_strategy.py
for rep in 1 2; do
  step c3_new_$rep 300 python tools/config_bench.py C3
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_head.so step c3_old_$rep 300 python tools/config_bench.py C3
done
step prof_c3v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3v -o run --output-format csv -- python3 tools/config_bench.py C3
echo done
