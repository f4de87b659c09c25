#!/usr/bin/env bash
# Round-4 session H: HyParView vertex groups of 8 per wave (default) vs 64
# (exp_hv64.so): lockstep parity, C2 and HyParView at 1M.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400; [ $rc -le 1 ] || exit $rc; }
step t_hv 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_hyparview.py
step c2_g8 300 python tools/config_bench.py C2
PSIM_LIB_PATH=$PWD/partisan_amd/exp_hv64.so step c2_g64 300 python tools/config_bench.py C2
step hv_g8 300 python tools/probe_engines.py hv 1000000
PSIM_LIB_PATH=$PWD/partisan_amd/exp_hv64.so step hv_g64 300 python tools/probe_engines.py hv 1000000
echo done
