#!/usr/bin/env bash
# Round-4 session H2: HyParView groups sized to the vertex count (hv_group).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400; [ $rc -le 1 ] || exit $rc; }
step t_hv 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_hyparview.py
step c2_auto 300 python tools/config_bench.py C2
step hv_auto 300 python tools/probe_engines.py hv 1000000
step hv_100k 300 python tools/probe_engines.py hv 100000
echo done
