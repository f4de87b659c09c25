#!/usr/bin/env bash
# GPU box: parity of the record-queue engines (HyParView, SCAMP, C3, window
# lanes), then their throughput (HyParView 1M steady rounds, C3 1M churn).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local n=$1 s=$2; shift 2; echo "=== $n"; timeout -k 10 "$s" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; tail -3 "gpurun_out/$n.log"; [ $rc -eq 0 ] || { echo "=== $n rc=$rc"; exit $rc; }; }
step pytest_eng 900 python -u -m pytest tests/test_hyparview.py tests/test_scamp.py tests/test_c3.py tests/test_plumtree_gpu.py -m gpu -x -q -k "not build_tree" --timeout 500 --timeout-method thread
step probe_hv 300 python tools/probe_engines.py hv
step cfg_c3 600 python tools/config_bench.py C3 C2
echo done
