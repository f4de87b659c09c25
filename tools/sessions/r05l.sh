#!/usr/bin/env bash
# Round-5: broadcast_run with max_rounds 0 settles the origin (the fix), then
# the tests that the whole-suite run failed on.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_plumtree_gpu.py tests/test_nif_harness.py > gpurun_out/l_parity.log 2>&1
rc=$?; echo "=== l_parity rc=$rc"; tail -3 gpurun_out/l_parity.log | cut -c1-300; exit $rc
