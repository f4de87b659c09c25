#!/usr/bin/env bash
# Round-5 session C: the configs' 8-way splits on one GPU (tests/test_world8.py).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 1150 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread -p no:cacheprovider -m gpu tests/test_world8.py > gpurun_out/world8.log 2>&1
rc=$?
echo "=== world8 rc=$rc"; grep -E "PASS|FAIL|passed|failed|Error|rounds" gpurun_out/world8.log | tail -12
exit $rc
