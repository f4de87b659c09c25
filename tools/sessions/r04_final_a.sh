#!/usr/bin/env bash
# Round-4 final, part A: the whole -m gpu suite and smoke() on this build.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
echo "== pytest"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_final.log 2>&1
rc=$?
echo "== pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu_final.log
[ $rc -le 1 ] || exit $rc
echo "== smoke"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1
echo "== smoke rc=$?"; tail -2 gpurun_out/smoke_final.log
