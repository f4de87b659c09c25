#!/usr/bin/env bash
# Round-5 final session, part 1: the whole -m gpu suite and smoke() on this tree.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 1020 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "=== pytest_gpu rc=$rc"; tail -6 gpurun_out/pytest_gpu.log | cut -c1-300
if grep -qiE "illegal memory|memory access fault|HSA_STATUS_ERROR|core dumped" gpurun_out/pytest_gpu.log; then echo "=== GPU fault"; exit 3; fi
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc2=$?
echo "=== smoke rc=$rc2"; tail -2 gpurun_out/smoke.log
exit $(( rc > rc2 ? rc : rc2 ))
