#!/usr/bin/env bash
# Round-5 session E: the WaveQ microtest, then SCAMP parity (small n).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # name seconds cmd...  (stops the session on a GPU fault, abort, kill or timeout)
    local name=$1 secs=$2; shift 2
    echo "=== $name" ; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-600
    if grep -qiE "illegal memory|memory access fault|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "gpurun_out/$name.log"; then
        echo "=== GPU fault in $name: stopping"; exit 3
    fi
    [ $rc -le 1 ] || exit $rc
}
step wq 60 ./tools/mb/mb_wq
step scamp 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_scamp.py
echo "=== session done"
