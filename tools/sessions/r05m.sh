#!/usr/bin/env bash
# Round-5: SCAMP calls radix-sorted on the host, crash duplicates by stamps:
# SCAMP / C3 parity and the C3 line (wall per round).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # name seconds cmd...  (stops the session on a GPU fault, abort, kill or timeout)
    local name=$1 secs=$2; shift 2
    echo "=== $name" ; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-500
    if grep -qiE "illegal memory|memory access fault|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "gpurun_out/$name.log"; then
        echo "=== GPU fault in $name: stopping"; exit 3
    fi
    [ $rc -le 1 ] || exit $rc
}
step sc_parity 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_scamp.py tests/test_c3.py
grep -q " passed" gpurun_out/sc_parity.log && ! grep -q "failed" gpurun_out/sc_parity.log || { echo "=== parity not green: stopping"; exit 4; }
step c3_1 200 python tools/config_bench.py C3
step c3_2 200 python tools/config_bench.py C3
echo "=== session done"
