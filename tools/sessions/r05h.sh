#!/usr/bin/env bash
# Round-5 session H: C3 with the device call index and round prep kernels:
# SCAMP / C3 parity, C3 lines, the phase split, rocprof stats.
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
step sc_parity 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_scamp.py tests/test_c3.py
grep -q " passed" gpurun_out/sc_parity.log && ! grep -q "failed" gpurun_out/sc_parity.log || { echo "=== parity not green: stopping"; exit 4; }
step win_parity 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_plumtree_gpu.py -k "overlapping or window"
step c3_1 200 python tools/config_bench.py C3
step c3_2 200 python tools/config_bench.py C3
step c3prof 300 python tools/c3_prof.py 1000000 30
step prof_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 tools/config_bench.py C3
echo "=== session done"
