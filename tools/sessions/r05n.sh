#!/usr/bin/env bash
# Round-5: the origin by a wave (one lane per peer slot): Plumtree parity, bench A/B, a trace.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # name seconds cmd...  (stops the session on a GPU fault, abort, kill or timeout)
    local name=$1 secs=$2; shift 2
    echo "=== $name" ; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
    if grep -qiE "illegal memory|memory access fault|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "gpurun_out/$name.log"; then
        echo "=== GPU fault in $name: stopping"; exit 3
    fi
    [ $rc -le 1 ] || exit $rc
}
OLD=$PWD/partisan_amd/exp_pre_origin.so
step parity 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_plumtree_gpu.py tests/test_worklist_parity.py tests/test_forest.py tests/test_nif_harness.py
grep -q " passed" gpurun_out/parity.log && ! grep -q "failed" gpurun_out/parity.log || { echo "=== parity not green: stopping"; exit 4; }
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --sustain-s 2"
for rep in 1 2 3; do
  step b_new_$rep 200 $B
  PSIM_LIB_PATH=$OLD step b_old_$rep 200 $B
done
step trace 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --sustain-s 0
echo "=== session done"
