#!/usr/bin/env bash
# Round-5 session F: WaveQ microtest (wavefront-scope count), SCAMP / C3
# parity, Plumtree parity with the chunk prep kernel and broadcast_run, then
# C3 lines new vs exp_prewq.so and the bench.
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
OLD=$PWD/partisan_amd/exp_prewq.so
step wq 60 ./tools/mb/mb_wq
step sc_parity 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_scamp.py tests/test_c3.py
grep -q " passed" gpurun_out/sc_parity.log && ! grep -q "failed" gpurun_out/sc_parity.log || { echo "=== sc parity not green: stopping"; exit 4; }
step pt_parity 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_plumtree_gpu.py tests/test_worklist_parity.py tests/test_forest.py
for rep in 1 2; do
  step c3_new_$rep 200 python tools/config_bench.py C3
  PSIM_LIB_PATH=$OLD step c3_old_$rep 200 python tools/config_bench.py C3
done
step bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
echo "=== session done"
