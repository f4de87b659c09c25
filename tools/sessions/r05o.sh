#!/usr/bin/env bash
# Round-5: every per-round host wait by polling an event (new) vs blocking
# stream syncs (old = exp_pre_spin.so): parity of the engines, config lines A/B.
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
OLD=$PWD/partisan_amd/exp_pre_spin.so
step parity 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_hyparview.py tests/test_scamp.py tests/test_c3.py tests/test_demers.py tests/test_causal.py tests/test_forest.py tests/test_fullmem.py
grep -q " passed" gpurun_out/parity.log && ! grep -q "failed" gpurun_out/parity.log || { echo "=== parity not green: stopping"; exit 4; }
for rep in 1 2; do
  step cfg_new_$rep 400 python tools/config_bench.py C2 C3 C4 C5
  PSIM_LIB_PATH=$OLD step cfg_old_$rep 400 python tools/config_bench.py C2 C3 C4 C5
done
echo "=== session done"
