#!/usr/bin/env bash
# Round-5 (session 2): C3 host path -- crash lists uploaded once through pinned
# staging with no waits, one wait per round for the SCAMP + Plumtree rounds,
# sorted call lists not re-sorted (new) vs the head (old = exp_c3_old.so):
# SCAMP / C3 / NIF parity, then the C3 wall split and config line A/B.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # name seconds cmd...  (stops the session on a GPU fault, abort, kill or timeout)
    local name=$1 secs=$2; shift 2
    echo "=== $name" ; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400
    if grep -qiE "illegal memory|memory access fault|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "gpurun_out/$name.log"; then
        echo "=== GPU fault in $name: stopping"; exit 3
    fi
    [ $rc -le 1 ] || exit $rc
}
OLD=$PWD/partisan_amd/exp_c3_old.so
step parity 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_scamp.py tests/test_c3.py tests/test_membership_strategy.py tests/test_nif_harness.py
grep -q " passed" gpurun_out/parity.log && ! grep -q "failed" gpurun_out/parity.log || { echo "=== parity not green: stopping"; exit 4; }
for rep in 1 2; do
  step c3w_new_$rep 240 python tools/c3_wall.py 1000000 30
  PSIM_LIB_PATH=$OLD step c3w_old_$rep 240 python tools/c3_wall.py 1000000 30
done
step cfg_c3_new 300 python tools/config_bench.py C3
PSIM_LIB_PATH=$OLD step cfg_c3_old 300 python tools/config_bench.py C3
echo "=== session done"
