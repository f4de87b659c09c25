#!/usr/bin/env bash
# Round-5 (session 2): C5 arrivals in batches of 4 (arrive_batch, new) vs
# one at a time (old = exp_c5_old.so): causal parity, then the C5 line A/B.
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
OLD=$PWD/partisan_amd/exp_c5_old.so
step parity 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_causal.py tests/test_causal_shard.py
grep -q " passed" gpurun_out/parity.log && ! grep -q "failed" gpurun_out/parity.log || { echo "=== parity not green: stopping"; exit 4; }
for rep in 1 2; do
  step c5_new_$rep 300 python tools/config_bench.py C5
  PSIM_LIB_PATH=$OLD step c5_old_$rep 300 python tools/config_bench.py C5
done
grep -h '"C5"' gpurun_out/c5_*.log
echo "=== session done"
