#!/usr/bin/env bash
# Round-5 session D: C3 with per-wave LDS send buffers (one atomic per 64
# sends), register top-k selection and no row snapshots: SCAMP / C3 parity,
# then C3 lines new vs exp_prewq.so (the tree before).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # name seconds cmd...
    local name=$1 secs=$2; shift 2
    echo "=== $name" ; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-600
    [ $rc -le 1 ] || exit $rc
}
OLD=$PWD/partisan_amd/exp_prewq.so
step d_parity 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_scamp.py tests/test_c3.py
for rep in 1 2; do
  step c3_new_$rep 200 python tools/config_bench.py C3
  PSIM_LIB_PATH=$OLD step c3_old_$rep 200 python tools/config_bench.py C3
done
step prof_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 tools/config_bench.py C3
echo "=== session done"
