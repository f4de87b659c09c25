#!/usr/bin/env bash
# Round-5 (session 11, final): small-overlay HyParView rounds bucket their
# messages in one workgroup (hv_bucket_small) instead of two fills + five
# launches: the C2 line new vs old (= exp_head.so) twice each; then on this
# build the whole GPU suite (HyParView parity on both paths: <= 12,288 and
# larger overlays) and smoke, PMC FETCH / WRITE keyed to its sha256, the
# bench and rocprof kernel stats.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # name seconds cmd...  (stops the session on a GPU fault, abort, kill or timeout)
    local name=$1 secs=$2; shift 2
    echo "=== $name" ; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-400
    if grep -qiE "illegal memory|memory access fault|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "gpurun_out/$name.log"; then
        echo "=== GPU fault in $name: stopping"; exit 3
    fi
    [ $rc -le 1 ] || exit $rc
}
OLD=$PWD/partisan_amd/exp_head.so
for rep in 1 2; do
  step c2h_new_$rep 300 python tools/config_bench.py C2
  PSIM_LIB_PATH=$OLD step c2h_old_$rep 300 python tools/config_bench.py C2
done
step gpu_suite 1500 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider
grep -q " passed" gpurun_out/gpu_suite.log && ! grep -q "failed" gpurun_out/gpu_suite.log || { echo "=== suite not green: stopping"; exit 4; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --sustain-s 0
step pmc_write 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --sustain-s 0
python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --n 10000000 --peers 5 --rounds-per-step 16 --steps 4 --source profiles/r05 --out gpurun_out/pmc_traffic.json > gpurun_out/pmc_traffic.log 2>&1 || exit 5
step bench 600 python bench.py --steps 20 --warmup 5 --traffic-json gpurun_out/pmc_traffic.json
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --sustain-s 0
echo "=== session done"
