#!/usr/bin/env bash
# Round-5 session A: the -m gpu suite on the cleaned-up build (frontier kernel
# and PT_* variants deleted, word counter, vclock ops, collective agreement),
# smoke, the bench with the per-round roofline, rocprof stats, PMC passes.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # name seconds cmd...
    local name=$1 secs=$2; shift 2
    echo "=== $name" ; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
    [ $rc -le 1 ] || exit $rc
}
step pytest_forest 400 python -u -m pytest tests/test_forest.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider
step pytest_gpu 1100 python -u -m pytest tests -m gpu --ignore=tests/test_forest.py -q -x --timeout 400 --timeout-method thread -p no:cacheprovider
step smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py --steps 20 --warmup 3
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline
step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_write 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
echo "=== session done"
