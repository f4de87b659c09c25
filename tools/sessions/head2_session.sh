#!/usr/bin/env bash
# GPU box: full -m gpu suite, smoke, two benches and a kernel trace (gaps).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local n=$1 s=$2; shift 2; echo "=== $n"; timeout -k 10 "$s" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; tail -2 "gpurun_out/$n.log" | cut -c1-400; [ $rc -eq 0 ] || { echo "=== $n rc=$rc"; exit $rc; }; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench1 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
step bench2 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline
step trace 300 rocprofv3 --kernel-trace -d gpurun_out/trace2 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
echo "=== session done"
