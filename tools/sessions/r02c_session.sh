#!/usr/bin/env bash
# GPU box: artefacts of the current head -- kernel trace (per-dispatch start /
# end, for the gaps between rounds), PMC FETCH / WRITE passes, the bench with
# that traffic and its rocprof stats, and the 8-shard projection.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local n=$1 s=$2; shift 2; echo "=== $n"; timeout -k 10 "$s" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; tail -3 "gpurun_out/$n.log"; [ $rc -eq 0 ] || { echo "=== $n rc=$rc"; exit $rc; }; }
step trace 300 rocprofv3 --kernel-trace -d gpurun_out/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --n 10000000 --peers 5 --rounds-per-step 16 --steps 3 --out gpurun_out/pmc_traffic.json || exit 1
step bench 600 python bench.py --steps 10 --warmup 2 --traffic-json gpurun_out/pmc_traffic.json
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
step proj 600 python tools/shard_projection.py
echo "=== session done"
