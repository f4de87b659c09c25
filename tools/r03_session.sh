#!/usr/bin/env bash
# Round-3 measurement session on one MI355X (run through gpurun):
# kernel trace, PMC FETCH/WRITE passes keyed to this libpsim build, the bench
# line, the rocprof --stats summary of the same command, and the C2-C5
# config lines (tools/config_bench.py).
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "step $name failed: $?"; exit 1; }; }
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --n 10000000 --peers 5 --rounds-per-step 16 --steps 3 --source profiles/r03 --out gpurun_out/pmc_traffic.json || exit 1
step bench 600 python bench.py --steps 20 --warmup 3 --traffic-json gpurun_out/pmc_traffic.json
step configs 900 python tools/config_bench.py C2 C3 C4 C5
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline
echo done
