#!/usr/bin/env bash
# Round-4 final, part B: PMC FETCH/WRITE passes keyed to this libpsim build,
# the bench line, the rocprof --kernel-trace --stats summary of the same
# command, and the C2-C5 / RELAY config lines.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --n 10000000 --peers 5 --rounds-per-step 16 --steps 3 --source profiles/r04 --out gpurun_out/pmc_traffic.json || exit 1
step bench 600 python bench.py --steps 20 --warmup 3 --traffic-json gpurun_out/pmc_traffic.json
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline
step configs 600 python tools/config_bench.py C2 C3 C4 C5 RELAY
echo done
