#!/usr/bin/env bash
# Round 3: kernel stats and FETCH_SIZE / WRITE_SIZE passes over the C3-C5
# config runs (tools/config_bench.py), summarised by tools/engine_traffic.py.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "step $name failed: $?"; exit 1; }; }
step prof_cfg 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg -o run --output-format csv -- python3 tools/config_bench.py C3 C4 C5
step pmc_cfg_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_cfg_fetch -o run --output-format csv -- python3 tools/config_bench.py C3 C4 C5
step pmc_cfg_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_cfg_write -o run --output-format csv -- python3 tools/config_bench.py C3 C4 C5
python tools/engine_traffic.py gpurun_out/prof_cfg gpurun_out/pmc_cfg_fetch gpurun_out/pmc_cfg_write --out gpurun_out/engine_traffic.json > /dev/null || exit 1
echo done
