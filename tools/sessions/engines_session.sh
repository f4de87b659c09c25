#!/usr/bin/env bash
# Runs on the GPU box: throughput of C2-C5 (tools/config_bench.py), their CPU
# oracle baselines (tools/cpu_configs.py, 1 process and 16), a rocprof kernel
# trace and FETCH_SIZE / WRITE_SIZE PMC passes over C3-C5.  Each GPU step has
# its own time limit; any failure ends the session.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local n=$1 s=$2; shift 2; echo "=== $n"; timeout -k 10 "$s" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; tail -3 "gpurun_out/$n.log"; [ $rc -eq 0 ] || { echo "=== $n rc=$rc"; exit $rc; }; }
step configs 600 python tools/config_bench.py C2 C3 C4 C5
step cpu_configs 900 python tools/cpu_configs.py --workers 16
step prof_cfg 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg -o run --output-format csv -- python3 tools/config_bench.py C2 C3 C4 C5
step pmc_cfg_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_cfg_fetch -o run --output-format csv -- python3 tools/config_bench.py C3 C4 C5
step pmc_cfg_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_cfg_write -o run --output-format csv -- python3 tools/config_bench.py C3 C4 C5
python tools/engine_traffic.py gpurun_out/prof_cfg gpurun_out/pmc_cfg_fetch gpurun_out/pmc_cfg_write --out gpurun_out/engine_traffic.json > /dev/null
echo done
