#!/usr/bin/env bash
# Round 3: HyParView at 1M peers (200 join waves of 5000, then 40 rounds,
# tools/probe_engines.py hv) -- kernel stats and FETCH/WRITE passes.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "step $name failed: $?"; exit 1; }; }
step hv_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/hv_prof -o run --output-format csv -- python3 tools/probe_engines.py hv
step hv_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/hv_fetch -o run --output-format csv -- python3 tools/probe_engines.py hv
step hv_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/hv_write -o run --output-format csv -- python3 tools/probe_engines.py hv
python tools/engine_traffic.py gpurun_out/hv_prof gpurun_out/hv_fetch gpurun_out/hv_write --out gpurun_out/hv_traffic.json > /dev/null || exit 1
echo done
