#!/usr/bin/env bash
# Round-4 session L: PC sampling (host trap) of the Plumtree flood, to find
# where the round kernel spends its issue slots.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
    --pc-sampling-interval 1 -d gpurun_out/pcs -o run --output-format csv -- python3 tools/round_profile.py --steps 3 > gpurun_out/pcs.log 2>&1
rc=$?
echo "pcs rc=$rc"; tail -5 gpurun_out/pcs.log | cut -c1-300; ls -la gpurun_out/pcs 2>/dev/null
