#!/usr/bin/env bash
# Round-5 session I: a kernel + copy trace of the bench (per-step timeline, gaps).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --sustain-s 0 > gpurun_out/trace.log 2>&1
rc=$?; echo "=== trace rc=$rc"; tail -2 gpurun_out/trace.log | cut -c1-300; exit $rc
