#!/usr/bin/env bash
# Round-4 session G: kernel-level time split of the secondary engines
# (C2 HyParView at 10k, C3 SCAMP + Plumtree repair at 1M, HyParView at 1M).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step prof_c2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 tools/config_bench.py C2
rm -f gpurun_out/prof_c2/run_kernel_trace.csv
step prof_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 tools/probe_engines.py c3
rm -f gpurun_out/prof_c3/run_kernel_trace.csv
step prof_hv 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_hv -o run --output-format csv -- python3 tools/probe_engines.py hv 1000000
rm -f gpurun_out/prof_hv/run_kernel_trace.csv
echo done
