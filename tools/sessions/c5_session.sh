#!/usr/bin/env bash
# GPU box: causal engine after the fold change -- parity tests, then C5 with
# the previous library (PSIM_LIB_PATH) and the new one.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local n=$1 s=$2; shift 2; echo "=== $n"; timeout -k 10 "$s" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; tail -2 "gpurun_out/$n.log" | cut -c1-500; [ $rc -eq 0 ] || { echo "=== $n rc=$rc"; exit $rc; }; }
step t_causal 600 python -u -m pytest tests/test_causal.py tests/test_causal_shard.py -m gpu -x -q --timeout 300 --timeout-method thread
step c5_new 300 python tools/config_bench.py C5
export PSIM_LIB_PATH=$PWD/tools/ab/libpsim_prev.so
step c5_prev 300 python tools/config_bench.py C5
unset PSIM_LIB_PATH
step c5_new2 300 python tools/config_bench.py C5
echo "=== session done"
