#!/usr/bin/env bash
# GPU box: sharded handles on ELL rows -- the sharded / NIF / membership GPU
# tests, then the 8-shard projection with ELL and with CSR rows.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local n=$1 s=$2; shift 2; echo "=== $n"; timeout -k 10 "$s" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; tail -3 "gpurun_out/$n.log"; [ $rc -eq 0 ] || { echo "=== $n rc=$rc"; exit $rc; }; }
step pytest_shard 600 python -u -m pytest tests/test_shard.py tests/test_nif_harness.py tests/test_membership_strategy.py tests/test_plumtree_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread
step proj_ell 600 python tools/shard_projection.py
step proj_csr 600 python tools/shard_projection.py --csr
echo "=== session done"
