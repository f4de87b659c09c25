#!/usr/bin/env bash
# Round-5 (session 2): psim_hv_join_seq (C2's sequential joins in one call):
# HyParView parity (C2 against the oracle through join_seq, join_seq = join +
# step), then the C2 line.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400; [ $rc -le 1 ] || exit $rc; }
step hv_parity 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu tests/test_hyparview.py tests/test_nif_harness.py
grep -q " passed" gpurun_out/hv_parity.log && ! grep -q "failed" gpurun_out/hv_parity.log || { echo "=== parity not green: stopping"; exit 4; }
step c2_1 300 python tools/config_bench.py C2
step c2_2 300 python tools/config_bench.py C2
echo "=== session done"
