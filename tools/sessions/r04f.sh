#!/usr/bin/env bash
# Round-4 session F: the causal round kernel's branch-free arrival path --
# lockstep parity, C5 time, SQ counters.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; [ $rc -le 1 ] || exit $rc; }
step t_causal 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_causal.py tests/test_causal_shard.py
step c5_f 200 python tools/config_bench.py C5

step pmc_c5f 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    --kernel-include-regex cs_round -d gpurun_out/pmc_c5f -o run --output-format csv -- python3 tools/c5_probe.py
echo done
