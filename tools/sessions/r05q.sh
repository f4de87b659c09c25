#!/usr/bin/env bash
# Round-5 (session 2): SQ counters of cs_round_kernel, batched arrivals (new)
# vs one at a time (old = exp_c5_old.so), C5 probe.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; [ $rc -le 1 ] || exit $rc; }
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
step pmc_c5_new 180 rocprofv3 --pmc $C --kernel-include-regex cs_round -d gpurun_out/pmc_c5_new -o run --output-format csv -- python3 tools/c5_probe.py
PSIM_LIB_PATH=$PWD/partisan_amd/exp_c5_old.so step pmc_c5_old 180 rocprofv3 --pmc $C --kernel-include-regex cs_round -d gpurun_out/pmc_c5_old -o run --output-format csv -- python3 tools/c5_probe.py
for x in new old; do f=$(find gpurun_out/pmc_c5_$x -name '*counter_collection.csv' | head -1); echo "== $x"; python3 tools/pmc_summary.py "$f" cs_round 1000000 4; done
echo done
