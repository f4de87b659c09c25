#!/usr/bin/env bash
# Round-4 session T: SQ counters of the C3 process kernels (sc_process,
# pd_process) -- issue-bound or waiting?
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
step pmc_c3 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
    --kernel-include-regex "sc_process|pd_process" -d gpurun_out/pmc_c3 -o run --output-format csv -- python3 tools/config_bench.py C3
step pmc_c3b 240 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU TCC_HIT_sum TCC_MISS_sum \
    --kernel-include-regex "sc_process|pd_process" -d gpurun_out/pmc_c3b -o run --output-format csv -- python3 tools/config_bench.py C3
echo done
