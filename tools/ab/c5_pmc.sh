#!/usr/bin/env bash
# PMC passes on the causal round kernel (one pass per counter group).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/c5pmc${C5TAG:-}$i -o run --output-format csv -- python3 tools/c5_probe.py ${C5N:-1000000} 8 > gpurun_out/c5pmc${C5TAG:-}$i.log 2>&1 || { echo "pass $i failed: $?"; tail -5 gpurun_out/c5pmc${C5TAG:-}$i.log; exit 1; }
done
echo done
