#!/usr/bin/env bash
# Round-4 session I: per-round SQ / L2 counters of the Plumtree round kernel
# over one 10M flood (which rounds wait, which issue).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pmc_r1 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
    --kernel-include-regex pt_round_ell -d gpurun_out/pmc_r1 -o run --output-format csv -- python3 tools/round_profile.py --steps 1
step pmc_r2 180 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM TCC_HIT_sum TCC_MISS_sum \
    --kernel-include-regex pt_round_ell -d gpurun_out/pmc_r2 -o run --output-format csv -- python3 tools/round_profile.py --steps 1
echo done
