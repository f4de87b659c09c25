#!/usr/bin/env bash
# Round-4 session K: the A/B of the working tree (default) against the last commit
# vs the per-slot FIFO walk (exp_prevhead.so): parity, bench A/B, per-round.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300; [ $rc -le 1 ] || exit $rc; }
step t_pt 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_worklist_parity.py tests/test_plumtree_gpu.py
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
for rep in 1 2; do
  step bk_new_$rep 300 $B
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_prevhead.so step bk_old_$rep 300 $B
done
step rpk_new 300 python tools/round_profile.py --steps 2
PSIM_LIB_PATH=$PWD/partisan_amd/exp_prevhead.so step rpk_old 300 python tools/round_profile.py --steps 2
step pmck_r1 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
    --kernel-include-regex pt_round_ell -d gpurun_out/pmck_r1 -o run --output-format csv -- python3 tools/round_profile.py --steps 1
echo done
