#!/usr/bin/env bash
# Round-4 session Q: light/heavy candidate order + output skip (working tree), order only (exp_sort.so), against
# the head (exp_full.so): parity, bench A/B, per-round profile, round PMC.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -h '^{' "gpurun_out/$name.log" | python3 -c "import json,sys;[print('  ms_per_step', json.loads(l)['ms_per_step']) for l in sys.stdin]" 2>/dev/null; tail -1 "gpurun_out/$name.log" | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
step t_pt 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_worklist_parity.py tests/test_plumtree_gpu.py tests/test_frontier.py tests/test_shard.py
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
for rep in 1 2 3; do
  step bk_new_$rep 300 $B
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_sort.so step bk_sort_$rep 300 $B
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_full.so step bk_head_$rep 300 $B
done
step rp_new 300 python tools/round_profile.py --steps 2
PSIM_LIB_PATH=$PWD/partisan_amd/exp_sort.so step rp_sort 300 python tools/round_profile.py --steps 2
PSIM_LIB_PATH=$PWD/partisan_amd/exp_full.so step rp_head 300 python tools/round_profile.py --steps 2
step pmc_new 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
    --kernel-include-regex pt_round_ell -d gpurun_out/pmc_new -o run --output-format csv -- python3 tools/round_profile.py --steps 1
echo done
