#!/usr/bin/env bash
# Round-4 session P: mostly-flagged chunks read whole (working tree: >= 48 of 64 groups; exp_t32.so: >= 32) against
# all-flagged chunks only (exp_full.so): parity, bench A/B, per-round profile.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -h '^{' "gpurun_out/$name.log" | python3 -c "import json,sys;[print('  ms_per_step', json.loads(l)['ms_per_step']) for l in sys.stdin]" 2>/dev/null; tail -1 "gpurun_out/$name.log" | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
step t_pt 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_worklist_parity.py tests/test_plumtree_gpu.py
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
for rep in 1 2 3; do
  step bk_t48_$rep 300 $B
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_t32.so step bk_t32_$rep 300 $B
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_full.so step bk_t64_$rep 300 $B
done
step rp_t48 300 python tools/round_profile.py --steps 2
PSIM_LIB_PATH=$PWD/partisan_amd/exp_t32.so step rp_t32 300 python tools/round_profile.py --steps 2
PSIM_LIB_PATH=$PWD/partisan_amd/exp_full.so step rp_t64 300 python tools/round_profile.py --steps 2
echo done
