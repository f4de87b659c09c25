#!/usr/bin/env bash
# Round-4 session M: what a sparse round's floor is made of (tools/mb_launch),
# then persistent rounds (PSIM_PERSIST=1, one launch per 16-round chunk with a
# device barrier between rounds): parity, bench A/B, per-round profile.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300; [ $rc -le 1 ] || exit $rc; }
step mb_launch 200 ./tools/mb_launch
PSIM_PERSIST=1 step t_pst 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_worklist_parity.py tests/test_plumtree_gpu.py
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
for rep in 1 2; do
  PSIM_PERSIST=1 step bk_pst_$rep 300 $B
  step bk_base_$rep 300 $B
done
PSIM_PERSIST=1 step rp_pst 300 python tools/round_profile.py --steps 2
step rp_base 300 python tools/round_profile.py --steps 2
echo done
