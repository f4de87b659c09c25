#!/usr/bin/env bash
# Round-4 session N: the flag-free threshold (PSIM_DENSE_DIV: a round after
# >= n / d messages writes no group flags; head d = 4) and the list threshold
# (PSIM_WL_THR; head ng / 8 = 78125 at 10M): bench A/B on one box, parity.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -h '^{' "gpurun_out/$name.log" | python3 -c "import json,sys;[print('  ms_per_step', json.loads(l)['ms_per_step']) for l in sys.stdin]" 2>/dev/null; tail -1 "gpurun_out/$name.log" | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
PSIM_DENSE_DIV=16 step t_dense16 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_worklist_parity.py
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
for rep in 1 2; do
  for d in 4 8 16 32; do PSIM_DENSE_DIV=$d step bk_d${d}_$rep 300 $B; done
  for w in 20000 200000 400000; do PSIM_WL_THR=$w step bk_w${w}_$rep 300 $B; done
done
PSIM_DENSE_DIV=16 step rp_d16 300 python tools/round_profile.py --steps 2
PSIM_WL_THR=400000 step rp_w400000 300 python tools/round_profile.py --steps 2
step rp_base 300 python tools/round_profile.py --steps 2
echo done
