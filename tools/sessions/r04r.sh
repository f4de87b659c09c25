#!/usr/bin/env bash
# Round-4 session R: the ELL round kernel at 6 waves per SIMD (exp_w6.so: 80
# VGPRs, ~23 spilled) against the head's 5 (96 VGPRs): bench A/B, per round.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -h '^{' "gpurun_out/$name.log" | python3 -c "import json,sys;[print('  ms_per_step', json.loads(l)['ms_per_step']) for l in sys.stdin]" 2>/dev/null; tail -1 "gpurun_out/$name.log" | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
for rep in 1 2 3; do
  step bk_head_$rep 300 $B
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_w6.so step bk_w6_$rep 300 $B
done
step rp_head 300 python tools/round_profile.py --steps 2
PSIM_LIB_PATH=$PWD/partisan_amd/exp_w6.so step rp_w6 300 python tools/round_profile.py --steps 2
echo done
