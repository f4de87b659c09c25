#!/usr/bin/env bash
# Round-4 session B: the 3-pass LDS transport micro-benchmark; C3 rows and
# in-library Demers exchange tests; A/B of the mark-2 claims issued before
# the word stores (default) vs after them (PT_CLAIMS_AFTER_STORES build).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; [ $rc -le 1 ] || exit $rc; }
step mbb 180 tools/mb_binned
step t_wl 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_worklist_parity.py tests/test_frontier.py
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
OLD=$PWD/partisan_amd/exp_claims_after.so
for rep in 1 2; do
  step b_new_$rep 300 $B
  PSIM_LIB_PATH=$OLD step b_old_$rep 300 $B
done
step rp_new 300 python tools/round_profile.py --steps 2
PSIM_LIB_PATH=$OLD step rp_old 300 python tools/round_profile.py --steps 2
step t_b 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
    tests/test_c3.py tests/test_demers_shard.py tests/test_configs_at_scale.py -k "c3 or demers or c4"
echo done
