#!/usr/bin/env bash
# Round-4 session D: batched candidate loads (PT_BATCH=2, default build) vs
# PT_BATCH=1 (exp_b1.so) vs the committed head (exp_head.so); the 3-pass
# transport micro-benchmark; session C's tests.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; [ $rc -le 1 ] || exit $rc; }
step t_wl 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_worklist_parity.py
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
for rep in 1 2; do
  step b_b2_$rep 300 $B
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_b1.so step b_b1_$rep 300 $B
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_head.so step b_head_$rep 300 $B
done
step rp_b2 300 python tools/round_profile.py --steps 2
PSIM_LIB_PATH=$PWD/partisan_amd/exp_head.so step rp_head 300 python tools/round_profile.py --steps 2
step mbb2 180 tools/mb_binned
step t_c 1200 python -u -m pytest -v --timeout 900 --timeout-method thread -m gpu \
    tests/test_causal_shard.py tests/test_nif_harness.py tests/test_shard.py::test_sharded_set_delays_busy_on_every_rank \
    tests/test_c3.py::test_gpu_c3_many_grafts_per_vertex_round tests/test_configs_at_scale.py::test_bench_config_10m_oracle_parity
echo done
