#!/usr/bin/env bash
# Round-4 session A (gpurun): the new parity tests, the bench line with the
# 10M oracle parity, the dense-round transport micro-benchmark.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; [ $rc -le 1 ] || exit $rc; }
step t_new 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
    tests/test_bench_launch.py tests/test_fullmem.py tests/test_nif_harness.py \
    tests/test_c3.py::test_gpu_c3_many_grafts_per_vertex_round tests/test_shard.py::test_sharded_set_delays_busy_on_every_rank \
    tests/test_configs_at_scale.py::test_bench_config_10m_oracle_parity
step bench 600 python bench.py --steps 10 --warmup 2 --cpu-workers 0
step mbt 180 tools/mb_transpose 0.54
echo done
