#!/usr/bin/env bash
# Round-4 session C: 3-pass transport micro-benchmark (prefetched loads);
# the in-library causal exchange, the NIF harness, collective set_delays, 10M oracle parity.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; [ $rc -le 1 ] || exit $rc; }
step mbb2 180 tools/mb_binned
step t_c 1200 python -u -m pytest -v --timeout 900 --timeout-method thread -m gpu \
    tests/test_causal_shard.py tests/test_nif_harness.py tests/test_shard.py::test_sharded_set_delays_busy_on_every_rank \
    tests/test_c3.py::test_gpu_c3_many_grafts_per_vertex_round tests/test_configs_at_scale.py::test_bench_config_10m_oracle_parity
echo done
