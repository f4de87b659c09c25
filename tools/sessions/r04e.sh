#!/usr/bin/env bash
# Round-4 session E: the Demers exchange forms (records / dense / auto) and
# the causal shard paths on the GPU; SQ instruction counters of the
# rewritten causal round kernel (C5) and of the Demers round kernel (C4).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; [ $rc -le 1 ] || exit $rc; }
step t_dm 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_demers_shard.py
step t_cs 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_causal_shard.py tests/test_nif_harness.py
step t_dly 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_shard.py -k "delay or overlapping" tests/test_plumtree_gpu.py
step c4 200 python tools/config_bench.py C4
step mbt 240 tools/mb_transpose
step pmc_c5 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    --kernel-include-regex cs_round -d gpurun_out/pmc_c5 -o run --output-format csv -- python3 tools/c5_probe.py
step pmc_c4 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY \
    --kernel-include-regex dm_round -d gpurun_out/pmc_c4 -o run --output-format csv -- python3 tools/config_bench.py C4
echo done
