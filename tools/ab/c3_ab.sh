#!/usr/bin/env bash
# A/B (round 3): C3's Plumtree kernel without scratch memory (pd_process:
# context in registers) vs the previous build (exp_pd_old: 400 B of scratch
# per thread); parity first, then C3 lines and FETCH/WRITE passes of each.
set -u
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "step $name failed: $?"; exit 1; }; }
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OLD=$PWD/partisan_amd/exp_pd_old.so
step pytest_c3 600 python -m pytest tests/test_c3.py tests/test_configs_at_scale.py -m gpu -x -q -k "c3 or C3"
for rep in 1 2; do
  step c3_new_$rep 300 python tools/config_bench.py C3
  PSIM_LIB_PATH=$OLD step c3_old_$rep 300 python tools/config_bench.py C3
done
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_new_$c 300 rocprofv3 --pmc $c -d gpurun_out/pmc_new_$c -o run --output-format csv -- python3 tools/config_bench.py C3
  PSIM_LIB_PATH=$OLD step pmc_old_$c 300 rocprofv3 --pmc $c -d gpurun_out/pmc_old_$c -o run --output-format csv -- python3 tools/config_bench.py C3
done
step prof_new 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_new -o run --output-format csv -- python3 tools/config_bench.py C3
echo done
