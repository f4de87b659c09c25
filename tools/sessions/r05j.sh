#!/usr/bin/env bash
# Round-5 session J: the round kernel's branch-light vertex path (one
# divergent region per row / per vertex's LDS words, a select-only reply path
# for flood replies) vs exp_base5.so: parity, bench A/B, per-round SQ counters.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # name seconds cmd...  (stops the session on a GPU fault, abort, kill or timeout)
    local name=$1 secs=$2; shift 2
    echo "=== $name" ; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
    if grep -qiE "illegal memory|memory access fault|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "gpurun_out/$name.log"; then
        echo "=== GPU fault in $name: stopping"; exit 3
    fi
    [ $rc -le 1 ] || exit $rc
}
OLD=$PWD/partisan_amd/exp_base5.so
step parity 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_plumtree_gpu.py tests/test_worklist_parity.py
grep -q " passed" gpurun_out/parity.log && ! grep -q "failed" gpurun_out/parity.log || { echo "=== parity not green: stopping"; exit 4; }
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --sustain-s 2"
for rep in 1 2 3; do
  step b_new_$rep 200 $B
  PSIM_LIB_PATH=$OLD step b_old_$rep 200 $B
done
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
step pmc_new 180 rocprofv3 --pmc $SQ --kernel-include-regex pt_round_ell -d gpurun_out/pmc_new -o run --output-format csv -- python3 tools/round_profile.py --steps 1
PSIM_LIB_PATH=$OLD step pmc_old 180 rocprofv3 --pmc $SQ --kernel-include-regex pt_round_ell -d gpurun_out/pmc_old -o run --output-format csv -- python3 tools/round_profile.py --steps 1
echo "=== session done"
