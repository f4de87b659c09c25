#!/usr/bin/env bash
# Round-5 session B: parity of the dense-round candidate loop (mark 0 and
# one-GPU stores specialised) + the forest fix; bench A/B against
# exp_premark.so (the same tree without the specialisation); per-round SQ
# counters of both; the C2 all-roots line; the C3 phase split; the 8-way
# splits on one GPU.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # name seconds cmd...
    local name=$1 secs=$2; shift 2
    echo "=== $name" ; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400
    [ $rc -le 1 ] || exit $rc
}
OLD=$PWD/partisan_amd/exp_premark.so
step b_parity 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread -p no:cacheprovider -m gpu tests/test_plumtree_gpu.py tests/test_worklist_parity.py tests/test_forest.py
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
for rep in 1 2; do
  step b_new_$rep 200 $B
  PSIM_LIB_PATH=$OLD step b_old_$rep 200 $B
done
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
step pmc_new 180 rocprofv3 --pmc $SQ --kernel-include-regex pt_round_ell -d gpurun_out/pmc_new -o run --output-format csv -- python3 tools/round_profile.py --steps 1
PSIM_LIB_PATH=$OLD step pmc_old 180 rocprofv3 --pmc $SQ --kernel-include-regex pt_round_ell -d gpurun_out/pmc_old -o run --output-format csv -- python3 tools/round_profile.py --steps 1
step c2all 400 python tools/config_bench.py C2ALL
step c3prof 400 python tools/c3_prof.py 1000000 30
step c3line 300 python tools/config_bench.py C3
echo "(world8 tests: session C)"
echo "=== session done"
