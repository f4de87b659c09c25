#!/usr/bin/env bash
# Round-5 (session 4): A/B of the round kernel: flag-mode chunks load the
# next chunk's group flags during their own work (new) vs at the chunk's start
# (old = exp_head.so): Plumtree lockstep parity, bench A/B, per-round SQ
# counters.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # name seconds cmd...  (stops the session on a GPU fault, abort, kill or timeout)
    local name=$1 secs=$2; shift 2
    echo "=== $name" ; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300
    if grep -qiE "illegal memory|memory access fault|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "gpurun_out/$name.log"; then
        echo "=== GPU fault in $name: stopping"; exit 3
    fi
    [ $rc -le 1 ] || exit $rc
}
OLD=$PWD/partisan_amd/exp_head.so
step parity 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_plumtree_gpu.py tests/test_worklist_parity.py tests/test_golden_traces.py tests/test_run_n.py
grep -q " passed" gpurun_out/parity.log && ! grep -q "failed" gpurun_out/parity.log || { echo "=== parity not green: stopping"; exit 4; }
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --sustain-s 2"
for rep in 1 2 3; do
  step z_new_$rep 200 $B
  PSIM_LIB_PATH=$OLD step z_old_$rep 200 $B
done
SQ="SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES"
step pmc_new 180 rocprofv3 --pmc $SQ --kernel-include-regex pt_round_ell -d gpurun_out/pmcz_new -o run --output-format csv -- python3 tools/round_profile.py --steps 1
PSIM_LIB_PATH=$OLD step pmc_old 180 rocprofv3 --pmc $SQ --kernel-include-regex pt_round_ell -d gpurun_out/pmcz_old -o run --output-format csv -- python3 tools/round_profile.py --steps 1
for x in new old; do echo "== $x"; python3 tools/pmc_rounds.py pt_round_ell "$(find gpurun_out/pmcz_$x -name '*counter_collection.csv' | head -1)"; done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/z_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); rf = d["roofline"]
            print(f, round(d["ms_per_step"], 4), round(d["sustained"]["ms_per_step"], 4), "kernel/step", round(rf["avg_launch_us"] * 16 / 1e3, 4))
PY
echo "=== session done"
