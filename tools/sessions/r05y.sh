#!/usr/bin/env bash
# Round-5 (session 3): a pipelined interval's leading rounds as one burst
# launch (pt_burst_ell_kernel) -- parity of run_n against the per-round loop,
# bench A/B on the same library (PSIM_BURST_WORDS=0 = one launch per round),
# rocprof kernel stats of the burst build.
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
step parity 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_run_n.py
PSIM_BURST_GRID=1 PSIM_BURST_WORDS=100000 step parity1 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_run_n.py
grep -q " passed" gpurun_out/parity.log && ! grep -q "failed" gpurun_out/parity.log || { echo "=== parity not green: stopping"; exit 4; }
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --sustain-s 2"
for rep in 1 2; do
  PSIM_BURST_WORDS=0 step y_old_$rep 200 $B
  PSIM_BURST_GRID=1 PSIM_BURST_WORDS=100 step y_g1w100_$rep 200 $B
  PSIM_BURST_GRID=1 PSIM_BURST_WORDS=400 step y_g1w400_$rep 200 $B
  PSIM_BURST_GRID=1 PSIM_BURST_WORDS=1500 step y_g1w1500_$rep 200 $B
done
PSIM_BURST_GRID=1 PSIM_BURST_WORDS=400 step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_y1 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --sustain-s 0
find gpurun_out/prof_y1 -name '*kernel_stats.csv' -exec cat {} \;
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/y_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f, round(d["ms_per_step"], 4), round(d["sustained"]["ms_per_step"], 4), d.get("parity_10m", {}).get("ok") if isinstance(d.get("parity_10m"), dict) else d.get("parity_10m"))
PY
echo "=== session done"
