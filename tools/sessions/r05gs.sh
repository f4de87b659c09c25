#!/usr/bin/env bash
# Round-5 (session 6): the bench round kernel's grid below the resident one
# (PSIM_ELL_GRID: 1280 = 5 workgroups per CU, the default; 1024, 768, 512):
# the bench's per-round table for each, to see which rounds (if any) gain
# from fewer chunks in flight.
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
PSIM_ELL_GRID=300 step parity 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_run_n.py tests/test_worklist_parity.py
grep -q " passed" gpurun_out/parity.log && ! grep -q "failed" gpurun_out/parity.log || { echo "=== parity not green: stopping"; exit 4; }
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --sustain-s 1"
for g in 1280 1024 768 512; do
  PSIM_ELL_GRID=$g step g_$g 200 $B
done
step g_def 200 $B
python3 - <<'PY'
import json, glob
rows = {}
for f in sorted(glob.glob("gpurun_out/g_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f, round(d["ms_per_step"], 4), round(d["sustained"]["ms_per_step"], 4))
            rows[f] = [r["us"] for r in d["roofline"]["per_round"]]
for f, r in rows.items():
    print(f.split("/")[-1], " ".join("%6.1f" % x for x in r))
PY
echo "=== session done"
