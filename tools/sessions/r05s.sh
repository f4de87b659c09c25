#!/usr/bin/env bash
# Round-5 (session 2): bench.py with the per-step bookkeeping after the timed
# region (new) vs the head's bench.py (bench_old.py), same library; then a
# kernel + copy trace of a few steps for the time between steps.
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
for rep in 1 2 3; do
  step b_new_$rep 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --sustain-s 2
  step b_old_$rep 200 python bench_old.py --steps 20 --warmup 5 --no-cpu-baseline --sustain-s 2
done
step trace 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/trace_s -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --sustain-s 0
python3 tools/trace_gaps.py "$(dirname $(find gpurun_out/trace_s -name 'run_kernel_trace.csv' | head -1))" > gpurun_out/trace_s_gaps.txt 2>&1
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/b_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); print(f, round(d["ms_per_step"], 4), round(d["sustained"]["ms_per_step"], 4))
PY
grep -E "^step|between" gpurun_out/trace_s_gaps.txt | head -20
echo "=== session done"
