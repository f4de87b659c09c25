#!/usr/bin/env bash
# Round-5 (session 2): psim_plumtree_broadcast_run_n (pipelined intervals inside the
# library) vs the loop; bench with the timed steps in one call (new) vs the
# head's bench.py loop (bench_old.py), same library; a trace of the steps.
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
step runn 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_run_n.py tests/test_plumtree_gpu.py tests/test_worklist_parity.py tests/test_forest.py tests/test_shard.py tests/test_golden_traces.py
grep -q " passed" gpurun_out/runn.log && ! grep -q "failed" gpurun_out/runn.log || { echo "=== parity not green: stopping"; exit 4; }
for rep in 1 2 3; do
  step b_new_$rep 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --sustain-s 2
  step b_old_$rep 200 python bench_old.py --steps 20 --warmup 5 --no-cpu-baseline --sustain-s 2
done
step trace 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/trace_t -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --sustain-s 0
python3 tools/trace_gaps.py "$(dirname $(find gpurun_out/trace_t -name 'run_kernel_trace.csv' | head -1))" > gpurun_out/trace_t_gaps.txt 2>&1
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/b_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); print(f, round(d["ms_per_step"], 4), round(d["sustained"]["ms_per_step"], 4), d["config"]["verified_after_timing"])
PY
grep -E "between" gpurun_out/trace_t_gaps.txt | head -8
echo "=== session done"
