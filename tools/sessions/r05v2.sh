#!/usr/bin/env bash
# Round-5 final session (session 3): list-mode workgroup cap A/B on this
# build (PSIM_WL_WGS=0 = the whole grid vs the default 256), then the whole
# GPU suite and smoke, PMC FETCH / WRITE keyed to its sha256, the bench with
# CPU baselines and traffic, rocprof kernel stats of the bench, the config
# lines, and a world-2 launch rehearsal.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # name seconds cmd...  (stops the session on a GPU fault, abort, kill or timeout)
    local name=$1 secs=$2; shift 2
    echo "=== $name" ; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400
    if grep -qiE "illegal memory|memory access fault|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "gpurun_out/$name.log"; then
        echo "=== GPU fault in $name: stopping"; exit 3
    fi
    [ $rc -le 1 ] || exit $rc
}
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --sustain-s 1"
for rep in 1 2 3; do
  step ab_new_$rep 200 $B
  PSIM_WL_WGS=0 step ab_old_$rep 200 $B
done
python3 - <<'PY'
import json, glob
rows = {}
for f in sorted(glob.glob("gpurun_out/ab_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f, round(d["ms_per_step"], 4), round(d["sustained"]["ms_per_step"], 4))
            rows[f] = [r["us"] for r in d["roofline"]["per_round"]]
for f, r in rows.items():
    print(f.split("/")[-1], " ".join("%6.1f" % x for x in r))
PY
step gpu_suite 1500 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider
grep -q " passed" gpurun_out/gpu_suite.log && ! grep -q "failed" gpurun_out/gpu_suite.log || { echo "=== suite not green: stopping"; exit 4; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --sustain-s 0
step pmc_write 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --sustain-s 0
python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --n 10000000 --peers 5 --rounds-per-step 16 --steps 4 --source profiles/r05 --out gpurun_out/pmc_traffic.json > gpurun_out/pmc_traffic.log 2>&1 || exit 5
step bench 600 python bench.py --steps 20 --warmup 5 --traffic-json gpurun_out/pmc_traffic.json
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --sustain-s 0
step configs 700 python tools/config_bench.py C2 C3 C4 C5 RELAY C2ALL
step tr_w2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --transport gloo --all-on-device0 --no-cpu-baseline --sustain-s 1
echo "=== session done"
