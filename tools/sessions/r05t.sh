#!/usr/bin/env bash
# Round-5 (session 10): with list-mode rounds on 256 workgroups, the list
# threshold (PSIM_WL_THR; default ng / 8 = 78,125 at 10M) raised so that
# round 8 (81,785 words read) also reads a list: per-round tables.
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
echo "=== session 10"

B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --sustain-s 1"
for rep in 1 2; do
for g in 78125 160000 320000; do
  PSIM_WL_THR=$g step t_${g}_$rep 200 $B
done
done
python3 - <<'PY'
import json, glob
rows = {}
for f in sorted(glob.glob("gpurun_out/t_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f, round(d["ms_per_step"], 4), round(d["sustained"]["ms_per_step"], 4))
            rows[f] = [r["us"] for r in d["roofline"]["per_round"]]
for f, r in rows.items():
    print(f.split("/")[-1], " ".join("%6.1f" % x for x in r))
PY
echo "=== session done"
