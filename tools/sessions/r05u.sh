#!/usr/bin/env bash
# Round-5 (session 2): where the pipelined intervals' ~1 us per round goes --
# head (guard test in every round kernel, read-back on a copy stream) vs
# exp_nospec.so (no guard test in the round kernels: timing only) vs
# exp_nocs.so (read-back on the rounds' stream); bench.py, same box, alternated.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --sustain-s 2"
for rep in 1 2; do
  step u_head_$rep 200 $B
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_nospec.so step u_nospec_$rep 200 $B
  PSIM_LIB_PATH=$PWD/partisan_amd/exp_nocs.so step u_nocs_$rep 200 $B
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/u_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); rf = d["roofline"]
            print(f, round(d["ms_per_step"], 4), round(d["sustained"]["ms_per_step"], 4), "kernel/step", round(rf["avg_launch_us"] * 16 / 1e3, 4))
PY
