#!/usr/bin/env bash
# A/B of the worklist threshold (PSIM_WL_THR; default ng/8 = 78125 groups' worth of messages at 10M)
set -u
mkdir -p gpurun_out
line() { python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],round(d['ms_per_step'],3),round(d['roofline']['avg_launch_us'],1),round(d['roofline']['frac'],4))" "$@"; }
for t in default 312500 625000 2499999 default 312500 625000 2499999; do
  if [ "$t" = default ]; then unset PSIM_WL_THR; else export PSIM_WL_THR=$t; fi
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit $?
  line gpurun_out/ab.log "thr_$t"
done
