#!/usr/bin/env bash
set -u
mkdir -p gpurun_out
line() { python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],round(d['ms_per_step'],3),round(d['roofline']['avg_launch_us'],1),round(d['roofline']['frac'],4))" "$@"; }
for v in ${VARIANTS:-prev:x cur:x prev:x cur:x cur:--csr}; do
  lib=${v%%:*}; f=${v#*:}; [ "$f" = x ] && f=""
  PSIM_LIB_PATH=$PWD/tools/ab/libpsim_$lib.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $f > gpurun_out/ab.log 2>&1 || exit $?
  line gpurun_out/ab.log "$lib$f"
done
