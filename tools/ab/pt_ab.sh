#!/usr/bin/env bash
# A/B of Plumtree round-kernel variants (tools/ab/libpsim_*.so) on the 10M bench, then a
# rocprof trace of the default for per-round launch times.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
line() { python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],round(d['ms_per_step'],3),round(d['roofline']['avg_launch_us'],1),round(d['roofline']['frac'],4))" "$@"; }
for v in ${VARIANTS:-d4 d2 d8 d16 d4}; do
  PSIM_LIB_PATH=$PWD/tools/ab/libpsim_$v.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || exit $?
  line gpurun_out/ab_$v.log $v
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/trace.log 2>&1 || exit $?
echo done
