#!/usr/bin/env bash
# A/B session on the GPU box: parity tests of the Plumtree engines, then
# bench variants (each line: variant ms/step avg_launch_us frac), then a
# rocprof kernel trace of the default.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_plumtree_gpu.py tests/test_golden_traces.py tests/test_shard.py tests/test_configs_at_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_tests.log 2>&1; rc=$?
tail -3 gpurun_out/pt_tests.log
[ $rc -le 1 ] || exit $rc
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],round(d['ms_per_step'],3),round(d['roofline']['avg_launch_us'],1),round(d['roofline']['frac'],4))" "$@"; }
for v in "ell:" "csr:--csr" "ell2:" "csr2:--csr"; do
  name=${v%%:*}; flags=${v#*:}
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $flags > gpurun_out/bench_$name.log 2>&1 || exit $?
  line gpurun_out/bench_$name.log $name
done
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit $?
echo done
