set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_plumtree_gpu.py tests/test_golden_traces.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_tests.log 2>&1; rc=$?
tail -3 gpurun_out/pt_tests.log
[ $rc -le 1 ] || exit $rc
for mode in never auto always; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --buckets $mode > gpurun_out/bench_$mode.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bench_$mode.log').read().strip().splitlines()[-1]);print('$mode',d['ms_per_step'],d['roofline']['avg_launch_us'],d['roofline']['frac'])"
done
for th in 1000000 5000000; do
  PSIM_BK_MIN_BCAST=$th timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_th$th.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bench_th$th.log').read().strip().splitlines()[-1]);print('th$th',d['ms_per_step'],d['roofline']['avg_launch_us'],d['roofline']['frac'])"
done
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit $?
echo done
