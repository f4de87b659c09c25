#!/usr/bin/env bash
# Runs on the GPU box (via gpurun) from the repo root.  Each GPU step has its
# own time limit; a crash / abort / timeout ends the session immediately,
# a plain test failure (exit 1) does not.
#   usage: tools/gpu_session.sh [steps...]   steps: build test t:<name> smoke bench prof pmc
set -u
mkdir -p gpurun_out
STEPS=${*:-"test smoke bench prof"}
export PYTHONUNBUFFERED=1

run() {  # name seconds cmd...
    local name=$1 secs=$2; shift 2
    echo "=== $name: $*" | tee -a gpurun_out/session.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
    tail -5 "gpurun_out/$name.log"
    case $rc in
        0|1) return 0 ;;
        *) echo "=== stopping: $name ended with $rc"; exit $rc ;;
    esac
}

for s in $STEPS; do
    case $s in
        build) run build 600 python -c "import __graft_entry__ as g; g.build()" ;;
        test)  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
        t:*)   f=${s#t:}; run "pytest_${f}" 900 python -u -m pytest "tests/test_${f}.py" -m gpu -x -q --timeout 300 --timeout-method thread ;;
        tv:*)  # tv:<test file>:<variant>: a test file against tools/ab/libpsim_<variant>.so
               x=${s#tv:}; f=${x%%:*}; v=${x#*:}
               PSIM_LIB_PATH=$PWD/tools/ab/libpsim_$v.so run "pytest_${f}_$v" 900 python -u -m pytest "tests/test_${f}.py" \
                   -m gpu -x -q --timeout 300 --timeout-method thread ;;
        te:*)  # te:<test file>:<ENV=VAL>: a test file with one environment setting
               x=${s#te:}; f=${x%%:*}; e=${x#*:}
               run "pytest_${f}_${e%%=*}" 900 env "$e" python -u -m pytest "tests/test_${f}.py" -m gpu -x -q \
                   --timeout 300 --timeout-method thread ;;
        ab)    run ab 1100 bash tools/ab/gs_ab.sh ;;
        proj)  run shard_projection 600 python tools/shard_projection.py --rccl-latency ;;
        c3prof)
            export TMPDIR=/tmp
            run c3prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/c3prof -o run --output-format csv \
                -- python3 tools/c3_wall.py 1000000 30 ;;
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run bench 600 python bench.py --steps 5 --warmup 2 ;;
        benchq) run benchq 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity ;;
        rprof) run round_profile 300 python tools/round_profile.py --steps 3 ;;
        frprof) PSIM_FRONTIER=1 PSIM_FR_PROFILE=1 run fr_profile 300 python tools/round_profile.py --steps 2 ;;
        prof)
            export TMPDIR=/tmp
            run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv \
                -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity ;;
        pmc)
            export TMPDIR=/tmp
            run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv \
                -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --sustain-s 0
            run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv \
                -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --sustain-s 0 ;;
        *) echo "unknown step $s" ;;
    esac
done
echo "=== session done"
