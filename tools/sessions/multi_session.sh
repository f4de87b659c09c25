#!/usr/bin/env bash
# GPU box: the driver's multi-GPU bench command shape rehearsed on ONE GPU --
# torchrun world 2 with the gloo transport, both ranks on device 0 (RCCL
# refuses two ranks on one device), and world 1 under torchrun with nccl.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local n=$1 s=$2; shift 2; echo "=== $n"; timeout -k 10 "$s" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; tail -2 "gpurun_out/$n.log" | cut -c1-600; [ $rc -eq 0 ] || { echo "=== $n rc=$rc"; exit $rc; }; }
step tr_w1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline
step tr_w2_gloo 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 2 --steps 3 --warmup 1 --transport gloo --all-on-device0 --no-cpu-baseline
step tr_w2_gloo_csr 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29515 bench.py --gpus 2 --steps 3 --warmup 1 --transport gloo --all-on-device0 --no-cpu-baseline --csr
echo "=== session done"
