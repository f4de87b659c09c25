set -u
mkdir -p gpurun_out
true
echo "tests rc=$?"; tail -5 gpurun_out/shard_tests.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --transport gloo --all-on-device0 --num-peers 2000000 > gpurun_out/bench_shard2.log 2>&1
echo "bench2 rc=$?"; tail -3 gpurun_out/bench_shard2.log | cut -c1-1500
