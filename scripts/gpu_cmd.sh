set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_shadow_shard.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_shard.log 2>&1 || { tail -30 gpurun_out/t_shard.log; exit 1; }
export NR_BENCH_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 3 --warmup 1 --config cfg5 --light-shard > gpurun_out/dist2c5s.json 2> gpurun_out/dist2c5s.err || { tail -20 gpurun_out/dist2c5s.err; exit 3; }
cut -c1-400 gpurun_out/dist2c5s.json
