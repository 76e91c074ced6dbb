set -o pipefail
mkdir -p gpurun_out
export NR_BENCH_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/dist2.json 2> gpurun_out/dist2.err || { tail -20 gpurun_out/dist2.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --scaling strong > gpurun_out/dist2s.json 2> gpurun_out/dist2s.err || { tail -20 gpurun_out/dist2s.err; exit 2; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 3 --warmup 1 --config cfg5 > gpurun_out/dist2c5.json 2> gpurun_out/dist2c5.err || { tail -20 gpurun_out/dist2c5.err; exit 3; }
cat gpurun_out/dist2.json gpurun_out/dist2s.json gpurun_out/dist2c5.json | cut -c1-300
