set -u
mkdir -p gpurun_out/r04/distdbg
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
export NR_BENCH_DIST_BACKEND=gloo NR_BENCH_WATCHDOG=30
timeout -k 10 100 $TR --nproc-per-node 2 --master-port 29631 bench.py --gpus 2 --config cfg4 --steps 3 --warmup 1 --fp32-leg-steps 0 > gpurun_out/r04/distdbg/cfg4_gloo2.json 2> gpurun_out/r04/distdbg/cfg4_gloo2.log
echo "cfg4_gloo2 rc=$?"
timeout -k 10 100 $TR --nproc-per-node 4 --master-port 29632 bench.py --gpus 4 --steps 3 --warmup 1 --fp32-leg-steps 0 > gpurun_out/r04/distdbg/cfg2_gloo4.json 2> gpurun_out/r04/distdbg/cfg2_gloo4.log
echo "cfg2_gloo4 rc=$?"
timeout -k 10 100 $TR --nproc-per-node 4 --master-port 29633 bench.py --gpus 4 --config cfg4 --steps 3 --warmup 1 --fp32-leg-steps 0 > gpurun_out/r04/distdbg/cfg4_gloo4.json 2> gpurun_out/r04/distdbg/cfg4_gloo4.log
echo "cfg4_gloo4 rc=$?"
