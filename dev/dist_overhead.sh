# same-box A/B: bench without and with the distributed path at one rank (RCCL)
set -e
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --cpu-baseline-seconds 0 --no-kernel-timing | tail -1 >> gpurun_out/dist_ab.jsonl
  NR_BENCH_FORCE_DIST=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2951$i bench.py --steps 30 --warmup 5 --cpu-baseline-seconds 0 --no-kernel-timing 2>/dev/null | tail -1 >> gpurun_out/dist_ab.jsonl
done
