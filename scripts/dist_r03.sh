#!/bin/bash
# Multi-rank rehearsal on the one-GPU box (the driver's 8-GPU run uses RCCL):
# 2 gloo ranks sharing the GPU (RCCL refuses two ranks on one device) through
# bench.py's distributed path -- cfg2 with the DistributedSampler partition, and
# cfg5 --grad-on-light with the light image sharded (differentiable gather) and
# the Light_N_importance = -1 schedule -- plus the RCCL path at one rank.
set -u
mkdir -p gpurun_out/dist
run() {  # run <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/dist/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(grep '^{' gpurun_out/dist/$name.log | tail -c 300)"
    if [ $rc -ne 0 ]; then tail -20 "gpurun_out/dist/$name.log"; exit $rc; fi
}
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
want() { [ $# -eq 0 ] || [[ " $ALL " == *" $1 "* ]]; }
ALL="$*"
want cfg2_gloo2 && NR_BENCH_DIST_BACKEND=gloo run cfg2_gloo2 300 $TR --nproc-per-node 2 --master-port 29611 \
    bench.py --gpus 2 --steps 5 --warmup 2 --fp32-leg-steps 0
want cfg5_gol_shard_gloo2 && NR_BENCH_DIST_BACKEND=gloo run cfg5_gol_shard_gloo2 300 $TR --nproc-per-node 2 --master-port 29612 \
    bench.py --gpus 2 --config cfg5 --grad-on-light --light-shard --light-importance -1 --steps 5 --warmup 2 --fp32-leg-steps 0
want cfg2_rccl1 && NR_BENCH_FORCE_DIST=1 run cfg2_rccl1 300 $TR --nproc-per-node 1 --master-port 29613 \
    bench.py --steps 10 --warmup 3 --cpu-baseline-seconds 0 --fp32-leg-steps 0
# cfg4 (800^2, 4096 rays per rank) at 4 ranks sharing the GPU: the sampler's
# padded partition of the 64M-ray pool, the bucketed all-reduce, and the
# max-over-ranks timing at more than two ranks
want cfg4_gloo4 && NR_BENCH_DIST_BACKEND=gloo run cfg4_gloo4 400 $TR --nproc-per-node 4 --master-port 29614 \
    bench.py --gpus 4 --config cfg4 --steps 5 --warmup 2 --fp32-leg-steps 0
want cfg5_gol_shard_gloo4 && NR_BENCH_DIST_BACKEND=gloo run cfg5_gol_shard_gloo4 400 $TR --nproc-per-node 4 --master-port 29615 \
    bench.py --gpus 4 --config cfg5 --grad-on-light --light-shard --steps 5 --warmup 2 --fp32-leg-steps 0
echo done
