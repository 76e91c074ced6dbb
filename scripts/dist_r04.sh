#!/bin/bash
# Multi-rank rehearsal on the one-GPU box (the driver's 8-GPU run uses RCCL):
# bench.py's distributed path with N gloo ranks sharing the GPU (RCCL refuses
# two ranks on one device), each rank printing a progress line per phase to
# stderr, plus the RCCL path at one rank.  The driver's command line exactly
# (default steps / warmup / exact-fp32 leg) unless a case says otherwise.
#   bash scripts/dist_r04.sh [case...]   cases: cfg4_gloo4 cfg2_gloo2 cfg5_gol_shard_gloo4 cfg2_rccl1
set -u
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r04/dist
mkdir -p "$out"
run() {  # run <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$to" "$@" > "$out/$name.json" 2> "$out/$name.log"
    local rc=$?
    echo "== $name rc=$rc $(tail -c 300 "$out/$name.json")"
    if [ $rc -ne 0 ]; then tail -20 "$out/$name.log"; exit $rc; fi
}
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
want() { [ -z "$ALL" ] || [[ " $ALL " == *" $1 "* ]]; }
ALL="$*"
want cfg4_gloo4 && NR_BENCH_DIST_BACKEND=gloo run cfg4_gloo4 500 $TR --nproc-per-node 4 --master-port 29621 \
    bench.py --gpus 4 --config cfg4
want cfg2_gloo2 && NR_BENCH_DIST_BACKEND=gloo run cfg2_gloo2 300 $TR --nproc-per-node 2 --master-port 29622 \
    bench.py --gpus 2
want cfg5_gol_shard_gloo4 && NR_BENCH_DIST_BACKEND=gloo run cfg5_gol_shard_gloo4 500 $TR --nproc-per-node 4 --master-port 29623 \
    bench.py --gpus 4 --config cfg5 --grad-on-light --light-shard --light-importance -1
want cfg2_rccl1 && NR_BENCH_FORCE_DIST=1 run cfg2_rccl1 300 $TR --nproc-per-node 1 --master-port 29624 \
    bench.py --cpu-baseline-seconds 0
echo done
