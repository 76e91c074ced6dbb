set -u
cd "${GRAFT_REPO_ROOT:-.}"
echo "box env GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
out=gpurun_out/r06/qcheck; mkdir -p $out
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
NR_BENCH_FORCE_DIST=1 timeout -k 10 300 $TR --nproc-per-node 1 --master-port 29791 bench.py --cpu-baseline-seconds 0 > $out/cfg2_rccl1.log 2>&1 || exit 1
grep -h '^{' $out/cfg2_rccl1.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); m=j["mlp_stage"]; print("rccl1", j["value"], m["ms_per_step"], m["launch_ms_sum_per_step"])'
