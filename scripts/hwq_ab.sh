# RCCL one-rank vs standalone bench lines with HIP's default 4 hardware queues
# per process and with 8 (the backward chains and the pipelined step need their
# streams on distinct queues; RCCL's streams take queues too) -- DESIGN.md 15
set -u
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r06/hwqab; mkdir -p $out
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
val() { grep -h '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); m=j["mlp_stage"]; print(j["value"], "union", m["ms_per_step"], "sum", m["launch_ms_sum_per_step"])'; }
for i in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q NR_BENCH_FORCE_DIST=1 timeout -k 10 200 $TR --nproc-per-node 1 --master-port $((29710+i*10+q)) bench.py --cpu-baseline-seconds 0 --fp32-leg-steps 0 > $out/rccl_q${q}_$i.log 2>&1 || exit 1
    echo "rccl q$q $i $(val $out/rccl_q${q}_$i.log)"
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --fp32-leg-steps 0 > $out/solo_q${q}_$i.log 2>&1 || exit 1
    echo "solo q$q $i $(val $out/solo_q${q}_$i.log)"
  done
done
