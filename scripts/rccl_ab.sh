set -u
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r06/rcclab; mkdir -p $out
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for i in 1 2; do
  for v in pipe nopipe; do
    e=1; [ $v = nopipe ] && e=0
    NR_BENCH_PIPELINE=$e NR_BENCH_FORCE_DIST=1 timeout -k 10 200 $TR --nproc-per-node 1 --master-port $((29700+i)) bench.py --cpu-baseline-seconds 0 --fp32-leg-steps 0 > $out/rccl_${v}_$i.log 2>&1 || exit 1
    NR_BENCH_PIPELINE=$e timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --fp32-leg-steps 0 > $out/solo_${v}_$i.log 2>&1 || exit 1
    echo "$v $i rccl $(grep -h '^{' $out/rccl_${v}_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])') solo $(grep -h '^{' $out/solo_${v}_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
