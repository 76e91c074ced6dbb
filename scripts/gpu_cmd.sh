set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_bf16.log 2>&1 || { tail -30 gpurun_out/t_bf16.log; exit 1; }
: > gpurun_out/wg.log
for m in bf16 f16x3; do
  timeout -k 10 100 python dev/time_wgrad.py $m >> gpurun_out/wg.log 2>&1 || exit 1
done
for t in 12 13; do
    NR_WGRAD_TASKMASK=$((1<<t)) timeout -k 10 100 python dev/time_wgrad.py bf16 >> gpurun_out/wg.log 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --math bf16 --steps 20 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/bench_bf16.json 2> gpurun_out/bench_bf16.err || exit 2
