set -u
mkdir -p gpurun_out/r04/v2
timeout -k 10 400 python -u -m pytest tests/test_gpu_sigma_train.py tests/test_gpu_active.py tests/test_gpu_shadow.py tests/test_gpu_shadow_random.py tests/test_gpu_shadow_shard.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -s > gpurun_out/r04/v2/tests_defer.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && { tail -30 gpurun_out/r04/v2/tests_defer.log; exit $rc; }
for c in "cfg5" "cfg5 --grad-on-light"; do
  n=$(echo $c | tr -d ' -')
  timeout -k 10 200 python bench.py --config $c --cpu-baseline-seconds 0 > gpurun_out/r04/v2/bench_$n.log 2>&1
  rc=$?; echo "bench $n rc=$rc $(grep -h '^{' gpurun_out/r04/v2/bench_$n.log | head -c 200)"; [ $rc -ne 0 ] && exit $rc
done
bash scripts/distdbg_r04.sh
