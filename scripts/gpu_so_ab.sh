set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sigma_train.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -s > gpurun_out/so_test.log 2>&1
rc=$?; echo "so_test rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest tests/test_gpu_shadow.py tests/test_gpu_shadow_shard.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/shadow_test.log 2>&1
rc=$?; echo "shadow rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in 0 1; do
  NERF_PL_AMD_SIGMA_TRAIN=$v timeout -k 10 200 python bench.py --config cfg5 --grad-on-light --steps 10 --warmup 3 --cpu-baseline-seconds 0 --fp32-leg-steps 0 > gpurun_out/cfg5gol_so$v.log 2>&1
  rc=$?; echo "bench so=$v rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  NERF_PL_AMD_SIGMA_TRAIN=$v timeout -k 10 200 python bench.py --config cfg5 --steps 10 --warmup 3 --cpu-baseline-seconds 0 --fp32-leg-steps 0 > gpurun_out/cfg5_so$v.log 2>&1
  rc=$?; echo "bench cfg5 so=$v rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
