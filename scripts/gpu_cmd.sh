set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_bf16.log 2>&1 || { tail -30 gpurun_out/t_bf16.log; exit 1; }
timeout -k 10 200 python bench.py --math bf16 --steps 20 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/bench_bf16.json 2> gpurun_out/bench_bf16.err || exit 2
for s in 7 8 9; do NERF_PL_AMD_MATH=bf16 timeout -k 10 120 python scripts/psnr_compare.py --impl ours --steps 2000 --draw-seed $s --out gpurun_out/psnr_ours_bf16_s$s.json > gpurun_out/psnr_bf16_s$s.log 2>&1 || exit 3; done
