# scratch GPU command (gpurun): same-box A/B of the saved-activation layouts,
# and the step on trained weights
set -o pipefail
mkdir -p gpurun_out/ab
B="python bench.py --steps 10 --warmup 3 --cpu-baseline-seconds 0 --fp32-leg-steps 0"
for v in n16 rows rowplain; do
  case $v in n16) L=dev/ab/libnerf_pl_amd_n16.so ;; rows) L=nerf_pl_amd/libnerf_pl_amd.so ;; rowplain) L=dev/ab/libnerf_pl_amd_rowplain.so ;; esac
  NERF_PL_AMD_LIB=$L timeout -k 10 200 $B > gpurun_out/ab/cfg2_${v}.log 2>&1 || exit $?
  NERF_PL_AMD_LIB=$L timeout -k 10 200 $B --config cfg5 --grad-on-light > gpurun_out/ab/cfg5gol_${v}.log 2>&1 || exit $?
done
timeout -k 10 150 python scripts/psnr_compare.py --impl ours --steps 2000 --eval-every 1000 --draw-seed 7 --save-weights gpurun_out/w7.safetensors --out gpurun_out/ab/train_s7.json > gpurun_out/ab/train.log 2>&1 || exit $?
timeout -k 10 200 python dev/trained_step.py gpurun_out/w7.safetensors --out gpurun_out/ab/trained_step.json > gpurun_out/ab/trained_step.log 2>&1
rc=$?; rm -f gpurun_out/w7.safetensors; exit $rc
