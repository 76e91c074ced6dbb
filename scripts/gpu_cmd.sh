# scratch GPU command (gpurun): same-box A/B of the saved-activation layouts
set -o pipefail
mkdir -p gpurun_out/ab
B="python bench.py --steps 10 --warmup 3 --cpu-baseline-seconds 0 --fp32-leg-steps 0"
for r in 1 2; do
for v in n16 rows rowplain; do
  case $v in n16) L=dev/ab/libnerf_pl_amd_n16.so ;; rows) L=nerf_pl_amd/libnerf_pl_amd.so ;; rowplain) L=dev/ab/libnerf_pl_amd_rowplain.so ;; esac
  NERF_PL_AMD_LIB=$L timeout -k 10 200 $B > gpurun_out/ab/cfg2_${v}_$r.log 2>&1 || exit $?
  if [ $r = 1 ]; then NERF_PL_AMD_LIB=$L timeout -k 10 200 $B --config cfg5 --grad-on-light > gpurun_out/ab/cfg5gol_${v}.log 2>&1 || exit $?; fi
done
done
