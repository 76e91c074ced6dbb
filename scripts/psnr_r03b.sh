#!/bin/bash
# More PSNR seeds in few processes (the scene is built once per process):
#   bash scripts/psnr_r03b.sh <impl> <lo-hi> [<timeout-s>]
# impl: f16x3 | fp32 | bf16 (this package) or oracle (the reference's algorithm
# in PyTorch fp32 on the GPU); JSONs to gpurun_out/psnr/<impl>_s<seed>.json.
set -u
impl=$1; seeds=$2; to=${3:-900}
mkdir -p gpurun_out/psnr
if [ "$impl" = oracle ]; then
  timeout -k 10 "$to" python scripts/psnr_compare.py --impl oracle --steps 2000 --eval-every 500 \
    --draw-seeds "$seeds" --out-dir gpurun_out/psnr > "gpurun_out/psnr/oracle_$seeds.log" 2>&1
else
  NERF_PL_AMD_MATH=$impl timeout -k 10 "$to" python scripts/psnr_compare.py --impl ours --steps 2000 \
    --eval-every 500 --draw-seeds "$seeds" --out-dir gpurun_out/psnr > "gpurun_out/psnr/${impl}_$seeds.log" 2>&1
fi
rc=$?
echo "$impl $seeds rc=$rc $(grep -c '"psnr"' gpurun_out/psnr/${impl}_$seeds.log) evals"
exit $rc
