#!/bin/bash
# PSNR over draw seeds on the MI355X box:
#   bash scripts/psnr_r03.sh <out-dir> <impl> <seed> [<seed> ...]
# impl: f16x3 | fp32 | bf16 (this package, NERF_PL_AMD_MATH) or oracle (the
# reference's algorithm in PyTorch fp32 on the GPU).  2000 steps, PSNR every 500.
set -u
out=$1; impl=$2; shift 2
mkdir -p "$out"
for s in "$@"; do
  if [ "$impl" = oracle ]; then
    timeout -k 10 600 python scripts/psnr_compare.py --impl oracle --steps 2000 --eval-every 500 \
      --draw-seed "$s" --out "$out/oracle_s$s.json" > "$out/oracle_s$s.log" 2>&1
  else
    NERF_PL_AMD_MATH=$impl timeout -k 10 300 python scripts/psnr_compare.py --impl ours --steps 2000 \
      --eval-every 500 --draw-seed "$s" --out "$out/${impl}_s$s.json" > "$out/${impl}_s$s.log" 2>&1
  fi
  rc=$?
  echo "$impl seed $s rc=$rc $(tail -n 1 $out/*_s$s.log | tail -c 200)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
