#!/bin/bash
# Paired PSNR seeds in parallel on one GPU (the 1,024-ray training step is
# launch-bound, so several processes share the card):
#   bash scripts/psnr_par.sh <first-seed> <seeds-per-proc> <procs-per-impl> <deadline-s> <impl>...
# impl: f16x3 | fp32 | bf16 (this package) or oracle (the reference's algorithm in
# PyTorch fp32 on the GPU).  Process p of every impl runs the same seed range, so
# the groups stay paired whatever the deadline cuts.  JSONs: gpurun_out/psnr/.
set -u
first=$1; per=$2; procs=$3; deadline=$4; shift 4
mkdir -p gpurun_out/psnr
pids=()
for impl in "$@"; do
  for ((p = 0; p < procs; p++)); do
    lo=$((first + p * per)); hi=$((lo + per - 1))
    if [ "$impl" = oracle ]; then
      args=(--impl oracle); envm=()
    else
      args=(--impl ours); envm=(NERF_PL_AMD_MATH=$impl)
    fi
    env "${envm[@]}" timeout -k 10 $((deadline + 240)) python scripts/psnr_compare.py "${args[@]}" \
      --steps 2000 --eval-every 500 --threads 1 --draw-seeds "$lo-$hi" --deadline-s "$deadline" \
      --out-dir gpurun_out/psnr > "gpurun_out/psnr/${impl}_$lo-$hi.log" 2>&1 &
    pids+=($!)
  done
done
rc=0
for pid in "${pids[@]}"; do wait "$pid" || rc=$?; done
echo "runs: $(ls gpurun_out/psnr/*_s*.json 2>/dev/null | wc -l) rc=$rc"
exit $rc
