#!/bin/bash
# PSNR runs of one impl over explicit seed lists, one process per list, all on
# one GPU (scripts/psnr_par.sh runs paired ranges; this fills in the seeds one
# group is missing):
#   bash scripts/psnr_list.sh <impl> <deadline-s> <seeds,...> [<seeds,...> ...]
# impl: f16x3 | fp32 | bf16 | oracle.  JSONs: gpurun_out/psnr/<impl>_s<seed>.json.
set -u
impl=$1; deadline=$2; shift 2
mkdir -p gpurun_out/psnr
if [ "$impl" = oracle ]; then args=(--impl oracle); envm=(); else args=(--impl ours); envm=(NERF_PL_AMD_MATH=$impl); fi
pids=(); p=0
for list in "$@"; do
  p=$((p + 1))
  env "${envm[@]}" timeout -k 10 $((deadline + 300)) python scripts/psnr_compare.py "${args[@]}" \
    --steps 2000 --eval-every 500 --threads 1 --draw-seeds "$list" --deadline-s "$deadline" \
    --out-dir gpurun_out/psnr > "gpurun_out/psnr/${impl}_list$p.log" 2>&1 &
  pids+=($!)
done
rc=0
for pid in "${pids[@]}"; do wait "$pid" || rc=$?; done
echo "runs: $(ls gpurun_out/psnr/${impl}_s*.json 2>/dev/null | wc -l) rc=$rc"
exit $rc
