#!/bin/bash
# Four lanes of scripts/psnr_r03.sh side by side on the one GPU (each run is a
# small 1024-ray training loop that leaves the GPU mostly idle), one impl after
# another:  bash scripts/psnr_parallel.sh <out-dir> <first-seed> <last-seed> <impl>...
set -u
out=$1; first=$2; last=$3; shift 3
mkdir -p "$out"
export OMP_NUM_THREADS=4
for impl in "$@"; do
  pids=()
  for lane in 0 1 2 3; do
    seeds=$(seq $((first + lane)) 4 "$last")
    [ -z "$seeds" ] && continue
    bash scripts/psnr_r03.sh "$out" "$impl" $seeds > "$out/lane_${impl}_$lane.log" 2>&1 &
    pids+=($!)
  done
  rc=0
  for p in "${pids[@]}"; do wait "$p" || rc=$?; done
  echo "$impl done rc=$rc"
  cat "$out"/lane_"$impl"_*.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
