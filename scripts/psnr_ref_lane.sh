#!/bin/bash
# One lane of reference CPU training runs (here only: imports /root/reference),
# 2000 steps each, PSNR every 500.  Two lanes run side by side
# at low priority while the container is used for other work:
#   bash scripts/psnr_ref_lane.sh 3 11 13 15 &  bash scripts/psnr_ref_lane.sh 3 12 14 16 &
set -u
threads=$1; shift
out=profiles/r03/psnr
mkdir -p "$out"
for s in "$@"; do
  nice -n 15 python scripts/psnr_compare.py --impl reference --steps 2000 --eval-every 500 \
    --threads "$threads" --draw-seed "$s" --out "$out/reference_s$s.json" > "$out/reference_s$s.log" 2>&1
done
