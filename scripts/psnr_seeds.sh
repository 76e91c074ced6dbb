#!/bin/bash
# PSNR spread of this package over draw seeds + chaos controls + same-weights
# evaluation.  Run on the MI355X box:
#   bash scripts/psnr_seeds.sh gpurun_out/psnr
# then, here, the reference on the saved weights:
#   python scripts/psnr_compare.py --impl reference --eval-weights <dir>/w_s7.safetensors ...
set -eu
out=${1:-gpurun_out/psnr}
mkdir -p "$out"
run() { timeout -k 10 120 python scripts/psnr_compare.py --impl ours --steps 2000 --eval-every 500 "$@"; }
run --draw-seed 7 --save-weights "$out/w_s7.safetensors" --out "$out/ours_s7.json" > "$out/ours_s7.log" 2>&1
run --draw-seed 8 --save-weights "$out/w_s8.safetensors" --out "$out/ours_s8.json" > "$out/ours_s8.log" 2>&1
for s in 7 8; do
  run --draw-seed $s --perturb-ulp --out "$out/ours_s${s}_ulp.json" > "$out/ours_s${s}_ulp.log" 2>&1
  run --draw-seed 77 --eval-weights "$out/w_s$s.safetensors" --out "$out/eval_ours_w$s.json" > "$out/eval_ours_w$s.log" 2>&1
done
for s in $(seq 9 20); do
  run --draw-seed $s --out "$out/ours_s$s.json" > "$out/ours_s$s.log" 2>&1
done
echo done
