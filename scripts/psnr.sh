#!/bin/bash
# PSNR against the reference (BASELINE north star: within 0.1 dB; DESIGN.md
# sections 2, 9, 10).  One driver for every leg of scripts/psnr_compare.py:
#
#   bash scripts/psnr.sh pairs <out> <first-seed> <seeds-per-proc> <procs> <deadline-s> <impl>...
#       on the MI355X box: paired seed ranges, <procs> processes per impl on one GPU
#       (the 1,024-ray step is launch-bound, so processes share the card); process p
#       of every impl runs the same seed range, so the groups stay paired whatever
#       the deadline cuts.  impl: f16x3 | fp32 | bf16 (this package) or oracle (the
#       reference's algorithm in PyTorch fp32 on the GPU).
#   bash scripts/psnr.sh list <out> <impl> <deadline-s> <seeds,...> [<seeds,...> ...]
#       on the box: explicit seed lists, one process per list (fills in a group).
#   bash scripts/psnr.sh reference <out> <threads> <seed>...
#       here only (imports /root/reference): the reference itself on the CPU, one
#       seed after another at low priority -- run two lanes side by side.
#   bash scripts/psnr.sh controls <out>
#       on the box: same-weights evaluation and one-ulp chaos controls.
#
# Every run: 2000 steps, PSNR of the fine rgb on the held-out views every 500;
# JSONs <out>/<impl>_s<seed>.json; summary: scripts/psnr_summary.py.
set -u
mode=$1; out=$2; shift 2
mkdir -p "$out"

impl_args() {   # impl -> psnr_compare.py arguments and environment
  if [ "$1" = oracle ]; then args=(--impl oracle); envm=(); else args=(--impl ours); envm=(NERF_PL_AMD_MATH=$1); fi
}

case "$mode" in
pairs)
  first=$1; per=$2; procs=$3; deadline=$4; shift 4
  pids=()
  for impl in "$@"; do
    impl_args "$impl"
    for ((p = 0; p < procs; p++)); do
      lo=$((first + p * per)); hi=$((lo + per - 1))
      env "${envm[@]}" timeout -k 10 $((deadline + 240)) python scripts/psnr_compare.py "${args[@]}" \
        --steps 2000 --eval-every 500 --threads 1 --draw-seeds "$lo-$hi" --deadline-s "$deadline" \
        --out-dir "$out" > "$out/${impl}_$lo-$hi.log" 2>&1 &
      pids+=($!)
    done
  done
  rc=0
  for pid in "${pids[@]}"; do wait "$pid" || rc=$?; done
  echo "runs: $(ls "$out"/*_s*.json 2>/dev/null | wc -l) rc=$rc"
  exit $rc ;;
list)
  impl=$1; deadline=$2; shift 2
  impl_args "$impl"
  pids=(); p=0
  for seeds in "$@"; do
    p=$((p + 1))
    env "${envm[@]}" timeout -k 10 $((deadline + 300)) python scripts/psnr_compare.py "${args[@]}" \
      --steps 2000 --eval-every 500 --threads 1 --draw-seeds "$seeds" --deadline-s "$deadline" \
      --out-dir "$out" > "$out/${impl}_list$p.log" 2>&1 &
    pids+=($!)
  done
  rc=0
  for pid in "${pids[@]}"; do wait "$pid" || rc=$?; done
  echo "runs: $(ls "$out"/"${impl}"_s*.json 2>/dev/null | wc -l) rc=$rc"
  exit $rc ;;
reference)
  threads=$1; shift
  for s in "$@"; do
    nice -n 15 python scripts/psnr_compare.py --impl reference --steps 2000 --eval-every 500 \
      --threads "$threads" --draw-seed "$s" --out "$out/reference_s$s.json" > "$out/reference_s$s.log" 2>&1
  done ;;
controls)
  run() { timeout -k 10 120 python scripts/psnr_compare.py --impl ours --steps 2000 --eval-every 500 "$@"; }
  set -e
  for s in 7 8; do
    run --draw-seed $s --save-weights "$out/w_s$s.safetensors" --out "$out/ours_s$s.json" > "$out/ours_s$s.log" 2>&1
    run --draw-seed $s --perturb-ulp --out "$out/ours_s${s}_ulp.json" > "$out/ours_s${s}_ulp.log" 2>&1
    run --draw-seed 77 --eval-weights "$out/w_s$s.safetensors" --out "$out/eval_ours_w$s.json" > "$out/eval_ours_w$s.log" 2>&1
  done
  echo "then, here: python scripts/psnr_compare.py --impl reference --eval-weights $out/w_s7.safetensors ..." ;;
*)
  echo "usage: scripts/psnr.sh pairs|list|reference|controls <out> ..." >&2; exit 2 ;;
esac
