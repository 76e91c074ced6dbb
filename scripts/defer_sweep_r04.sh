#!/bin/bash
# Deferred-save crossover: the training step with every forward deferring
# (all) vs saving (none) on weights after 100 / 300 / 1000 / 2000 training
# steps (scripts/psnr_compare.py --save-weights), dev/trained_step.py.
# Outputs under gpurun_out/r04/defer_sweep/.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r04/defer_sweep
mkdir -p "$out"
for st in 100 300 1000 2000; do
    timeout -k 10 200 python scripts/psnr_compare.py --impl ours --steps $st --eval-every $st --draw-seed 7 \
        --save-weights "$out/w_$st.safetensors" --out "$out/train_$st.json" > "$out/train_$st.log" 2>&1 || exit $?
    timeout -k 10 200 python dev/trained_step.py "$out/w_$st.safetensors" --steps 40 --modes all,none,auto \
        --out "$out/step_$st.json" > "$out/step_$st.log" 2>&1 || exit $?
    echo "== $st"; cat "$out/step_$st.log"
done
