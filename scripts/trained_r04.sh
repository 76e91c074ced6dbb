#!/bin/bash
# Round-4 check of the adaptive deferred save on the MI355X box: its GPU tests,
# a 2000-step training run that saves its weights, the training step on those
# weights (dev/trained_step.py: auto / none / every-sample), the default bench
# line.  Outputs under gpurun_out/r04/trained/.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r04/trained
mkdir -p "$out"
run() {  # run <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -15 "$out/$name.log"; exit $rc; fi
}
run tests 600 python -u -m pytest tests/test_gpu_active.py tests/test_gpu_sigma_train.py tests/test_gpu_render.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider
run train 300 python scripts/psnr_compare.py --impl ours --steps 2000 --eval-every 500 --draw-seed 7 --save-weights "$out/w7.safetensors" --out "$out/train_s7.json"
run step 300 python dev/trained_step.py "$out/w7.safetensors" --steps 40 --out "$out/trained_step.json"
run bench 300 python bench.py --cpu-baseline-seconds 0
grep -h '^{' "$out/bench.log" | head -c 300; echo
cat "$out/trained_step.json"
