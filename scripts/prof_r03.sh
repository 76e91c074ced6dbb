#!/bin/bash
# Round-3 profiles (run on the MI355X box; outputs under gpurun_out/, copied to
# profiles/r03/ afterwards):
#   1. rocprofv3 --kernel-trace --stats of the default bench command (f16x3 cfg2
#      + its exact-fp32 leg) and of cfg5 --grad-on-light;
#   2. separate --pmc FETCH_SIZE and WRITE_SIZE passes over the isolated fused
#      MLP kernels at the cfg2 fine-pass size, f16x3 and fp32 (scripts/kbench.py)
#      -> scripts/traffic.py -> gpurun_out/traffic_r03.json
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name"
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
run stats_cfg2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stats_cfg2 -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 3 --cpu-baseline-seconds 0 --no-kernel-timing
run stats_cfg5gol 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stats_cfg5gol -o run --output-format csv -- \
    python bench.py --config cfg5 --grad-on-light --steps 5 --warmup 2 --cpu-baseline-seconds 0 --no-kernel-timing --fp32-leg-steps 0
for c in FETCH_SIZE WRITE_SIZE; do
    run pmc_h3_$c 120 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/pmc_h3/p_$c -o run --output-format csv -- \
        python scripts/kbench.py fwdh3save,bwdh3,wgradh3 3
    run pmc_f32_$c 180 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/pmc_f32/p_$c -o run --output-format csv -- \
        python scripts/kbench.py fwdsave,bwd,wgrad 3
done
python scripts/traffic.py gpurun_out/pmc_f32 gpurun_out/traffic_r03.json --fwd-save-only > gpurun_out/traffic_f32.log 2>&1
python scripts/traffic.py gpurun_out/pmc_h3 gpurun_out/traffic_r03.json --arith f16x3 --fwd-save-only > gpurun_out/traffic_h3.log 2>&1
echo done
