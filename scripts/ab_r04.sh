#!/bin/bash
# A/B of library variants on the MI355X box (round 4): for each ablibs/ variant
# (and the shipped library), a parity check, a short bench line and one
# WRITE_SIZE / FETCH_SIZE pass over the bench step.
#   bash scripts/ab_r04.sh <tag> <variant>...     (variant "base" = nerf_pl_amd/libnerf_pl_amd.so)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
tag=$1; shift
out=gpurun_out/r04/ab_$tag
mkdir -p "$out"
export TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -8 "$out/$name.log"; exit $rc; fi
}
B="bench.py --steps 3 --warmup 2 --fp32-leg-steps 0 --cpu-baseline-seconds 0 --no-kernel-timing"
for v in "$@"; do
    if [ "$v" = base ]; then unset NERF_PL_AMD_LIB; else export NERF_PL_AMD_LIB=$PWD/ablibs/libnerf_pl_amd_$v.so; fi
    run "test_$v" 300 python -m pytest tests/test_gpu_active.py::test_active_backward_in_render_rays \
        "tests/test_gpu_render.py" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
    run "bench_$v" 200 python bench.py --steps 20 --warmup 5 --fp32-leg-steps 0 --cpu-baseline-seconds 0
    run "write_$v" 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$out/write_$v" -o run --output-format csv -- python $B
    run "fetch_$v" 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$out/fetch_$v" -o run --output-format csv -- python $B
done
unset NERF_PL_AMD_LIB
echo done
