#!/bin/bash
# Kernel traces of short bench runs (one per workload) for the idle-GPU gap
# analysis of scripts/gaps.py: bash scripts/gaps_r04.sh <tag> "<bench args>"...
set -u
cd "${GRAFT_REPO_ROOT:-.}"
tag=$1; shift
export TMPDIR=/tmp
i=0
for a in "$@"; do
    i=$((i + 1))
    out=gpurun_out/r04/gaps_$tag/$i
    mkdir -p "$out"
    echo "$a" > "$out/args.txt"
    timeout -k 10 240 rocprofv3 --kernel-trace -d "$out" -o run --output-format csv -- \
        python bench.py $a --steps 10 --warmup 3 --fp32-leg-steps 0 --cpu-baseline-seconds 0 \
        --no-kernel-timing > "$out/bench.log" 2>&1 || exit $?
    echo "$i rc=0 $a"
done
