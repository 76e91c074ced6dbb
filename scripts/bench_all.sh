#!/bin/bash
# Every bench.py config on one GPU (dev/judging aid): scripts/bench_all.sh [steps] [cpu_seconds]
# Writes gpurun_out/bench_<config>.json; stops at the first failing config.
set -u
mkdir -p gpurun_out
steps=${1:-20}; cpu=${2:-12}
for c in cfg2 cfg3 cfg4 cfg5 cfg5gol eval; do
    args="--config $c"
    [ $c = cfg5gol ] && args="--config cfg5 --grad-on-light"
    timeout -k 10 300 python bench.py $args --steps $steps --warmup 5 \
        --cpu-baseline-seconds $cpu > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
    rc=$?
    echo "$c rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_$c.err; exit $rc; fi
done
