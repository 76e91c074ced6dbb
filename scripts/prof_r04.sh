#!/bin/bash
# Round-4 profiles over bench.py's own cfg2 training step (run on the MI355X
# box; outputs under gpurun_out/r04/<tag>/, copied to profiles/r04/ afterwards).
#   scripts/prof_r04.sh <tag> [bench] [stats] [sq] [traffic]
#   bench   : the default bench line (rank 0 JSON) -> bench.json
#   stats   : rocprofv3 --kernel-trace --stats of a short bench run
#   sq      : two SQ counter passes (issue / stall / MFMA / LDS / VMEM counts)
#   traffic : FETCH_SIZE and WRITE_SIZE passes (separate runs)
# Every pass is its own rocprofv3 run with --kernel-trace only besides --pmc.
# The bench runs cover the f16x3 kernels (main region) and the exact-fp32
# kernels (the fp32 leg) in one process.  Extra bench flags: $BENCH_ARGS.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
tag=$1; shift
out=gpurun_out/r04/$tag
mkdir -p "$out"
export TMPDIR=/tmp
want() { [ $# -eq 0 ] || [[ " $ALL " == *" $1 "* ]]; }
ALL="$*"
run() {  # run <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -8 "$out/$name.log"; exit $rc; fi
}
B="bench.py --steps 3 --warmup 2 --fp32-leg-steps 3 --cpu-baseline-seconds 0 --no-kernel-timing ${BENCH_ARGS:-}"
if want bench; then
    run bench 300 python bench.py ${BENCH_ARGS:-}
    grep '^{' "$out/bench.log" > "$out/bench.json"
fi
if want stats; then
    run stats 300 rocprofv3 --kernel-trace --stats -d "$out/stats" -o run --output-format csv -- \
        python bench.py --steps 10 --warmup 3 --cpu-baseline-seconds 0 --no-kernel-timing ${BENCH_ARGS:-}
fi
if want sq; then
    run sq_a 180 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
        SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU \
        GRBM_GUI_ACTIVE -d "$out/sq_a" -o run --output-format csv -- python $B
    run sq_b 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
        SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
        -d "$out/sq_b" -o run --output-format csv -- python $B
fi
if want traffic; then
    run fetch 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$out/fetch" -o run --output-format csv -- python $B
    run write 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$out/write" -o run --output-format csv -- python $B
fi
echo done
