#!/bin/bash
# Round-4 check of the tree on the MI355X box: GPU tests, smoke, the other
# BASELINE configs' bench lines.  Outputs under gpurun_out/r04/<tag>/.
#   bash scripts/gpu_r04.sh <tag> [tests] [smoke] [benches]
set -u
cd "${GRAFT_REPO_ROOT:-.}"
tag=$1; shift
out=gpurun_out/r04/$tag
mkdir -p "$out"
want() { [ -z "$ALL" ] || [[ " $ALL " == *" $1 "* ]]; }
ALL="$*"
run() {  # run <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(grep -h '^{' "$out/$name.log" | head -c 160)"
    if [ $rc -ne 0 ]; then tail -15 "$out/$name.log"; exit $rc; fi
}
want tests && run tests 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider
want smoke && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
if want benches; then
    run bench_cfg3 300 python bench.py --config cfg3 --cpu-baseline-seconds 0
    run bench_cfg4 300 python bench.py --config cfg4 --cpu-baseline-seconds 0
    run bench_cfg5 300 python bench.py --config cfg5 --cpu-baseline-seconds 0
    run bench_cfg5gol 300 python bench.py --config cfg5 --grad-on-light --cpu-baseline-seconds 0
    run bench_eval 300 python bench.py --config eval --cpu-baseline-seconds 0
fi
echo done
