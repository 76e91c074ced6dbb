#!/bin/bash
# GPU check used with gpurun: tests, bench, then (optionally) rocprof.
# Stops at the first step that faults, aborts or times out (rc not in {0,1}).
set -u
mkdir -p gpurun_out
step() {  # step <name> <timeout-seconds> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name: $*" | tee -a gpurun_out/steps.log
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
n=0
for s in "$@"; do
    case $s in
        tests) step tests 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread ;;
        testsall) step testsall 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
        bench) step bench 600 python bench.py --steps 20 --warmup 5 ;;
        benchq) step benchq 300 python bench.py --steps 10 --warmup 3 --cpu-baseline-seconds 0 ;;
        prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-baseline-seconds 0 --no-kernel-timing ;;
        smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        *) n=$((n+1)); step custom$n 600 bash -c "$s" ;;
    esac
done
