# scratch GPU command (gpurun): full check of the tree + profiles of the
# zero-gradient-sample backward
set -o pipefail
mkdir -p gpurun_out/pmcb
B="python bench.py --steps 3 --warmup 2 --cpu-baseline-seconds 0 --fp32-leg-steps 0 --no-kernel-timing"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config cfg5 --grad-on-light --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/bench_cfg5gol.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-baseline-seconds 0 --no-kernel-timing > gpurun_out/prof.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmcb/fetch -o run --output-format csv -- $B > gpurun_out/pmcb/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmcb/write -o run --output-format csv -- $B > gpurun_out/pmcb/write.log 2>&1
