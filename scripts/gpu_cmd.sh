# scratch GPU command (gpurun): check of the tree with the per-graph layouts
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config cfg5 --grad-on-light --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/bench_cfg5gol.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config cfg5 --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/bench_cfg5.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config cfg3 --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/bench_cfg3.log 2>&1
