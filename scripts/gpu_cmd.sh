set -o pipefail
mkdir -p gpurun_out
for tag in h3 b1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/pmc_r02_$tag/$c -o run --output-format csv -- python scripts/kbench.py $tag 3 > gpurun_out/pmc_r02_${tag}_$c.log 2>&1 || { tail -5 gpurun_out/pmc_r02_${tag}_$c.log; exit 1; }
  done
done
python scripts/kbench.py h3 10 > gpurun_out/kbench_h3.log 2>&1 && python scripts/kbench.py b1 10 > gpurun_out/kbench_b1.log 2>&1
