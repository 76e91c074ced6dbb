set -e
mkdir -p gpurun_out
for r in 1024 2048 3072 4096 6144 8192 16384; do
  NR_KB_RAYS=$r timeout -k 10 120 python scripts/kbench.py h3 10 >> gpurun_out/sweep.txt 2>&1
done
