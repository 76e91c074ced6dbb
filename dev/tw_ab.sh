set -e
mkdir -p gpurun_out
for r in 1365 4096; do
  NR_VAR_RAYS=$r timeout -k 10 200 python dev/time_h3var.py tw760,tw380,tw512,tw1024,tw760,tw380,tw512,tw1024 20 >> gpurun_out/tw.txt 2>&1
done
