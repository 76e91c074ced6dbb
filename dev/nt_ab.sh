set -e
mkdir -p gpurun_out
timeout -k 10 200 python dev/time_h3var.py nt,nont,nt,nont,nt,nont 20 > gpurun_out/nt_ab_h3.txt 2>&1
NR_VAR_MATH=bf16 timeout -k 10 200 python dev/time_h3var.py b1nt,b1nont,b1nt,b1nont,b1nt,b1nont 20 > gpurun_out/nt_ab_b1.txt 2>&1
