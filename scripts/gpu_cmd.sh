set -o pipefail
for v in mb_w8 mb_w8_dma0 mb_w8_dma2; do echo "== $v"; timeout -k 5 120 ./dev/$v 20; done > gpurun_out/w8dma.log 2>&1
