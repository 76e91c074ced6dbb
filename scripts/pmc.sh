#!/bin/bash
# PMC passes over the isolated kernels (each pass its own rocprofv3 run, no tracing
# domains besides the kernel trace).  Usage: scripts/pmc.sh <tag> [kernel]
set -u
tag=$1; k=${2:-all}
out=gpurun_out/pmc_$tag
mkdir -p $out
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" \
            "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
            "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TA_BUSY_avr"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d $out/p$i -o run --output-format csv -- python scripts/kbench.py $k ${REPS:-3} > $out/p$i.log 2>&1
    rc=$?
    echo "pass $i ($ctrs) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $out/p$i.log; fi
    if [ $rc -ge 124 ]; then exit $rc; fi
done
