#!/bin/bash
# wgrad3 schedule variants; dev only
set -e
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950"
S="nerf_pl_amd/csrc/wgrad.hip nerf_pl_amd/csrc/errors.hip"
/opt/rocm/bin/hipcc $F -DNR_W3_SGB=0 -DNR_W3_MULTI=0 -shared -o dev/libw3dbg0.so $S &
/opt/rocm/bin/hipcc $F -DNR_W3_SGB=1 -DNR_W3_MULTI=0 -shared -o dev/libw3dbg1.so $S &
/opt/rocm/bin/hipcc $F -DNR_W3_SGB=0 -DNR_W3_MULTI=1 -shared -o dev/libw3dbg2.so $S &
/opt/rocm/bin/hipcc $F -DNR_W3_SGB=1 -DNR_W3_MULTI=1 -shared -o dev/libw3dbg3.so $S &
wait
