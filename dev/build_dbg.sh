#!/bin/bash
# timing-experiment variants of the bf16x6 forward (x3.h NR_X3_DBG); dev only
set -e
for v in 0 1 2 3; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 -DNR_X3_DBG=$v \
    -shared -o dev/libx3dbg$v.so nerf_pl_amd/csrc/mlp_fwd3.hip nerf_pl_amd/csrc/mlp_bwd3.hip nerf_pl_amd/csrc/errors.hip &
done
wait
