#!/bin/bash
# wgrad3 timing-experiment variants (NR_W3_DBG); dev only
set -e
for v in 0 1 2 3; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 -DNR_W3_DBG=$v \
    -shared -o dev/libw3dbg$v.so nerf_pl_amd/csrc/wgrad.hip nerf_pl_amd/csrc/errors.hip &
done
wait
