#!/bin/bash
# timing-experiment variants of the bf16x6 kernels (x3.h NR_X3_DBG, NR_X3_SGB); dev only
set -e
build() {  # build <suffix> <flags...>
  local suf=$1; shift
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 "$@" \
    -shared -o dev/libx3dbg$suf.so nerf_pl_amd/csrc/mlp_fwd3.hip nerf_pl_amd/csrc/mlp_bwd3.hip nerf_pl_amd/csrc/errors.hip
}
for v in 0 1 2 3 4 5 8; do build $v -DNR_X3_DBG=$v & done
build s0 -DNR_X3_SGB=0 &
build s2 -DNR_X3_SGB=2 &
wait
