#!/bin/bash
# f16x3 timing-experiment variants (dev only): dev/h3var.sh <name> <flags...>
# builds dev/libh3_<name>.so (fwd3 + bwd3 + wgrad, NR_F16=1) for dev/time_h3var.py
set -e
name=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 \
  -DNR_F16=${NR_F16:-1} "$@" -shared -o dev/libh3_$name.so nerf_pl_amd/csrc/mlp_fwd3.hip \
  nerf_pl_amd/csrc/mlp_bwd3.hip nerf_pl_amd/csrc/wgrad.hip nerf_pl_amd/csrc/errors.hip
