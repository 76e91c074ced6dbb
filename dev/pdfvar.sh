#!/bin/bash
# sample_pdf timing variants (dev only): dev/pdfvar.sh <name> <flags...> -> dev/libpdf_<name>.so
set -e
name=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 \
  "$@" -shared -o dev/libpdf_$name.so nerf_pl_amd/csrc/render.hip nerf_pl_amd/csrc/errors.hip
