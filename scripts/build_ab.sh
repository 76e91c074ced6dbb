#!/bin/bash
# A/B build of the library with extra defines on the f16x3 objects (default)
# or on the base objects (bf16x6 + exact fp32 + shared kernels, 4th arg "base"):
#   bash scripts/build_ab.sh <name> "<object...: mlp_fwd3 mlp_bwd3 wgrad ...>" "<-DFLAGS>" [base]
# -> ablibs/libnerf_pl_amd_<name>.so (selected at run time with NERF_PL_AMD_LIB)
set -eu
name=$1; objs_ab=$2; flags=$3; kind=${4:-h3}
HIPFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 -Wall -Wno-unused-function"
mkdir -p build_ab ablibs
make -s -j8
objs=$(ls build/*.o)
for obj in $objs_ab; do
    if [ "$kind" = base ]; then
        /opt/rocm/bin/hipcc $HIPFLAGS $flags -c nerf_pl_amd/csrc/$obj.hip -o build_ab/${obj}_$name.o
        objs=$(echo "$objs" | grep -v "/${obj}.o")
        objs="$objs build_ab/${obj}_$name.o"
    else
        /opt/rocm/bin/hipcc $HIPFLAGS -DNR_F16=1 $flags -c nerf_pl_amd/csrc/$obj.hip -o build_ab/${obj}_h3_$name.o
        objs=$(echo "$objs" | grep -v "/${obj}_h3.o")
        objs="$objs build_ab/${obj}_h3_$name.o"
    fi
done
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o ablibs/libnerf_pl_amd_$name.so $objs
echo "ablibs/libnerf_pl_amd_$name.so"
