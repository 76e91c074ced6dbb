# Builds the C-ABI library nerf_pl_amd/libnerf_pl_amd.so for gfx950 (MI355X)
# and the C pieces of the oracle.  `make -j8`
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize --offload-arch=$(ARCH) -Wall -Wno-unused-function
SRC := $(wildcard nerf_pl_amd/csrc/*.hip)
HDR := $(wildcard nerf_pl_amd/csrc/*.h)
OBJ := $(patsubst nerf_pl_amd/csrc/%.hip,build/%.o,$(SRC))
# the split-operand kernels built a second time as f16x3 (x3.h NR_F16, *_h3 entry points)
H3 := mlp_fwd3 mlp_bwd3 wgrad
OBJ += $(patsubst %,build/%_h3.o,$(H3))
# ... and a third time as plain bf16 (x3.h NR_BF1, *_b1 entry points)
OBJ += $(patsubst %,build/%_b1.o,$(H3))
LIB := nerf_pl_amd/libnerf_pl_amd.so

all: $(LIB)

build/%.o: nerf_pl_amd/csrc/%.hip $(HDR) | build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/%_h3.o: nerf_pl_amd/csrc/%.hip $(HDR) | build
	$(HIPCC) $(HIPFLAGS) -DNR_F16=1 -c $< -o $@

build/%_b1.o: nerf_pl_amd/csrc/%.hip $(HDR) | build
	$(HIPCC) $(HIPFLAGS) -DNR_BF1=1 -c $< -o $@

build:
	mkdir -p build

$(LIB): $(OBJ)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)

clean:
	rm -rf build $(LIB)

.PHONY: all clean
