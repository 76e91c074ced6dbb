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
# host-side AddressSanitizer build of the same sources (the C-ABI
# argument checks and error paths, run by tests/test_abi_asan.py on the CPU).
# The sanitizer instruments host code only (-Xarch_host); device code is built
# as usual and GPU sanitizers are not used.
ASAN_FLAGS := -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer
ASAN_OBJ := $(patsubst build/%.o,build/asan/%.o,$(OBJ))
ASAN_LIB := build/asan/libnerf_pl_amd_asan.so

all: $(LIB)

asan: $(ASAN_LIB)

build/asan/%.o: nerf_pl_amd/csrc/%.hip $(HDR) | build/asan
	$(HIPCC) $(HIPFLAGS) $(ASAN_FLAGS) -c $< -o $@

build/asan/%_h3.o: nerf_pl_amd/csrc/%.hip $(HDR) | build/asan
	$(HIPCC) $(HIPFLAGS) $(ASAN_FLAGS) -DNR_F16=1 -c $< -o $@

build/asan/%_b1.o: nerf_pl_amd/csrc/%.hip $(HDR) | build/asan
	$(HIPCC) $(HIPFLAGS) $(ASAN_FLAGS) -DNR_BF1=1 -c $< -o $@

build/asan:
	mkdir -p build/asan

$(ASAN_LIB): $(ASAN_OBJ)
	$(HIPCC) $(HIPFLAGS) $(ASAN_FLAGS) -shared -o $@ $(ASAN_OBJ)

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

.PHONY: all clean asan
