# Build for MI355X (gfx950). No cmake: plain hipcc / gcc.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
# -disable-machine-licm: MachineLICM hoists the f64 exp/log polynomial constants of
# phase 2 into ~60 VGPRs live across the whole batch loop (kernels.hip), halving occupancy.
HIPFLAGS = --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-result \
           -mllvm -disable-machine-licm
LIB = meyda_amd/libmeyda_gpu.so
SRC = meyda_amd/csrc/kernels.hip meyda_amd/csrc/plan.cpp meyda_amd/csrc/group.cpp
HDR = include/meyda_gpu.h meyda_amd/csrc/mgx_internal.h

all: $(LIB) oracle

$(LIB): $(SRC) $(HDR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ -x hip $(SRC) -ldl

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -f $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
