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

# Host-side sanitizer build: the library with ASan + UBSan on its host code
# (the GPU code is not instrumented: -Xarch_host), a host-only driver (WAV-parser fuzz corpus,
# host tables, arithmetic, validation) and the N-API addon, all against clang's shared ASan
# runtime; tests/test_asan.py runs them with that runtime preloaded.
ASAN_DIR = build/asan
SAN = -fsanitize=address -fsanitize=undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -shared-libsan
CLANG = /opt/rocm/lib/llvm/bin/clang
asan: $(ASAN_DIR)/libmeyda_gpu.so $(ASAN_DIR)/host_checks $(ASAN_DIR)/addon/meyda_napi.node

$(ASAN_DIR)/libmeyda_gpu.so: $(SRC) $(HDR)
	mkdir -p $(ASAN_DIR)
	$(HIPCC) $(HIPFLAGS) $(foreach f,$(SAN),-Xarch_host $(f)) -shared -o $@ -x hip $(SRC) -ldl

$(ASAN_DIR)/host_checks: tools/asan/host_checks.cpp $(ASAN_DIR)/libmeyda_gpu.so include/meyda_gpu.h
	$(CLANG)++ -O1 -g -std=c++17 $(SAN) -o $@ $< -L$(ASAN_DIR) -l:libmeyda_gpu.so -Wl,-rpath,'$$ORIGIN'

$(ASAN_DIR)/addon/meyda_napi.node: meyda_amd/addon/meyda_napi.c $(ASAN_DIR)/libmeyda_gpu.so include/meyda_gpu.h
	mkdir -p $(ASAN_DIR)/addon
	$(CLANG) -O1 -g -fPIC -std=c11 -I/usr/include/node -DNODE_GYP_MODULE_NAME=meyda_napi $(SAN) -mllvm -asan-globals=0 -shared -o $@ $< \
	  -L$(ASAN_DIR) -l:libmeyda_gpu.so -Wl,-rpath,'$$ORIGIN/..'

$(LIB): $(SRC) $(HDR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ -x hip $(SRC) -ldl

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -f $(LIB)
	rm -rf $(ASAN_DIR)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean asan
