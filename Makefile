# Builds the C-ABI shared library of the MI355X (gfx950) hot path.
#   make            -> medvae_disentangled_multimodal_amd/libmvae_hip.so
#   make oracle     -> oracle/_ref (nothing to build: the reference is pure Python, see oracle/README)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := medvae_disentangled_multimodal_amd
SRC := $(wildcard $(PKG)/csrc/*.hip) $(PKG)/csrc/errors.cpp
OBJ := $(patsubst $(PKG)/csrc/%,build/%.o,$(SRC))
CXXFLAGS := -O3 -std=c++17 -fPIC -fno-slp-vectorize --offload-arch=$(ARCH) -Wall -Wno-unused-function -Wno-unused-variable

all: $(PKG)/libmvae_hip.so

build/%.o: $(PKG)/csrc/% $(PKG)/csrc/common.h $(PKG)/csrc/gemm_core.h
	@mkdir -p build
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(PKG)/libmvae_hip.so: $(OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(OBJ) -o $@

clean:
	rm -rf build $(PKG)/libmvae_hip.so

.PHONY: all clean
