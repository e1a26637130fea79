# Builds the C-ABI shared library of the MI355X (gfx950) hot path.
#   make            -> medvae_disentangled_multimodal_amd/libmvae_hip.so
#   make oracle     -> oracle/_ref (nothing to build: the reference is pure Python, see oracle/README)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := medvae_disentangled_multimodal_amd
SRC := $(wildcard $(PKG)/csrc/*.hip) $(PKG)/csrc/errors.cpp
OBJ := $(patsubst $(PKG)/csrc/%,build/%.o,$(SRC))
CXXFLAGS := -O3 -std=c++17 -fPIC -fno-slp-vectorize --offload-arch=$(ARCH) -Wall -Wno-unused-function -Wno-unused-variable

PYINC := $(shell python3 -c "import sysconfig; print(sysconfig.get_paths()['include'])")
PYEXT := $(shell python3 -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")

all: $(PKG)/libmvae_hip.so $(PKG)/_mvae_fast$(PYEXT)

# host-side call path (Python -> C ABI) without ctypes argument conversion: csrc/pyfast.c
$(PKG)/_mvae_fast$(PYEXT): $(PKG)/csrc/pyfast.c
	gcc -O2 -shared -fPIC -Wall -I$(PYINC) $< -o $@

build/%.o: $(PKG)/csrc/% $(PKG)/csrc/common.h $(PKG)/csrc/gemm_core.h
	@mkdir -p build
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(PKG)/libmvae_hip.so: $(OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(OBJ) -o $@

clean:
	rm -rf build $(PKG)/libmvae_hip.so $(PKG)/_mvae_fast*.so

.PHONY: all clean
