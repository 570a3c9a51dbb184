# Builds the in-tree native library (gfx950 only) and the CPU parity oracle.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
CXX ?= g++
CXXFLAGS ?= -O2 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter
HDR = include/jsplace.h include/jsk_host.h jobset_amd/csrc/jsp_internal.h
HOST_SRC = $(wildcard jobset_amd/csrc/host/*.cc)
HOST_HDR = $(wildcard jobset_amd/csrc/host/*.h)
HOST_OBJ = $(patsubst jobset_amd/csrc/host/%.cc,build/host_%.o,$(HOST_SRC))
LIB = jobset_amd/libjsplace.so
OBJ = build/jsp_kernels.o build/jsp_engine.o $(HOST_OBJ)

all: $(LIB) oracle

build/jsp_kernels.o: jobset_amd/csrc/jsp_kernels.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

build/jsp_engine.o: jobset_amd/csrc/jsp_engine.cc $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c -o $@ $<

build/host_%.o: jobset_amd/csrc/host/%.cc $(HOST_HDR) $(HDR)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -c -o $@ $<

$(LIB): $(OBJ)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf build $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
