# Builds the in-tree native library (gfx950 only) and the CPU parity oracle.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
SRC = jobset_amd/csrc/jsp_kernels.hip jobset_amd/csrc/jsp_engine.cc
HDR = include/jsplace.h jobset_amd/csrc/jsp_internal.h
LIB = jobset_amd/libjsplace.so
OBJ = build/jsp_kernels.o build/jsp_engine.o

all: $(LIB) oracle

build/jsp_kernels.o: jobset_amd/csrc/jsp_kernels.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

build/jsp_engine.o: jobset_amd/csrc/jsp_engine.cc $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c -o $@ $<

$(LIB): $(OBJ)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf build $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
