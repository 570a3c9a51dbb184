# Builds the in-tree native library (gfx950 only) and the CPU parity oracle.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
CXX ?= g++
CXXFLAGS ?= -O2 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter
HDR = include/jsplace.h include/jsplace_bench.h include/jsk_host.h jobset_amd/csrc/jsp_internal.h jobset_amd/csrc/jsp_walk.h jobset_amd/csrc/jsp_multi.h
HOST_SRC = $(wildcard jobset_amd/csrc/host/*.cc)
HOST_HDR = $(wildcard jobset_amd/csrc/host/*.h)
HOST_OBJ = $(patsubst jobset_amd/csrc/host/%.cc,build/host_%.o,$(HOST_SRC))
LIB = jobset_amd/libjsplace.so
OBJ = build/jsp_kernels.o build/jsp_engine.o build/jsp_walk.o build/jsp_multi.o $(HOST_OBJ)

all: $(LIB) oracle

# -ffinite-math-only: the kernels' only floating point is the tally's f64
# capacity minimum (finite, non-negative): v_min_f64 without the NaN-quieting
# v_max_f64 the IEEE minNum semantics would put before each operand
KFLAGS = -ffinite-math-only
build/jsp_kernels.o: jobset_amd/csrc/jsp_kernels.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) $(KFLAGS) -c -o $@ $<

build/jsp_engine.o: jobset_amd/csrc/jsp_engine.cc jobset_amd/csrc/jsp_walk.h $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c -o $@ $<

build/jsp_walk.o: jobset_amd/csrc/jsp_walk.cc jobset_amd/csrc/jsp_walk.h $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c -o $@ $<

build/jsp_multi.o: jobset_amd/csrc/jsp_multi.cc jobset_amd/csrc/jsp_multi.h $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c -o $@ $<

build/host_%.o: jobset_amd/csrc/host/%.cc $(HOST_HDR) $(HDR)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -c -o $@ $<

$(LIB): $(OBJ)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ) -ldl

oracle:
	$(MAKE) -s -C oracle

# diagnostic build with in-kernel phase stamps (tools/stamps.py); never the product library
diag: tools/diag/libjsplace.so tools/bin/dispatch_probe tools/bin/stream_ceiling
# probes that run on the GPU box live in tools/bin (shipped); the diagnostic
# library stays in tools/diag (.gpurunignore: 4 MB per push)
tools/bin/dispatch_probe: tools/dispatch_probe.hip
	@mkdir -p tools/bin
	$(HIPCC) --offload-arch=gfx950 -O3 -o $@ $<
tools/diag/libjsplace.so: jobset_amd/csrc/jsp_kernels.hip jobset_amd/csrc/jsp_engine.cc $(HOST_SRC) $(HDR) $(HOST_HDR)
	@mkdir -p build/diag tools/diag
	$(HIPCC) $(HIPFLAGS) $(KFLAGS) -DJSP_STAMPS -c -o build/diag/k.o jobset_amd/csrc/jsp_kernels.hip
	$(HIPCC) $(HIPFLAGS) -DJSP_STAMPS -x hip -c -o build/diag/e.o jobset_amd/csrc/jsp_engine.cc
	$(HIPCC) $(HIPFLAGS) -shared -o $@ build/diag/k.o build/diag/e.o build/jsp_walk.o build/jsp_multi.o $(HOST_OBJ)

# ASan + UBSan build of the host mirror (webhook / reconciler / planner / JSON)
# linked with the product engine objects, and of the C oracles; tests/
# test_sanitizers.py runs the host and oracle suites against them under a
# preloaded libasan. Host code only: GPU sanitizers are not used.
SANFLAGS = -O1 -g -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -fsanitize=address,undefined \
	-fno-omit-frame-pointer -fno-sanitize-recover=undefined
ASAN_OBJ = $(patsubst jobset_amd/csrc/host/%.cc,build/asan/host_%.o,$(HOST_SRC))
sanitize: build/asan/libjsplace.so
	$(MAKE) -s -C oracle sanitize
build/asan/host_%.o: jobset_amd/csrc/host/%.cc $(HOST_HDR) $(HDR)
	@mkdir -p build/asan
	$(CXX) $(SANFLAGS) -c -o $@ $<
build/asan/libjsplace.so: build/jsp_kernels.o build/jsp_engine.o build/jsp_walk.o build/jsp_multi.o $(ASAN_OBJ)
	$(CXX) -shared -fsanitize=address,undefined -o $@ $^ -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lamdhip64

# ThreadSanitizer build of the host mirror (the engine objects as built):
# tests/test_concurrency.py runs its concurrent host-mirror callers against it
# with libtsan preloaded. Host code only.
TSANFLAGS = -O1 -g -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -fsanitize=thread -fno-omit-frame-pointer
TSAN_OBJ = $(patsubst jobset_amd/csrc/host/%.cc,build/tsan/host_%.o,$(HOST_SRC))
tsan: build/tsan/libjsplace.so
build/tsan/host_%.o: jobset_amd/csrc/host/%.cc $(HOST_HDR) $(HDR)
	@mkdir -p build/tsan
	$(CXX) $(TSANFLAGS) -c -o $@ $<
build/tsan/libjsplace.so: build/jsp_kernels.o build/jsp_engine.o build/jsp_walk.o build/jsp_multi.o $(TSAN_OBJ)
	$(CXX) -shared -fsanitize=thread -o $@ $^ -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lamdhip64 -ldl

clean:
	rm -rf build $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean diag sanitize tsan

# achievable streaming ceiling (read-only and copy, cold and warm) at the placement kernels' byte counts
tools/bin/stream_ceiling: tools/stream_ceiling.hip
	@mkdir -p tools/bin
	$(HIPCC) --offload-arch=gfx950 -O3 -std=c++17 -o $@ $<
tools/bin/layout_probe: tools/layout_probe.hip
	@mkdir -p tools/bin
	$(HIPCC) --offload-arch=gfx950 -O3 -std=c++17 -o $@ $<
tools/bin/mailbox_probe: tools/mailbox_probe.hip
	@mkdir -p tools/bin
	$(HIPCC) --offload-arch=gfx950 -O3 -std=c++17 -o $@ $< -lhsa-runtime64
tools/bin/valu_rate: tools/valu_rate.hip
	@mkdir -p tools/bin
	$(HIPCC) --offload-arch=gfx950 -O3 -std=c++17 -o $@ $<

# A/B builds of the kernels with one build flag (a probe loads them
# through JSP_LIB_PATH): tools/ablib/<name>/libjsplace.so
AB_FLAGS_fakedesc = -DJSP_AB_FAKE_DESC
tools/ablib/%/libjsplace.so: jobset_amd/csrc/jsp_kernels.hip build/jsp_engine.o build/jsp_walk.o build/jsp_multi.o $(HOST_OBJ) $(HDR)
	@mkdir -p build/ab_$* tools/ablib/$*
	$(HIPCC) $(HIPFLAGS) $(KFLAGS) $(AB_FLAGS_$*) -c -o build/ab_$*/k.o jobset_amd/csrc/jsp_kernels.hip
	$(HIPCC) $(HIPFLAGS) -shared -o $@ build/ab_$*/k.o build/jsp_engine.o build/jsp_walk.o build/jsp_multi.o $(HOST_OBJ) -ldl
tools/bin/block_probe: tools/block_probe.hip
	@mkdir -p tools/bin
	$(HIPCC) --offload-arch=gfx950 -O3 -std=c++17 -o $@ $<
# A/B build: the service's row/leaf-pass stamps carry the shader clock (diagnostic)
tools/bin/ab_clk/libjsplace.so: jobset_amd/csrc/jsp_kernels.hip build/jsp_engine.o build/jsp_walk.o build/jsp_multi.o $(HOST_OBJ) $(HDR)
	@mkdir -p build/ab_clk tools/bin/ab_clk
	$(HIPCC) $(HIPFLAGS) $(KFLAGS) -DJSP_AB_CLKFREQ -c -o build/ab_clk/k.o jobset_amd/csrc/jsp_kernels.hip
	$(HIPCC) $(HIPFLAGS) -shared -o $@ build/ab_clk/k.o build/jsp_engine.o build/jsp_walk.o build/jsp_multi.o $(HOST_OBJ) -ldl
# A/B build: service stamps 2-4 inside the row pass (loop start, class record, first scan)
tools/bin/ab_fine/libjsplace.so: jobset_amd/csrc/jsp_kernels.hip build/jsp_engine.o build/jsp_walk.o build/jsp_multi.o $(HOST_OBJ) $(HDR)
	@mkdir -p build/ab_fine tools/bin/ab_fine
	$(HIPCC) $(HIPFLAGS) $(KFLAGS) -DJSP_AB_FINESTAMP -c -o build/ab_fine/k.o jobset_amd/csrc/jsp_kernels.hip
	$(HIPCC) $(HIPFLAGS) -shared -o $@ build/ab_fine/k.o build/jsp_engine.o build/jsp_walk.o build/jsp_multi.o $(HOST_OBJ) -ldl
# A/B build: split-service stamps 2-4 at tally_block's entry, after its row copy, after its first barrier
tools/bin/ab_entry/libjsplace.so: jobset_amd/csrc/jsp_kernels.hip build/jsp_engine.o build/jsp_walk.o build/jsp_multi.o $(HOST_OBJ) $(HDR)
	@mkdir -p build/ab_entry tools/bin/ab_entry
	$(HIPCC) $(HIPFLAGS) $(KFLAGS) -DJSP_AB_ENTRYSTAMP -c -o build/ab_entry/k.o jobset_amd/csrc/jsp_kernels.hip
	$(HIPCC) $(HIPFLAGS) -shared -o $@ build/ab_entry/k.o build/jsp_engine.o build/jsp_walk.o build/jsp_multi.o $(HOST_OBJ) -ldl
AB_FLAGS_noinv = -DJSP_AB_NOINV
AB_FLAGS_entrynoinv = -DJSP_AB_NOINV -DJSP_AB_ENTRYSTAMP
# diagnostic stamp build shipped to the GPU box (tools/bin is not gpurun-ignored)
tools/bin/diag/libjsplace.so: jobset_amd/csrc/jsp_kernels.hip build/jsp_engine.o build/jsp_walk.o build/jsp_multi.o $(HOST_OBJ) $(HDR)
	@mkdir -p build/diag2 tools/bin/diag
	$(HIPCC) $(HIPFLAGS) $(KFLAGS) -DJSP_STAMPS -c -o build/diag2/k.o jobset_amd/csrc/jsp_kernels.hip
	$(HIPCC) $(HIPFLAGS) -shared -o $@ build/diag2/k.o build/jsp_engine.o build/jsp_walk.o build/jsp_multi.o $(HOST_OBJ) -ldl
# A/B build: the recovery's wake runs inside the patch call instead of the
# waker thread (tools/cold_probe4.py loads it through JSP_LIB_PATH)
tools/bin/ab_inlinewake/libjsplace.so: jobset_amd/csrc/jsp_engine.cc build/jsp_kernels.o build/jsp_walk.o build/jsp_multi.o $(HOST_OBJ) $(HDR)
	@mkdir -p build/ab_iw tools/bin/ab_inlinewake
	$(HIPCC) $(HIPFLAGS) -DJSP_AB_INLINE_WAKE -x hip -c -o build/ab_iw/e.o jobset_amd/csrc/jsp_engine.cc
	$(HIPCC) $(HIPFLAGS) -shared -o $@ build/jsp_kernels.o build/ab_iw/e.o build/jsp_walk.o build/jsp_multi.o $(HOST_OBJ) -ldl
tools/bin/stop_anatomy: tools/stop_anatomy.hip
	@mkdir -p tools/bin
	$(HIPCC) --offload-arch=gfx950 -O3 -std=c++17 -o $@ $<
# A/B build: real-time stamps inside the resident evaluation (slots 3, 4, 6, 7)
tools/bin/ab_eval/libjsplace.so: jobset_amd/csrc/jsp_kernels.hip build/jsp_engine.o build/jsp_walk.o build/jsp_multi.o $(HOST_OBJ) $(HDR)
	@mkdir -p build/ab_eval tools/bin/ab_eval
	$(HIPCC) $(HIPFLAGS) $(KFLAGS) -DJSP_AB_EVALSTAMP -c -o build/ab_eval/k.o jobset_amd/csrc/jsp_kernels.hip
	$(HIPCC) $(HIPFLAGS) -shared -o $@ build/ab_eval/k.o build/jsp_engine.o build/jsp_walk.o build/jsp_multi.o $(HOST_OBJ) -ldl
