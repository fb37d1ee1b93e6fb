# Builds the product library (HIP, gfx950 only) and the CPU oracle (test infrastructure).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-result --offload-arch=$(ARCH)
CSRC := dragonboat_amd/csrc
LIBDIR := dragonboat_amd/lib
LIB := $(LIBDIR)/libhipquorum.so
OBJS := $(LIBDIR)/hq_runtime.o $(LIBDIR)/hq_kernels.o $(LIBDIR)/hq_table.o $(LIBDIR)/hq_pack.o \
        $(LIBDIR)/hq_worker.o $(LIBDIR)/hq_wire.o $(LIBDIR)/hq_stream.o $(LIBDIR)/hq_jobs.o $(LIBDIR)/hq_dstep.o \
        $(LIBDIR)/hq_engine.o
SRCS := $(CSRC)/hq_kernels.hip $(CSRC)/hq_table.hip $(CSRC)/hq_runtime.hip $(CSRC)/hq_pack.cpp \
        $(CSRC)/hq_worker.cpp $(CSRC)/hq_wire.cpp $(CSRC)/hq_stream.cpp $(CSRC)/hq_jobs.cpp $(CSRC)/hq_dstep.hip \
        $(CSRC)/hq_engine.hip
DEPS := $(wildcard $(CSRC)/*.h) include/hipquorum.h
CXX ?= g++
CXXFLAGS ?= -O3 -std=c++17 -fPIC -pthread -Wall -Wextra

all: $(LIB) oracle tools/link_probe

# the host-link probe bench.py's step legs run beside them (their link roofline)
tools/link_probe: tools/link_probe.cpp
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -o $@ $<

$(LIBDIR)/%.o: $(CSRC)/%.hip $(DEPS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

# host-only sources (packers): plain C++
$(LIBDIR)/%.o: $(CSRC)/%.cpp $(DEPS)
	@mkdir -p $(LIBDIR)
	$(CXX) $(CXXFLAGS) -c -o $@ $<

$(LIB): $(OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -pthread -o $@ $(OBJS)

oracle:
	$(MAKE) -C oracle

# tuning variants (one library each, for A/B runs via HQ_LIB_PATH, tools/ab_libs.sh):
#   lib_vec2   lag kernels with 2 groups per lane (8-byte loads)
#   lib_b512   every commit kernel with 512-thread blocks
#   lib_mbN    grid cap (in 256-thread units) raised N x
#   lib_ivN    records per lane of the table ingest kernels
#   lib_b3tpwN tiles per wave of the 3-byte bitmap kernel
#   lib_pltpwN tiles per wave of the bit-plane kernel, lib_plblkN its block size
#   lib_swN    the device step engine's kernels asked for N waves per SIMD
#   lib_rinet0 multi-ctx ReadIndex with the 28-CE transposition sort instead of Batcher's 19-CE network
#   lib_tilecopy / lib_b3copy / lib_plcopy the commit tile / 3-byte / bit-plane kernel's loads and stores without the
#              decision (their floors)
#   lib_ingnostore / lib_ingnoload the grouped table ingest without its table stores / loads (timing probes: wrong output)
#   lib_encspawn the threaded event encoder spawning its threads per call (before the task pool)
#   lib_encprof the threaded encoder's per-range start / barrier arrival per call (stderr)
#   lib_engprof the engine's per-workgroup clocks and tile counts (hq_engine_wgprof; tools/engine_wgprof.py)
#   lib_notakerun the device step taking every run member one event at a time (no take_run; A/B)
define variant
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) $(1) -shared -o $@ $(SRCS)
endef
tools/lib_vec2/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_LAG_VEC=2)
tools/lib_b512/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_COMMIT_BLOCK_BIG=512)
tools/lib_mb%/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_MAX_BLOCKS=$*)
tools/lib_iv%/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_INGEST_V=$*)
tools/lib_b3tpw%/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_BITS3_TPW=$*)
tools/lib_pltpw%/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_PLANES_TPW=$*)
tools/lib_plblk%/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_PLANES_BLK=$*)
tools/lib_plplain/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_PLANES_PLAIN)
tools/lib_plcopy/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_PLANES_COPY)
tools/lib_tilecopy/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_TILE_COPY)
tools/lib_b3copy/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_BITS3_COPY)

variants: tools/lib_vec2/libhipquorum.so tools/lib_b512/libhipquorum.so

clean:
	rm -rf $(LIBDIR) oracle/build

.PHONY: all oracle clean variants
tools/lib_encspawn/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_ENCODE_SPAWN)
tools/lib_ingnostore/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_INGEST_NOSTORE)
tools/lib_ingnoload/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_INGEST_NOLOAD)
tools/lib_rinet0/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_RI_NET=0)
tools/lib_encprof/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_ENC_PROF)
tools/lib_engprof/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_ENGINE_WGPROF)
tools/lib_notakerun/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_NO_TAKE_RUN)
tools/lib_sw%/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_STEP_WAVES=$*)
# binned-ingest A/B (tools/ab_bin.sh): kernel parts removed (HQ_BIN_AB) or smaller regions
tools/lib_binab%/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_BIN_AB=$*)
tools/lib_bintpb%/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_BIN_TPB_SHIFT=$*)
# phase timestamps of the binned ingest (tools/binprof.hip includes hq_table.hip with HQ_BIN_PROF)
tools/binprof: tools/binprof.hip $(SRCS) $(DEPS) $(OBJS)
	$(HIPCC) $(HIPFLAGS) -c -o tools/binprof.o tools/binprof.hip
	$(HIPCC) $(HIPFLAGS) -pthread -o $@ tools/binprof.o $(filter-out $(LIBDIR)/hq_table.o,$(OBJS))
tools/lib_plcqtpw%/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_PLCQ_TPW=$*)
tools/lib_stepchunks%/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_STEP_CHUNKS=$*)
tools/lib_plcqzero%/libhipquorum.so: $(SRCS) $(DEPS)
	$(call variant,-DHQ_PLCQ_ZERO_EARLY=$*)
# persistent-engine experiments (tools/ab_engine.py): multi-batch loop / flat / claim kernels beside
# the engine, in a library of their own linked against the product library
tools/lib_engexp/libengexp.so: tools/engine_exp.hip $(LIB) $(DEPS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ tools/engine_exp.hip -L$(LIBDIR) -lhipquorum -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'

