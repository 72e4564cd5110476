# Build everything in-tree (the built files travel to the GPU box with the gpurun snapshot).
#   make            -> raytracingc_amd/_lib/librtc.so, raytracingc_amd/_lib/rtc (CLI), oracle/liboracle.so,
#                      oracle/_ref/rtc_ref (only when /root/reference is present)
# Device code: gfx950 only, -ffp-contract=off, no fast-math.

HIPCC    ?= /opt/rocm/bin/hipcc
CC       ?= gcc
CXX      ?= g++
ARCH     ?= gfx950
BUILD    := build
LIBDIR   := raytracingc_amd/_lib
CSRC     := raytracingc_amd/csrc
REF      ?= /root/reference

HIPFLAGS := --offload-arch=$(ARCH) -O3 -ffp-contract=off -fno-slp-vectorize -fPIC -std=c++17 -Wall
CFLAGS   := -std=gnu11 -O2 -fPIC -ffp-contract=off -Wall -Wextra

LIB      := $(LIBDIR)/librtc.so
CLI      := $(LIBDIR)/rtc
ORACLE   := oracle/liboracle.so
REFBIN   := oracle/_ref/rtc_ref
PROBE    := $(LIBDIR)/exact_probe

all: $(LIB) $(CLI) $(ORACLE) $(PROBE) ref

$(BUILD):
	mkdir -p $(BUILD) $(LIBDIR) oracle/_ref

$(BUILD)/scene_build.o: $(CSRC)/scene_build.c $(CSRC)/rtc_internal.h include/rtc.h | $(BUILD)
	$(CC) $(CFLAGS) -c $< -o $@

# header dependencies: explicit below, and generated (-MMD) for anything the explicit lists miss
HDRS     := $(CSRC)/rtc_layout.h $(CSRC)/rtc_plan.h $(CSRC)/rtc_device.h $(CSRC)/rtc_math.h $(CSRC)/rtc_bm_tables.h $(CSRC)/rtc_hip_util.h $(CSRC)/rtc_internal.h include/rtc.h
-include $(wildcard $(BUILD)/*.d)

$(BUILD)/rtc_render.o: $(CSRC)/rtc_render.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -MMD -MP -c $< -o $@

$(BUILD)/rtc_frame.o: $(CSRC)/rtc_frame.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -MMD -MP -c $< -o $@

$(BUILD)/rtc_scene.o: $(CSRC)/rtc_scene.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -MMD -MP -c $< -o $@

$(BUILD)/rtc_probe.o: $(CSRC)/rtc_probe.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -MMD -MP -c $< -o $@

# the launch planner: pure host C++ (rtc_plan.h), no HIP
$(BUILD)/rtc_plan.o: $(CSRC)/rtc_plan.cpp $(CSRC)/rtc_plan.h include/rtc.h | $(BUILD)
	$(CXX) -std=c++17 -O2 -fPIC -Wall -Wextra -c $< -o $@

# the objects every library variant shares (the render kernels are rtc_render.o, or a variant of it)
COMMON   := $(BUILD)/rtc_frame.o $(BUILD)/rtc_scene.o $(BUILD)/rtc_probe.o $(BUILD)/rtc_plan.o $(BUILD)/scene_build.o

$(LIB): $(BUILD)/rtc_render.o $(COMMON)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -o $@ -Wl,-soname,librtc.so -ldl -L/opt/rocm/lib -lhsa-runtime64

# diagnostic variant (per-wave cycle stamps); never the measured product
DIAGLIB  := $(LIBDIR)/librtc_diag.so
$(BUILD)/rtc_render_diag.o: $(CSRC)/rtc_render.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DRTC_DIAG -MMD -MP -c $< -o $@

$(DIAGLIB): $(BUILD)/rtc_render_diag.o $(COMMON)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -o $@ -ldl -L/opt/rocm/lib -lhsa-runtime64

diag: $(DIAGLIB)

# exhaustive GPU check of the exact f32 shortcuts (tests/test_gpu_exact.py)
$(PROBE): tools/exact_probe.hip $(HDRS) | $(BUILD)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -ffp-contract=off -std=c++17 $< -o $@

probe: $(PROBE)

$(BUILD)/rtc_main.o: $(CSRC)/rtc_main.c include/rtc.h | $(BUILD)
	$(CC) $(CFLAGS) -c $< -o $@

$(CLI): $(BUILD)/rtc_main.o $(LIB)
	$(CC) $< -o $@ -L$(LIBDIR) -lrtc -Wl,-rpath,'$$ORIGIN' -lm

# CPU restatement (test infrastructure + timed CPU baseline); gcc, SSE2, no FMA contraction
$(ORACLE): oracle/rtc_oracle.c include/rtc.h | $(BUILD)
	$(CC) -std=gnu11 -O3 -fPIC -shared -ffp-contract=off -Wall $< -o $@ -lm -lpthread

# The reference's own sources, built where they lie (no copy), deterministic variant (oracle/ref_unity.c)
ref: | $(BUILD)
	@if [ -d $(REF) ]; then \
	  $(CC) -std=gnu99 -O3 -w -I$(REF) oracle/ref_unity.c -o $(REFBIN) -lm -lpthread && echo "built $(REFBIN)"; \
	else echo "no $(REF): keeping prebuilt $(REFBIN) if any"; fi

clean:
	rm -rf $(BUILD) $(LIB) $(CLI) $(ORACLE) $(REFBIN)

.PHONY: all ref clean diag
