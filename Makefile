# Builds libcocoa_hip.so (gfx950) and the CPU oracle.  Used by
# __graft_entry__.build(); `make -j8` works standalone too.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := cocoa_amd/csrc
OUT := cocoa_amd/libcocoa_hip.so
BUILD := build/obj
COMMON := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Iinclude -I$(CSRC)
HDRS := $(wildcard $(CSRC)/*.h) include/cocoa_capi.h

all: $(OUT) oracle/liboracle.so cocoa_amd/cocoa_driver ubench

$(BUILD)/%.strict.o: $(CSRC)/%.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(COMMON) -ffp-contract=off -c $< -o $@

$(BUILD)/%.fast.o: $(CSRC)/%.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(COMMON) -ffp-contract=fast -munsafe-fp-atomics -c $< -o $@

$(BUILD)/dataset.o: $(CSRC)/dataset.cpp $(HDRS) | $(BUILD)
	$(HIPCC) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Iinclude -I$(CSRC) -x c++ -c $< -o $@

$(BUILD)/comm.o: $(CSRC)/comm.cpp $(HDRS) | $(BUILD)
	$(HIPCC) -O2 -std=c++17 -fPIC -Wall -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -I$(CSRC) -x c++ -c $< -o $@

OBJS := $(BUILD)/kernels_strict.strict.o $(BUILD)/kernels_fast.fast.o $(BUILD)/engine.strict.o $(BUILD)/dataset.o \
        $(BUILD)/comm.o $(BUILD)/ingest.strict.o

$(OUT): $(OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(OBJS) -lpthread -ldl

cocoa_amd/cocoa_driver: $(CSRC)/driver_main.cpp $(CSRC)/jdouble.h $(OUT) include/cocoa_capi.h
	$(HIPCC) -O2 -std=c++17 -ffp-contract=off -Iinclude -I$(CSRC) -x c++ $< -o $@ -Lcocoa_amd -lcocoa_hip -Wl,-rpath,'$$ORIGIN'

# diagnostic build with per-step phase stamps in the local solver
DIAG := build/diag
diag: $(DIAG)/libcocoa_hip.so
$(DIAG)/libcocoa_hip.so: $(CSRC)/*.hip $(CSRC)/*.cpp $(HDRS)
	mkdir -p $(DIAG)
	$(HIPCC) $(COMMON) -DCOCOA_STEP_PROF -ffp-contract=off -c $(CSRC)/kernels_strict.hip -o $(DIAG)/ks.o
	$(HIPCC) $(COMMON) -DCOCOA_STEP_PROF -DCOCOA_DIAG -ffp-contract=fast -munsafe-fp-atomics -c $(CSRC)/kernels_fast.hip -o $(DIAG)/kf.o
	$(HIPCC) $(COMMON) -DCOCOA_DIAG -ffp-contract=off -c $(CSRC)/engine.hip -o $(DIAG)/en.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(DIAG)/ks.o $(DIAG)/kf.o $(DIAG)/en.o $(BUILD)/dataset.o $(BUILD)/comm.o \
	    $(BUILD)/ingest.strict.o -lpthread -ldl

oracle/liboracle.so: oracle/cocoa_oracle.c
	$(MAKE) -s -C oracle

$(BUILD):
	mkdir -p $(BUILD)

# PMC calibration / latency micro-benchmarks (tools/gpu_run.sh pmc)
ubench: tools/ubench/calib tools/ubench/lat
tools/ubench/%: tools/ubench/%.hip
	$(HIPCC) -O2 --offload-arch=$(ARCH) $< -o $@

clean:
	rm -rf build $(OUT) cocoa_amd/cocoa_driver oracle/liboracle.so

.PHONY: all clean diag ubench
