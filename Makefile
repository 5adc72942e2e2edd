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
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@.tmp $(OBJS) -lpthread -ldl && mv -f $@.tmp $@

cocoa_amd/cocoa_driver: $(CSRC)/driver_main.cpp $(CSRC)/jdouble.h $(OUT) include/cocoa_capi.h
	$(HIPCC) -O2 -std=c++17 -ffp-contract=off -Iinclude -I$(CSRC) -x c++ $< -o $@ -Lcocoa_amd -lcocoa_hip -Wl,-rpath,'$$ORIGIN'

# diagnostic build with per-step phase stamps in the local solver (always
# rebuilt; DEFS="-DFOO" adds defines, e.g. an A/B variant's)
DIAG := build/diag
diag:
	mkdir -p $(DIAG)
	$(HIPCC) $(COMMON) $(DEFS) -DCOCOA_STEP_PROF -ffp-contract=off -c $(CSRC)/kernels_strict.hip -o $(DIAG)/ks.o
	$(HIPCC) $(COMMON) $(DEFS) -DCOCOA_STEP_PROF -DCOCOA_DIAG -ffp-contract=fast -munsafe-fp-atomics -c $(CSRC)/kernels_fast.hip -o $(DIAG)/kf.o
	$(HIPCC) $(COMMON) $(DEFS) -DCOCOA_DIAG -ffp-contract=off -c $(CSRC)/engine.hip -o $(DIAG)/en.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $(DIAG)/libcocoa_hip.so $(DIAG)/ks.o $(DIAG)/kf.o $(DIAG)/en.o $(BUILD)/dataset.o $(BUILD)/comm.o \
	    $(BUILD)/ingest.strict.o -lpthread -ldl

oracle/liboracle.so: oracle/cocoa_oracle.c
	$(MAKE) -s -C oracle

$(BUILD):
	mkdir -p $(BUILD)

# A/B variant of the library: make variant V=name DEFS="-DFOO=1" -> build/v_name/libcocoa_hip.so
# (COCOA_LIB=build/v_name/libcocoa_hip.so selects it; tools/gpu_run.sh ab)
variant:
	mkdir -p build/v_$(V)
	$(HIPCC) $(COMMON) $(DEFS) -ffp-contract=off -c $(CSRC)/kernels_strict.hip -o build/v_$(V)/ks.o
	$(HIPCC) $(COMMON) $(DEFS) -ffp-contract=fast -munsafe-fp-atomics -c $(CSRC)/kernels_fast.hip -o build/v_$(V)/kf.o
	$(HIPCC) $(COMMON) $(DEFS) -ffp-contract=off -c $(CSRC)/engine.hip -o build/v_$(V)/en.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o build/v_$(V)/libcocoa_hip.so build/v_$(V)/ks.o build/v_$(V)/kf.o \
	    build/v_$(V)/en.o $(BUILD)/dataset.o $(BUILD)/comm.o $(BUILD)/ingest.strict.o -lpthread -ldl

# PMC calibration / latency micro-benchmarks (tools/gpu_run.sh pmc)
ubench: tools/ubench/calib tools/ubench/lat tools/ubench/ldsdma tools/ubench/dma_layout tools/ubench/evalspmv tools/ubench/cumask
# eval-pass variants on the C2 shape (links the library for the generator and the shipped eval)
tools/ubench/evalspmv: tools/ubench/evalspmv.hip $(CSRC)/eval_wave.h $(OUT)
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -ffp-contract=fast -Iinclude -I$(CSRC) $< -o $@.tmp -Lcocoa_amd -lcocoa_hip \
	    -Wl,-rpath,'$$ORIGIN/../../cocoa_amd' && mv -f $@.tmp $@
tools/ubench/%: tools/ubench/%.hip
	$(HIPCC) -O2 --offload-arch=$(ARCH) $< -o $@

clean:
	rm -rf build $(OUT) cocoa_amd/cocoa_driver oracle/liboracle.so

.PHONY: all clean diag ubench variant
