# Builds the MI355X engine (narwhal_amd/libnarwhal_amd.so, gfx950 only), the CPU oracle
# (test infrastructure) and the host arithmetic check library (test infrastructure).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Iinclude -Inarwhal_amd/csrc -Wall -Wno-unused-function
CSRC := narwhal_amd/csrc
HDRS := $(wildcard $(CSRC)/*.hpp) $(CSRC)/nw_kernels.h $(CSRC)/nw_runtime.h $(CSRC)/nw_host.h include/narwhal_amd.h
LIB := narwhal_amd/libnarwhal_amd.so
BUILD := build

all: $(LIB) oracle hostcheck loadgen

$(BUILD)/nw_kernels.o: $(CSRC)/nw_kernels.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/nw_batch.o: $(CSRC)/nw_batch.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/nw_cert.o: $(CSRC)/nw_cert.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/nw_small.o: $(CSRC)/nw_small.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/nw_jobs.o: $(CSRC)/nw_jobs.cpp $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(BUILD)/nw_wire.o: $(CSRC)/nw_wire.cpp $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(BUILD)/nw_service.o: $(CSRC)/nw_service.cpp $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(BUILD)/nw_host.o: $(CSRC)/nw_host.cpp $(CSRC)/nw_host.h $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(BUILD)/nw_api.o: $(CSRC)/nw_api.cpp $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(BUILD)/nw_kernels.o $(BUILD)/nw_batch.o $(BUILD)/nw_cert.o $(BUILD)/nw_small.o $(BUILD)/nw_api.o $(BUILD)/nw_jobs.o $(BUILD)/nw_wire.o $(BUILD)/nw_service.o $(BUILD)/nw_host.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

oracle:
	$(MAKE) -s -C oracle

hostcheck: tools/libnw_hostcheck.so
tools/libnw_hostcheck.so: tools/hostcheck.hip $(HDRS)
	$(HIPCC) --cuda-host-only -O2 -std=c++17 -fPIC -shared -Iinclude $< -o $@

loadgen: tools/libnw_loadgen.so
tools/libnw_loadgen.so: tools/nw_loadgen.cpp include/narwhal_amd.h $(LIB)
	g++ -O2 -std=c++17 -fPIC -shared -Iinclude $< -o $@ -Lnarwhal_amd -lnarwhal_amd -Wl,-rpath,'$$ORIGIN/../narwhal_amd' -pthread

# CPU harness of the service's host logic over test doubles of the device entry points
# (tests/test_service_stress.py); _tsan: the same under ThreadSanitizer
STRESS_FLAGS := -std=c++17 -pthread -D__HIP_PLATFORM_AMD__ -Iinclude -I$(CSRC) -I/opt/rocm/include
stress: tools/service_stress tools/service_stress_tsan
tools/service_stress: tools/service_stress.cpp $(CSRC)/nw_service.cpp $(HDRS)
	g++ -O2 $(STRESS_FLAGS) tools/service_stress.cpp $(CSRC)/nw_service.cpp -o $@
tools/service_stress_tsan: tools/service_stress.cpp $(CSRC)/nw_service.cpp $(HDRS)
	g++ -O1 -g -fsanitize=thread -DNW_SERVICE_SYSTEM_CLOCK_WAIT $(STRESS_FLAGS) tools/service_stress.cpp $(CSRC)/nw_service.cpp -o $@

ubench: tools/ubench_valu
tools/ubench_valu: tools/ubench_valu.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 $< -o $@

clean:
	rm -rf $(BUILD) $(LIB) tools/libnw_hostcheck.so tools/libnw_loadgen.so tools/service_stress tools/service_stress_tsan
	$(MAKE) -s -C oracle clean

.PHONY: all oracle hostcheck loadgen stress ubench clean
