# Native build: HIP kernels (hipcc, gfx950 only) + C++17 host runtime (g++) +
# pybind11 module + mcg-cg CLI.   `make -j8`  (also driven by __graft_entry__.build()).
ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
CXX       ?= g++
ARCH      ?= gfx950
PYTHON    ?= python3

PY_INC    := $(shell $(PYTHON) -c "import sysconfig; print(sysconfig.get_paths()['include'])")
PYBIND_INC:= $(shell $(PYTHON) -c "import pybind11; print(pybind11.get_include())")
EXT_SUFFIX:= $(shell $(PYTHON) -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")

BUILD     := build
PKG       := cuda_mpi_parallel_amd
PYMOD     := $(PKG)/_C$(EXT_SUFFIX)
CLI       := bin/mcg-cg
TESTBIN   := $(BUILD)/test_host

COMMON    := -O3 -std=c++17 -fPIC -Icsrc/include -Wall -Wno-unused-function
HIPFLAGS  := $(COMMON) --offload-arch=$(ARCH) -munsafe-fp-atomics $(EXTRA_HIPFLAGS)
CXXFLAGS  := $(COMMON) -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include -pthread
LDLIBS    := -L$(ROCM)/lib -lamdhip64 -lrccl -Wl,-rpath,$(ROCM)/lib -pthread -ldl
# One RCCL (and HIP runtime) for every entry point: the Python extension binds to the copies torch
# ships (torch is imported first, the SONAMEs match), so the CLI is pointed at the same files
# through in-tree links under build/rt searched before /opt/rocm/lib (DT_RPATH, transitive).
TORCH_LIB := $(shell $(PYTHON) -c "import os, torch; print(os.path.dirname(torch.__file__) + '/lib')" 2>/dev/null)
RT        := $(BUILD)/rt
RT_LIBS   := librccl.so.1:librccl.so libamdhip64.so.7:libamdhip64.so libhsa-runtime64.so.1:libhsa-runtime64.so \
             libroctx64.so.4:libroctx64.so librccl.so:librccl.so libamdhip64.so:libamdhip64.so \
             libhsa-runtime64.so:libhsa-runtime64.so libroctx64.so:libroctx64.so
CLI_LDLIBS:= -Wl,--disable-new-dtags -Wl,-rpath,'$$ORIGIN/../$(RT)' $(LDLIBS)

HIP_SRC   := $(wildcard csrc/gpu/*.hip)
HOST_SRC  := $(wildcard csrc/host/*.cpp)
GPU_CPP   := $(wildcard csrc/gpu/*.cpp)

HIP_OBJ   := $(patsubst csrc/%.hip,$(BUILD)/%.o,$(HIP_SRC))
HOST_OBJ  := $(patsubst csrc/%.cpp,$(BUILD)/%.o,$(HOST_SRC) $(GPU_CPP))
CORE_OBJ  := $(HIP_OBJ) $(HOST_OBJ)
HEADERS   := $(wildcard csrc/include/mcg/*.hpp) $(wildcard csrc/gpu/*.hpp)

all: $(PYMOD) $(CLI) $(TESTBIN) $(BUILD)/streamop_capture $(BUILD)/persist_probe

$(BUILD)/%.o: csrc/%.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/%.o: csrc/%.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(BUILD)/python/bindings.o: csrc/python/bindings.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -I$(PY_INC) -I$(PYBIND_INC) -fvisibility=hidden -c $< -o $@

$(PYMOD): $(CORE_OBJ) $(BUILD)/python/bindings.o
	$(CXX) -shared -o $@ $^ $(LDLIBS)

$(RT)/.stamp:
	@mkdir -p $(RT)
	@if [ -n "$(TORCH_LIB)" ]; then for m in $(RT_LIBS); do \
	  so=$${m%%:*}; f=$${m##*:}; [ -e "$(TORCH_LIB)/$$f" ] && ln -sfn "$(TORCH_LIB)/$$f" "$(RT)/$$so"; done; true; fi
	@touch $@

$(CLI): $(CORE_OBJ) $(BUILD)/cli/main.o | $(RT)/.stamp
	@mkdir -p bin
	$(CXX) -o $@ $^ $(CLI_LDLIBS)

$(TESTBIN): $(HOST_OBJ:$(BUILD)/gpu/%=) $(BUILD)/tests/test_host.o
	$(CXX) -o $@ $(filter-out $(BUILD)/gpu/%,$(HOST_OBJ)) $(BUILD)/tests/test_host.o -pthread -ldl

$(BUILD)/tests/test_host.o: tests/native/test_host.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

# repro of the stream memory operations / copy-engine copies under graph capture (bench/)
$(BUILD)/streamop_capture: bench/streamop_capture.cpp
	@mkdir -p $(BUILD)
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 $< -o $@

# grid barrier between resident passes vs the kernel boundary (bench/)
$(BUILD)/persist_probe: bench/persist_probe.hip
	@mkdir -p $(BUILD)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 $< -o $@

# host-only sanitizer build of the CPU reference path / partitioner / halo plan tests
# (GPU sanitizers are not available on this pool: host code only)
ASAN_SRC  := $(wildcard csrc/host/*.cpp) tests/native/test_host.cpp
$(BUILD)/test_host_asan: $(ASAN_SRC) $(HEADERS)
	@mkdir -p $(BUILD)
	$(CXX) -O1 -g -std=c++17 -Icsrc/include -fsanitize=address,undefined -fno-omit-frame-pointer \
	  -fno-sanitize-recover=undefined $(ASAN_SRC) -o $@ -pthread -ldl

asan: $(BUILD)/test_host_asan

clean:
	rm -rf $(BUILD) $(PYMOD) $(CLI)

.PHONY: all clean asan
