# Build of libstrom (engine + CDNA4 kernels) and the CLI tools, for gfx950.
# `make -j16` (or `python -m nvme_strom_amd.build`).  Output lands in-tree
# (nvme_strom_amd/lib) so the GPU box snapshot carries it.
ROCM     ?= /opt/rocm
HIPCC    ?= $(ROCM)/bin/hipcc
ARCH     ?= gfx950
OUT      := nvme_strom_amd/lib
OBJ      := build/obj
CXXFLAGS := -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Icsrc/include -Icsrc/engine
HIPFLAGS := $(CXXFLAGS) --offload-arch=$(ARCH) -munsafe-fp-atomics
LDFLAGS  := -shared -fPIC -lpthread

ENGINE_SRC := $(wildcard csrc/engine/*.cc)
KERNEL_SRC := $(wildcard csrc/kernels/*.hip)
ENGINE_OBJ := $(patsubst csrc/engine/%.cc,$(OBJ)/engine/%.o,$(ENGINE_SRC))
KERNEL_OBJ := $(patsubst csrc/kernels/%.hip,$(OBJ)/kernels/%.o,$(KERNEL_SRC))
TOOLS      := $(patsubst csrc/tools/%.cc,$(OUT)/%,$(wildcard csrc/tools/*.cc))

all: $(OUT)/libstrom.so tools

tools: $(TOOLS)

$(OBJ)/engine/%.o: csrc/engine/%.cc csrc/engine/engine.h csrc/include/strom/uapi.h csrc/include/strom/strom.h
	@mkdir -p $(dir $@)
	$(HIPCC) $(CXXFLAGS) -D__HIP_PLATFORM_AMD__ -c $< -o $@

$(OBJ)/kernels/%.o: csrc/kernels/%.hip csrc/include/strom/strom.h
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OUT)/libstrom.so: $(ENGINE_OBJ) $(KERNEL_OBJ)
	@mkdir -p $(OUT)
	$(HIPCC) $(LDFLAGS) --offload-arch=$(ARCH) -o $@ $^

$(OUT)/%: csrc/tools/%.cc $(OUT)/libstrom.so
	$(HIPCC) $(HIPFLAGS) -x hip -o $@ $< -L$(OUT) -lstrom -Wl,-rpath,'$$ORIGIN' -lpthread

clean:
	rm -rf build $(OUT)/libstrom.so $(TOOLS)

.PHONY: all tools clean
