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
LDFLAGS  := -shared -fPIC -lpthread -L$(ROCM)/lib -lrocprofiler-sdk-roctx -lhsa-runtime64

ENGINE_SRC := $(wildcard csrc/engine/*.cc)
KERNEL_SRC := $(wildcard csrc/kernels/*.hip)
# the kernel-free core shared with the kernel module (planner, raid0, PRPs)
CORE_SRC   := kmod/strom_core.c
CORE_OBJ   := $(OBJ)/core/strom_core.o
ENGINE_OBJ := $(patsubst csrc/engine/%.cc,$(OBJ)/engine/%.o,$(ENGINE_SRC))
KERNEL_OBJ := $(patsubst csrc/kernels/%.hip,$(OBJ)/kernels/%.o,$(KERNEL_SRC))
TOOLS      := $(patsubst csrc/tools/%.cc,$(OUT)/%,$(wildcard csrc/tools/*.cc))

all: $(OUT)/libstrom.so tools $(OUT)/libstrom_decprof.so $(OUT)/libstrom_lz4par512_host.so \
     $(OUT)/libstrom_lz4par512b_host.so \
     $(OUT)/libstrom_zstdprof.so

tools: $(TOOLS)

$(CORE_OBJ): $(CORE_SRC) kmod/strom_core.h
	@mkdir -p $(dir $@)
	gcc -O2 -std=gnu11 -fPIC -Wall -Wextra -Wno-unused-parameter -c $< -o $@

$(OBJ)/engine/%.o: csrc/engine/%.cc csrc/engine/engine.h csrc/include/strom/uapi.h csrc/include/strom/strom.h kmod/strom_core.h
	@mkdir -p $(dir $@)
	$(HIPCC) $(CXXFLAGS) -D__HIP_PLATFORM_AMD__ -c $< -o $@

$(OBJ)/kernels/%.o: csrc/kernels/%.hip csrc/include/strom/strom.h
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# the 512-thread decoder build is lz4par.hip compiled again
$(OBJ)/kernels/lz4par_nt512.o: csrc/kernels/lz4par.hip
$(OBJ)/kernels/lz4par_nt512_ob8k.o: csrc/kernels/lz4par.hip

$(OUT)/libstrom.so: $(ENGINE_OBJ) $(KERNEL_OBJ) $(CORE_OBJ)
	@mkdir -p $(OUT)
	$(HIPCC) $(LDFLAGS) --offload-arch=$(ARCH) -o $@ $^

# the LZ4/snappy decoder with its cycle profile compiled in (tools/decomp_prof.py)
$(OUT)/libstrom_decprof.so: csrc/kernels/decompress.hip csrc/kernels/lz4par.hip csrc/include/strom/strom.h
	@mkdir -p $(OUT)
	$(HIPCC) $(HIPFLAGS) -DSTROM_DECOMP_PROF -shared -o $@ csrc/kernels/decompress.hip csrc/kernels/lz4par.hip

# the zstd decoder with its phase profile compiled in (tools/zstd_bench.py --prof)
$(OUT)/libstrom_zstdprof.so: csrc/kernels/zstd.hip csrc/include/strom/strom.h
	@mkdir -p $(OUT)
	$(HIPCC) $(HIPFLAGS) -DZS_PROF -shared -o $@ $<

# zstd geometry variants for A/B timing (tools/zstd_bench.py --lib):
# make zv ZV="name:-DZS_OB=1024 ..." -> $(OUT)/zv/<name>.so
ZV ?= base:-DZS_OB=512
zv:
	@rm -rf $(OUT)/zv && mkdir -p $(OUT)/zv
	@for v in $(ZV); do name=$${v%%:*}; defs=$$(echo $${v#*:} | tr , ' '); \
	  $(HIPCC) $(HIPFLAGS) -Icsrc/include $$defs -shared -o $(OUT)/zv/$$name.so \
	    csrc/kernels/zstd.hip || exit 1; done
.PHONY: zv

# a standalone decoder build for same-box A/B runs (tools/decomp_ab.py):
# make ab AB=name [SRC=path/to/decompress.hip]
SRC ?= csrc/kernels/decompress.hip
WSRC ?= csrc/kernels/lz4par.hip
ab:
	@mkdir -p $(OUT)/ab
	$(HIPCC) $(HIPFLAGS) -Icsrc/include -shared -o $(OUT)/ab/$(AB).so $(SRC) $(WSRC)
	$(HIPCC) $(HIPFLAGS) -Icsrc/include -DSTROM_DECOMP_PROF -shared -o $(OUT)/ab/$(AB)_prof.so $(SRC) $(WSRC)

$(OUT)/%: csrc/tools/%.cc $(OUT)/libstrom.so
	$(HIPCC) $(HIPFLAGS) -x hip -o $@ $< -L$(OUT) -lstrom -Wl,-rpath,'$$ORIGIN' -lpthread

clean:
	rm -rf build $(OUT)/libstrom.so $(OUT)/libstrom_decprof.so $(OUT)/libstrom_lz4par512_host.so \
	  $(OUT)/libstrom_lz4par512b_host.so \
	  $(OUT)/libstrom_zstdprof.so $(TOOLS)

.PHONY: all tools clean ab

# ---- host-only engine self-test, plain and under sanitizers ---------------
# The engine's host code builds with g++ (HIP host API only); device kernels
# are not part of these builds.  GPU sanitizers are not used on this pool.
SELFTEST_SRC := csrc/tests/engine_selftest.cc $(ENGINE_SRC) $(CORE_SRC)
SELFTEST_FLAGS := -std=c++17 -g -O1 -Icsrc/include -Icsrc/engine -I$(ROCM)/include -D__HIP_PLATFORM_AMD__
SELFTEST_LIBS := -L$(ROCM)/lib -lamdhip64 -lhsa-runtime64 -lrocprofiler-sdk-roctx -lpthread -Wl,-rpath,$(ROCM)/lib

build/selftest: $(SELFTEST_SRC) csrc/engine/engine.h
	@mkdir -p build
	g++ $(SELFTEST_FLAGS) -o $@ $(SELFTEST_SRC) $(SELFTEST_LIBS)

build/selftest-asan: $(SELFTEST_SRC) csrc/engine/engine.h
	@mkdir -p build
	g++ $(SELFTEST_FLAGS) -fsanitize=address,undefined -fno-omit-frame-pointer -o $@ $(SELFTEST_SRC) $(SELFTEST_LIBS)

# TSAN uses ROCm's clang runtime: gcc-11's libtsan lacks the
# pthread_cond_clockwait interceptor that condition_variable::wait_until
# compiles to, which yields false "double lock" reports on the task table.
build/selftest-tsan: $(SELFTEST_SRC) csrc/engine/engine.h
	@mkdir -p build
	$(ROCM)/llvm/bin/clang++ $(SELFTEST_FLAGS) -fsanitize=thread -o $@ $(SELFTEST_SRC) $(SELFTEST_LIBS)

# the 512-thread build of the block-parallel decoder WITH its host copy:
# the CPU tests run its phases thread by thread (tests/test_codecs_cpu.py)
$(OUT)/libstrom_lz4par512_host.so: csrc/kernels/lz4par.hip csrc/include/strom/strom.h
	$(HIPCC) $(HIPFLAGS) -Icsrc/include -DLZ4PAR_NT=512 -DLZ4PAR_LOADU=8 -DLZ4PAR_WPE_LZ4=6 -DLZ4P_NS=lz4p512 -DLZ4PAR_SN_LOOKBACK=64 -DLZ4PAR_SN_WLOOKBACK=32 \
	  -DLZ4PAR_ENTRY=strom_decompress_par512 -shared -o $@ $<

# ... and of the 8 KiB-batch build (lz4par_nt512_ob8k.hip)
$(OUT)/libstrom_lz4par512b_host.so: csrc/kernels/lz4par.hip csrc/include/strom/strom.h
	$(HIPCC) $(HIPFLAGS) -Icsrc/include -DLZ4PAR_NT=512 -DLZ4PAR_LOADU=8 -DLZ4PAR_OB=8192 -DLZ4PAR_WPE_LZ4=4 -DLZ4PAR_WPE=4 -DLZ4P_NS=lz4p512b -DLZ4PAR_SN_LOOKBACK=64 -DLZ4PAR_SN_WLOOKBACK=32 \
	  -DLZ4PAR_ENTRY=strom_decompress_par512b -shared -o $@ $<

# lz4par geometry variants for A/B timing (tools/lz4par_bench.py --variants):
# make lz4v LZ4V="name:-DX=1,-DY=2 ..." -> $(OUT)/lz4v/<name>.so (lz4par.hip
# with those macros: LZ4PAR_NT / _PW / _OB / _HR / _LOOKBACK / _WALKERS / _WLOOKBACK /
# _WALK_AFTER / _WALK_EARLY / _SN_WALK / _SN_LOOKBACK / _SN_WLOOKBACK / _WPE / _WPE_LZ4)
LZ4V ?= base:-DLZ4PAR_HR=0
lz4v:
	@rm -rf $(OUT)/lz4v && mkdir -p $(OUT)/lz4v
	@for v in $(LZ4V); do name=$${v%%:*}; defs=$$(echo $${v#*:} | tr , ' '); \
	  $(HIPCC) $(HIPFLAGS) -Icsrc/include $$defs -shared -o $(OUT)/lz4v/$$name.so \
	    csrc/kernels/lz4par.hip || exit 1; done
.PHONY: lz4v

build/arrow_meta_fuzz: csrc/tests/arrow_meta_fuzz.cc csrc/engine/arrow_meta.cc
	@mkdir -p build
	$(CXX) -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all -o $@ $^ -lpthread

# the zstd decoder's host copy, host-only with ASan + UBSan (mutation test);
# built with the literals-only direct path on, so the mutants cover it too
build/zstd_fuzz: csrc/tests/zstd_fuzz.cc csrc/kernels/zstd.hip csrc/include/strom/strom.h
	@mkdir -p build
	$(HIPCC) -std=c++17 -O1 -g -Icsrc/include --offload-arch=$(ARCH) -DZS_LITDIRECT=1 \
	  -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
	  -Xarch_host -fno-sanitize-recover=all -fno-omit-frame-pointer \
	  -o $@ csrc/tests/zstd_fuzz.cc csrc/kernels/zstd.hip

# the block-parallel LZ4 / snappy decoder's host copy, host-only with ASan + UBSan
build/lz4par_fuzz: csrc/tests/lz4par_fuzz.cc csrc/kernels/lz4par.hip csrc/include/strom/strom.h
	@mkdir -p build
	$(HIPCC) -std=c++17 -O1 -g -Icsrc/include --offload-arch=$(ARCH) \
	  -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
	  -Xarch_host -fno-sanitize-recover=all -fno-omit-frame-pointer \
	  -o $@ csrc/tests/lz4par_fuzz.cc csrc/kernels/lz4par.hip

selftest: build/selftest build/selftest-asan build/selftest-tsan
	STROM_STAT_SHM=0 ./build/selftest && STROM_STAT_SHM=0 ./build/selftest-asan && STROM_STAT_SHM=0 TSAN_OPTIONS=report_signal_unsafe=0 ./build/selftest-tsan

.PHONY: selftest

# ---- kernel provider executed on the CPU ----------------------------------
# The real kmod/strom_*.c linked against the behavioural kernel model
# (kmod/testshim/kshim_rt.c) and driven by kmod/testshim/kmod_exec.c, plain,
# ASAN+UBSAN and TSAN (tests/test_kmod_exec_cpu.py).
KMOD_SRC  := $(wildcard kmod/strom_*.c) kmod/testshim/kshim_rt.c
KMOD_HDR  := $(wildcard kmod/*.h) $(wildcard kmod/testshim/*.h) csrc/include/strom/uapi.h
KSIM_KFLAGS := -std=gnu11 -g -D__KERNEL__ -Ikmod/testshim -Ikmod -Icsrc/include -Wall \
               -Wno-unused-function -Wno-address-of-packed-member
KSIM_UFLAGS := -std=gnu11 -g -Ikmod/testshim -Icsrc/include -Wall
KSIM_DRV  := kmod/testshim/kmod_exec.c

define ksim_build
	@mkdir -p build/ksim$(2)
	for f in $(KMOD_SRC); do $(1) $(KSIM_KFLAGS) $(3) -c $$f -o build/ksim$(2)/$$(basename $$f .c).o || exit 1; done
	$(1) $(KSIM_UFLAGS) $(3) -c $(KSIM_DRV) -o build/ksim$(2)/kmod_exec.o
	$(1) $(3) -o $@ build/ksim$(2)/*.o -lpthread
endef

build/kmod_exec: $(KMOD_SRC) $(KMOD_HDR) $(KSIM_DRV)
	$(call ksim_build,gcc,,-O1)

build/kmod_exec-asan: $(KMOD_SRC) $(KMOD_HDR) $(KSIM_DRV)
	$(call ksim_build,gcc,-asan,-O1 -fsanitize=address$(comma)undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined)

build/kmod_exec-tsan: $(KMOD_SRC) $(KMOD_HDR) $(KSIM_DRV)
	$(call ksim_build,$(ROCM)/llvm/bin/clang,-tsan,-O1 -fsanitize=thread)

comma := ,
# the same, as a library for the ctypes differential test against libstrom
build/libkmodsim.so: $(KMOD_SRC) $(KMOD_HDR)
	@mkdir -p build/ksim-so
	for f in $(KMOD_SRC); do gcc $(KSIM_KFLAGS) -O1 -fPIC -c $$f -o build/ksim-so/$$(basename $$f .c).o || exit 1; done
	gcc -shared -o $@ build/ksim-so/*.o -lpthread

kmod-exec: build/kmod_exec build/kmod_exec-asan build/kmod_exec-tsan
	./build/kmod_exec && ./build/kmod_exec-asan && TSAN_OPTIONS=halt_on_error=1 ./build/kmod_exec-tsan

.PHONY: kmod-exec
