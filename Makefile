# Build for AMD Instinct MI355X (gfx950). One build, backend chosen at run
# time (--backend rccl|cpu); no PROXY_ENABLE_* configurations.
#
# Reference equivalent: Makefile.common / Makefile.flags.mk / Makefile.<SYSTEM>
# (SURVEY.md C16-C18), which compiled one binary set per backend config.
#
#   make              # library + CLI binaries (+ *_loop aliases)
#   make lib          # dlnetbench_amd/_lib/libdlnb.so only
#   make clean
#   make ARCH=gfx950 HIPCC=/opt/rocm/bin/hipcc -j8

ROCM    ?= /opt/rocm
HIPCC   ?= $(ROCM)/bin/hipcc
ARCH    ?= gfx950
BUILD   ?= build
OPT     ?= -O3
CXXFLAGS = $(OPT) -std=c++17 -fPIC -Wall -Wno-unused-result -Icsrc/include --offload-arch=$(ARCH)
LDLIBS   = -L$(ROCM)/lib -lrccl -lamdhip64 -lpthread -lrt -Wl,-rpath,$(ROCM)/lib

LIB_SRCS := $(wildcard csrc/src/*.cpp) $(wildcard csrc/kernels/*.hip)
# host-only C++ (no device pass): the CPU backend's multiversioned SIMD loops
HOST_SRCS := $(wildcard csrc/host/*.cpp)
HOSTCXX  ?= $(ROCM)/llvm/bin/clang++
LIB_OBJS := $(patsubst csrc/%,$(BUILD)/obj/%.o,$(LIB_SRCS)) $(patsubst csrc/%,$(BUILD)/obj/%.o,$(HOST_SRCS))
APPS     := dp fsdp hybrid_2d hybrid_3d hybrid_3d_moe hybrid_cp hybrid_4d dlnb
LOOPS    := dp_loop fsdp_loop hybrid_2d_loop hybrid_3d_loop hybrid_3d_moe_loop hybrid_cp_loop hybrid_4d_loop
LIB      := $(BUILD)/libdlnb.so
PYLIB    := dlnetbench_amd/_lib/libdlnb.so

.PHONY: all lib apps clean asan tsan probes
all: lib apps

lib: $(PYLIB)

$(BUILD)/obj/host/%.o: csrc/host/%
	@mkdir -p $(dir $@)
	$(HOSTCXX) $(subst -Xarch_host,,$(OPT)) -std=c++17 -fPIC -Wall -Icsrc/include -MMD -MP -c $< -o $@

$(BUILD)/obj/%.o: csrc/%
	@mkdir -p $(dir $@)
	$(HIPCC) $(CXXFLAGS) -MMD -MP -c $< -o $@

# header dependencies (every object is rebuilt when a header it includes changes)
-include $(LIB_OBJS:.o=.d)

$(LIB): $(LIB_OBJS)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $^ $(LDLIBS) -Wl,-soname,libdlnb.so

$(PYLIB): $(LIB)
	@mkdir -p $(dir $@)
	cp $< $@

apps: $(addprefix $(BUILD)/bin/,$(APPS)) $(addprefix $(BUILD)/bin/,$(LOOPS))

$(BUILD)/bin/%: csrc/apps/%.cpp $(LIB) $(wildcard csrc/include/dlnb/*.hpp)
	@mkdir -p $(dir $@)
	$(HIPCC) $(CXXFLAGS) $< -o $@ -L$(BUILD) -ldlnb $(LDLIBS) -Wl,-rpath,'$$ORIGIN/..'

# The reference builds separate *_loop binaries with -DPROXY_LOOP; here the
# same binary switches to loop mode when invoked under a *_loop name.
$(BUILD)/bin/%_loop: $(BUILD)/bin/%
	ln -sf $(notdir $<) $@

# Small measurement programs (scripts/probes/*.cpp) linked against the library.
probes: $(BUILD)/bin/boundary_cost
$(BUILD)/bin/boundary_cost: scripts/probes/boundary_cost.cpp $(LIB)
	@mkdir -p $(dir $@)
	$(HIPCC) $(CXXFLAGS) $< -o $@ -L$(BUILD) -ldlnb $(LDLIBS) -Wl,-rpath,'$$ORIGIN/..'

# Host AddressSanitizer build of the library + binaries into build-asan/
# (device code is not instrumented: GPU ASan is not available on the pool).
asan:
	$(MAKE) BUILD=build-asan OPT="-O1 -g -fno-omit-frame-pointer -Xarch_host -fsanitize=address" \
	  LDLIBS="$(LDLIBS) -fsanitize=address" PYLIB=build-asan/unused.so apps

# Host ThreadSanitizer build into build-tsan/: the loopback backend's rank
# threads, the CPU device's worker-thread streams and the energy sampler.
tsan:
	$(MAKE) BUILD=build-tsan OPT="-O1 -g -fno-omit-frame-pointer -Xarch_host -fsanitize=thread" \
	  LDLIBS="$(LDLIBS) -fsanitize=thread" PYLIB=build-tsan/unused.so apps

clean:
	rm -rf $(BUILD) build-asan build-tsan $(PYLIB)
