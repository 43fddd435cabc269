# xrabit native build: host runtime (g++) + gfx950 HIP kernels (hipcc), linked against
# libamdhip64 and librccl.  Outputs land in-tree (rabit_amd/lib) so they travel with the
# repository snapshot to the GPU box.
#
#   make -j8            libraries (robust/base/mock/empty flavours, same names as rabit)
#   make tests          C++ unit-test and integration programs in build/bin
#   make lint           style / hygiene checks of C++, HIP and Python (tools/lint.py)
#   make doc            API reference docs/api.md from the sources (tools/gendoc.py)
#   make clean

ROCM      ?= /opt/rocm
CXX       ?= g++
HIPCC     ?= $(ROCM)/bin/hipcc
ARCH      ?= gfx950
OPT       ?= -O3
SAN       ?=

BUILD     := build
OBJ       := $(BUILD)/obj
LIBDIR    := rabit_amd/lib
BIN       := $(BUILD)/bin

INC       := -Icsrc/include -Icsrc/src -I$(ROCM)/include
CXXFLAGS  := $(OPT) -g -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -pthread \
             -D__HIP_PLATFORM_AMD__ $(INC) $(SAN)
HIPFLAGS  := $(OPT) -std=c++17 -fPIC --offload-arch=$(ARCH) -munsafe-fp-atomics $(INC)
# -z defs: a symbol declared but never defined fails the link, not the first dlopen
LDLIBS    := -Wl,-z,defs -L$(ROCM)/lib -lamdhip64 -lhsa-runtime64 -lrccl -lrocprofiler-sdk-roctx -pthread -Wl,-rpath,$(ROCM)/lib $(SAN)

CORE_SRCS := csrc/src/core/log.cc csrc/src/core/trace.cc csrc/src/core/exit.cc csrc/src/net/socket.cc csrc/src/net/tracker_client.cc csrc/src/net/link_reset.cc \
             csrc/src/coll/host_coll.cc csrc/src/coll/shm_coll.cc csrc/src/device/device_plane.cc csrc/src/device/device_checkpoint.cc csrc/src/device/dma_copier.cc csrc/src/device/peer_coll.cc csrc/src/device/peer_registry.cc csrc/src/device/host_stager.cc \
             csrc/src/engine/engine_base.cc csrc/src/engine/device_setup.cc csrc/src/engine/engine_robust.cc \
             csrc/src/engine/recovery.cc csrc/src/engine/local_replicas.cc csrc/src/engine/local_recovery.cc \
             csrc/src/capi/c_api.cc csrc/src/capi/build_info.cc
CORE_OBJS := $(patsubst csrc/src/%.cc,$(OBJ)/%.o,$(CORE_SRCS))
# every source of the libraries, in byte order; their sha256 is compiled into build_info.o
# (rabit_amd/_lib.py:source_hash computes the same over the working tree)
ALL_SRCS  := $(shell find csrc -type f \( -name '*.cc' -o -name '*.h' -o -name '*.hip' \) | LC_ALL=C sort)
KERN_OBJ  := $(OBJ)/device/kernels.o $(OBJ)/device/peer_kernels.o $(OBJ)/device/fused_allreduce.o
HEADERS   := $(shell find csrc -name '*.h')

FLAVOURS  := rabit rabit_base rabit_mock rabit_empty
LIBS      := $(foreach f,$(FLAVOURS),$(LIBDIR)/lib$(f).so) $(LIBDIR)/librabit_mock.a

.PHONY: all libs tests clean asan tsan lint doc
all: libs
libs: $(LIBS)

$(OBJ)/%.o: csrc/src/%.cc $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(OBJ)/device/%.o: csrc/src/device/%.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/capi/build_info.o: csrc/src/capi/build_info.cc $(ALL_SRCS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -DXRABIT_ARCH='"$(ARCH)"' \
	  -DXRABIT_SRC_HASH='"'"$$(cat $(ALL_SRCS) | sha256sum | cut -d' ' -f1)"'"' -c $< -o $@

# one registry object per flavour: only the default engine differs
$(OBJ)/registry_%.o: csrc/src/engine/registry.cc $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -DXRABIT_DEFAULT_ENGINE='"$*"' -c $< -o $@

$(LIBDIR)/librabit.so: $(CORE_OBJS) $(KERN_OBJ) $(OBJ)/registry_robust.o
	@mkdir -p $(LIBDIR)
	$(CXX) -shared -o $@ $^ $(LDLIBS)
$(LIBDIR)/librabit_base.so: $(CORE_OBJS) $(KERN_OBJ) $(OBJ)/registry_base.o
	@mkdir -p $(LIBDIR)
	$(CXX) -shared -o $@ $^ $(LDLIBS)
$(LIBDIR)/librabit_mock.so: $(CORE_OBJS) $(KERN_OBJ) $(OBJ)/registry_mock.o
	@mkdir -p $(LIBDIR)
	$(CXX) -shared -o $@ $^ $(LDLIBS)
$(LIBDIR)/librabit_empty.so: $(CORE_OBJS) $(KERN_OBJ) $(OBJ)/registry_empty.o
	@mkdir -p $(LIBDIR)
	$(CXX) -shared -o $@ $^ $(LDLIBS)
$(LIBDIR)/librabit_mock.a: $(CORE_OBJS) $(KERN_OBJ) $(OBJ)/registry_mock.o
	@mkdir -p $(LIBDIR)
	rm -f $@ && ar rcs $@ $^

# ---------------------------------------------------------------- test / example programs
TEST_PROGS := unit_tests recover_test speed_test basic broadcast lazy_allreduce device_reducer_test \
              rccl_lifecycle_test
tests: $(foreach p,$(TEST_PROGS),$(BIN)/$(p))

# -Wno-array-bounds -Wno-stringop-overflow: a test writes past a fixed buffer on purpose (the write throws first)
$(BIN)/unit_tests: tests/cpp/unit_tests.cc $(LIBDIR)/librabit_mock.a $(HEADERS)
	@mkdir -p $(BIN)
	$(CXX) $(CXXFLAGS) -Wno-array-bounds -Wno-stringop-overflow $< $(LIBDIR)/librabit_mock.a -o $@ $(LDLIBS)
# GPU test of the RCCL communicator lifecycle: drives DevicePlane directly (internal API)
$(BIN)/rccl_lifecycle_test: tests/cpp/rccl_lifecycle_test.cc $(LIBDIR)/librabit_mock.a $(HEADERS)
	@mkdir -p $(BIN)
	$(CXX) $(CXXFLAGS) $< $(LIBDIR)/librabit_mock.a -o $@ $(LDLIBS)
# a HIP program: the user's reduction is instantiated as a gfx950 kernel in its own TU
$(BIN)/device_reducer_test: tests/cpp/device_reducer_test.hip $(LIBDIR)/librabit_mock.so $(HEADERS)
	@mkdir -p $(BIN)
	$(HIPCC) $(HIPFLAGS) $< -o $@ -L$(LIBDIR) -lrabit_mock -Wl,-rpath,$(abspath $(LIBDIR)) $(LDLIBS)
$(BIN)/%: tests/cpp/%.cc $(LIBDIR)/librabit_mock.so $(HEADERS)
	@mkdir -p $(BIN)
	$(CXX) $(CXXFLAGS) $< -o $@ -L$(LIBDIR) -lrabit_mock -Wl,-rpath,$(abspath $(LIBDIR)) $(LDLIBS)
$(BIN)/%: examples/%.cc $(LIBDIR)/librabit.so $(HEADERS)
	@mkdir -p $(BIN)
	$(CXX) $(CXXFLAGS) $< -o $@ -L$(LIBDIR) -lrabit -Wl,-rpath,$(abspath $(LIBDIR)) $(LDLIBS)

# host sanitizer builds in their own tree (device code is not instrumented: GPU ASan / XNACK
# are not available on the target pool).  tests/test_sanitizers.py runs the results.
asan:
	$(MAKE) BUILD=build/asan LIBDIR=build/asan/lib OPT=-O1 \
	  SAN="-fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined" \
	  libs tests
tsan:
	$(MAKE) BUILD=build/tsan LIBDIR=build/tsan/lib OPT=-O1 SAN="-fsanitize=thread" libs tests

# the reference's `make lint` / `make doc` (Makefile:97-104) ran cpplint / pylint and
# Doxygen / Sphinx, none of which this image has: tools/lint.py and tools/gendoc.py do the job
lint:
	python3 tools/lint.py
doc:
	python3 tools/gendoc.py

clean:
	rm -rf $(BUILD) $(LIBDIR)/*.so $(LIBDIR)/*.a
