# mireduce native build (gfx950 / MI355X). Replaces the reference's cuda/C/common/common.mk +
# cuda/C/src/reduction/Makefile (sm_10/13/20) and mpi/Makefile (mpixlc / mpicc).
#
#   make            shared library (build/lib/libmireduce.so: every kernel + the host runtime), the python
#                   extension and the apps (reduction, reduce_xgmi, bandwidth_test, reduce_mpi), all linked
#                   against that one library — the kernel table is not embedded in every binary
#   make static     build/lib/libmireduce.a (the same objects, for static consumers)
#   make python     only the python extension (cuda_mpi_reductions_amd/_C*.so)
#   make asan       host-code ASan/UBSan build of the CPU-only apps + unit tests (GPU code untouched)
#   make tsan       ThreadSanitizer build of the threaded host reference reducers (race_unit)
#   make clean
#
# Variables: ARCH=gfx950  DEBUG=1  MPI_HOME=/opt/conda  SAVE_TEMPS=1 (keep .s for inspection)

ARCH      ?= gfx950
ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
HOSTCXX   ?= $(ROCM)/lib/llvm/bin/clang++
MPI_HOME  ?= /opt/conda
PYTHON    ?= python3
BUILD     ?= build

OPT       := $(if $(DEBUG),-O0 -g,-O3)
CXXSTD    := -std=c++17
INCLUDES  := -Icsrc/include -I$(BUILD)/gen -I$(ROCM)/include
WARN      := -Wall -Wno-unused-result
COMMON    := $(CXXSTD) $(OPT) $(WARN) -fPIC $(INCLUDES)
HIPFLAGS  := $(COMMON) -x hip --offload-arch=$(ARCH) -munsafe-fp-atomics $(if $(SAVE_TEMPS),-save-temps=obj,)
HOSTFLAGS := $(COMMON) -D__HIP_PLATFORM_AMD__
LDLIBS    := -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64 -lrocprofiler-sdk-roctx -lpthread

PY_INC    := $(shell $(PYTHON) -c "import sysconfig; print(sysconfig.get_paths()['include'])")
PYBIND_INC:= $(shell $(PYTHON) -c "import pybind11; print(pybind11.get_include())")
PY_EXT    := $(shell $(PYTHON) -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYEXT     := cuda_mpi_reductions_amd/_C$(PY_EXT)

KERNEL_SRC  := $(wildcard csrc/kernels/*.hip)
RUNTIME_SRC := $(wildcard csrc/runtime/*.cpp)
COMM_SRC    := $(wildcard csrc/comm/*.cpp)
COMM_HIP    := $(wildcard csrc/comm/*.hip)

KERNEL_OBJ  := $(patsubst csrc/%.hip,$(BUILD)/obj/%.o,$(KERNEL_SRC))
RUNTIME_OBJ := $(patsubst csrc/%.cpp,$(BUILD)/obj/%.o,$(RUNTIME_SRC))
COMM_OBJ    := $(patsubst csrc/%.cpp,$(BUILD)/obj/%.o,$(COMM_SRC)) $(patsubst csrc/%.hip,$(BUILD)/obj/%.o,$(COMM_HIP))
LIB         := $(BUILD)/lib/libmireduce.a
SHLIB       := $(BUILD)/lib/libmireduce.so
COMMLIB     := $(BUILD)/lib/libmireduce_comm.a
# binaries in build/bin and the extension in cuda_mpi_reductions_amd/ find the library next to them
LINK_BIN    := -L$(BUILD)/lib -lmireduce -Wl,-rpath,'$$ORIGIN/../lib'
LINK_PY     := -L$(BUILD)/lib -lmireduce -Wl,-rpath,'$$ORIGIN/../$(BUILD)/lib'

APPS := $(BUILD)/bin/reduction $(BUILD)/bin/reduce_xgmi $(BUILD)/bin/bandwidth_test
MPI_APP := $(BUILD)/bin/reduce_mpi

.PHONY: all python apps mpi clean asan tsan unit diag examples window_ab dyntail_ab i32sum_ab launch_floor static shared
static: $(LIB)
shared: $(SHLIB)
all: python apps mpi unit diag examples

python: $(PYEXT)
apps: $(APPS)
mpi: $(MPI_APP)

HEADERS := $(wildcard csrc/include/mireduce/*.hpp) $(wildcard csrc/kernels/*.hpp)

$(BUILD)/obj/%.o: csrc/%.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/obj/%.o: csrc/%.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(HOSTCXX) $(HOSTFLAGS) -c $< -o $@

# Build provenance (csrc/include/mireduce/version.hpp): the source hash header is regenerated on
# every make but replaced only when the hash changed, so version.o (and the links) rebuild exactly
# when some csrc file did.
SRC_HASH_H := $(BUILD)/gen/mireduce_source_hash.h
.PHONY: FORCE
FORCE:
$(SRC_HASH_H): FORCE
	@mkdir -p $(dir $@)
	@$(PYTHON) tools/source_hash.py --header > $@.tmp && { cmp -s $@.tmp $@ || mv $@.tmp $@; }; rm -f $@.tmp
$(BUILD)/obj/runtime/version.o: $(SRC_HASH_H)

# core: kernels + host runtime (no RCCL: the python extension shares a process with torch's RCCL)
$(LIB): $(KERNEL_OBJ) $(RUNTIME_OBJ)
	@mkdir -p $(dir $@)
	rm -f $@
	ar rcs $@ $^

$(SHLIB): $(KERNEL_OBJ) $(RUNTIME_OBJ)
	@mkdir -p $(dir $@)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $^ -Wl,-soname,libmireduce.so $(LDLIBS) -o $@

$(COMMLIB): $(COMM_OBJ)
	@mkdir -p $(dir $@)
	rm -f $@
	ar rcs $@ $^

$(BUILD)/obj/python/module.o: csrc/python/module.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(HOSTCXX) $(HOSTFLAGS) -I$(PY_INC) -I$(PYBIND_INC) -fvisibility=hidden -c $< -o $@

$(PYEXT): $(BUILD)/obj/python/module.o $(SHLIB)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $< $(LINK_PY) $(LDLIBS) -o $@

$(BUILD)/bin/%: csrc/apps/%.cpp $(SHLIB) $(COMMLIB) $(HEADERS)
	@mkdir -p $(dir $@)
	$(HOSTCXX) $(HOSTFLAGS) $< -Wl,--whole-archive $(COMMLIB) -Wl,--no-whole-archive $(LINK_BIN) \
	    -L$(ROCM)/lib -lrccl $(LDLIBS) -o $@

# reduce.c parity app: plain C++ against MPICH (CPU buffers only; no HIP needed).
MPI_SRCS := csrc/apps/reduce_mpi.cpp csrc/runtime/fault.cpp csrc/runtime/mt19937.cpp csrc/runtime/cli.cpp csrc/runtime/report.cpp csrc/runtime/timer.cpp csrc/runtime/types.cpp csrc/runtime/version.cpp
$(MPI_APP): $(MPI_SRCS) $(HEADERS) $(SRC_HASH_H)
	@mkdir -p $(dir $@)
	g++ $(CXXSTD) -O3 -Wall -Icsrc/include -I$(BUILD)/gen -DMIREDUCE_NO_HIP -I$(MPI_HOME)/include \
	    $(MPI_SRCS) -static-libstdc++ -static-libgcc $(MPI_HOME)/lib/libmpi.so -Wl,-rpath,$(MPI_HOME)/lib -o $@

# Diagnostic: per-workgroup timeline of streaming-body variants (docs/TUNING.md).
diag: $(BUILD)/bin/wg_timeline
$(BUILD)/bin/wg_timeline: tools/wg_timeline.hip
	@mkdir -p $(dir $@)
	$(HIPCC) -std=c++17 -O3 --offload-arch=$(ARCH) $< -o $@

# Production-kernel A/B of the streaming body's load schedule (profiles/r3_window/).
window_ab: $(BUILD)/bin/window_ab
$(BUILD)/obj/tools/window_ab.o: tools/window_ab.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@
$(BUILD)/bin/window_ab: $(BUILD)/obj/tools/window_ab.o $(SHLIB)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) $< $(LINK_BIN) $(LDLIBS) -o $@

# Experiment: a workgroup-level dynamic tail vs the static XCD-weighted split (tools/dyntail_ab.hip).
dyntail_ab: $(BUILD)/bin/dyntail_ab
$(BUILD)/obj/tools/dyntail_ab.o: tools/dyntail_ab.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@
$(BUILD)/bin/dyntail_ab: $(BUILD)/obj/tools/dyntail_ab.o $(SHLIB)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) $< $(LINK_BIN) $(LDLIBS) -o $@

# Where the per-launch fixed cost goes: empty / args / fan-in-only kernels vs the production
# reduction, graph-replayed (tools/launch_floor.hip).
launch_floor: $(BUILD)/bin/launch_floor
$(BUILD)/obj/tools/launch_floor.o: tools/launch_floor.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@
$(BUILD)/bin/launch_floor: $(BUILD)/obj/tools/launch_floor.o $(SHLIB)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) $< $(LINK_BIN) $(LDLIBS) -o $@

# Experiment: int32 SUM with dot2 half-sums (tools/i32sum_ab.hip).
i32sum_ab: $(BUILD)/bin/i32sum_ab
$(BUILD)/obj/tools/i32sum_ab.o: tools/i32sum_ab.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@
$(BUILD)/bin/i32sum_ab: $(BUILD)/obj/tools/i32sum_ab.o $(SHLIB)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) $< $(LINK_BIN) $(LDLIBS) -o $@

# C++ library consumer example (examples/cpp_consumer; the CMake build links it via find_package).
examples: $(BUILD)/bin/cpp_consumer
$(BUILD)/bin/cpp_consumer: examples/cpp_consumer/main.cpp $(SHLIB) $(HEADERS)
	@mkdir -p $(dir $@)
	$(HOSTCXX) $(HOSTFLAGS) $< $(LINK_BIN) $(LDLIBS) -o $@

# Native unit tests (host code only) and the bootstrap multi-process test.
UNIT := $(BUILD)/bin/host_unit $(BUILD)/bin/bootstrap_test
unit: $(UNIT)

UNIT_SRCS := $(filter-out csrc/apps/reduce_mpi.cpp,$(MPI_SRCS)) csrc/runtime/peer_access.cpp
$(BUILD)/bin/host_unit: tests/native/host_unit.cpp $(UNIT_SRCS) $(HEADERS)
	@mkdir -p $(dir $@)
	g++ $(CXXSTD) -O2 -Wall -Icsrc/include -I$(BUILD)/gen -DMIREDUCE_NO_HIP tests/native/host_unit.cpp \
	    $(UNIT_SRCS) -o $@

$(BUILD)/bin/bootstrap_test: tests/native/bootstrap_test.cpp $(COMMLIB) $(SHLIB) $(HEADERS)
	@mkdir -p $(dir $@)
	$(HOSTCXX) $(HOSTFLAGS) $< -Wl,--whole-archive $(COMMLIB) -Wl,--no-whole-archive $(LINK_BIN) \
	    -L$(ROCM)/lib -lrccl $(LDLIBS) -o $@

# Host sanitizers: CPU-only code paths under ASan+UBSan.
asan: csrc/apps/reduce_mpi.cpp
	@mkdir -p $(BUILD)/asan
	g++ $(CXXSTD) -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -Icsrc/include -I$(BUILD)/gen -DMIREDUCE_NO_HIP \
	    -I$(MPI_HOME)/include $(MPI_SRCS) -static-libstdc++ -static-libgcc $(MPI_HOME)/lib/libmpi.so -Wl,-rpath,$(MPI_HOME)/lib \
	    -o $(BUILD)/asan/reduce_mpi
	g++ $(CXXSTD) -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -Icsrc/include -I$(BUILD)/gen -DMIREDUCE_NO_HIP \
	    tests/native/host_unit.cpp $(UNIT_SRCS) -o $(BUILD)/asan/host_unit

# Race detection: the threaded host reference reducers / arg-reductions under
# ThreadSanitizer (tests/native/race_unit.cpp; exits non-zero on any report).
TSAN_SRCS := csrc/runtime/cpu_reference.cpp csrc/runtime/arg_reduce_cpu.cpp csrc/runtime/types.cpp
tsan: $(BUILD)/tsan/race_unit
$(BUILD)/tsan/race_unit: tests/native/race_unit.cpp $(TSAN_SRCS) $(HEADERS)
	@mkdir -p $(dir $@)
	g++ $(CXXSTD) -O1 -g -fsanitize=thread -fno-omit-frame-pointer -Icsrc/include -I$(ROCM)/include \
	    -D__HIP_PLATFORM_AMD__ -DMIREDUCE_NO_HIP tests/native/race_unit.cpp $(TSAN_SRCS) -o $@

clean:
	rm -rf $(BUILD) $(PYEXT)
