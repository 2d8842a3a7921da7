# libsplinter_amd native build (host C++ with g++, device code with hipcc for gfx950).
# Outputs stay in-tree (libsplinter_amd/lib, libsplinter_amd/bin) so they travel
# with the repo snapshot to the GPU box; every link writes NAME.tmp and renames it into place, so a
# snapshot taken during a build never holds a half-written library.
CXX      ?= g++
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG      := libsplinter_amd
SRC      := $(PKG)/csrc
LIB      := $(PKG)/lib
BIN      := $(PKG)/bin
BUILD_ID := $(shell git rev-parse --short HEAD 2>/dev/null || echo dev)

CXXFLAGS := -O3 -std=c++17 -Wall -Wextra -fPIC -D_GNU_SOURCE -I$(SRC)/include -I$(SRC)/core \
            -DSPL_BUILD_ID=\"$(BUILD_ID)\"
HIPFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -D_GNU_SOURCE -I$(SRC)/include -I$(SRC)/core \
            -I$(SRC)/hip -Wno-unused-result -munsafe-fp-atomics
LDLIBS   := -ldl -lrt -lpthread

CORE_SRCS := $(SRC)/core/store_host.cpp $(SRC)/core/node_store.cpp $(SRC)/core/capi.cpp $(SRC)/core/wordpiece.cpp $(SRC)/core/batch_host.cpp
CORE_HDRS := $(wildcard $(SRC)/include/*.h $(SRC)/include/*.hpp $(SRC)/core/*.hpp)
HIP_SRCS  := $(wildcard $(SRC)/hip/*.hip)
HIP_HDRS  := $(wildcard $(SRC)/hip/*.hpp) $(CORE_HDRS)
HIP_OBJS  := $(patsubst $(SRC)/hip/%.hip,build/hip/%.o,$(HIP_SRCS))

HOST_LIBS := $(LIB)/libsplinter.so $(LIB)/libsplinter_p.so
TOOLS     := $(patsubst $(SRC)/tools/%.cpp,$(BIN)/%,$(wildcard $(SRC)/tools/*.cpp)) \
             $(if $(wildcard $(SRC)/cli/*.cpp),$(BIN)/splinterctl)

.PHONY: all host hip tools clean test tsan asan hip-variant
all: host hip tools
host: $(HOST_LIBS)
hip: $(LIB)/libsplinter_hip.so
tools: $(TOOLS)

$(LIB) $(BIN) build/hip:
	mkdir -p $@

$(LIB)/libsplinter.so: $(CORE_SRCS) $(CORE_HDRS) | $(LIB)
	$(CXX) $(CXXFLAGS) -shared -o $@.tmp $(CORE_SRCS) $(LDLIBS) && mv -f $@.tmp $@

$(LIB)/libsplinter_p.so: $(CORE_SRCS) $(CORE_HDRS) | $(LIB)
	$(CXX) $(CXXFLAGS) -DSPLINTER_PERSISTENT -shared -o $@.tmp $(CORE_SRCS) $(LDLIBS) && mv -f $@.tmp $@

build/hip/%.o: $(SRC)/hip/%.hip $(HIP_HDRS) | build/hip
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

# attention: keep MFMA accumulators in VGPRs (the default AGPR form costs 128 v_accvgpr copies per
# K/V tile around the online-softmax rescale); per file: the flag crashes the compiler on
# search_kernels.hip (ROCm 7.2)
build/hip/nomic_kernels.o: HIPFLAGS += -mllvm -amdgpu-mfma-vgpr-form -fno-honor-nans
build/hip/decoder_kernels.o: HIPFLAGS += -mllvm -amdgpu-mfma-vgpr-form

$(LIB)/libsplinter_hip.so: $(HIP_OBJS) $(LIB)/libsplinter.so | $(LIB)
	$(HIPCC) $(HIPFLAGS) -shared -o $@.tmp $(HIP_OBJS) -L$(LIB) -lsplinter -Wl,-rpath,'$$ORIGIN' $(LDLIBS) && mv -f $@.tmp $@

# A/B builds of the HIP backend for one process-level switch (SPLINTER_HIP_VARIANT=<V> loads
# lib/libsplinter_hip_<V>.so): make hip-variant V=name VFLAGS="-DSOMETHING"
hip-variant: $(LIB)/libsplinter.so | $(LIB)
	mkdir -p build/hip_$(V)
	for f in $(HIP_SRCS); do o=build/hip_$(V)/$$(basename $$f .hip).o; x=""; \
	  case $$f in *nomic_kernels.hip) x="-mllvm -amdgpu-mfma-vgpr-form -fno-honor-nans";; *decoder_kernels.hip) x="-mllvm -amdgpu-mfma-vgpr-form";; esac; \
	  $(HIPCC) $(HIPFLAGS) $$x $(VFLAGS) -c -o $$o $$f || exit 1; done
	$(HIPCC) $(HIPFLAGS) -shared -o $(LIB)/libsplinter_hip_$(V).so build/hip_$(V)/*.o -L$(LIB) -lsplinter \
	  -Wl,-rpath,'$$ORIGIN' $(LDLIBS)

$(BIN)/%: $(SRC)/tools/%.cpp $(LIB)/libsplinter.so $(CORE_HDRS) | $(BIN)
	$(CXX) $(CXXFLAGS) -o $@.tmp $< -L$(LIB) -lsplinter -Wl,-rpath,'$$ORIGIN/../lib' $(LDLIBS) && mv -f $@.tmp $@

$(BIN)/splinterctl: $(wildcard $(SRC)/cli/*.cpp $(SRC)/cli/*.hpp) $(LIB)/libsplinter.so | $(BIN)
	$(CXX) $(CXXFLAGS) -I$(SRC)/cli -o $@.tmp $(filter %.cpp,$^) -L$(LIB) -lsplinter -Wl,-rpath,'$$ORIGIN/../lib' $(LDLIBS) && mv -f $@.tmp $@
	ln -sf splinterctl $(BIN)/splinter_cli

test: host tools
	$(BIN)/splinter_test

# ThreadSanitizer builds of the host store + TAP/stress tools (SURVEY §5 race detection);
# the seqlock payload copies are the only exempt accesses (store_host.cpp seq_copy).
TSAN_TOOLS := $(BIN)/tsan/splinter_test $(BIN)/tsan/splinter_stress $(BIN)/tsan/splinter_chi_sao
tsan: $(TSAN_TOOLS)
$(BIN)/tsan:
	mkdir -p $@
$(BIN)/tsan/%: $(SRC)/tools/%.cpp $(CORE_SRCS) $(CORE_HDRS) | $(BIN)/tsan
	$(CXX) -O1 -g -std=c++17 -fsanitize=thread -Wno-tsan -fPIC -D_GNU_SOURCE -I$(SRC)/include -I$(SRC)/core \
	  -o $@ $< $(CORE_SRCS) $(LDLIBS)

# AddressSanitizer + UndefinedBehaviorSanitizer builds of the host store, the TAP / stress tools and
# the CLI (with its Lua and WASM interpreters): the memory-error checks the reference runs as
# valgrind memcheck ctests (reference CMakeLists.txt:316-329).  Host code only (-fno-gpu-sanitize
# is implied: these are g++ builds; libsplinter_hip.so is never loaded by them).
ASAN_FLAGS := -O1 -g -std=c++17 -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined \
              -fPIC -D_GNU_SOURCE -I$(SRC)/include -I$(SRC)/core -DSPL_BUILD_ID=\"asan\"
ASAN_TOOLS := $(BIN)/asan/splinter_test $(BIN)/asan/splinter_stress $(BIN)/asan/splinter_chi_sao \
              $(BIN)/asan/splinterctl $(BIN)/asan/splinter_hostapi_bench
asan: $(ASAN_TOOLS)
$(BIN)/asan:
	mkdir -p $@
$(BIN)/asan/splinterctl: $(wildcard $(SRC)/cli/*.cpp $(SRC)/cli/*.hpp) $(CORE_SRCS) $(CORE_HDRS) | $(BIN)/asan
	$(CXX) $(ASAN_FLAGS) -I$(SRC)/cli -o $@ $(filter %.cpp,$^) $(LDLIBS)
	ln -sf splinterctl $(BIN)/asan/splinter_cli
$(BIN)/asan/%: $(SRC)/tools/%.cpp $(CORE_SRCS) $(CORE_HDRS) | $(BIN)/asan
	$(CXX) $(ASAN_FLAGS) -o $@ $< $(CORE_SRCS) $(LDLIBS)

clean:
	rm -rf build $(LIB)/*.so $(BIN)
