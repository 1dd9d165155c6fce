# Build for MI355X (gfx950).  `make` builds the product library and the CPU oracle.
#   lumo_amd/liblumo_amd.so   product: host scene builder (C++) + HIP wavefront kernels + C ABI
#   oracle/_build/liblumo_oracle.so   test infrastructure (CPU restatement), never linked by the product
# Strict IEEE f64: no FMA contraction anywhere (parity with the scalar restatement).

HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
ARCH     ?= gfx950
JOBS     ?= 8
FPFLAGS  := -ffp-contract=off -fno-fast-math
CXXFLAGS := -O2 -std=c++17 -fPIC $(FPFLAGS) -Wall -Wextra -Wno-unused-parameter
HIPFLAGS := -O3 -std=c++17 -fPIC $(FPFLAGS) --offload-arch=$(ARCH) -Wall -Wno-unused-parameter \
            -munsafe-fp-atomics

HOST_SRC := $(wildcard lumo_amd/csrc/host/*.cpp)
BUILD    ?= build
HOST_OBJ := $(patsubst lumo_amd/csrc/host/%.cpp,build/host/%.o,$(HOST_SRC))
# kernels.hip: host orchestration, C ABI and the non-traversal kernels.  The traversal kernels
# are instantiated once per kd stack class (launch.h STACK_CLASSES) in their own translation
# units, so they compile in parallel: inst_pt.hip / inst_bd.hip built with -DLUMO_STK=<class>.
STK_CLASSES := 0 4 8 16 24 32 48 64
DEV_OBJ  := $(BUILD)/device/kernels.o $(foreach k,$(STK_CLASSES),$(BUILD)/device/inst_pt_$(k).o $(BUILD)/device/inst_bd_$(k).o)
DEV_H    := $(wildcard lumo_amd/csrc/device/*.h)
COMMON_H := $(wildcard lumo_amd/csrc/common/*.h) include/lumo_amd.h include/lumo_host.h

LIB      ?= lumo_amd/liblumo_amd.so
ORACLE   := oracle/_build/liblumo_oracle.so
ORACLE_G := oracle/_build/liblumo_oracle_glibc.so

all: $(LIB) $(ORACLE) $(ORACLE_G)

build/host/%.o: lumo_amd/csrc/host/%.cpp $(COMMON_H) $(wildcard lumo_amd/csrc/host/*.h)
	@mkdir -p build/host
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(BUILD)/device/kernels.o: lumo_amd/csrc/device/kernels.hip $(COMMON_H) $(DEV_H)
	@mkdir -p $(BUILD)/device
	$(HIPCC) $(HIPFLAGS) $(DEVFLAGS) -c $< -o $@

$(BUILD)/device/inst_pt_%.o: lumo_amd/csrc/device/inst_pt.hip $(COMMON_H) $(DEV_H)
	@mkdir -p $(BUILD)/device
	$(HIPCC) $(HIPFLAGS) $(DEVFLAGS) -DLUMO_STK=$* -c $< -o $@

$(BUILD)/device/inst_bd_%.o: lumo_amd/csrc/device/inst_bd.hip $(COMMON_H) $(DEV_H)
	@mkdir -p $(BUILD)/device
	$(HIPCC) $(HIPFLAGS) $(DEVFLAGS) -DLUMO_STK=$* -c $< -o $@

$(LIB): $(HOST_OBJ) $(DEV_OBJ)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $^ -lpthread -lz

$(ORACLE): oracle/src/oracle.cpp oracle/oracle.h $(COMMON_H)
	@mkdir -p oracle/_build
	$(CXX) $(CXXFLAGS) -O2 -shared -o $@ oracle/src/oracle.cpp -lpthread

$(ORACLE_G): oracle/src/oracle.cpp oracle/oracle.h $(COMMON_H)
	@mkdir -p oracle/_build
	$(CXX) $(CXXFLAGS) -O2 -DLUMO_ORACLE_GLIBC -shared -o $@ oracle/src/oracle.cpp -lpthread

# Sanitizer build (CPU only): the host library sources and the oracle under ASan + UBSan, driven by
# tools/sanitize/main.cpp (scene builds, both integrators, textures, hostile PNG / HDR / OBJ input).
SAN_FLAGS := -O1 -g -std=c++17 $(FPFLAGS) -fsanitize=address,undefined -fno-sanitize-recover=all \
             -fno-omit-frame-pointer -Wall -Wno-unused-parameter
build/sanitize/lumo_sanitize: tools/sanitize/main.cpp $(HOST_SRC) oracle/src/oracle.cpp oracle/oracle.h $(COMMON_H) \
                              $(wildcard lumo_amd/csrc/host/*.h)
	@mkdir -p build/sanitize
	$(CXX) $(SAN_FLAGS) -o $@ tools/sanitize/main.cpp $(HOST_SRC) oracle/src/oracle.cpp -lpthread -lz

sanitize: build/sanitize/lumo_sanitize
	ASAN_OPTIONS=halt_on_error=1:detect_leaks=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
	    ./build/sanitize/lumo_sanitize

# A/B builds of the device code (perf experiments, loaded with LUMO_AMD_LIB=<path>):
#   make variant NAME=rs0 DEVFLAGS=-DLUMO_KD_REG=0   ->  lumo_amd/var/liblumo_amd_rs0.so
variant:
	@mkdir -p lumo_amd/var
	$(MAKE) BUILD=build/var_$(NAME) LIB=lumo_amd/var/liblumo_amd_$(NAME).so DEVFLAGS="$(DEVFLAGS)" lumo_amd/var/liblumo_amd_$(NAME).so


clean:
	rm -rf build $(LIB) oracle/_build lumo_amd/var

.PHONY: all clean variant sanitize
