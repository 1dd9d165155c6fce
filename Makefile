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
HOST_OBJ := $(patsubst lumo_amd/csrc/host/%.cpp,build/host/%.o,$(HOST_SRC))
# kernels.hip: host orchestration, C ABI and the non-traversal kernels.  The traversal kernels
# are instantiated once per kd stack class (launch.h STACK_CLASSES) in their own translation
# units, so they compile in parallel: inst_pt.hip / inst_bd.hip built with -DLUMO_STK=<class>.
STK_CLASSES := 4 8 16 24 32 48 64
DEV_OBJ  := build/device/kernels.o $(foreach k,$(STK_CLASSES),build/device/inst_pt_$(k).o build/device/inst_bd_$(k).o)
DEV_H    := $(wildcard lumo_amd/csrc/device/*.h)
COMMON_H := $(wildcard lumo_amd/csrc/common/*.h) include/lumo_amd.h include/lumo_host.h

LIB      := lumo_amd/liblumo_amd.so
ORACLE   := oracle/_build/liblumo_oracle.so
ORACLE_G := oracle/_build/liblumo_oracle_glibc.so

all: $(LIB) $(ORACLE) $(ORACLE_G)

build/host/%.o: lumo_amd/csrc/host/%.cpp $(COMMON_H) $(wildcard lumo_amd/csrc/host/*.h)
	@mkdir -p build/host
	$(CXX) $(CXXFLAGS) -c $< -o $@

build/device/kernels.o: lumo_amd/csrc/device/kernels.hip $(COMMON_H) $(DEV_H)
	@mkdir -p build/device
	$(HIPCC) $(HIPFLAGS) $(DEVFLAGS) -c $< -o $@

build/device/inst_pt_%.o: lumo_amd/csrc/device/inst_pt.hip $(COMMON_H) $(DEV_H)
	@mkdir -p build/device
	$(HIPCC) $(HIPFLAGS) $(DEVFLAGS) -DLUMO_STK=$* -c $< -o $@

build/device/inst_bd_%.o: lumo_amd/csrc/device/inst_bd.hip $(COMMON_H) $(DEV_H)
	@mkdir -p build/device
	$(HIPCC) $(HIPFLAGS) $(DEVFLAGS) -DLUMO_STK=$* -c $< -o $@

$(LIB): $(HOST_OBJ) $(DEV_OBJ)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $^ -lpthread

$(ORACLE): oracle/src/oracle.cpp oracle/oracle.h $(COMMON_H)
	@mkdir -p oracle/_build
	$(CXX) $(CXXFLAGS) -O2 -shared -o $@ oracle/src/oracle.cpp -lpthread

$(ORACLE_G): oracle/src/oracle.cpp oracle/oracle.h $(COMMON_H)
	@mkdir -p oracle/_build
	$(CXX) $(CXXFLAGS) -O2 -DLUMO_ORACLE_GLIBC -shared -o $@ oracle/src/oracle.cpp -lpthread

# DEVFLAGS: extra device defines for A/B builds, e.g. make DEVFLAGS=-DLUMO_TRAVERSAL_WAVES=4

clean:
	rm -rf build $(LIB) oracle/_build

.PHONY: all clean
