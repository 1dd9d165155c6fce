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
DEV_SRC  := $(wildcard lumo_amd/csrc/device/*.hip)
DEV_OBJ  := $(patsubst lumo_amd/csrc/device/%.hip,build/device/%.o,$(DEV_SRC))
COMMON_H := $(wildcard lumo_amd/csrc/common/*.h) include/lumo_amd.h include/lumo_host.h

LIB      := lumo_amd/liblumo_amd.so
ORACLE   := oracle/_build/liblumo_oracle.so
ORACLE_G := oracle/_build/liblumo_oracle_glibc.so

all: $(LIB) $(ORACLE) $(ORACLE_G)

build/host/%.o: lumo_amd/csrc/host/%.cpp $(COMMON_H) $(wildcard lumo_amd/csrc/host/*.h)
	@mkdir -p build/host
	$(CXX) $(CXXFLAGS) -c $< -o $@

build/device/%.o: lumo_amd/csrc/device/%.hip $(COMMON_H) $(wildcard lumo_amd/csrc/device/*.h)
	@mkdir -p build/device
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(HOST_OBJ) $(DEV_OBJ)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $^ -lpthread

$(ORACLE): oracle/src/oracle.cpp oracle/oracle.h $(COMMON_H)
	@mkdir -p oracle/_build
	$(CXX) $(CXXFLAGS) -O2 -shared -o $@ oracle/src/oracle.cpp -lpthread

$(ORACLE_G): oracle/src/oracle.cpp oracle/oracle.h $(COMMON_H)
	@mkdir -p oracle/_build
	$(CXX) $(CXXFLAGS) -O2 -DLUMO_ORACLE_GLIBC -shared -o $@ oracle/src/oracle.cpp -lpthread

# A/B variants of the device code (perf experiments): lumo_amd/liblumo_amd_<name>.so
VARIANTS ?= lb4:-DLUMO_TRAVERSAL_WAVES=4 noinl:-DLUMO_NOINLINE_KD
variants: $(HOST_OBJ)
	@for v in $(VARIANTS); do n=$${v%%:*}; f=$${v#*:}; f=$$(echo $$f | tr ',' ' '); \
	  echo "variant $$n: $$f"; \
	  $(HIPCC) $(HIPFLAGS) $$f -c lumo_amd/csrc/device/kernels.hip -o build/device/kernels_$$n.o && \
	  $(HIPCC) -shared --offload-arch=$(ARCH) -o lumo_amd/liblumo_amd_$$n.so $(HOST_OBJ) build/device/kernels_$$n.o -lpthread; done

clean:
	rm -rf build $(LIB) oracle/_build

.PHONY: all clean variants
