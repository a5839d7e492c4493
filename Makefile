# Top-level build (no cmake): everything lands in tempi_amd/lib/.
#   libtempi_hip.so : gfx950 HIP kernels + HIP runtime C ABI (include/tempi_hip.h)
#   libtempi.so     : the MPI interposer, C++17, links libtempi_hip + the MPI library
#   oracle          : CPU restatement used by tests only (oracle/Makefile)
MPI_HOME ?= /opt/conda
ROCM ?= /opt/rocm
LIB := tempi_amd/lib
HIPCC := $(ROCM)/bin/hipcc
JOBS ?= 8

HIP_SRC := $(wildcard tempi_amd/csrc/hip/*.hip)
CORE_SRC := $(wildcard tempi_amd/csrc/core/*.cpp)
CORE_HDR := $(wildcard tempi_amd/csrc/core/*.hpp) $(wildcard include/*.h)
CORE_OBJ := $(patsubst tempi_amd/csrc/core/%.cpp,build/core/%.o,$(CORE_SRC))
HIP_OBJ := $(patsubst tempi_amd/csrc/hip/%.hip,build/hip/%.o,$(HIP_SRC))

HIPFLAGS := --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Wall
CXXFLAGS := -std=c++17 -O2 -g1 -fPIC -fvisibility=hidden -Wall -Wextra -Wno-unused-parameter \
            -Iinclude -I$(MPI_HOME)/include

APPS := $(LIB)/libtempi_apps.so $(LIB)/halo_exchange $(LIB)/pingpong_nd $(LIB)/pingpong_1d $(LIB)/alltoallv_sparse \
        $(LIB)/measure_system \
        $(LIB)/type_commit $(LIB)/mpi_pack $(LIB)/mpi_isend $(LIB)/pack_bench

all: $(LIB)/libtempi.so $(APPS) oracle

build/hip/%.o: tempi_amd/csrc/hip/%.hip include/tempi_hip.h
	@mkdir -p build/hip
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB)/libtempi_hip.so: $(HIP_OBJ)
	@mkdir -p $(LIB)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $^ -Wl,-rpath,$(ROCM)/lib

build/core/%.o: tempi_amd/csrc/core/%.cpp $(CORE_HDR)
	@mkdir -p build/core
	g++ $(CXXFLAGS) -c $< -o $@

# libstdc++ is linked statically and hidden: the MPI library's directory
# (/opt/conda/lib) is on our RUNPATH and carries an older libstdc++
$(LIB)/libtempi.so: $(CORE_OBJ) $(LIB)/libtempi_hip.so
	g++ -shared -o $@ $(CORE_OBJ) -L$(LIB) -ltempi_hip $(MPI_HOME)/lib/libmpi.so -ldl -lpthread \
	    -static-libstdc++ -static-libgcc -Wl,--exclude-libs,ALL \
	    -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(MPI_HOME)/lib -Wl,--enable-new-dtags

# applications link -ltempi BEFORE the MPI library, like any TEMPI user
$(LIB)/libtempi_apps.so: apps/halo_lib.cpp apps/bench_lib.cpp $(LIB)/libtempi.so
	$(HIPCC) --offload-arch=gfx950 -O2 -std=c++17 -fPIC -shared -Iinclude -I$(MPI_HOME)/include -o $@ apps/halo_lib.cpp apps/bench_lib.cpp \
	    -L$(LIB) -ltempi -ltempi_hip -L$(MPI_HOME)/lib -lmpi -static-libstdc++ -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(MPI_HOME)/lib

$(LIB)/halo_exchange: apps/halo_exchange_main.cpp $(LIB)/libtempi_apps.so
	$(HIPCC) --offload-arch=gfx950 -O2 -std=c++17 -Iinclude -I$(MPI_HOME)/include -o $@ $< -L$(LIB) -ltempi_apps \
	    -ltempi -ltempi_hip -L$(MPI_HOME)/lib -lmpi -static-libstdc++ -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(MPI_HOME)/lib

$(LIB)/pingpong_nd: apps/pingpong_nd.cpp $(LIB)/libtempi_apps.so
	$(HIPCC) --offload-arch=gfx950 -O2 -std=c++17 -Iinclude -I$(MPI_HOME)/include -o $@ $< -L$(LIB) -ltempi_apps \
	    -ltempi -ltempi_hip -L$(MPI_HOME)/lib -lmpi -static-libstdc++ -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(MPI_HOME)/lib

$(LIB)/pingpong_1d: apps/pingpong_1d.cpp $(LIB)/libtempi_apps.so
	$(HIPCC) --offload-arch=gfx950 -O2 -std=c++17 -Iinclude -I$(MPI_HOME)/include -o $@ $< -L$(LIB) -ltempi_apps \
	    -ltempi -ltempi_hip -L$(MPI_HOME)/lib -lmpi -static-libstdc++ -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(MPI_HOME)/lib

$(LIB)/alltoallv_sparse: apps/alltoallv_sparse.cpp $(LIB)/libtempi_apps.so
	$(HIPCC) --offload-arch=gfx950 -O2 -std=c++17 -Iinclude -I$(MPI_HOME)/include -o $@ $< -L$(LIB) -ltempi_apps \
	    -ltempi -ltempi_hip -L$(MPI_HOME)/lib -lmpi -static-libstdc++ -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(MPI_HOME)/lib

$(LIB)/mpi_isend: apps/mpi_isend.cpp $(LIB)/libtempi_apps.so
	$(HIPCC) --offload-arch=gfx950 -O2 -std=c++17 -Iinclude -I$(MPI_HOME)/include -o $@ $< -L$(LIB) -ltempi_apps \
	    -ltempi -ltempi_hip -L$(MPI_HOME)/lib -lmpi -static-libstdc++ -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(MPI_HOME)/lib

# packer level, no MPI: the C-ABI alone
$(LIB)/pack_bench: apps/pack_bench.cpp $(LIB)/libtempi_hip.so
	$(HIPCC) --offload-arch=gfx950 -O2 -std=c++17 -Iinclude -o $@ $< -L$(LIB) -ltempi_hip -Wl,-rpath,'$$ORIGIN'

$(LIB)/%: apps/%.cpp $(LIB)/libtempi.so
	$(HIPCC) --offload-arch=gfx950 -O2 -std=c++17 -Iinclude -I$(MPI_HOME)/include -o $@ $< -L$(LIB) -ltempi -ltempi_hip -L$(MPI_HOME)/lib -lmpi \
	    -static-libstdc++ -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(MPI_HOME)/lib

oracle:
	$(MAKE) -s -C oracle all

clean:
	rm -rf build $(LIB)/*.so $(APPS)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
