# Native build for the MI355X Gray-Scott framework.
#   make            -> grayscott_amd/_lib/libgs_core.so (CPU/OpenMP backend, BP4 I/O)
#                      grayscott_amd/_lib/libgs_hip.so  (gfx950 kernels + RCCL transport)
#   make tools      -> build/bin/* native CLI helpers
ROCM     ?= /opt/rocm
ARCH     ?= gfx950
HIPCC    ?= $(ROCM)/bin/hipcc
CXX      ?= g++
OUT      := grayscott_amd/_lib
INC      := -Icsrc/include
CXXFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-parameter \
            -Wno-unused-result

CORE_SRC := csrc/cpu/backend_cpu.cpp csrc/io/bp4.cpp
HIP_SRC  := csrc/hip/backend_hip.hip
HDRS     := $(wildcard csrc/include/gs/*.h) $(wildcard csrc/hip/*.hpp)

all: $(OUT)/libgs_core.so $(OUT)/libgs_hip.so

$(OUT)/libgs_core.so: $(CORE_SRC) $(HDRS)
	@mkdir -p $(OUT)
	$(CXX) $(CXXFLAGS) -fopenmp $(INC) -shared -o $@ $(CORE_SRC)

$(OUT)/libgs_hip.so: $(HIP_SRC) $(HDRS)
	@mkdir -p $(OUT)
	$(HIPCC) $(HIPFLAGS) $(INC) -shared -o $@ $(HIP_SRC) -L$(ROCM)/lib -lrccl -Wl,-rpath,$(ROCM)/lib

clean:
	rm -f $(OUT)/*.so

.PHONY: all clean tools
