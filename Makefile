# Native build for the MI355X Gray-Scott framework.
#   make            -> grayscott_amd/_lib/libgs_core.so (CPU/OpenMP backend, BP4 I/O)
#                      grayscott_amd/_lib/libgs_hip.so  (gfx950 kernels + RCCL transport)
#   make selftest   -> build/bin/core_selftest (threads-as-ranks runtime self-test)
#   make tools      -> build/bin/ubench_valu (gfx950 VALU issue-rate micro-benchmark)
#   make ablation   -> grayscott_amd/_lib/libgs_hip_abl.so: the HIP library plus the fused
#                      kernel's ablation variants (results WRONG by design; timing experiments
#                      only, loaded with GS_HIP_VARIANT=abl by scripts/power_probe.py etc.)
#   make asan/tsan  -> the same self-test under AddressSanitizer+UBSan / ThreadSanitizer (host
#                      code only: GPU sanitizers are not available on the MI355X pool)
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
# the heavy template instantiations (fused kernel per precision, overlap shell) in their own
# translation units, compiled in parallel (make -j)
HIP_INST := $(wildcard csrc/hip/inst/*.hip)
HDRS     := $(wildcard csrc/include/gs/*.h) $(wildcard csrc/hip/*.hpp)
HIP_OBJ  := $(patsubst csrc/hip/%.hip,build/obj/%.o,$(HIP_SRC) $(HIP_INST))

all: $(OUT)/libgs_core.so $(OUT)/libgs_hip.so

$(OUT)/libgs_core.so: $(CORE_SRC) $(HDRS)
	@mkdir -p $(OUT)
	$(CXX) $(CXXFLAGS) -fopenmp $(INC) -shared -o $@ $(CORE_SRC)

build/obj/%.o: csrc/hip/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) $(INC) -c -o $@ $<

$(OUT)/libgs_hip.so: $(HIP_OBJ)
	@mkdir -p $(OUT)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(HIP_OBJ) -L$(ROCM)/lib -lrccl -Wl,-rpath,$(ROCM)/lib

$(OUT)/libgs_hip_abl.so: $(HIP_SRC) $(HIP_INST) $(HDRS)
	@mkdir -p $(OUT)
	$(HIPCC) $(HIPFLAGS) -DGS_ABLATION $(INC) -shared -o $@ $(HIP_SRC) $(HIP_INST) -L$(ROCM)/lib -lrccl -Wl,-rpath,$(ROCM)/lib

ablation: $(OUT)/libgs_hip_abl.so

# no VALU-write -> DPP-read hazard in the shipped code object (the fused kernel's DPP sums are
# inline asm without wait states; scripts/check_dpp_hazards.py, tests/test_isa_hazards.py)
check-isa: $(OUT)/libgs_hip.so
	python3 scripts/check_dpp_hazards.py $(OUT)/libgs_hip.so

SELFTEST_TMP ?= /tmp
SELFTEST_SRC := csrc/tools/core_selftest.cpp $(CORE_SRC)

build/bin/core_selftest: $(SELFTEST_SRC) $(HDRS)
	@mkdir -p build/bin
	$(CXX) -O2 -g -std=c++17 -fopenmp $(INC) -o $@ $(SELFTEST_SRC) -lpthread

build/asan/core_selftest: $(SELFTEST_SRC) $(HDRS)
	@mkdir -p build/asan
	$(CXX) -O1 -g -std=c++17 -fopenmp -fsanitize=address,undefined -fno-omit-frame-pointer \
	  -fno-sanitize-recover=undefined $(INC) -o $@ $(SELFTEST_SRC) -lpthread

# no -fopenmp: libgomp is not TSan-instrumented; the rank threads are what is checked
build/tsan/core_selftest: $(SELFTEST_SRC) $(HDRS)
	@mkdir -p build/tsan
	$(CXX) -O1 -g -std=c++17 -Wno-unknown-pragmas -fsanitize=thread $(INC) -o $@ $(SELFTEST_SRC) -lpthread

# VALU issue-rate micro-benchmark (profiles/r1_ubench_valu.txt)
build/bin/ubench_valu: csrc/tools/ubench_valu.hip
	@mkdir -p build/bin
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -o $@ $<

tools: build/bin/ubench_valu

selftest: build/bin/core_selftest
	build/bin/core_selftest $(SELFTEST_TMP)
asan: build/asan/core_selftest
	ASAN_OPTIONS=detect_leaks=1 build/asan/core_selftest $(SELFTEST_TMP)
tsan: build/tsan/core_selftest
	build/tsan/core_selftest $(SELFTEST_TMP)

clean:
	rm -f $(OUT)/*.so
	rm -rf build

.PHONY: all clean selftest asan tsan tools ablation check-isa
