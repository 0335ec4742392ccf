# Builds the gfx950 HIP library kelpie_amd/libkelpie_hip.so (C ABI: include/kelpie_hip.h)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC := $(wildcard kelpie_amd/csrc/*.hip)
CPP := $(wildcard kelpie_amd/csrc/*.cpp)
OBJ := $(patsubst kelpie_amd/csrc/%.hip,build/%.o,$(SRC)) $(patsubst kelpie_amd/csrc/%.cpp,build/%.cpp.o,$(CPP))
CXX ?= g++
FLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
         -Wno-unused-result -Iinclude -Xarch_host -mavx2
LIB := kelpie_amd/libkelpie_hip.so

all: $(LIB)

build/%.o: kelpie_amd/csrc/%.hip kelpie_amd/csrc/kp_common.hpp kelpie_amd/csrc/kp_attn.hpp kelpie_amd/csrc/kp_attn3.hpp kelpie_amd/csrc/kp_cv_fused.hpp include/kelpie_hip.h
	@mkdir -p build
	$(HIPCC) $(FLAGS) -c $< -o $@

# host-only C++ (prefilter graphs)
build/%.cpp.o: kelpie_amd/csrc/%.cpp include/kelpie_hip.h
	@mkdir -p build
	$(CXX) -O3 -std=c++17 -fPIC -Wall -mavx2 -pthread -Iinclude $(if $(findstring kp_rng,$<),-ffp-contract=off -mfma) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -pthread -o $@ $(OBJ)

resources: $(SRC)
	@mkdir -p build
	for f in $(SRC); do $(HIPCC) $(FLAGS) -c $$f -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs|Spill|Occupancy|LDS" ; done

# diagnostic build: kp_attn phase timestamps (s_memtime), kelpie_amd/libkelpie_hip_stamps.so
stamps:
	@mkdir -p build/stamps
	for f in $(SRC); do $(HIPCC) $(FLAGS) -DKP_ATTN_STAMPS -DKP_TE_STAMPS -c $$f -o build/stamps/$$(basename $$f .hip).o || exit 1; done
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -pthread -o kelpie_amd/libkelpie_hip_stamps.so build/stamps/*.o $(patsubst kelpie_amd/csrc/%.cpp,build/%.cpp.o,$(CPP))

# timing-only diagnostic variants (wrong results), never the product library:
#   make diag DIAG="nos:-DKP_DIAG_NO_S noo:-DKP_DIAG_NO_O nodma:-DKP_ATTN_NODMA"  (commas: several defines)
# builds variants/lib_<name>.so, loaded by tools/attn_phase_ab.sh through KELPIE_HIP_LIB
DIAG ?= nos:-DKP_DIAG_NO_S noo:-DKP_DIAG_NO_O nodma:-DKP_ATTN_NODMA
diag: $(patsubst kelpie_amd/csrc/%.cpp,build/%.cpp.o,$(CPP))
	@mkdir -p variants
	for v in $(DIAG); do n=$${v%%:*}; d=$$(echo $${v#*:} | tr , ' '); mkdir -p build/diag_$$n; \
	  for f in $(SRC); do $(HIPCC) $(FLAGS) -DKP_DIAGNOSTIC_BUILD $$d -c $$f -o build/diag_$$n/$$(basename $$f .hip).o || exit 1; done; \
	  $(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -pthread -o variants/lib_$$n.so build/diag_$$n/*.o $^ || exit 1; done

clean:
	rm -rf build $(LIB)

.PHONY: all clean resources stamps diag

# host sanitizer builds of the library's host C++ (kp_rng.cpp worker pool / arenas,
# kp_graph.cpp) linked into tests/native/host_san_driver.cpp; run by
# tests/test_host_sanitizers.py (CPU suite), or by hand: make asan tsan
SAN_SRC := kelpie_amd/csrc/kp_rng.cpp kelpie_amd/csrc/kp_graph.cpp kelpie_amd/csrc/kp_sched.cpp tests/native/host_san_driver.cpp
SAN_FLAGS := -O1 -g -std=c++17 -fno-omit-frame-pointer -mavx2 -mfma -ffp-contract=off -pthread -Iinclude
asan: build/san/host_asan
tsan: build/san/host_tsan
build/san/host_asan: $(SAN_SRC) include/kelpie_hip.h
	@mkdir -p build/san
	$(CXX) $(SAN_FLAGS) -fsanitize=address,undefined -fno-sanitize-recover=undefined $(SAN_SRC) -o $@
build/san/host_tsan: $(SAN_SRC) include/kelpie_hip.h
	@mkdir -p build/san
	$(CXX) $(SAN_FLAGS) -fsanitize=thread $(SAN_SRC) -o $@

.PHONY: asan tsan
