# Build of the MI355X-native library + CLIs (gfx950 only). `make -j8`.
#   deepreadmapper_amd/libdrm_hip.so : C ABI (include/drm_hip.h), HIP kernels + host C++
#   bin/pipeline, bin/hnswpq_index   : drop-in CLIs for src/main.cpp and src/hnswpq/index.cpp
#   oracle/*.so                      : TEST-ONLY checker (oracle/Makefile)
ROCM ?= /opt/rocm
HIPCC ?= $(ROCM)/bin/hipcc
ARCH ?= gfx950
CXX ?= g++
BUILD := build
PKG := deepreadmapper_amd
SRC := $(PKG)/csrc

COMMON := -O3 -std=c++17 -fPIC -Iinclude -I$(SRC) -Wall -Wno-unused-result
HIPFLAGS := $(COMMON) --offload-arch=$(ARCH) -ffp-contract=off -munsafe-fp-atomics
HOSTFLAGS := $(COMMON) -fopenmp -ffp-contract=off -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include

LIB := $(PKG)/libdrm_hip.so
HIP_OBJS := $(BUILD)/hnsw_search.o $(BUILD)/hnsw_pq_fast.o $(BUILD)/builder_gpu.o $(BUILD)/embed_gpu.o $(BUILD)/hnsw_search_lds.o $(BUILD)/hnsw_flat_search.o $(BUILD)/sw_rerank.o $(BUILD)/l2_rerank.o \
            $(BUILD)/encoder_gru.o $(BUILD)/capi.o $(BUILD)/exec.o
HOST_OBJS := $(BUILD)/faiss_io.o $(BUILD)/formats.o $(BUILD)/builder.o $(BUILD)/embed.o $(BUILD)/hnswlib_io.o \
             $(BUILD)/builder_flat.o $(BUILD)/encoder.o
HDRS := include/drm_hip.h $(SRC)/drm_internal.h $(SRC)/drm_device.h $(SRC)/pq_common.h

all: $(LIB) bin/pipeline bin/hnswpq_index oracle

$(BUILD):
	mkdir -p $(BUILD) bin

$(BUILD)/%.o: $(SRC)/%.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# the search kernel: loops aligned to 16 bytes (103.7 -> 103.5 ms at C5, profiles/r04/ab_search_loop_align.txt);
# the default machine scheduler (max-ILP, kept in round 4, is 0.8 % slower with the round-5 code,
# profiles/r05/ab_search_sched_strategy_r05*.txt)
$(BUILD)/hnsw_pq_fast.o: $(SRC)/hnsw_pq_fast.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -falign-loops=16 -c $< -o $@

# the SW rerank under the iterative-ILP machine scheduler: 28.1 -> 27.6 ms on the 152-column probe, equal at 64
# (profiles/r05/ab_sw_sched_strategy.txt)
$(BUILD)/sw_rerank.o: $(SRC)/sw_rerank.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -mllvm -amdgpu-sched-strategy=iterative-ilp -c $< -o $@

$(BUILD)/capi.o: $(SRC)/capi.cpp $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(BUILD)/exec.o: $(SRC)/exec.cpp $(HDRS) | $(BUILD)
	$(CXX) $(HOSTFLAGS) -c $< -o $@

$(BUILD)/%.o: $(SRC)/%.cpp $(HDRS) | $(BUILD)
	$(CXX) $(HOSTFLAGS) -c $< -o $@

$(LIB): $(HIP_OBJS) $(HOST_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -L$(ROCM)/lib -lamdhip64 -lrccl -lgomp -Wl,-soname,libdrm_hip.so

bin/%: tools/%.cpp $(LIB) $(HDRS) | $(BUILD)
	$(CXX) $(HOSTFLAGS) -o $@ $< -L$(PKG) -ldrm_hip -L$(ROCM)/lib -lamdhip64 -Wl,-rpath,'$$ORIGIN/../$(PKG)' -Wl,-rpath,$(ROCM)/lib

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD) bin $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
