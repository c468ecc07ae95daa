# Builds the in-tree engine library trivy_amd/libtrivy_secret_gpu.so for gfx950.
# (hipcc cross-compiles without a GPU; the .so travels to the GPU box.)
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
CXXFLAGS = -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude -Itrivy_amd/csrc
HIPFLAGS = $(CXXFLAGS) -x hip --offload-arch=$(ARCH) -munsafe-fp-atomics
SRC_DIR  = trivy_amd/csrc
BUILD    = build
LIB      = trivy_amd/libtrivy_secret_gpu.so

HOST_SRCS = $(SRC_DIR)/gre.cpp $(SRC_DIR)/ruleset.cpp $(SRC_DIR)/follow.cpp $(SRC_DIR)/dfa.cpp $(SRC_DIR)/nfa.cpp $(SRC_DIR)/layertar.cpp
HIP_SRCS  = $(SRC_DIR)/engine.hip
HDRS      = $(wildcard $(SRC_DIR)/*.h) $(wildcard include/*.h)

OBJS = $(patsubst $(SRC_DIR)/%.cpp,$(BUILD)/%.o,$(HOST_SRCS)) $(patsubst $(SRC_DIR)/%.hip,$(BUILD)/%.o,$(HIP_SRCS))

# bench-only CPU baseline (bench.py cpu_baseline): not part of the product library
BENCH_LIB = bench_cpu/libtsg_cpu_scan.so
# bench / test corpus generator (bench.py, tests): not part of the product library
GEN_LIB   = bench_gen/libtsg_corpus.so

all: $(LIB) $(BENCH_LIB) $(GEN_LIB)

$(GEN_LIB): bench_gen/corpus.hip bench_gen/tsg_corpus.h include/trivy_secret_gpu.h
	$(HIPCC) $(HIPFLAGS) -Ibench_gen -shared -o $@ $<

$(BENCH_LIB): bench_cpu/cpu_scan.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $< -lpthread

$(BUILD)/%.o: $(SRC_DIR)/%.cpp $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/%.o: $(SRC_DIR)/%.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(OBJS) -lamdhip64 -lhsa-runtime64

# ablation build for tools/*.sh A/B runs (TSG_LIB_VARIANT=exp selects it in
# trivy_amd/_native.py): dead kernel shapes + getenv switches, some of which
# give wrong results by design.  Never the product library.
EXP_LIB  = trivy_amd/libtrivy_secret_gpu_exp.so
EXP_OBJS = $(patsubst $(SRC_DIR)/%.cpp,build_exp/%.o,$(HOST_SRCS)) $(patsubst $(SRC_DIR)/%.hip,build_exp/%.o,$(HIP_SRCS))

exp: $(EXP_LIB)

build_exp/%.o: $(SRC_DIR)/%.cpp $(HDRS)
	@mkdir -p build_exp
	$(HIPCC) $(HIPFLAGS) -DTSG_EXPERIMENTS -c $< -o $@

build_exp/%.o: $(SRC_DIR)/%.hip $(HDRS)
	@mkdir -p build_exp
	$(HIPCC) $(HIPFLAGS) -DTSG_EXPERIMENTS -c $< -o $@

$(EXP_LIB): $(EXP_OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(EXP_OBJS) -lamdhip64 -lhsa-runtime64

clean:
	rm -rf $(BUILD) build_exp $(LIB) $(BENCH_LIB) $(GEN_LIB) $(EXP_LIB)

.PHONY: all clean exp alt

# product build of another revision's sources (tools/build_alt.sh exports them
# to build_<ALT>/src): TSG_LIB_VARIANT=<ALT> (alt, alt2, ...) loads it, for
# same-box A/B runs
ALT      ?= alt
ALT_SRC  = build_$(ALT)/src
ALT_LIB  = trivy_amd/libtrivy_secret_gpu_$(ALT).so
ALT_OBJS = $(patsubst $(SRC_DIR)/%.cpp,build_$(ALT)/%.o,$(HOST_SRCS)) $(patsubst $(SRC_DIR)/%.hip,build_$(ALT)/%.o,$(HIP_SRCS))
ALT_FLAGS = -O3 -std=c++17 -fPIC -Wno-unused-function -I$(ALT_SRC)/include -I$(ALT_SRC)/$(SRC_DIR)

alt: $(ALT_LIB)

build_$(ALT)/%.o: $(ALT_SRC)/$(SRC_DIR)/%.cpp
	$(HIPCC) $(ALT_FLAGS) -x hip --offload-arch=$(ARCH) -munsafe-fp-atomics -c $< -o $@

build_$(ALT)/%.o: $(ALT_SRC)/$(SRC_DIR)/%.hip
	$(HIPCC) $(ALT_FLAGS) -x hip --offload-arch=$(ARCH) -munsafe-fp-atomics -c $< -o $@

$(ALT_LIB): $(ALT_OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(ALT_OBJS) -lamdhip64 -lhsa-runtime64
