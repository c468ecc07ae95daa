# Host-side ASan + UBSan build of the whole C ABI (sanitizers
# on host code only — the GPU pool has no device ASan).  Device code is
# compiled as usual; every host translation unit is instrumented.
#   make -f tools/asan.mk            -> trivy_amd/libtrivy_secret_gpu_asan.so
# tests/test_asan.py loads it (TSG_LIB_VARIANT=asan) under the clang runtime
# and runs the host-only tests (regex compiler/VM, rule compiler, tar walker,
# malformed-tar fuzz, threaded reentrancy) against it.  CPU only.
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
SAN      = -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined
FLAGS    = -O1 -g -fno-omit-frame-pointer -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude -Itrivy_amd/csrc \
           -x hip --offload-arch=$(ARCH) -munsafe-fp-atomics $(SAN)
SRC_DIR  = trivy_amd/csrc
SRCS     = gre.cpp ruleset.cpp follow.cpp dfa.cpp nfa.cpp layertar.cpp engine.hip
OBJS     = $(patsubst %,build_asan/%.o,$(SRCS))
LIB      = trivy_amd/libtrivy_secret_gpu_asan.so
HDRS     = $(wildcard $(SRC_DIR)/*.h) $(wildcard include/*.h)

$(LIB): $(OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -shared-libsan $(SAN) -o $@ $(OBJS) -lamdhip64 -lhsa-runtime64

build_asan/%.o: $(SRC_DIR)/% $(HDRS)
	@mkdir -p build_asan
	$(HIPCC) $(FLAGS) -c $< -o $@
