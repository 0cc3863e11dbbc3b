# Builds the MI355X-native library (gfx950 only) in-tree:
#   dependence_free_rl_amd/libxylo_hip.so   (C ABI: include/xylo_hip.h)
# and the test-only CPU oracle (oracle/liboracle.so, oracle/_ref/ when the
# reference tree is present).
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG      := dependence_free_rl_amd
SRC      := $(PKG)/csrc
LIB      := $(PKG)/libxylo_hip.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall \
            -Wno-unused-result -Iinclude -I$(SRC)
OBJS     := $(SRC)/policy_kernels.o $(SRC)/value_kernels.o \
            $(SRC)/env_kernels.o $(SRC)/kl_kernels.o \
            $(SRC)/heuristic_kernels.o $(SRC)/dense_kernels.o \
            $(SRC)/pg_kernels.o $(SRC)/venv_kernels.o $(SRC)/value_net_kernels.o \
            $(SRC)/policy_spec8_kernels.o $(SRC)/policy_spec8_kl_kernels.o \
            $(SRC)/policy_spec4_kernels.o \
            $(SRC)/policy_split8wh_kernels.o $(SRC)/policy_split8wh_kl_kernels.o \
            $(SRC)/policy_split8x_kernels.o $(SRC)/policy_split8x_kl_kernels.o \
            $(SRC)/policy_split4h_kernels.o $(SRC)/policy_split4h_kl_kernels.o \
            $(SRC)/loss_kernels.o $(SRC)/tensor_kernels.o \
            $(SRC)/train_select.o $(SRC)/model_api.o $(SRC)/tensor_api.o \
            $(SRC)/xylo_hip.o
# superseded train kernels (the config-3 / config-5
# epoch's earlier forms), kept for A/B runs in the variant library only
VARIANT_KERNELS := policy_split_kernels policy_split128_kernels \
            policy_split8w_kernels policy_split8wp_kernels \
            policy_split4p_kernels policy_split8wg_kernels
HDRS     := $(SRC)/xh_device.h $(SRC)/xh_kernels.h $(SRC)/xh_split.h \
            $(SRC)/spec8_layout.h \
            $(SRC)/xh_host.h include/xylo_hip.h

# Drop-in C++20 layer (include/xylo_compat): the reference's unmodified
# apps/bin_packing drivers (when the reference tree is present) and our own
# examples/ drivers, compiled against it and linked to the library.
CXX20    ?= /opt/rocm/lib/llvm/bin/clang++
REF      ?= /root/reference
COMPAT   := build/compat
CXXFLAGS20 := -std=c++20 -O2 -Wall -Wno-unused-variable -Iinclude/xylo_compat \
              -Iinclude
LDCOMPAT := -L$(PKG) -lxylo_hip -Wl,-rpath,'$$ORIGIN/../../$(PKG)'
REF_APPS := ppo_training ac_training ppo2_training pg_training deep_agent \
            random_agent firstfit_agent bestfit_agent minwaste_agent
EXAMPLES := $(patsubst examples/%.cc,$(COMPAT)/%,$(wildcard examples/*.cc))
COMPAT_HDRS := $(shell find include/xylo_compat -name '*.h') include/xylo_hip.h

.PHONY: all lib oracle compat clean diag variant variants
all: lib oracle compat

lib: $(LIB)

# per-file code-generation flags, measured per kernel: the
# split train kernels with the VGPR form of the MFMAs (the accumulators need
# not live in AGPRs: 64-row kernel 0 B of spills and 8% faster; the 128-row
# one keeps half 0's pre-activations in registers with it, 6% faster)
FLAGS_policy_split_kernels := -mllvm -amdgpu-mfma-vgpr-form
FLAGS_policy_split128_kernels := -mllvm -amdgpu-mfma-vgpr-form
FLAGS_policy_split8w_kernels := -mllvm -amdgpu-mfma-vgpr-form
FLAGS_policy_split8wp_kernels := -mllvm -amdgpu-mfma-vgpr-form
FLAGS_policy_split4p_kernels := -mllvm -amdgpu-mfma-vgpr-form
FLAGS_policy_split8wh_kernels := -mllvm -amdgpu-mfma-vgpr-form
FLAGS_policy_split8x_kernels := -mllvm -amdgpu-mfma-vgpr-form
FLAGS_policy_split4h_kernels := -mllvm -amdgpu-mfma-vgpr-form
FLAGS_policy_split8wg_kernels := -mllvm -amdgpu-mfma-vgpr-form
FLAGS_policy_spec8_kernels := -mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize
FLAGS_policy_spec4_kernels := -mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize

$(SRC)/%.o: $(SRC)/%.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) $(FLAGS_$*) -c $< -o $@

# the KL-PPO builds of the 64-, 128- and 32-bin train kernels (their own objects:
# the full unroll of their task lambdas needs a threshold the other builds
# are not made with, policy_split8wh_kernels.hip)
$(SRC)/policy_split8wh_kl_kernels.o: $(SRC)/policy_split8wh_kernels.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) $(FLAGS_policy_split8wh_kernels) -DXH_8WH_KL_TU=1 \
	    -mllvm -pragma-unroll-threshold=200000 -c $< -o $@
$(SRC)/policy_split8x_kl_kernels.o: $(SRC)/policy_split8x_kernels.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) $(FLAGS_policy_split8x_kernels) -DXH_8X_KL_TU=1 \
	    -mllvm -pragma-unroll-threshold=200000 -c $< -o $@
$(SRC)/policy_spec8_kl_kernels.o: $(SRC)/policy_spec8_kernels.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) $(FLAGS_policy_spec8_kernels) -DXH_SP8_KL_TU=1 -c $< -o $@
$(SRC)/policy_split4h_kl_kernels.o: $(SRC)/policy_split4h_kernels.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) $(FLAGS_policy_split4h_kernels) -DXH_4H_KL_TU=1 \
	    -mllvm -pragma-unroll-threshold=200000 -c $< -o $@

$(SRC)/xylo_hip.o: $(SRC)/xylo_hip.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SRC)/train_select.o: $(SRC)/train_select.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SRC)/model_api.o: $(SRC)/model_api.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SRC)/tensor_api.o: $(SRC)/tensor_api.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# the variant library: the product objects + the superseded train kernels,
# with the dispatch that reaches them (XH_TRAIN_KERNEL=split4w / split8w /
# split8wp / split4p / split8wg / split128); loaded through XH_LIB_PATH only
VDIR := build/variants
VOBJS := $(patsubst %,$(VDIR)/%.o,$(VARIANT_KERNELS))
$(VDIR)/%.o: research/variants/%.hip $(HDRS)
	@mkdir -p $(VDIR)
	$(HIPCC) $(HIPFLAGS) $(FLAGS_$*) -c $< -o $@
$(VDIR)/train_select.o: $(SRC)/train_select.cpp $(HDRS)
	@mkdir -p $(VDIR)
	$(HIPCC) $(HIPFLAGS) -DXH_VARIANT_KERNELS=1 -c $< -o $@
variants: $(OBJS) $(VOBJS) $(VDIR)/train_select.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $(VDIR)/libxylo_hip.so \
	    $(filter-out $(SRC)/train_select.o,$(OBJS)) $(VOBJS) $(VDIR)/train_select.o \
	    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJS) -L/opt/rocm/lib -lrccl \
	    -Wl,-rpath,/opt/rocm/lib

# diagnostic library with the phase-ablation bits compiled in (tools/ablate.sh;
# loaded through XH_LIB_PATH, never by the product path)
DIAG := build/diag
diag: $(OBJS)
	@mkdir -p $(DIAG)
	$(HIPCC) $(HIPFLAGS) -DXH_DIAG_ABLATE=1 -c $(SRC)/policy_kernels.hip -o $(DIAG)/policy_kernels.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $(DIAG)/libxylo_hip.so $(DIAG)/policy_kernels.o \
	    $(filter-out $(SRC)/policy_kernels.o,$(OBJS)) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -C oracle port
	@if [ -d /root/reference ]; then $(MAKE) -C oracle ref; fi

# test programs of the drop-in layer (tests/compat), prebuilt so the GPU box
# runs them without a compiler step
COMPAT_TESTS := $(COMPAT)/bound_env_by_hand $(COMPAT)/save_weights \
                $(COMPAT)/composed_learner $(COMPAT)/tensor_ops \
                $(COMPAT)/tensor_device

compat: $(EXAMPLES) $(COMPAT_TESTS)
	@mkdir -p $(COMPAT)
	@if [ -d $(REF)/apps/bin_packing ]; then \
	  for a in $(REF_APPS); do \
	    $(CXX20) $(CXXFLAGS20) -Wno-logical-op-parentheses \
	      $(REF)/apps/bin_packing/$$a.cc $(LDCOMPAT) -o $(COMPAT)/$$a || exit 1; \
	  done; fi

$(COMPAT)/bound_env_by_hand: tests/compat/bound_env_by_hand.cc $(COMPAT_HDRS) $(LIB)
	@mkdir -p $(COMPAT)
	$(CXX20) $(CXXFLAGS20) $< $(LDCOMPAT) -o $@

$(COMPAT)/save_weights: tests/compat/save_weights.cc $(COMPAT_HDRS) $(LIB)
	@mkdir -p $(COMPAT)
	$(CXX20) $(CXXFLAGS20) $< $(LDCOMPAT) -o $@

$(COMPAT)/composed_learner: tests/compat/composed_learner.cc $(COMPAT_HDRS) $(LIB)
	@mkdir -p $(COMPAT)
	$(CXX20) $(CXXFLAGS20) $< $(LDCOMPAT) -o $@

$(COMPAT)/tensor_ops: tests/compat/tensor_ops.cc $(COMPAT_HDRS) $(LIB)
	@mkdir -p $(COMPAT)
	$(CXX20) $(CXXFLAGS20) $< $(LDCOMPAT) -o $@

$(COMPAT)/tensor_device: tests/compat/tensor_device.cc $(COMPAT_HDRS) $(LIB)
	@mkdir -p $(COMPAT)
	$(CXX20) $(CXXFLAGS20) $< $(LDCOMPAT) -o $@

# the host paths of the drop-in tensor layer under AddressSanitizer +
# UndefinedBehaviorSanitizer (tests/test_tensor_compat.py runs it
# with every operation kept on the host)
$(COMPAT)/tensor_ops_asan: tests/compat/tensor_ops.cc $(COMPAT_HDRS) $(LIB)
	@mkdir -p $(COMPAT)
	$(CXX20) $(CXXFLAGS20) -O1 -g -fsanitize=address,undefined \
	    -fno-omit-frame-pointer -fno-sanitize-recover=undefined $< $(LDCOMPAT) -o $@

$(COMPAT)/%: examples/%.cc $(COMPAT_HDRS) $(LIB)
	@mkdir -p $(COMPAT)
	$(CXX20) $(CXXFLAGS20) $< $(LDCOMPAT) -o $@

clean:
	rm -f $(OBJS) $(LIB)

# performance variants of the policy kernels for A/B runs on one box
# (tools/gpu_variants.sh; loaded through XH_LIB_PATH, never by the product):
#   make variant V=name VFLAGS="-DXH_DIAG_TRACE=1 ..."
#   make variant V=name VSRC=dense_kernels VFLAGS="..."  (another source file)
VSRC ?= policy_kernels
variant: $(OBJS)
	@mkdir -p build/$(V)
	$(HIPCC) $(HIPFLAGS) $(FLAGS_$(VSRC)) $(VFLAGS) -c $(SRC)/$(VSRC).hip -o build/$(V)/$(VSRC).o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o build/$(V)/libxylo_hip.so build/$(V)/$(VSRC).o \
	    $(filter-out $(SRC)/$(VSRC).o,$(OBJS)) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
