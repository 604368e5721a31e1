# Builds libdmip.so (gfx950) in-tree. Used by __graft_entry__.build(); `make -j2` by hand.
PKG := diffusion-modelling-for-inverse-problems_amd
CSRC := $(PKG)/csrc
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-parameter
F32OBJS := $(CSRC)/dmip_f32.o $(CSRC)/dmip_f32_cde.o $(CSRC)/dmip_f32_post.o $(CSRC)/dmip_f32_cdiffe.o
X3OBJS := $(CSRC)/dmip_x3.o $(CSRC)/dmip_x3_cde.o $(CSRC)/dmip_x3_post.o $(CSRC)/dmip_x3_cdiffe.o $(CSRC)/dmip_x3k.o \
          $(CSRC)/dmip_dps_x3.o
OBJS := $(CSRC)/dmip_kernels.o $(CSRC)/dmip_train.o $(CSRC)/dmip_eval.o $(CSRC)/dmip_surrogate.o $(CSRC)/dmip_gemm.o $(CSRC)/dmip_jets.o $(CSRC)/dmip_step.o $(F32OBJS) $(X3OBJS) $(CSRC)/dmip_capi.o
HDRS := $(CSRC)/dmip_device.h $(CSRC)/dmip_internal.h include/dmip.h

all: $(PKG)/libdmip.so

# no SLP vectorisation in the sampler: packed f32 FMAs (v_pk_fma_f32) beside MFMAs cost more than
# the scalar pair (MI355X_MICROARCH.md, filler prices); bf16 packing is written out pairwise instead
$(CSRC)/dmip_kernels.o: $(CSRC)/dmip_kernels.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -fno-slp-vectorize -c $< -o $@

$(CSRC)/dmip_train.o: $(CSRC)/dmip_train.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/dmip_eval.o: $(CSRC)/dmip_eval.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/dmip_surrogate.o: $(CSRC)/dmip_surrogate.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/dmip_gemm.o: $(CSRC)/dmip_gemm.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/dmip_jets.o: $(CSRC)/dmip_jets.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/dmip_step.o: $(CSRC)/dmip_step.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# exact-f32 parity engine: one header, four translation units compiled in parallel
$(CSRC)/dmip_f32.o: $(CSRC)/dmip_f32.hip $(CSRC)/dmip_f32.h $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/dmip_f32_%.o: $(CSRC)/dmip_f32_%.hip $(CSRC)/dmip_f32.h $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# fp32-accurate split-fp16 engine (DMIP_PREC_F32X3): one header, four translation units; no SLP
# vectorisation (it packs the split's f32 subtractions into v_pk_add_f32, an anti-lever beside MFMAs)
$(CSRC)/dmip_x3.o: $(CSRC)/dmip_x3.hip $(CSRC)/dmip_x3.h $(HDRS)
	$(HIPCC) $(HIPFLAGS) -fno-slp-vectorize -c $< -o $@

$(CSRC)/dmip_x3_%.o: $(CSRC)/dmip_x3_%.hip $(CSRC)/dmip_x3.h $(CSRC)/dmip_x3s.h $(HDRS)
	$(HIPCC) $(HIPFLAGS) -fno-slp-vectorize -c $< -o $@

# the k-major multi-tile fp32x3 CDE engine (width 256): its own header
$(CSRC)/dmip_x3k.o: $(CSRC)/dmip_x3k.hip $(CSRC)/dmip_x3k.h $(CSRC)/dmip_x3.h $(HDRS)
	$(HIPCC) $(HIPFLAGS) -fno-slp-vectorize -c $< -o $@

# DPS (config 4) on the split-fp16 arithmetic
$(CSRC)/dmip_dps_x3.o: $(CSRC)/dmip_dps_x3.hip $(CSRC)/dmip_x3.h $(HDRS)
	$(HIPCC) $(HIPFLAGS) -fno-slp-vectorize -c $< -o $@

$(CSRC)/dmip_capi.o: $(CSRC)/dmip_capi.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(PKG)/libdmip.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJS) -o $@

# A/B + diagnostic library (never the product): the samplers' timing ablations and per-phase cycle stamps behind
# -DDMIP_DIAG (run-time DMIP_X3_DIAG for the x3 / x3k engines, scripts/x3k_stamps.py), and the paired-tile 32x32
# fp32x3 engine (dmip_x3p.h, opt-in DMIP_X3P=1; it measured slower than x3k, so libdmip.so does not hold it).
# Load it with DMIP_LIB=abv/diag/libdmip_diag.so (tests/test_gpu_x3p.py runs there). The paired engine's
# per-chunk stamps (scripts/x3p_stamps.py) replace its snapshots, so they need their own build:
# make diag X3P_DIAG=-DDMIP_X3P_DIAG
DIAG_DIR := abv/diag
DIAG_SRCS := dmip_x3_cde dmip_x3k dmip_capi
diag: $(DIAG_DIR)/libdmip_diag.so
$(DIAG_DIR)/%_diag.o: $(CSRC)/%.hip $(CSRC)/dmip_x3k.h $(CSRC)/dmip_x3.h $(CSRC)/dmip_x3s.h $(HDRS)
	@mkdir -p $(DIAG_DIR)
	$(HIPCC) $(HIPFLAGS) -fno-slp-vectorize -DDMIP_DIAG -c $< -o $@
X3P_DIAG ?=
$(DIAG_DIR)/dmip_x3p_diag.o: $(CSRC)/dmip_x3p.hip $(CSRC)/dmip_x3p.h $(CSRC)/dmip_x3.h $(HDRS)
	@mkdir -p $(DIAG_DIR)
	$(HIPCC) $(HIPFLAGS) -fno-slp-vectorize $(X3P_DIAG) -c $< -o $@
$(DIAG_DIR)/dmip_capi_diag.o: $(CSRC)/dmip_capi.cpp $(HDRS)
	@mkdir -p $(DIAG_DIR)
	$(HIPCC) $(HIPFLAGS) -DDMIP_WITH_X3P -c $< -o $@
$(DIAG_DIR)/libdmip_diag.so: $(filter-out $(patsubst %,$(CSRC)/%.o,$(DIAG_SRCS)),$(OBJS)) $(patsubst %,$(DIAG_DIR)/%_diag.o,$(DIAG_SRCS)) $(DIAG_DIR)/dmip_x3p_diag.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -o $@

# microbenchmarks (scripts/ubench): built here, never committed
UBENCH := scripts/ubench/valu_mix scripts/ubench/valu_rates
ubench: $(UBENCH)
scripts/ubench/%: scripts/ubench/%.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 $< -o $@

# Host-only AddressSanitizer build of the C-ABI layer (argument validation, packing, handle
# management): dmip_capi.cpp instrumented on the host side only (-Xarch_host), linked with the same
# kernel objects, driven by tests/asan/capi_args.cpp through the calls that need no GPU.
# dmip_capi.cpp has no device code: it compiles as plain host C++ against the HIP runtime headers.
ASAN_DIR := build/asan
HOSTCXX ?= /opt/rocm/lib/llvm/bin/clang++
ASANFLAGS := -O1 -g -std=c++17 -fPIC -fsanitize=address -fno-omit-frame-pointer
asan: $(ASAN_DIR)/capi_args
$(ASAN_DIR)/dmip_capi_asan.o: $(CSRC)/dmip_capi.cpp $(HDRS)
	@mkdir -p $(ASAN_DIR)
	$(HOSTCXX) -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include $(ASANFLAGS) -c $< -o $@
$(ASAN_DIR)/libdmip_asan.so: $(filter-out $(CSRC)/dmip_capi.o,$(OBJS)) $(ASAN_DIR)/dmip_capi_asan.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -fsanitize=address $^ -o $@
$(ASAN_DIR)/capi_args: tests/asan/capi_args.cpp $(ASAN_DIR)/libdmip_asan.so include/dmip.h
	$(HOSTCXX) $(ASANFLAGS) $< -L$(ASAN_DIR) -ldmip_asan -Wl,-rpath,$(abspath $(ASAN_DIR)) -lpthread -o $@

clean:
	rm -f $(OBJS) $(PKG)/libdmip.so $(UBENCH)
	rm -rf $(ASAN_DIR)

.PHONY: all clean ubench asan diag
