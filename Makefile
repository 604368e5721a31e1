# Builds libdmip.so (gfx950) in-tree. Used by __graft_entry__.build(); `make -j2` by hand.
PKG := diffusion-modelling-for-inverse-problems_amd
CSRC := $(PKG)/csrc
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-parameter
F32OBJS := $(CSRC)/dmip_f32.o $(CSRC)/dmip_f32_cde.o $(CSRC)/dmip_f32_post.o $(CSRC)/dmip_f32_cdiffe.o
OBJS := $(CSRC)/dmip_kernels.o $(CSRC)/dmip_train.o $(CSRC)/dmip_eval.o $(CSRC)/dmip_surrogate.o $(F32OBJS) $(CSRC)/dmip_capi.o
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

# exact-f32 parity engine: one header, four translation units compiled in parallel
$(CSRC)/dmip_f32.o: $(CSRC)/dmip_f32.hip $(CSRC)/dmip_f32.h $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/dmip_f32_%.o: $(CSRC)/dmip_f32_%.hip $(CSRC)/dmip_f32.h $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/dmip_capi.o: $(CSRC)/dmip_capi.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(PKG)/libdmip.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJS) -o $@

clean:
	rm -f $(OBJS) $(PKG)/libdmip.so

.PHONY: all clean
