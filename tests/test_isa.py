"""Static checks of the built gfx950 code objects (scripts/check_isa.py; CPU only): no kernel calls an
outlined device function or needs a dynamic stack (an outlined score evaluation once put the f32
sampler's activation arrays on an undersized scratch stack and faulted on the GPU), and the product
samplers (16-bit, fp32x3 one-tile) and the config-5 training kernels run without any scratch (a
register spill in them would be a silent slowdown); the k-major fp32x3 kernels within a small cap."""
import importlib
import os

import pytest

from conftest import ROOT


def _analyse(path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    mod = importlib.import_module("check_isa")
    return mod.analyse(path)


@pytest.fixture(scope="module")
def isa(dmip):
    if not os.path.exists(dmip._lib.LIB_PATH):
        pytest.skip("libdmip.so not built")
    res = _analyse(dmip._lib.LIB_PATH)
    # the A/B library's paired-tile engine (make diag) is held to the same static checks
    diag = os.path.join(ROOT, "abv", "diag", "libdmip_diag.so")
    if os.path.exists(diag):
        res.update({k: v for k, v in _analyse(diag).items() if "x3p_sampler_kernel" in k})
    return res


def test_every_kernel_found(isa):
    names = " ".join(isa)
    for k in ("em_sampler_kernel", "f32_sampler_kernel", "f32_forward_kernel", "mlp_forward_kernel",
              "loss_grad_kernel", "mh_kernel", "dps_kernel", "x3_sampler_kernel", "x3k_sampler_kernel"):
        assert k in names, k


def test_product_library_holds_no_ab_engine(dmip):
    """The paired-tile engine measured slower (profiles/r4_ab_x3p_vs_x3k.json): only the A/B library holds it."""
    if not os.path.exists(dmip._lib.LIB_PATH):
        pytest.skip("libdmip.so not built")
    assert not any("x3p_sampler_kernel" in k for k in _analyse(dmip._lib.LIB_PATH))


def test_no_outlined_calls_or_dynamic_stack(isa):
    bad = {k: v for k, v in isa.items() if v.get("calls", 0) or v.get("uses_dynamic_stack")}
    assert not bad, bad


def test_bf16_samplers_have_no_scratch(isa):
    samplers = {k: v for k, v in isa.items() if "em_sampler_kernel" in k}
    assert samplers
    spill = {k: v["private_segment_fixed_size"] for k, v in samplers.items() if v.get("private_segment_fixed_size")}
    assert not spill, spill


# the k-major kernels hold ~460 registers; at NT = 3 the compiler parks ~20 dwords of per-segment state
# (chain indices, output pointers) in scratch. Their loads and stores sit in the segment setup, the
# hand-over epilogue and the snapshot branch, none in the step loop's hot path (checked in the ISA,
# round 3); the cap keeps that from growing unnoticed.
# The paired-tile kernels (x3p, 185 VGPRs + 256 AGPRs) have none. One-tile x3: none, except CDiffE (3, 23) at width
# 512, whose layer 1 streams through the ring (L1R, one wave per SIMD at ~512 registers): round 4 spilled ~17 dwords
# of segment state, reloaded a handful of times per step; round 5 cut that to 3 dwords of schedule setup (the chain
# index recomputed from the wave-uniform job and the lane id after the step loop), and the buffer LDS-DMA refills
# (no per-piece 64-bit addresses) to none.
# The fp32x3 DPS and MH kernels: none since the running range max is pinned (round 5; it had kept every tracked value
# alive, 176 B in DPS); the three-tile MH kernel (launched when its workgroup rounds are full) spills 20 B.
_SCRATCH_CAP = {"x3_sampler_kernel": 0, "x3k_sampler_kernel": 128, "loss_grad_kernel": 0, "x3p_sampler_kernel": 0,
                "dps_x3_kernel": 0, "mh_x3_kernel": 0, "mh_x3_mt_kernel": 0}
# The config-5 forward half (loss_grad_kernel<NL, 1>, two waves per SIMD, 256 registers) writes the record reverse half's
# per-layer records since round 6: about 26 dwords of its state spill (104-112 B), reloaded once per tile; the kernel
# without the record writes has none
_SCRATCH_CAP_KERNEL = {"mh_x3_mt_kernelILi3E": 24, "loss_grad_kernelILi3ELi1E": 128, "loss_grad_kernelILi2ELi1E": 128}


@pytest.mark.parametrize("family", list(_SCRATCH_CAP))
def test_fp32x3_samplers_and_training_kernels_scratch(isa, family):
    kernels = {k: v for k, v in isa.items() if family in k}
    if not kernels and family == "x3p_sampler_kernel":
        pytest.skip("A/B library not built (make diag)")
    assert kernels, family
    def cap(k):
        return next((c for pat, c in _SCRATCH_CAP_KERNEL.items() if pat in k), _SCRATCH_CAP[family])
    over = {k: v["private_segment_fixed_size"] for k, v in kernels.items()
            if v.get("private_segment_fixed_size", 0) > cap(k)}
    assert not over, over
