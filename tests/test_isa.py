"""Static checks of the built gfx950 code objects (scripts/check_isa.py; CPU only): no kernel calls an
outlined device function or needs a dynamic stack (an outlined score evaluation once put the f32
sampler's activation arrays on an undersized scratch stack and faulted on the GPU), and the bf16
product samplers run without any scratch."""
import importlib
import os

import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def isa(dmip):
    if not os.path.exists(dmip._lib.LIB_PATH):
        pytest.skip("libdmip.so not built")
    import sys
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    mod = importlib.import_module("check_isa")
    return mod.analyse(dmip._lib.LIB_PATH)


def test_every_kernel_found(isa):
    names = " ".join(isa)
    for k in ("em_sampler_kernel", "f32_sampler_kernel", "f32_forward_kernel", "mlp_forward_kernel",
              "loss_grad_kernel", "mh_kernel", "dps_kernel"):
        assert k in names, k


def test_no_outlined_calls_or_dynamic_stack(isa):
    bad = {k: v for k, v in isa.items() if v.get("calls", 0) or v.get("uses_dynamic_stack")}
    assert not bad, bad


def test_bf16_samplers_have_no_scratch(isa):
    samplers = {k: v for k, v in isa.items() if "em_sampler_kernel" in k}
    assert samplers
    spill = {k: v["private_segment_fixed_size"] for k, v in samplers.items() if v.get("private_segment_fixed_size")}
    assert not spill, spill
