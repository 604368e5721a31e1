"""The SiLU activation chain on the host: the oracle's chain against the package's reference-layout MLP built
with nn.SiLU (eager torch, CPU), the activation detection that routes a network to its compiled chain, and
the sampler-precision choice for a SiLU network (no GPU needed)."""
import importlib

import numpy as np
import pytest
import torch

import oracle as O

PKG = "diffusion-modelling-for-inverse-problems_amd"


@pytest.fixture(scope="module")
def dmip():
    return importlib.import_module(PKG)


def _params(net):
    return [(l.weight.detach().numpy(), l.bias.detach().numpy()) for l in net if isinstance(l, torch.nn.Linear)]


@pytest.mark.parametrize("hl", [[64] * 3, [32, 32]])
def test_oracle_silu_chain_matches_reference_layout_mlp(dmip, hl):
    """nets.py:17-35 with activation=nn.SiLU(): Linear -> SiLU -> SiLU (the `act` re-registration) -> ... ->
    Linear; the oracle's activation(.., "silu") chain equals torch's module chain to fp32 rounding."""
    torch.manual_seed(3)
    net = dmip.MLP(2 + 2 + 1, 2, hl, torch.nn.SiLU())
    names = list(net._modules.keys())  # (named_children drops the repeated module)
    assert names[:3] == ["0", "1", "act"]  # the double activation on layer 1, as the reference registers it
    x, y, t = torch.randn(300, 2), torch.randn(300, 2), torch.rand(300)
    with torch.no_grad():
        ref = net(x, y, t).numpy()
    out = O.cde_a(_params(net), x.numpy(), y.numpy(), t.numpy(), act="silu")
    assert np.abs(out - ref).max() < 1e-5 * max(1.0, np.abs(ref).max())
    tanh = O.cde_a(_params(net), x.numpy(), y.numpy(), t.numpy())
    assert np.abs(tanh - ref).max() > 1e-2  # the activation is not silently tanh


def test_activation_detection(dmip):
    lib = dmip._lib
    assert dmip.MLP(5, 2, [64] * 2, torch.nn.Tanh()).dmip_act == lib.DMIP_ACT_TANH_TWICE_FIRST
    assert dmip.MLP(5, 2, [64] * 2, torch.nn.SiLU()).dmip_act == lib.DMIP_ACT_SILU_TWICE_FIRST
    relu = dmip.MLP(5, 2, [64] * 2, torch.nn.ReLU())
    assert relu.dmip_act is None
    with pytest.raises(NotImplementedError, match="ReLU"):
        relu.require_dmip_act()


def test_silu_sampler_precision_choice(dmip):
    """A SiLU network samples on the exact-f32 CDE kernel whatever the requested precision; the Posterior and
    CDiffE samplers have no SiLU kernel (per-step loop / refusal)."""
    est = importlib.import_module(PKG + ".estimators")
    lib = dmip._lib
    silu = [lib.DMIP_ACT_SILU_TWICE_FIRST]
    for prec in ("fp16", "fp32x3", "fp32"):
        assert est._fused_precision(prec, lib.DMIP_SAMPLER_CDE, 256, 3, 3, 23, silu) == "fp32"
        assert est._fused_precision(prec, lib.DMIP_SAMPLER_POSTERIOR, 256, 3, 3, 23, silu * 2) is None
        assert est._fused_precision(prec, lib.DMIP_SAMPLER_CDIFFE, 256, 3, 3, 23, silu) is None
    assert est._fused_precision("fp32x3", lib.DMIP_SAMPLER_CDE, 256, 3, 3, 23) == "fp32x3"


def test_fused_training_skips_non_tanh_networks(dmip):
    tr = importlib.import_module(PKG + ".training")
    assert tr._tanh_chain(dmip.MLP(5, 2, [64] * 3, torch.nn.Tanh()))
    assert not tr._tanh_chain(dmip.MLP(5, 2, [64] * 3, torch.nn.SiLU()))
