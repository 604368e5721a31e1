"""The SiLU activation chain on the device (include/dmip.h DMIP_ACT_SILU_TWICE_FIRST): a reference-layout MLP
built with nn.SiLU (nets.py:17's `activation` argument; layer 1 applies it twice by the same re-registration
as tanh) runs the exact-f32 forward and the exact-f32 CDE sampler; every other kernel computes tanh and refuses
it. Tolerances: forward 1e-5 of max|out| against torch's fp32 module chain on the device (a plain fp32
reference of the same op); sampler 1e-4 max(1, |x|) against oracle.cde_sample(act="silu") after 6 steps (the
exact-f32 CDE tests' bound, test_gpu_f32.py)."""
import importlib

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _params(net):
    return [(l.weight.detach().cpu().numpy(), l.bias.detach().cpu().numpy())
            for l in net if isinstance(l, torch.nn.Linear)]


def _silu_cde(dmip, W, seed, xdim=3, ydim=23):
    torch.manual_seed(seed)
    m = dmip.CDE(xdim, ydim, [W] * 3)
    m.sde.a = dmip.MLP(xdim + ydim + 1, xdim, [W] * 3, torch.nn.SiLU()).to(DEV)
    with torch.no_grad():  # a smooth, well-conditioned drift for a trajectory comparison
        last = [l for l in m.sde.a if isinstance(l, torch.nn.Linear)][-1]
        last.weight.mul_(0.1)
    return m


@pytest.mark.parametrize("W", [64, 256, 512])
def test_silu_forward_vs_torch_fp32(dmip, W):
    torch.manual_seed(W)
    net = dmip.MLP(3 + 23 + 1, 3, [W] * 3, torch.nn.SiLU()).to(DEV)
    x, y, t = torch.randn(777, 3, device=DEV), torch.rand(777, 23, device=DEV), torch.rand(777, device=DEV)
    ref = torch.nn.Sequential.forward(net, torch.cat([x, y, t[:, None]], 1)).detach()  # torch's module chain
    before = dmip._lib.calls["mlp_forward"]
    for prec in ("fp32", "fp16"):  # a 16-bit request still runs the SiLU chain's exact-f32 forward
        net.dmip_precision = prec
        with torch.no_grad():
            out = net(x, y, t)
        err = (out - ref).abs().max().item()
        assert err < 1e-5 * max(1.0, ref.abs().max().item()), (prec, err)
    assert dmip._lib.calls["mlp_forward"] == before + 2
    tanh = dmip.MLP(3 + 23 + 1, 3, [W] * 3, torch.nn.Tanh()).to(DEV)
    tanh.load_state_dict(net.state_dict())
    with torch.no_grad():
        assert (tanh(x, y, t) - out).abs().max().item() > 1e-3  # a different chain, not tanh


@pytest.mark.parametrize("W,xdim,ydim", [(64, 2, 2), (256, 3, 23), (512, 3, 23)])
def test_silu_cde_sampler_vs_oracle(dmip, W, xdim, ydim):
    """Every requested precision runs the fused exact-f32 CDE kernel for a SiLU network (one em_sample launch),
    chain for chain equal to the oracle's SiLU chain within 1e-4."""
    m = _silu_cde(dmip, W, 5 + W, xdim, ydim)
    y = np.random.default_rng(W).uniform(0, 1, ydim).astype(np.float32)
    n, S, seed = 500, 6, 9
    ref = O.cde_sample(_params(m.sde.a), y, n, S, seed, act="silu")
    for prec in ("fp32x3", "fp32", "fp16"):
        before = dmip._lib.calls["em_sample"]
        x = m.sample_device(torch.from_numpy(y).to(DEV), n, S, seed=seed, precision=prec)[0].cpu().numpy()
        assert dmip._lib.calls["em_sample"] == before + 1
        err = np.abs(x - ref).max()
        assert err < 1e-4 * max(1.0, np.abs(ref).max()), (prec, err)
    tanh = O.cde_sample(_params(m.sde.a), y, n, S, seed)
    assert np.abs(tanh - ref).max() > 1e-3


def test_silu_cde_shards_and_injected_noise(dmip):
    m = _silu_cde(dmip, 256, 31)
    ys = torch.from_numpy(np.random.default_rng(2).uniform(0, 1, (2, 23)).astype(np.float32)).to(DEV)
    full = m.sample_device(ys, 900, 5, seed=4)
    shard = m.sample_device(ys, 300, 5, seed=4, chain_offset=400)
    assert torch.equal(full[:, 400:700], shard) and torch.isfinite(full).all()
    # injected noise (the reference's randn draws): the fused SiLU kernel against the oracle's EM loop
    y = ys[0].cpu().numpy()
    noise = np.random.default_rng(7).standard_normal((6, 1, 200, 3)).astype(np.float32)
    x = m.sample_device(ys[:1], 200, 5, noise=torch.from_numpy(noise).to(DEV))[0].cpu().numpy()
    p = _params(m.sde.a)
    ref = O.em_sample(lambda xx, tau: O.cde_a(p, xx, y, tau, act="silu"), noise[0, 0], 5, noise=noise[1:, 0])
    assert np.abs(x - ref).max() < 1e-4 * max(1.0, np.abs(ref).max())


def test_silu_posterior_runs_the_device_loop(dmip):
    """No fused Posterior kernel has the SiLU chain: the estimator steps through the per-step loop of exact-f32
    forward launches (never the tanh kernel), shard-invariant like the fused samplers."""
    torch.manual_seed(6)
    m = dmip.PosteriorDiffusionEstimator(3, 23, [64] * 2)
    sc = m.sde.a
    for name in ("prior_net", "likelihood_net"):
        old = getattr(sc, name)
        new = type(old)(old.input_dim, old.output_dim, old.hidden_layers, torch.nn.SiLU()).to(DEV)
        setattr(sc, name, new)
    y = torch.from_numpy(np.random.default_rng(3).uniform(0, 1, 23).astype(np.float32)).to(DEV)
    b_post, b_fwd = dmip._lib.calls["em_sample_posterior"], dmip._lib.calls["mlp_forward"]
    full = m.sample_device(y, 400, 4, seed=2)
    assert dmip._lib.calls["em_sample_posterior"] == b_post and dmip._lib.calls["mlp_forward"] >= b_fwd + 8
    shard = m.sample_device(y, 100, 4, seed=2, chain_offset=150)
    assert torch.isfinite(full).all() and torch.equal(full[:, 150:250], shard)


def test_silu_refused_where_not_compiled(dmip, golden):
    """The tanh-only kernels refuse a SiLU network loudly (never a silent tanh): the 16-bit and fp32x3 samplers
    through the C-ABI, DPS, and an activation with no kernel at all (ReLU) at the estimator."""
    m = _silu_cde(dmip, 256, 8)
    h = m.sde.a.dmip_handle(torch.device(DEV), 3)
    ys = torch.rand(1, 23, device=DEV)
    _, _, sde, out = m._prepare(ys[0], 64, 2, [m.sde.a])
    for prec in ("fp16", "fp32x3"):
        with pytest.raises(ValueError, match="SiLU"):
            dmip._lib.em_sample(h, sde, ys, 64, 0, 2, 0.0, 1.0, 1, out, None, prec)
    z = golden("surrogate.npz")
    fm = torch.nn.Sequential(torch.nn.Linear(3, 256), torch.nn.ReLU(), torch.nn.Linear(256, 256), torch.nn.ReLU(),
                             torch.nn.Linear(256, 256), torch.nn.ReLU(), torch.nn.Linear(256, 23))
    fm.load_state_dict({k.replace("_", "."): torch.from_numpy(z[k]) for k in z.files})
    d = dmip.DPS(3, 23, [256] * 3, fm.to(DEV))
    pn = d.sde.a.prior_net
    d.sde.a.prior_net = type(pn)(pn.input_dim, pn.output_dim, pn.hidden_layers, torch.nn.SiLU()).to(DEV)
    for prec in ("fp32", "fp32x3"):
        with pytest.raises(ValueError, match="SiLU"):
            d.sample_device(ys[0], 64, 2, seed=1, precision=prec)
    m.sde.a = dmip.MLP(27, 3, [64] * 3, torch.nn.ReLU()).to(DEV)
    with pytest.raises(NotImplementedError, match="ReLU"):
        m.sample_device(ys[0], 64, 2, seed=1)


def test_silu_cde_trains_through_autograd(dmip):
    """The fused loss + gradient engines differentiate the tanh chain only: a SiLU CDE's train_epoch takes the
    autograd path (no fused loss launch) and its loss decreases."""
    m = _silu_cde(dmip, 64, 12, 2, 2)
    prob = dmip.LinearForwardProblem()
    x = torch.randn(4096, 2, device=DEV)
    yv = x @ prob.A.to(DEV).T + prob.b.to(DEV) + 0.3 * torch.randn(4096, 2, device=DEV)
    def loader():
        return [(x[i:i + 512], yv[i:i + 512]) for i in range(0, 4096, 512)]
    opt = torch.optim.Adam(m.sde.a.parameters(), lr=1e-3)
    calls = dict(dmip._lib.calls)
    l0 = float(m.train_epoch(opt, dmip.DSMLoss(), loader)[0])
    for _ in range(4):
        l1 = float(m.train_epoch(opt, dmip.DSMLoss(), loader)[0])
    assert dmip._lib.calls.get("loss_grad", 0) == calls.get("loss_grad", 0)
    assert dmip._lib.calls.get("loss_grad_f32", 0) == calls.get("loss_grad_f32", 0)
    assert np.isfinite(l1) and l1 < l0


def test_activation_without_kernel_forward_is_the_module_chain(dmip):
    """an MLP / MLP2 with an activation that has no HIP kernel (ReLU) evaluates as the reference does --
    the module chain, on the device -- instead of raising; only the fused samplers refuse it (test above)."""
    torch.manual_seed(3)
    for cls, args in ((dmip.MLP, (27, 3)), (dmip.MLP2, (4, 3))):
        net = cls(*args, [64] * 3, torch.nn.ReLU()).to(DEV)
        x = torch.randn(128, 3, device=DEV)
        y = torch.randn(128, 23, device=DEV)
        t = torch.rand(128, 1, device=DEV)
        inp = torch.cat([x, y, t], 1) if cls is dmip.MLP else torch.cat([x, t], 1)
        with torch.no_grad():
            out = net(x, y, t) if cls is dmip.MLP else net(x, t)
            ref = torch.nn.Sequential.forward(net, inp)
        assert torch.equal(out, ref)
