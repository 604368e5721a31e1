"""The exact-f32 training engine (dmip_loss_grad_f32: stacked jet streams through MFMA GEMMs) against the
reference's values and gradients -- at the linear fixture's width 64 (G5) and at the reference configs'
hidden_layers [512]*3 for both problems (G11) -- and against the oracle at other shapes.
Needs an MI355X: `pytest -m gpu`.

Tolerances: exact f32 arithmetic whose summation order differs from torch-CPU's, so the errors are
f32 rounding (measured, round 3: loss <= 7.5e-7 relative, every gradient tensor <= 9.2e-7 relative L2
against the reference's own values, <= 3.3e-7 against the float64 oracle; the L1 PDE metric's sign
flips did not show). Each bound is about 3-5x the measured value, stated beside it."""
import importlib

import numpy as np
import pytest
import torch

import oracle as O
from conftest import GOLDEN, state_from_npz

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _tr():
    return importlib.import_module("diffusion-modelling-for-inverse-problems_amd.training")


def _rel(a, b):
    return float(np.linalg.norm((np.asarray(a) - np.asarray(b)).ravel()) / max(1e-30, np.linalg.norm(np.asarray(b).ravel())))


def _step(dmip, m, lf, x, y, t, eps):
    cfg = _tr().fused_config(m, lf)
    assert cfg is not None
    before = dmip._lib.calls.get("loss_grad_f32", 0)
    loss, info = _tr().fused_loss_grad(m, lf, cfg, x, y, t, eps, precision="fp32")
    assert dmip._lib.calls["loss_grad_f32"] == before + 1
    return float(loss), {k: float(v) for k, v in info.items()}, [p.grad.detach().cpu().numpy() for p in m.sde.a.parameters()]


def _lin_losses(dmip):
    sp = dmip.LinearForwardProblem().score_posterior
    return {
        "pinn": dmip.PINNLoss(sp, lam=1e-3, lam2=0.1, pde_loss="FPE", ic_metric="L2", pde_metric="L1"),
        "pinn_l1l2": dmip.PINNLoss(sp, lam=0.5, lam2=0.3, pde_loss="FPE", ic_metric="L1", pde_metric="L2"),
        "dsmpde": dmip.DSM_PDELoss(lam=1e-2, pde_loss="FPE", pde_metric="L1"),
        "pinn_cfpe": dmip.PINNLoss(sp, lam=1e-3, lam2=0.1, pde_loss="cScoreFPE", ic_metric="L2", pde_metric="L2"),
        "dsm": dmip.DSMLoss(),
    }


@pytest.mark.parametrize("name", ["pinn", "pinn_l1l2", "dsmpde", "pinn_cfpe", "dsm"])
def test_f32_loss_grad_vs_reference_width64(dmip, golden, name):
    z = golden("pinn_linear.npz")
    m = dmip.CDE(2, 2, [64] * 3)
    m.sde.a.load_state_dict(state_from_npz(golden("ckpt_lin.npz")))
    args = [torch.from_numpy(z[k]).to(DEV) for k in ("x", "y", "t", "eps")]
    loss, info, grads = _step(dmip, m, _lin_losses(dmip)[name], *args)
    keys = ("0_weight", "0_bias", "3_weight", "3_bias", "5_weight", "5_bias", "7_weight", "7_bias")
    ref_grads = [z[f"{name}_grad_{k}"] for k in keys]
    ref_loss = float(z["dsm_rows"].mean()) if name == "dsm" else float(z[f"{name}_loss"])
    if name != "dsm":
        pde_rel = abs(info["PDE-Loss"] - float(z[f"{name}_PDE_Loss"])) / abs(float(z[f"{name}_PDE_Loss"]))
        print(f"\n[f32] G5 {name}: PDE component rel {pde_rel:.2e}")
        assert info["PDE-Loss"] == pytest.approx(float(z[f"{name}_PDE_Loss"]), rel=1e-4, abs=1e-7)
    errs = [_rel(g, r) for g, r in zip(grads, ref_grads)]
    print(f"\n[f32] G5 {name}: loss rel {abs(loss - ref_loss) / abs(ref_loss):.2e}, grad rel L2 {[f'{e:.2e}' for e in errs]}")
    assert loss == pytest.approx(ref_loss, rel=3e-6)  # measured <= 7.5e-7 (round 3)
    assert max(errs) < 3e-6, errs  # measured <= 9.2e-7 (round 3)


@pytest.mark.parametrize("tag", ["lin", "scat"])
def test_f32_loss_grad_vs_reference_width512(dmip, golden, tag):
    """PINNLoss at hidden_layers [512]*3 with each reference config's loss settings (G11). The
    scatterometry initial condition is the package's score_posterior on the device (the fused
    -energy_grad of get_log_posterior through the surrogate), exactly as the reference driver defines it."""
    z = golden("pinn_ref_configs.npz")
    xd, yd = (2, 2) if tag == "lin" else (3, 23)
    m = dmip.CDE(xd, yd, [512] * 3)
    lin = [l for l in m.sde.a if isinstance(l, torch.nn.Linear)]
    with torch.no_grad():
        for l, (W, b) in zip(lin, O.reference_weights([xd + yd + 1, 512, 512, 512, xd], int(z[f"{tag}_seed"]))):
            l.weight.copy_(torch.from_numpy(W))
            l.bias.copy_(torch.from_numpy(b))
    if tag == "lin":
        lf = dmip.PINNLoss(dmip.LinearForwardProblem().score_posterior, lam=1e-3, lam2=0.1, pde_loss="FPE",
                           ic_metric="L2", pde_metric="L1")
    else:
        fm, prm = dmip.load_forward_model(GOLDEN)
        fm = fm.to(DEV)
        sp = lambda x, y: -dmip.energy_grad(x, lambda v: dmip.get_log_posterior(v, fm, prm["a"], prm["b"], y,
                                                                                 prm["lambd_bd"]))[0]
        lf = dmip.PINNLoss(sp, lam=0.01, lam2=0.001, pde_loss="FPE", ic_metric="L2", pde_metric="L1")
    args = [torch.from_numpy(z[f"{tag}_{k}"]).to(DEV) for k in ("x", "y", "t", "eps")]
    loss, info, grads = _step(dmip, m, lf, *args)
    assert loss == pytest.approx(float(z[f"{tag}_loss"]), rel=2e-6)  # measured <= 3.5e-7 (round 3)
    assert info["Initial Condition"] == pytest.approx(float(z[f"{tag}_Initial_Condition"]), rel=1e-4)
    assert info["DSM-Loss"] == pytest.approx(float(z[f"{tag}_DSM_Loss"]), rel=1e-5)
    keys = ("0_weight", "0_bias", "3_weight", "3_bias", "5_weight", "5_bias", "7_weight", "7_bias")
    errs = [_rel(g, z[f"{tag}_grad_{k}"]) for g, k in zip(grads, keys)]
    print(f"\n[f32] G11 {tag}: loss rel {abs(loss - float(z[f'{tag}_loss'])) / abs(float(z[f'{tag}_loss'])):.2e}, "
          f"grad rel L2 {[f'{e:.2e}' for e in errs]}")
    assert max(errs) < 2e-6, errs  # measured <= 4.3e-7 (round 3)


@pytest.mark.parametrize("W,NL,n", [(100, 2, 777), (256, 3, 5003), (512, 1, 300)])
@pytest.mark.parametrize("name", ["pinn", "dsmpde", "pinn_cfpe"])
def test_f32_loss_grad_vs_oracle(dmip, W, NL, n, name):
    """Odd widths, other depths, ragged batches against the float64 oracle."""
    torch.manual_seed(W + NL)
    m = dmip.CDE(2, 2, [W] * NL)
    params = [(l.weight.detach().cpu().numpy(), l.bias.detach().cpu().numpy())
              for l in m.sde.a if isinstance(l, torch.nn.Linear)]
    g = np.random.default_rng(n)
    x = g.normal(size=(n, 2)).astype(np.float32)
    y = (x @ np.array([[1, 0.5], [0, 1]], np.float32).T + np.array([0.3, 0.5], np.float32)
         + 0.3 * g.normal(size=(n, 2))).astype(np.float32)
    t = (1e-4 + g.uniform(size=(n, 1)) * (1 - 1e-4)).astype(np.float32)
    eps = g.normal(size=(n, 2)).astype(np.float32)
    loss, info, grads = _step(dmip, m, _lin_losses(dmip)[name], *(torch.from_numpy(a).to(DEV) for a in (x, y, t, eps)))
    cfgs = {"pinn": dict(kind="pinn", pde="FPE", pde_metric="L1", ic_metric="L2", lam=1e-3, lam2=0.1),
            "dsmpde": dict(kind="dsm_pde", pde="FPE", pde_metric="L1", lam=1e-2),
            "pinn_cfpe": dict(kind="pinn", pde="cFPE", pde_metric="L2", ic_metric="L2", lam=1e-3, lam2=0.1)}
    ref_loss, _, ref = O.loss_grad(params, x, y, t, eps, **cfgs[name], ic_A=[[1, 0.5], [0, 1]], ic_b=[0.3, 0.5],
                                   ic_Sinv=np.eye(2) / 0.3)
    errs = [_rel(gk, rk) for gk, rk in zip(grads, [a for wb in ref for a in wb])]
    print(f"\n[f32] oracle W={W} L={NL} n={n} {name}: loss rel {abs(loss - ref_loss) / abs(ref_loss):.2e}, "
          f"grad rel L2 {[f'{e:.2e}' for e in errs]}")
    assert loss == pytest.approx(ref_loss, rel=3e-7)  # measured <= 4.3e-8 (round 3)
    assert max(errs) < 1e-6, errs  # measured <= 3.3e-7 (round 3)


@pytest.mark.parametrize("weights", ["trained", "init"])
def test_f32_config5_batch_65536_vs_oracle(dmip, golden, weights):
    """The exact-f32 engine on BASELINE config 5's batch (65,536, PINNLoss as bench.py) against the float64
    oracle: loss and every gradient tensor; the observed errors are printed (DESIGN.md §6 records them)."""
    if weights == "trained":
        m = dmip.CDE(2, 2, [64] * 3)
        m.sde.a.load_state_dict(state_from_npz(golden("ckpt_lin.npz")))
    else:
        torch.manual_seed(5)
        m = dmip.CDE(2, 2, [64] * 3)
    params = [(l.weight.detach().cpu().numpy(), l.bias.detach().cpu().numpy())
              for l in m.sde.a if isinstance(l, torch.nn.Linear)]
    g = np.random.default_rng(2024)
    n = 65536
    x = g.normal(size=(n, 2)).astype(np.float32)
    y = (x @ np.array([[1, 0.5], [0, 1]], np.float32).T + np.array([0.3, 0.5], np.float32)
         + 0.3 * g.normal(size=(n, 2))).astype(np.float32)
    t = (1e-4 + g.uniform(size=(n, 1)) * (1 - 1e-4)).astype(np.float32)
    eps = g.normal(size=(n, 2)).astype(np.float32)
    loss, info, grads = _step(dmip, m, _lin_losses(dmip)["pinn"], *(torch.from_numpy(a).to(DEV) for a in (x, y, t, eps)))
    ref_loss, _, ref = O.loss_grad(params, x, y, t, eps, kind="pinn", pde="FPE", pde_metric="L1", ic_metric="L2",
                                   lam=1e-3, lam2=0.1, ic_A=[[1, 0.5], [0, 1]], ic_b=[0.3, 0.5], ic_Sinv=np.eye(2) / 0.3)
    errs = [_rel(gk, rk) for gk, rk in zip(grads, [a for wb in ref for a in wb])]
    lrel = abs(loss - ref_loss) / abs(ref_loss)
    print(f"\n[f32] config5 B=65536 {weights}: loss rel {lrel:.2e}, grad rel L2 {[f'{e:.2e}' for e in errs]}")
    assert lrel < 2e-7, lrel  # measured 3.2e-8 / 8.8e-10 (round 3)
    assert max(errs) < 1e-6, errs  # measured <= 2.3e-7 (round 3)


def test_f32_loss_grad_deterministic(dmip, golden):
    z = golden("pinn_linear.npz")
    m = dmip.CDE(2, 2, [64] * 3)
    m.sde.a.load_state_dict(state_from_npz(golden("ckpt_lin.npz")))
    args = [torch.from_numpy(np.tile(z[k], (40, 1))).to(DEV) for k in ("x", "y", "t", "eps")]
    lf = _lin_losses(dmip)["pinn"]
    a = _step(dmip, m, lf, *args)
    b = _step(dmip, m, lf, *args)
    assert a[0] == b[0] and all(np.array_equal(u, v) for u, v in zip(a[2], b[2]))


def test_train_epoch_default_is_exact_f32_and_tracks_autograd(dmip, monkeypatch):
    """CDE.train_epoch at the reference width [512]*3 takes the f32 engine by default and follows the
    autograd path's losses (DMIP_TRAIN_FUSED=0) batch by batch from the same seeds."""
    monkeypatch.delenv("DMIP_TRAIN_PRECISION", raising=False)

    def run(fused):
        monkeypatch.setenv("DMIP_TRAIN_FUSED", "1" if fused else "0")
        torch.manual_seed(0)
        m = dmip.CDE(2, 2, [512] * 3)
        opt = torch.optim.Adam(m.sde.a.parameters(), lr=1e-4)
        gen = torch.Generator().manual_seed(1)
        x = torch.randn(2048, 2, generator=gen)
        y = x @ torch.tensor([[1, 0.5], [0, 1.]]).T + torch.tensor([0.3, 0.5]) + 0.3 * torch.randn(2048, 2, generator=gen)
        x, y = x.to(DEV), y.to(DEV)

        def loader():
            for i in range(0, 2048, 512):
                yield x[i:i + 512], y[i:i + 512]
        before = dmip._lib.calls.get("loss_grad_f32", 0)
        torch.manual_seed(5)
        loss, info = m.train_epoch(opt, _lin_losses(dmip)["pinn"], loader)
        return float(loss), info, dmip._lib.calls.get("loss_grad_f32", 0) - before
    lf, info_f, nf = run(True)
    la, info_a, na = run(False)
    assert nf == 4 and na == 0
    assert lf == pytest.approx(la, rel=1e-3)
    for k in info_a:
        assert info_f[k] == pytest.approx(info_a[k], rel=1e-2, abs=1e-6)


def _cdiffe_dsm_f64(m, z, t, eps):
    """CDiffE.train_epoch's DSM batch loss (models/diffusion.py:128-136, losses.py:50-52) by float64
    autograd on the CPU: the reference semantics at a precision well above the kernel's."""
    import copy
    net = copy.deepcopy(m.sde.a).cpu().double()
    base = m.sde.base_sde
    z, t, eps = (v.detach().cpu().double() for v in (z, t, eps))
    std = base.var(t) ** 0.5
    zt = eps * std + base.mean_weight(t) * z
    g = base.g(t, zt)
    score = net(zt[:, :m.xdim], zt[:, m.xdim:], t) / g
    loss = (((score * std + eps) ** 2).sum(1) / 2).mean()
    loss.backward()
    return float(loss), [p.grad.numpy() for p in net.parameters()]


@pytest.mark.parametrize("xd,yd,W,n", [(2, 2, 64, 1000), (2, 2, 512, 4096), (3, 23, 256, 777), (3, 23, 512, 2048)])
def test_cdiffe_joint_dsm_vs_autograd(dmip, xd, yd, W, n):
    """CDiffE's joint DSM (state z = (x, y), 26-D for scatterometry) through dmip_loss_grad_f32 with
    ydim 0, against float64 autograd of the reference loss on the same (z, t, eps). Tolerances: loss
    1e-4 relative, every gradient tensor 2e-3 relative L2 (exact f32 vs f64)."""
    torch.manual_seed(W + xd)
    m = dmip.CDiffE(xd, yd, [W] * 3)
    lf = dmip.DSMLoss()
    cfg = _tr().joint_fused_config(m, lf)
    assert cfg is not None
    g = torch.Generator().manual_seed(3)
    z = torch.randn(n, xd + yd, generator=g)
    t = (1e-4 + torch.rand(n, 1, generator=g)).clamp(max=1.0)
    eps = torch.randn(n, xd + yd, generator=g)
    before = dmip._lib.calls.get("loss_grad_f32", 0)
    loss, info = _tr().fused_loss_grad(m, lf, cfg, z.to(DEV), None, t.to(DEV), eps.to(DEV))
    assert dmip._lib.calls["loss_grad_f32"] == before + 1 and info == {}
    grads = [p.grad.detach().cpu().numpy() for p in m.sde.a.parameters()]
    ref_loss, ref_grads = _cdiffe_dsm_f64(m, z, t, eps)
    assert float(loss) == pytest.approx(ref_loss, rel=1e-4)
    errs = [_rel(gk, rk) for gk, rk in zip(grads, ref_grads)]
    assert max(errs) < 2e-3, errs


def test_cdiffe_train_epoch_fused_tracks_autograd(dmip, monkeypatch):
    """CDiffE.train_epoch (scatterometry shape, [256]*3, DSMLoss) takes the fused engine on the device and
    follows the autograd path (DMIP_TRAIN_FUSED=0) batch by batch from the same seeds."""
    def run(fused):
        monkeypatch.setenv("DMIP_TRAIN_FUSED", "1" if fused else "0")
        torch.manual_seed(0)
        m = dmip.CDiffE(3, 23, [256] * 3)
        opt = torch.optim.Adam(m.sde.a.parameters(), lr=1e-4)
        gen = torch.Generator().manual_seed(1)
        x = torch.rand(2048, 3, generator=gen).to(DEV)
        y = torch.randn(2048, 23, generator=gen).to(DEV)

        def loader():
            for i in range(0, 2048, 512):
                yield x[i:i + 512], y[i:i + 512]
        before = dmip._lib.calls.get("loss_grad_f32", 0)
        torch.manual_seed(5)
        loss, _ = m.train_epoch(opt, dmip.DSMLoss(), loader)
        return float(loss), dmip._lib.calls.get("loss_grad_f32", 0) - before
    lf, nf = run(True)
    la, na = run(False)
    assert nf == 4 and na == 0
    assert lf == pytest.approx(la, rel=1e-3)


@pytest.mark.parametrize("tag,xd,yd,W", [("lin", 2, 2, 64), ("scat", 3, 23, 128)])
def test_cdiffe_joint_dsm_vs_reference(dmip, golden, tag, xd, yd, W):
    """G12: the fused engine's CDiffE DSM loss and gradients against the reference's own
    (models/diffusion.py:128-136 on the same weights and draws); 1e-4 loss, 2e-3 gradient rel-L2."""
    z = golden("cdiffe_dsm.npz")
    m = dmip.CDiffE(xd, yd, [W] * 3)
    m.sde.a.load_state_dict({k: torch.from_numpy(z[f"{tag}_{k.replace('.', '_')}"])
                             for k in m.sde.a.state_dict().keys()})
    lf = dmip.DSMLoss()
    cfg = _tr().joint_fused_config(m, lf)
    args = [torch.from_numpy(z[f"{tag}_{k}"]).to(DEV) for k in ("z", "t", "eps")]
    loss, _ = _tr().fused_loss_grad(m, lf, cfg, args[0], None, args[1], args[2])
    assert float(loss) == pytest.approx(float(z[f"{tag}_loss"]), rel=1e-4)
    for name, p in m.sde.a.named_parameters():
        ref = z[f"{tag}_grad_{name.replace('.', '_')}"]
        assert _rel(p.grad.detach().cpu().numpy(), ref) < 2e-3, name
