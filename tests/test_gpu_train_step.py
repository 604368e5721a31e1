"""The whole CDE training step on the device (training.DeviceTrainStep: dmip_train_draws ->
dmip_loss_grad[_f32] -> dmip_adam_step). Needs an MI355X: `pytest -m gpu`.

  * dmip_train_draws against oracle.train_draws (same generator, float64 inverse CDF): t to 1e-4
    relative (+1e-6 absolute: float32 inverse CDF), eps to 2e-5 absolute (device log/sin/cos);
  * dmip_adam_step against torch.optim.Adam (the reference's optimizer) on the same gradients:
    parameters and both moments to 2e-6 relative (element-wise rounding of the same formula);
  * a DeviceTrainStep step equals fused_loss_grad on its (t, eps) followed by torch's Adam, and
    CDE.train_epoch with $DMIP_TRAIN_DEVICE_STEP=1 runs one fused launch per batch and no
    optimizer.step()."""
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


def _tr():
    return importlib.import_module("diffusion-modelling-for-inverse-problems_amd.training")


def _lib():
    return importlib.import_module("diffusion-modelling-for-inverse-problems_amd._lib")


def _lin_data(n, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 2, generator=g)
    y = x @ torch.tensor([[1, 0.5], [0, 1.]]).T + torch.tensor([0.3, 0.5]) + 0.3 * torch.randn(n, 2, generator=g)
    return x.to(DEV), y.to(DEV)


@pytest.mark.parametrize("debias", [True, False])
@pytest.mark.parametrize("xdim,B,k", [(2, 10007, 0), (3, 4099, 5), (1, 1, 7)])
def test_train_draws_vs_oracle(debias, xdim, B, k):
    import ctypes
    L = _lib()
    t = torch.empty(B, device=DEV)
    eps = torch.empty(B, xdim, device=DEV)
    sde = L.vpsde(0.1, 20.0, 1.0)
    seed = 0x1234_5678_9ABC + xdim
    L.check(L.lib().dmip_train_draws(ctypes.c_uint64(seed), ctypes.c_uint64(k), B, xdim, int(debias),
                                     ctypes.byref(sde), 1e-3, 1e-4, L.ptr(t), L.ptr(eps), L.stream_of(t.device)))
    torch.cuda.synchronize()
    rt, reps = O.train_draws(seed, k, B, xdim, debias)
    np.testing.assert_allclose(t.cpu().numpy(), rt, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(eps.cpu().numpy(), reps, rtol=0, atol=2e-5)
    assert float(t.min()) > 0 and float(t.max()) <= 1.0


def test_train_draws_distribution():
    """t follows the debiased density (mass below t_eps = t_eps r(t_eps) / Z) and eps is N(0, 1),
    independent of t -- over 2^20 draws."""
    import ctypes
    L = _lib()
    B = 1 << 20
    t = torch.empty(B, device=DEV)
    eps = torch.empty(B, 2, device=DEV)
    sde = L.vpsde(0.1, 20.0, 1.0)
    L.check(L.lib().dmip_train_draws(ctypes.c_uint64(99), ctypes.c_uint64(0), B, 2, 1, ctypes.byref(sde), 1e-3,
                                     1e-4, L.ptr(t), L.ptr(eps), L.stream_of(t.device)))
    t, e = t.double().cpu().numpy(), eps.double().cpu().numpy()
    # CDF at 0.5 of the density, from the oracle's inverse CDF by bisection on u
    lo, hi = 0.0, 1.0
    for _ in range(60):
        mid = 0.5 * (lo + hi)
        lo, hi = (mid, hi) if O.vp_truncated_q(mid) + 1e-4 < 0.5 else (lo, mid)
    assert abs((t < 0.5).mean() - lo) < 5 / np.sqrt(B)
    assert abs(e.mean()) < 5 / np.sqrt(B) and abs(e.std() - 1) < 5 / np.sqrt(B)
    assert abs(np.corrcoef(t, e[:, 0])[0, 1]) < 5 / np.sqrt(B)


@pytest.mark.parametrize("foreach", [False, True])
def test_adam_step_matches_torch(dmip, foreach):
    import ctypes
    L = _lib()
    torch.manual_seed(3)
    m = dmip.CDE(2, 2, [64] * 3)
    ref = [p.detach().clone().requires_grad_(True) for p in m.sde.a.parameters()]
    mine = [p.detach().clone() for p in m.sde.a.parameters()]
    opt = torch.optim.Adam(ref, lr=3e-3, betas=(0.9, 0.99), eps=1e-8, foreach=foreach)
    ma = [torch.zeros_like(p) for p in mine]
    va = [torch.zeros_like(p) for p in mine]
    n = len(mine)
    vp = lambda ts: (ctypes.c_void_p * n)(*[x.data_ptr() for x in ts])
    for step in range(1, 6):
        grads = [torch.randn_like(p) * 10 ** float(np.random.default_rng(step).uniform(-3, 1)) for p in mine]
        for p, g in zip(ref, grads):
            p.grad = g.clone()
        opt.step()
        L.check(L.lib().dmip_adam_step(n, vp(mine), vp(grads), vp(ma), vp(va), (L._i64 * n)(*[p.numel() for p in mine]),
                                       3e-3, 0.9, 0.99, 1e-8, step, L.stream_of(torch.device(DEV))))
    torch.cuda.synchronize()
    for p, q, a, v in zip(ref, mine, ma, va):
        st = opt.state[p]
        for x, y in ((p.detach(), q), (st["exp_avg"], a), (st["exp_avg_sq"], v)):
            err = float((x - y).abs().max() / x.abs().max().clamp_min(1e-30))
            assert err < 2e-6, err


@pytest.mark.parametrize("graph", ["1", "0"])
@pytest.mark.parametrize("precision,width", [("fp32", 512), ("fp32", 64), ("bf16", 64)])
def test_device_step_equals_fused_then_torch_adam(dmip, precision, width, graph, monkeypatch):
    """graph "1": the captured-graph step (dmip_train_plan; two batch sizes, so two plans and a
    counter re-sync), "0": the launch-by-launch step."""
    monkeypatch.setenv("DMIP_TRAIN_GRAPH", graph)
    tr = _tr()
    torch.manual_seed(11)
    a = dmip.CDE(2, 2, [width] * 3)
    b = dmip.CDE(2, 2, [width] * 3)
    b.sde.a.load_state_dict(a.sde.a.state_dict())
    sp = dmip.LinearForwardProblem().score_posterior
    lf = dmip.PINNLoss(sp, lam=1e-3, lam2=0.1, pde_loss="FPE", ic_metric="L2", pde_metric="L1")
    oa = torch.optim.Adam(a.sde.a.parameters(), lr=1e-3)
    ob = torch.optim.Adam(b.sde.a.parameters(), lr=1e-3)
    step = tr.DeviceTrainStep(a, lf, oa, precision=precision)
    assert step.graph == (graph == "1")
    cfg = tr.fused_config(b, lf)
    n_plan = dmip._lib.calls.get("train_plan_step", 0)
    for k, n in enumerate((4096, 4096, 1000, 4096)):
        x, y = _lin_data(n, k)
        out = step(x, y).clone()
        loss_b, _ = tr.fused_loss_grad(b, lf, cfg, x, y, step.t.clone(), step.eps.clone(), precision=precision)
        ob.step()
        assert float(out[0]) == pytest.approx(float(loss_b), rel=1e-6)
    for p, q in zip(a.sde.a.parameters(), b.sde.a.parameters()):
        err = float((p - q).abs().max() / q.abs().max())
        assert err < 1e-5, err
    assert int(oa.state[next(a.sde.a.parameters())]["step"]) == 4
    assert dmip._lib.calls.get("train_plan_step", 0) - n_plan == (4 if graph == "1" else 0)


def test_graph_step_matches_launch_by_launch_step(dmip, monkeypatch):
    """The captured step replays the launch-by-launch step: same draws (stream id from the device
    counter), same loss, parameters equal to 1e-6 relative after 6 steps over two batch sizes (Adam's
    bias corrections in device vs host double pow)."""
    tr = _tr()
    sp = dmip.LinearForwardProblem().score_posterior
    lf = dmip.PINNLoss(sp, lam=1e-3, lam2=0.1, pde_loss="FPE", ic_metric="L2", pde_metric="L1")
    runs = {}
    for graph in ("1", "0"):
        monkeypatch.setenv("DMIP_TRAIN_GRAPH", graph)
        torch.manual_seed(3)
        m = dmip.CDE(2, 2, [512] * 3)
        opt = torch.optim.Adam(m.sde.a.parameters(), lr=1e-3)
        st = tr.DeviceTrainStep(m, lf, opt)
        losses, ts = [], []
        for k, n in enumerate((1000, 1000, 1000, 357, 1000, 1000)):
            x, y = _lin_data(n, 20 + k)
            losses.append(st(x, y).clone())
            ts.append(st.t.clone())
        runs[graph] = (m, [float(v[0]) for v in losses], ts)
    (ma, la, ta), (mb, lb, tb) = runs["1"], runs["0"]
    assert all(torch.equal(u, v) for u, v in zip(ta, tb))
    assert la[0] == lb[0]
    np.testing.assert_allclose(la, lb, rtol=1e-5)
    for p, q in zip(ma.sde.a.parameters(), mb.sde.a.parameters()):
        assert float((p - q).abs().max() / q.abs().max()) < 1e-6


def test_train_epoch_device_step(dmip, monkeypatch):
    monkeypatch.setenv("DMIP_TRAIN_DEVICE_STEP", "1")
    monkeypatch.delenv("DMIP_TRAIN_PRECISION", raising=False)
    torch.manual_seed(0)
    m = dmip.CDE(2, 2, [512] * 3)
    opt = torch.optim.Adam(m.sde.a.parameters(), lr=1e-4)
    calls = {"n": 0}
    orig = opt.step

    def counted(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)
    opt.step = counted
    x, y = _lin_data(2048, 1)
    before = [p.detach().clone() for p in m.sde.a.parameters()]
    n0 = dmip._lib.calls.get("loss_grad_f32", 0)
    p0 = dmip._lib.calls.get("train_plan_step", 0)

    def loader():
        for i in range(0, 2048, 512):
            yield x[i:i + 512], y[i:i + 512]
    sp = dmip.LinearForwardProblem().score_posterior
    loss, info = m.train_epoch(opt, dmip.PINNLoss(sp, lam=1e-3, lam2=0.1, pde_loss="FPE", ic_metric="L2",
                                                  pde_metric="L1"), loader)
    n_fused = dmip._lib.calls.get("loss_grad_f32", 0) - n0 + dmip._lib.calls.get("train_plan_step", 0) - p0
    assert n_fused == 4 and calls["n"] == 0
    assert np.isfinite(float(loss)) and set(info) == {"PDE-Loss", "Initial Condition", "DSM-Loss"}
    assert all(not torch.equal(p, q) for p, q in zip(m.sde.a.parameters(), before))
    assert int(opt.state[next(m.sde.a.parameters())]["step"]) == 4


def test_bf16_graph_step_pipelined_matches_launch_by_launch(dmip, monkeypatch):
    """The config-5 captured step (four launches: draws + weight pack, forward half, reverse half, reduction +
    Adam + counter advance; the batch staged by the draws launch, its kernel node re-pointed at each step's x / y)
    against the launch-by-launch step: steps issued back to back with no host synchronisation and a new batch
    every step (a node update must not reach a replay still in flight), over two batch sizes. Same draws, same
    first loss, parameters within 1e-6 after 8 steps."""
    tr = _tr()
    sp = dmip.LinearForwardProblem().score_posterior
    lf = dmip.PINNLoss(sp, lam=1e-3, lam2=0.1, pde_loss="FPE", ic_metric="L2", pde_metric="L1")
    sizes = (4096, 4096, 4096, 1000, 4096, 4096, 65536, 4096)
    data = [tuple(v.to("cuda:0") for v in _lin_data(n, 40 + k)) for k, n in enumerate(sizes)]
    torch.cuda.synchronize()
    runs = {}
    for graph in ("1", "0"):
        monkeypatch.setenv("DMIP_TRAIN_GRAPH", graph)
        torch.manual_seed(9)
        m = dmip.CDE(2, 2, [64] * 3)
        opt = torch.optim.Adam(m.sde.a.parameters(), lr=1e-3)
        st = tr.DeviceTrainStep(m, lf, opt, precision="bf16")
        assert st.graph == (graph == "1")
        losses, ts = [], []
        for x, y in data:
            losses.append(st(x, y).clone())
            ts.append(st.t.clone())
        torch.cuda.synchronize()
        runs[graph] = (m, [float(v[0]) for v in losses], ts)
    (ma, la, ta), (mb, lb, tb) = runs["1"], runs["0"]
    assert all(torch.equal(u, v) for u, v in zip(ta, tb))
    assert la[0] == lb[0]
    np.testing.assert_allclose(la, lb, rtol=1e-5)
    for p, q in zip(ma.sde.a.parameters(), mb.sde.a.parameters()):
        assert float((p - q).abs().max() / q.abs().max()) < 1e-6
