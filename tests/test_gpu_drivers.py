"""The training and evaluation drivers end to end on the device: train_linear with
the reference config's PINNLoss through the fused exact-f32 train_epoch, then evaluate_linear on the
trained network; train_scatterometry with PINNLoss whose initial condition is the surrogate posterior's
-energy_grad (main_diffusion_scatterometry.py:142-145), also fused. Needs an MI355X: `pytest -m gpu`."""
import importlib

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _mods():
    return (importlib.import_module("diffusion-modelling-for-inverse-problems_amd.training"),
            importlib.import_module("diffusion-modelling-for-inverse-problems_amd.evaluate"))


def test_train_then_evaluate_linear_on_device(dmip, tmp_path, monkeypatch):
    import pandas as pd
    monkeypatch.delenv("DMIP_TRAIN_PRECISION", raising=False)
    tr, ev = _mods()
    torch.manual_seed(0)
    f = dmip.LinearForwardProblem()
    xs = torch.randn(4000, 2)
    ys = f(xs)
    m = dmip.CDE(2, 2, [64] * 3)
    loss_fn = dmip.PINNLoss(f.score_posterior, lam=1e-3, lam2=0.1, pde_loss="FPE", ic_metric="L2", pde_metric="L1")
    opt = torch.optim.Adam(m.sde.a.parameters(), lr=1e-3)
    before = dmip._lib.calls.get("loss_grad_f32", 0)
    tr.train_linear(m, opt, loss_fn, vars(f), str(tmp_path / "ckpt"), str(tmp_path / "log"), 3, 1000,
                    xs.to(DEV), ys.to(DEV))
    assert dmip._lib.calls["loss_grad_f32"] - before == 12  # 3 epochs x 4 batches, all fused
    sd = torch.load(tmp_path / "ckpt" / "current_model.pt", weights_only=True)
    assert set(sd) == {"0.weight", "0.bias", "3.weight", "3.bias", "5.weight", "5.bias", "7.weight", "7.bias"}
    ys_eval = f(torch.randn(2, 2)).to(DEV)
    kl, nll, mse = ev.evaluate_linear(m, ys_eval, f, str(tmp_path), [], n_samples_x=4000, n_repeats=2, num_steps=100)
    df = pd.read_csv(tmp_path / "results.csv")
    assert list(df.columns)[1:] == ["KL2", "NLL_true", "NLL_diffusion", "MSE"] and len(df) == 2
    assert np.isfinite([kl, nll, mse]).all()


def test_train_scatterometry_pinn_energy_grad_ic_fused(dmip, tmp_path, monkeypatch):
    monkeypatch.delenv("DMIP_TRAIN_PRECISION", raising=False)
    tr, _ = _mods()
    fm, prm = dmip.load_forward_model(GOLDEN)
    fm = fm.to(DEV)
    torch.manual_seed(1)
    m = dmip.CDE(3, 23, [64] * 3)
    sp = lambda x, y: -dmip.energy_grad(x, lambda v: dmip.get_log_posterior(v, fm, prm["a"], prm["b"], y,
                                                                             prm["lambd_bd"]))[0]
    loss_fn = dmip.PINNLoss(sp, lam=0.01, lam2=0.001, pde_loss="FPE", ic_metric="L2", pde_metric="L1")
    opt = torch.optim.Adam(m.sde.a.parameters(), lr=1e-4)
    before = dmip._lib.calls.get("loss_grad_f32", 0)
    w0 = [p.detach().clone() for p in m.sde.a.parameters()]
    tr.train_scatterometry(m, opt, loss_fn, dict(prm), str(tmp_path / "s"), str(tmp_path / "slog"), 1, 500, fm)
    assert dmip._lib.calls["loss_grad_f32"] - before == 8  # one epoch = 8 batches of prior samples
    assert (tmp_path / "s" / "diffusion.pt").exists()
    assert all(not torch.equal(a, b) and torch.isfinite(b).all() for a, b in zip(w0, m.sde.a.parameters()))
