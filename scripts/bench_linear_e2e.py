"""The reference's linear configuration (config/config_linear.yml) trained to completion on one MI355X and
evaluated at the reference's own sizes, through the package's reference-API functions.

Recipe (main_diffusion_linear.py:140-163 with config_linear.yml): dataset of 100,000 (x ~ N(0, I), y = f(x)),
train_test_split(train_size=.9, random_state=7); CDE [512]^3 + PINNLoss (lam 0.001, lam2 0.1, FPE, L1 PDE
metric, L2 IC metric, the analytic score_posterior as the initial condition); Adam lr 1e-4; 1500 epochs of
shuffled batches of 1000 with fresh observation noise (datasets.py:44-54) = 135,000 optimizer steps. Then
`evaluate` (main_diffusion_linear.py:53-137): the first 100 test ys, 10 repeats x 30,000 posterior samples
(200 SDE steps) against the analytic Gaussian posterior (KL2 of 75x75 histograms, NLPD, score MSE at t=0).
The config file itself is not read (the reference tree is not on the GPU box); its values are restated here.
With --fixture: no training; the CPU-trained fixture CDE [64]^3 (tests/golden/ckpt_lin.npz, DSMLoss with uniform t,
make_golden.py) is evaluated the same way, as the control for the trained model's scores.
    python scripts/bench_linear_e2e.py [--epochs 1500] [--n-y 100] [--n 30000] [--fixture]"""
import argparse
import importlib
import json
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIG = {  # config_linear.yml
    "dataset_size": 100000, "train_size": .9, "random_state": 7, "lr": 1e-4, "n_epochs": 1500,
    "model": "CDE", "loss_fn": "PINNLoss", "lam": 0.001, "lam2": 0.1, "pde_loss": "FPE", "pde_metric": "L1",
    "ic_metric": "L2", "batch_size": 1000, "hidden_layers": [512, 512, 512], "n_samples_y": 100,
    "n_samples_x": 30000, "n_repeats": 10,
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=CONFIG["n_epochs"])
    ap.add_argument("--n-y", type=int, default=CONFIG["n_samples_y"])
    ap.add_argument("--n", type=int, default=CONFIG["n_samples_x"])
    ap.add_argument("--repeats", type=int, default=CONFIG["n_repeats"])
    ap.add_argument("--fixture", action="store_true", help="evaluate the CPU-trained fixture checkpoint only")
    a = ap.parse_args()
    from sklearn.model_selection import train_test_split
    pkg = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
    ev = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.evaluate")
    pr = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.problems")
    tr = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.training")
    fac = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.factory")
    dev = torch.device("cuda:0")
    torch.manual_seed(0)

    f = pr.LinearForwardProblem()
    # datasets.py:37-41 on the CPU (same seed and draws): the reference's version moves x to the device but
    # keeps A on the CPU (linear_problem.py:14,27), so it fails on a CUDA host
    gen = torch.random.manual_seed(CONFIG["random_state"])
    xs = torch.randn(CONFIG["dataset_size"], f.xdim, generator=gen)
    ys = f(xs)
    x_train, x_test, y_train, y_test = train_test_split(xs.cpu(), ys.cpu(), train_size=CONFIG["train_size"],
                                                        random_state=CONFIG["random_state"])
    cfg = dict(CONFIG, hidden_layers=[64] * 3) if a.fixture else CONFIG
    model, loss_fn = fac.get_model_from_args(cfg, vars(f), f.score_posterior, f)
    if a.fixture:
        sys.path.insert(0, __import__("os").path.join(ROOT, "tests"))
        from conftest import state_from_npz
        model.sde.a.load_state_dict(state_from_npz(np.load(__import__("os").path.join(ROOT, "tests", "golden", "ckpt_lin.npz"))))
        a.epochs = 0
    model.sde.a.to(dev)
    opt = torch.optim.Adam(model.sde.a.parameters(), lr=CONFIG["lr"])
    x_train, y_train = x_train.to(dev), y_train.to(dev)

    n0 = pkg._lib.calls.get("loss_grad_f32", 0)
    losses = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model.sde.train()
    for ep in range(a.epochs):
        loader = pr.get_dataloader_linear(x_train, y_train, vars(f)["scale"], CONFIG["batch_size"])
        loss, _ = model.train_epoch(opt, loss_fn, loader)
        if ep % max(1, a.epochs // 40) == 0 or ep == a.epochs - 1:
            losses.append(float(loss))
            print(f"epoch {ep}: loss {losses[-1]:.4g}", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    t_train = time.perf_counter() - t0
    fused = pkg._lib.calls.get("loss_grad_f32", 0) - n0
    n_steps = a.epochs * ((len(x_train) + CONFIG["batch_size"] - 1) // CONFIG["batch_size"])

    with tempfile.TemporaryDirectory() as td:
        torch.manual_seed(1)
        t0 = time.perf_counter()
        kl, nlpd, mse = ev.evaluate_linear(model, y_test[:a.n_y], f, td, [], n_samples_x=a.n, n_repeats=a.repeats)
        torch.cuda.synchronize()
        t_ev = time.perf_counter() - t0
    print(json.dumps({
        "metric": "reference linear configuration trained and evaluated on one GPU",
        "config": {k: cfg[k] for k in ("hidden_layers", "loss_fn", "lam", "lam2", "lr", "batch_size")},
        "model": "CPU-trained fixture CDE [64]^3 (tests/golden/ckpt_lin.npz, DSMLoss)" if a.fixture else "trained here",
        "epochs": a.epochs, "optimizer_steps": n_steps, "fused_steps": fused, "train_s": t_train,
        "train_samples_per_s": n_steps * CONFIG["batch_size"] / t_train, "loss_trace": losses,
        "evaluate": {"n_y": a.n_y, "n_samples_x": a.n, "n_repeats": a.repeats, "sde_steps": 200,
                     "evaluate_s": t_ev, "KL2_mean": float(kl), "NLPD_mean": float(nlpd), "MSE_mean": float(mse)},
    }), flush=True)


if __name__ == "__main__":
    main()
