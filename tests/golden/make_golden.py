"""Generate the golden fixtures under tests/golden/ by importing the REFERENCE (read-only,
/root/reference) in this container.

This script is test infrastructure: it is the only place that touches the reference code, it
runs only in the build container (the reference does not exist on the GPU box), and what it
writes is data (inputs + expected outputs, .npz/.json), never reference source.

Import recipe: the reference is flat-imported with cwd on sys.path plus two
sys.modules stubs -- `overrides.override` (a no-op decorator, models/diffusion.py:9,158) and the
un-vendored `include.sdeflow_light.lib.utils` (sdes.py:6; only needed by sample_debiasing_t,
which the fixtures avoid by using the uniform-t branch of sample_t, models/diffusion.py:55-57).

Fixtures (SURVEY.md §8c "Golden fixtures"):
  G1 schedule.npz          ts / T-ts / beta / sqrt(beta) for S in {200, 1000}
  G2 mlp_io.npz            seeded MLP / MLP2 / PosteriorScore weights + 64-row I/O
  G3 traj_*.npz            EM trajectories with captured x0 and per-step noise
  G4 ckpt_*.npz, samples_*.npz   fixture-trained CDE checkpoints + reference posterior samples
  G5 pinn_linear.npz       PINNLoss / DSM_PDELoss / DSMLoss components and parameter grads
  G6 data_*.npz            y_test / x_test of both problems
  G7 surrogate.npz         scatterometry surrogate weights (fp32)
  G9 ckpt_prior_scat.npz   a scatterometry prior score network MLP2 [256]*3 (the PosteriorDiffusionEstimator's
                           prior) trained with the reference's DSMLoss on inverse_cdf_prior samples (the
                           prior half of PosteriorLoss, losses.py:373-377; uniform t) -- for the DPS sampler
  G10 posterior_loss.npz   PosteriorLoss (losses.py:293-386) value, components, likelihood target and every
                           parameter gradient of both networks (prior = G9 checkpoint, likelihood seeded,
                           surrogate = G7) on 256 rows with captured eps and t
  G11 pinn_ref_configs.npz PINNLoss value, components and every parameter gradient at the reference configs'
                           hidden_layers [512]*3 for both problems (config_linear.yml / config_scatterometry.yml
                           loss settings; the scatterometry IC target -energy_grad(get_log_posterior),
                           main_diffusion_scatterometry.py:142-145); weights from a numpy seed (reference_weights)
  G8 surrogate_io.npz      surrogate forward, get_log_posterior and its autograd input gradient
                           (energy_grad) on 256 seeded rows; anneal_to_energy (random-walk MH) with
                           its captured draws (64 chains x 50 steps) and a 4000-chain x 1000-step run

Usage:  python tests/golden/make_golden.py [--what all|schedule|mlp|data|train|traj|samples|pinn|posterior_loss]
"""
import argparse
import os
import sys
import time
import types

import numpy as np

REF = os.environ.get("DMIP_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def import_reference():
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    sys.dont_write_bytecode = True
    if REF not in sys.path:
        sys.path.insert(0, REF)
    ov = types.ModuleType("overrides")
    ov.override = lambda f: f
    sys.modules.setdefault("overrides", ov)
    for name in ["include", "include.sdeflow_light", "include.sdeflow_light.lib"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    u = types.ModuleType("include.sdeflow_light.lib.utils")

    def _missing(*a, **k):
        raise RuntimeError("sdeflow-light is not vendored in the reference")

    u.sample_v = u.log_normal = u.sample_vp_truncated_q = _missing
    sys.modules.setdefault("include.sdeflow_light.lib.utils", u)
    # FrEIA (the SNF/INN baselines' flow library) is not installed; models/SNF.py imports five of its
    # names at module level but anneal_to_energy / energy_grad (models/SNF.py:234-275) use torch only
    fr = types.ModuleType("FrEIA")
    frf = types.ModuleType("FrEIA.framework")
    for nm in ("InputNode", "OutputNode", "Node", "ReversibleGraphNet", "ConditionNode"):
        setattr(frf, nm, object)
    frm = types.ModuleType("FrEIA.modules")
    frm.GLOWCouplingBlock = object
    for nm, mod in (("FrEIA", fr), ("FrEIA.framework", frf), ("FrEIA.modules", frm)):
        sys.modules.setdefault(nm, mod)
    import torch  # noqa: F401
    import nets, sdes, losses, linear_problem, utils_scatterometry, datasets  # noqa: E401
    from models import diffusion, SNF
    return types.SimpleNamespace(nets=nets, sdes=sdes, losses=losses, diffusion=diffusion,
                                 linear_problem=linear_problem, scat=utils_scatterometry,
                                 datasets=datasets, snf=SNF)


def state_to_npz_dict(sd, prefix=""):
    return {prefix + k.replace(".", "_"): v.detach().cpu().numpy().astype(np.float32)
            for k, v in sd.items()}


def load_state(net, path, prefix=""):
    import torch
    z = np.load(path)
    sd = {}
    for k in net.state_dict().keys():
        sd[k] = torch.from_numpy(z[prefix + k.replace(".", "_")])
    net.load_state_dict(sd)


# ----------------------------------------------------------------------------------------- G1
def gen_schedule(R):
    import torch
    out = {}
    sde = R.sdes.VariancePreservingSDE()
    for S in (200, 1000):
        ts = torch.linspace(0, 1, S + 1) * 1  # models/diffusion.py:34 (T=1)
        tau = 1 - ts                          # sdes.py:78 self.T - t
        beta = sde.beta(tau)                  # sdes.py:21-22
        g = sde.g(tau, tau)                   # sdes.py:33-35
        out[f"ts_{S}"] = ts.numpy()
        out[f"tau_{S}"] = tau.numpy()
        out[f"beta_{S}"] = beta.numpy()
        out[f"g_{S}"] = g.numpy()
        out[f"mw_{S}"] = sde.mean_weight(tau).numpy()
        out[f"var_{S}"] = sde.var(tau).numpy()
        out[f"delta_{S}"] = np.float64(1 / S)
    np.savez(os.path.join(OUT, "schedule.npz"), **out)


# ----------------------------------------------------------------------------------------- G2
def gen_mlp(R):
    import torch
    out = {}
    for tag, (xd, yd, hl) in {"lin": (2, 2, [64] * 3), "scat": (3, 23, [256] * 3)}.items():
        torch.manual_seed(0)
        cde = R.diffusion.CDE(xd, yd, hl)
        net = cde.sde.a
        out.update(state_to_npz_dict(net.state_dict(), f"{tag}_"))
        g = torch.Generator().manual_seed(1)
        n = 64
        x = torch.randn(n, xd, generator=g)
        y = torch.randn(n, yd, generator=g)
        t = torch.rand(n, 1, generator=g)
        with torch.no_grad():
            a = net(x, y, t)
            out[f"{tag}_x"], out[f"{tag}_y"], out[f"{tag}_t"] = x.numpy(), y.numpy(), t.numpy()
            out[f"{tag}_a"] = a.numpy()
            # the score the evaluate() drivers use: a(x,y,t)/g(t) (main_diffusion_linear.py:79-81)
            out[f"{tag}_score"] = (a / cde.sde.base_sde.g(t, x)).numpy()
        # Posterior (two-net) estimator: prior MLP2(x,t) + likelihood MLP(x,y,t), g-scaled
        torch.manual_seed(2)
        post = R.diffusion.PosteriorDiffusionEstimator(xd, yd, hl)
        out.update(state_to_npz_dict(post.sde.a.prior_net.state_dict(), f"{tag}_prior_"))
        out.update(state_to_npz_dict(post.sde.a.likelihood_net.state_dict(), f"{tag}_lik_"))
        with torch.no_grad():
            out[f"{tag}_prior_out"] = post.sde.a.prior_net(x, t).numpy()
            out[f"{tag}_post_out"] = post.sde.a(x, y, t).numpy()
    np.savez(os.path.join(OUT, "mlp_io.npz"), **out)


# ----------------------------------------------------------------------------------------- G6/G7
def gen_data(R):
    import torch
    fm, params = R.scat.load_forward_model(os.path.join(REF, "trained_models/scatterometry"))
    np.savez(os.path.join(OUT, "surrogate.npz"), **state_to_npz_dict(fm.state_dict()))
    with torch.no_grad():
        xs, ys = R.datasets.generate_dataset_scatterometry(fm, params["a"], params["b"], 100)
    np.savez(os.path.join(OUT, "data_scat.npz"), x_test=xs.numpy(), y_test=ys.numpy())
    f = R.linear_problem.LinearForwardProblem()
    xs, ys = R.datasets.generate_dataset_linear(f.xdim, f, 100000)
    from sklearn.model_selection import train_test_split
    x_tr, x_te, y_tr, y_te = train_test_split(xs, ys, train_size=0.9, random_state=7)
    np.savez(os.path.join(OUT, "data_linear.npz"), x_test=x_te[:100].numpy(),
             y_test=y_te[:100].numpy())
    # analytic posterior of y_test[0] (linear_problem.py:41-46) for the linear sampler checks
    post = f.get_posterior(y_te[0], device="cpu")
    np.savez(os.path.join(OUT, "linear_posterior.npz"), y=y_te[0].numpy(),
             mean=post.mean.numpy(), cov=post.covariance_matrix.numpy())


# ----------------------------------------------------------------------------------------- G4a
def train_ckpt(R, tag, minutes):
    """Train a fixture checkpoint with the REFERENCE train_epoch + DSMLoss (uniform t, since
    sdeflow-light's debiased sampler is not vendored: models/diffusion.py:55-57)."""
    import torch
    torch.manual_seed(123)
    np.random.seed(123)
    if tag == "lin":
        f = R.linear_problem.LinearForwardProblem()
        model = R.diffusion.CDE(2, 2, [64] * 3)
        xs, ys = R.datasets.generate_dataset_linear(f.xdim, f, 100000)
        loader_fn = lambda: R.datasets.get_dataloader_linear(xs, ys.clone(), f.scale, 1000)
        lr0 = 2e-3
    else:
        fm, params = R.scat.load_forward_model(os.path.join(REF, "trained_models/scatterometry"))
        model = R.diffusion.CDE(3, 23, [256] * 3)
        loader_fn = lambda: R.datasets.get_dataloader_scatterometry(
            1000, fm, params["a"], params["b"], params["lambd_bd"])
        lr0 = 1e-3
    model.sde.debias = False
    loss_fn = R.losses.DSMLoss()
    opt = torch.optim.Adam(model.sde.a.parameters(), lr=lr0)
    t0 = time.time()
    ep = 0
    log = []
    while time.time() - t0 < minutes * 60:
        frac = (time.time() - t0) / (minutes * 60)
        for gr in opt.param_groups:
            gr["lr"] = lr0 * (0.05 + 0.95 * 0.5 * (1 + np.cos(np.pi * min(frac, 1.0))))
        loss, _ = model.train_epoch(opt, loss_fn, loader_fn())
        ep += 1
        if ep % 20 == 0:
            log.append((ep, float(loss)))
            print(tag, ep, float(loss), f"{time.time() - t0:.0f}s", flush=True)
    np.savez(os.path.join(OUT, f"ckpt_{tag}.npz"), **state_to_npz_dict(model.sde.a.state_dict()),
             train_log=np.array(log, dtype=np.float64))


def make_cde(R, tag):
    if tag == "lin":
        m = R.diffusion.CDE(2, 2, [64] * 3)
    else:
        m = R.diffusion.CDE(3, 23, [256] * 3)
    load_state(m.sde.a, os.path.join(OUT, f"ckpt_{tag}.npz"))
    return m


def y_of(tag, i=0):
    import torch
    z = np.load(os.path.join(OUT, "data_linear.npz" if tag == "lin" else "data_scat.npz"))
    return torch.from_numpy(z["y_test"][i])


# ----------------------------------------------------------------------------------------- G3
def gen_traj(R):
    import torch
    for tag, (n, S) in {"lin": (32, 200), "scat": (16, 1000)}.items():
        m = make_cde(R, tag)
        y = y_of(tag)
        torch.manual_seed(77)
        x0 = torch.randn(n, m.xdim)
        xi = torch.stack([torch.randn(n, m.xdim) for _ in range(S)])
        torch.manual_seed(77)
        xS = m(y, num_samples=n, num_steps=S)  # models/diffusion.py:27-46
        # a second, shorter trajectory (10 steps) isolates the per-step arithmetic
        torch.manual_seed(78)
        x0s = torch.randn(n, m.xdim)
        xis = torch.stack([torch.randn(n, m.xdim) for _ in range(10)])
        torch.manual_seed(78)
        xSs = m(y, num_samples=n, num_steps=10)
        np.savez(os.path.join(OUT, f"traj_{tag}.npz"), y=y.numpy(), x0=x0.numpy(),
                 xi=xi.numpy(), x_final=xS, num_steps=S,
                 x0_short=x0s.numpy(), xi_short=xis.numpy(), x_final_short=xSs, steps_short=10)


# ----------------------------------------------------------------------------------------- G4b
def gen_samples(R):
    import torch
    torch.set_num_threads(os.cpu_count())
    for tag, (n, S) in {"lin": (100000, 200), "scat": (100000, 1000)}.items():
        m = make_cde(R, tag)
        y = y_of(tag)
        torch.manual_seed(2024)
        t0 = time.time()
        xs = m(y, num_samples=n, num_steps=S)
        dt = time.time() - t0
        q = np.linspace(0, 1, 1001)
        np.savez(os.path.join(OUT, f"samples_{tag}.npz"), y=y.numpy(), num_steps=S,
                 n_total=n, samples=xs[:20000].astype(np.float32),
                 quantiles=np.quantile(xs, q, axis=0).astype(np.float32),
                 mean=xs.mean(0), std=xs.std(0), seconds=dt, threads=torch.get_num_threads())
        print(tag, "sampled", n, "x", S, "in", dt, "s")


# ----------------------------------------------------------------------------------------- G5
def gen_pinn(R):
    import torch
    f = R.linear_problem.LinearForwardProblem()
    m = R.diffusion.CDE(2, 2, [64] * 3)
    load_state(m.sde.a, os.path.join(OUT, "ckpt_lin.npz"))
    z = np.load(os.path.join(OUT, "data_linear.npz"))
    g = torch.Generator().manual_seed(5)
    B = 256
    x = torch.from_numpy(z["x_test"][:100]).repeat(3, 1)[:B].clone()
    y = (x @ f.A.T + f.b) + 0.3 * torch.randn(B, 2, generator=g)
    t = (1e-4 + torch.rand(B, 1, generator=g) * (1 - 1e-4)).requires_grad_(True)
    out = {"x": x.numpy(), "y": y.numpy(), "t": t.detach().numpy()}
    # base_sde.sample with its randn_like replaced by a captured draw (sdes.py:37-49)
    eps = torch.randn(B, 2, generator=g)
    out["eps"] = eps.numpy()
    sde = m.sde.base_sde
    mu = sde.mean_weight(t) * x
    std = sde.var(t) ** 0.5
    x_t = eps * std + mu
    gg = sde.g(t, x_t)
    cfgs = {
        "pinn": R.losses.PINNLoss(f.score_posterior, lam=1e-3, lam2=0.1, pde_loss="FPE",
                                  ic_metric="L2", pde_metric="L1"),
        "pinn_l1l2": R.losses.PINNLoss(f.score_posterior, lam=0.5, lam2=0.3, pde_loss="FPE",
                                       ic_metric="L1", pde_metric="L2"),
        "dsmpde": R.losses.DSM_PDELoss(lam=1e-2, pde_loss="FPE", pde_metric="L1"),
        "pinn_cfpe": R.losses.PINNLoss(f.score_posterior, lam=1e-3, lam2=0.1,
                                       pde_loss="cScoreFPE", ic_metric="L2", pde_metric="L2"),
    }
    for name, lf in cfgs.items():
        for p in m.sde.a.parameters():
            p.grad = None
        loss, info = lf(m.sde, x, y, x_t, t, eps, std, gg)
        loss.backward(retain_graph=True)
        out[f"{name}_loss"] = loss.detach().numpy()
        for k, v in info.items():
            out[f"{name}_{k.replace(' ', '_').replace('-', '_')}"] = v.detach().numpy()
        for k, p in m.sde.a.named_parameters():
            out[f"{name}_grad_{k.replace('.', '_')}"] = p.grad.numpy().copy()
    # DSM alone (models/diffusion.py:83-85)
    for p in m.sde.a.parameters():
        p.grad = None
    score = m.sde.a(x_t, y, t) / gg
    dsm = R.losses.DSMLoss()(score, std, eps)
    dsm.mean().backward()
    out["dsm_rows"] = dsm.detach().numpy()
    for k, p in m.sde.a.named_parameters():
        out[f"dsm_grad_{k.replace('.', '_')}"] = p.grad.numpy().copy()
    # ScoreFPE internals (losses.py:14-26,77-98) on a fresh x_t(t) graph
    x_t = eps * sde.var(t) ** 0.5 + sde.mean_weight(t) * x
    gg = sde.g(t, x_t)
    s = m.sde.a(x_t, y, t) / gg
    div = R.losses.divergence(s, x_t)
    dsdt = R.losses.batch_gradient(s, t)
    out["fpe_div"] = div.detach().numpy()
    out["fpe_dsdt"] = dsdt.detach().numpy()
    out["fpe_rows"] = R.losses.ScoreFPELoss("L1")(s, x_t, t, sde.beta(t)).detach().numpy()
    np.savez(os.path.join(OUT, "pinn_linear.npz"), **out)


# ----------------------------------------------------------------------------------------- G8
def gen_surrogate(R):
    import torch
    torch.set_num_threads(os.cpu_count())
    fm, prm = R.scat.load_forward_model(os.path.join(REF, "trained_models/scatterometry"))
    a, b, lam = prm["a"], prm["b"], prm["lambd_bd"]
    z = np.load(os.path.join(OUT, "data_scat.npz"))
    ys = torch.from_numpy(z["y_test"])
    g = torch.Generator().manual_seed(8)
    n = 256
    # mostly inside the prior box, some outside (boundary penalty and its gradient)
    x = (torch.rand(n, 3, generator=g) * 2.2 - 1.1)
    y = ys[torch.arange(n) % ys.shape[0]]
    out = {"x": x.numpy(), "y": y.numpy(), "a": a, "b": b, "lambd_bd": lam}
    with torch.no_grad():
        out["f"] = fm(x).numpy()
    # energy_grad (models/SNF.py:234-237) on get_log_posterior (utils_scatterometry.py:30-38)
    energy = lambda v: R.scat.get_log_posterior(v, fm, a, b, y, lam)
    grad, e = R.snf.energy_grad(x.clone(), energy)
    out["energy"] = e.detach().numpy()
    out["grad"] = grad.detach().numpy()
    # anneal_to_energy with captured draws: generate_gt_samples draws x0 = rand*2-1, then every MH
    # step draws randn_like(x) (the proposal) and rand_like(e_diff) (the acceptance uniform)
    y0 = ys[0]
    for tag, (nc, S, ns) in {"mh": (64, 50, 0.5)}.items():
        inflated = y0[None, :].repeat(nc, 1)
        en = lambda v: R.scat.get_log_posterior(v, fm, a, b, inflated, lam)
        torch.manual_seed(31)
        x0 = torch.rand(nc, 3) * 2 - 1
        xi, u = [], []
        for _ in range(S):
            xi.append(torch.randn(nc, 3))
            u.append(torch.rand(nc))
        torch.manual_seed(31)
        x0b = torch.rand(nc, 3) * 2 - 1
        assert torch.equal(x0, x0b)
        xs, ediff = R.snf.anneal_to_energy(x0b, en, S, noise_std=ns)
        out.update({f"{tag}_y": y0.numpy(), f"{tag}_x0": x0.numpy(), f"{tag}_xi": torch.stack(xi).numpy(),
                    f"{tag}_u": torch.stack(u).numpy(), f"{tag}_x": xs.detach().numpy(),
                    f"{tag}_ediff": ediff.detach().numpy(), f"{tag}_noise_std": ns})
    # a ground-truth-style run (generate_scatterometry_ground_truth.py:27 with METR_STEPS = 1000,
    # NOISE_STD_MCMC = 0.5 of config_scatterometry.yml) for distributional parity
    nc, S = 4000, 1000
    inflated = y0[None, :].repeat(nc, 1)
    en = lambda v: R.scat.get_log_posterior(v, fm, a, b, inflated, lam)
    torch.manual_seed(2025)
    t0 = time.time()
    with torch.no_grad():
        xs, _ = R.snf.anneal_to_energy(torch.rand(nc, 3) * 2 - 1, en, S, noise_std=0.5)
    out["gt_samples"] = xs.numpy()
    out["gt_steps"] = S
    out["gt_seconds"] = time.time() - t0
    print("MH", nc, "x", S, "in", out["gt_seconds"], "s")
    np.savez(os.path.join(OUT, "surrogate_io.npz"), **out)


# ----------------------------------------------------------------------------------------- G9
def train_prior(R, minutes):
    import torch
    torch.set_num_threads(os.cpu_count())
    torch.manual_seed(321)
    np.random.seed(321)
    post = R.diffusion.PosteriorDiffusionEstimator(3, 23, [256] * 3)
    net = post.sde.a.prior_net
    sde = post.sde.base_sde
    loss_fn = R.losses.DSMLoss()
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    t0 = time.time()
    it, log = 0, []
    while time.time() - t0 < minutes * 60:
        frac = (time.time() - t0) / (minutes * 60)
        for gr in opt.param_groups:
            gr["lr"] = 1e-3 * (0.05 + 0.95 * 0.5 * (1 + np.cos(np.pi * min(frac, 1.0))))
        x = torch.tensor(R.scat.inverse_cdf_prior(np.random.uniform(size=(1000, 3)), 1000), dtype=torch.float)
        t = 1e-4 + torch.rand(1000, 1) * (1 - 1e-4)
        x_t, target, std, g = sde.sample(t, x, return_noise=True)
        loss = loss_fn(net(x_t, t), std, target).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        it += 1
        if it % 2000 == 0:
            log.append((it, float(loss)))
            print("prior", it, float(loss), f"{time.time() - t0:.0f}s", flush=True)
    np.savez(os.path.join(OUT, "ckpt_prior_scat.npz"), **state_to_npz_dict(net.state_dict()),
             train_log=np.array(log, dtype=np.float64))


# ---------------------------------------------------------------------------------------- G10
def gen_posterior_loss(R):
    """PosteriorLoss.forward + backward (losses.py:348-386) exactly as PosteriorDiffusionEstimator.train_epoch
    drives it (models/diffusion.py:204-229): loss_fn(model.sde, x, y, t) with t requiring grad."""
    import torch
    from torch import nn
    torch.set_num_threads(os.cpu_count())
    torch.manual_seed(41)
    post = R.diffusion.PosteriorDiffusionEstimator(3, 23, [256] * 3)
    load_state(post.sde.a.prior_net, os.path.join(OUT, "ckpt_prior_scat.npz"))
    zs = np.load(os.path.join(OUT, "surrogate.npz"))
    fm = nn.Sequential(nn.Linear(3, 256), nn.ReLU(), nn.Linear(256, 256), nn.ReLU(), nn.Linear(256, 256), nn.ReLU(),
                       nn.Linear(256, 23))
    fm.load_state_dict({k: torch.from_numpy(zs[k.replace(".", "_")]) for k in fm.state_dict().keys()})
    for prm in fm.parameters():
        prm.requires_grad = False
    a, b, lam = 0.2, 0.01, 0.01  # load_forward_model params; config_scatterometry.yml lam
    lf = R.losses.PosteriorLoss(fm, a, b, lam=lam)
    B = 256
    g = torch.Generator().manual_seed(10)
    x = torch.rand(B, 3, generator=g) * 2 - 1
    ys = torch.from_numpy(np.load(os.path.join(OUT, "data_scat.npz"))["y_test"])
    y = ys[torch.arange(B) % ys.shape[0]]
    t = (1e-4 + torch.rand(B, 1, generator=g) * (1 - 1e-4)).requires_grad_(True)
    torch.manual_seed(77)
    eps = torch.randn(B, 3)
    torch.manual_seed(77)  # base_sde.sample's randn_like(x) is the first draw in forward
    loss, info = lf(post.sde, x, y, t)
    loss.backward()
    out = {"x": x.numpy(), "y": y.numpy(), "t": t.detach().numpy(), "eps": eps.numpy(), "a": a, "b": b, "lam": lam,
           "loss": float(loss), "PriorLoss": float(info["PriorLoss"]), "LikelihoodLoss": float(info["LikelihoodLoss"])}
    for tag, net in (("prior", post.sde.a.prior_net), ("lik", post.sde.a.likelihood_net)):
        out.update(state_to_npz_dict(net.state_dict(), f"{tag}_"))
        for k, prm in net.named_parameters():
            out[f"{tag}_grad_{k.replace('.', '_')}"] = prm.grad.numpy().copy()
    # intermediates on the same inputs (a fresh graph): x_t, both scores, x0 and the likelihood target
    sde = post.sde.base_sde
    x_t = eps * sde.var(t) ** 0.5 + sde.mean_weight(t) * x
    std = sde.var(t) ** 0.5
    s_p = post.sde.a.prior_net(x_t, t)
    s_l = post.sde.a.likelihood_net(x_t, y, t)
    x_0 = 1 / sde.mean_weight(t) * (x_t + std ** 2 * s_p)
    T = lf.likelihood_target(x_0, y, x_t, s_p, std)
    out.update({"x_t": x_t.detach().numpy(), "s_prior": s_p.detach().numpy(), "s_lik": s_l.detach().numpy(),
                "x_0": x_0.detach().numpy(), "target": T.detach().numpy()})
    np.savez(os.path.join(OUT, "posterior_loss.npz"), **out)
    print("G10 loss", float(loss), {k: float(v) for k, v in info.items()})


# ---------------------------------------------------------------------------------------- G12
def gen_cdiffe_dsm(R):
    """CDiffE's joint DSM batch loss + backward exactly as CDiffE.train_epoch computes it
    (models/diffusion.py:128-136: z = [x, y], x_t / y_t from base_sde.sample, score = sde.a(x_t, y_t, t) / g,
    DSMLoss(...).mean()), with the draws t and eps given (the reference's debiased sample_t needs the
    un-vendored sdeflow-light). Reference networks, seeded; both problems' shapes."""
    import torch
    out = {}
    for tag, xd, yd, W, seed in (("lin", 2, 2, 64, 51), ("scat", 3, 23, 128, 52)):
        torch.manual_seed(seed)
        m = R.diffusion.CDiffE(xd, yd, [W] * 3)
        B = 512
        g = torch.Generator().manual_seed(seed + 100)
        z = torch.randn(B, xd + yd, generator=g)
        t = (1e-4 + torch.rand(B, 1, generator=g) * (1 - 1e-4)).requires_grad_(True)
        eps = torch.randn(B, xd + yd, generator=g)
        sde = m.sde.base_sde
        std = sde.var(t) ** 0.5
        diffused = eps * std + sde.mean_weight(t) * z  # base_sde.sample (sdes.py:37-49) with the draw given
        gt = sde.g(t, diffused)
        score = m.sde.a(diffused[:, :xd], diffused[:, xd:], t) / gt
        loss = R.losses.DSMLoss()(score, std, eps).mean()
        loss.backward()
        out.update({f"{tag}_z": z.numpy(), f"{tag}_t": t.detach().numpy(), f"{tag}_eps": eps.numpy(),
                    f"{tag}_loss": float(loss)})
        out.update(state_to_npz_dict(m.sde.a.state_dict(), f"{tag}_"))
        for k, prm in m.sde.a.named_parameters():
            out[f"{tag}_grad_{k.replace('.', '_')}"] = prm.grad.numpy().copy()
        print("G12", tag, float(loss))
    np.savez(os.path.join(OUT, "cdiffe_dsm.npz"), **out)


# ---------------------------------------------------------------------------------------- G11
def reference_weights(dims, seed):
    """Layer weights in nn.Linear's default range U(+-1/sqrt(fan_in)) from a numpy seed, so the tests can
    rebuild the same network without storing it (float32)."""
    g = np.random.default_rng(seed)
    out = []
    for i in range(len(dims) - 1):
        bd = 1.0 / np.sqrt(dims[i])
        out.append((g.uniform(-bd, bd, (dims[i + 1], dims[i])).astype(np.float32),
                    g.uniform(-bd, bd, dims[i + 1]).astype(np.float32)))
    return out


def gen_pinn_ref_configs(R):
    """PINNLoss forward + backward at hidden_layers [512]*3 (config_linear.yml:11-16,21 and
    config_scatterometry.yml:10-19), as CDE.train_epoch calls it (models/diffusion.py:80-89)."""
    import torch
    from torch import nn
    torch.set_num_threads(os.cpu_count())
    out = {}
    zs = np.load(os.path.join(OUT, "surrogate.npz"))
    fm = nn.Sequential(nn.Linear(3, 256), nn.ReLU(), nn.Linear(256, 256), nn.ReLU(), nn.Linear(256, 256), nn.ReLU(),
                       nn.Linear(256, 23))
    fm.load_state_dict({k: torch.from_numpy(zs[k.replace(".", "_")]) for k in fm.state_dict().keys()})
    for prm in fm.parameters():
        prm.requires_grad = False
    f = R.linear_problem.LinearForwardProblem()
    a_s, b_s, lbd = 0.2, 0.01, 1000.0
    for tag, (xd, yd, seed) in {"lin": (2, 2, 511), "scat": (3, 23, 512)}.items():
        m = R.diffusion.CDE(xd, yd, [512] * 3)
        lin = [l for l in m.sde.a if isinstance(l, nn.Linear)]
        for l, (W, bb) in zip(lin, reference_weights([xd + yd + 1, 512, 512, 512, xd], seed)):
            l.weight.data.copy_(torch.from_numpy(W))
            l.bias.data.copy_(torch.from_numpy(bb))
        g = torch.Generator().manual_seed(seed)
        B = 128
        if tag == "lin":
            x = torch.randn(B, 2, generator=g)
            y = (x @ f.A.T + f.b) + 0.3 * torch.randn(B, 2, generator=g)
            lf = R.losses.PINNLoss(f.score_posterior, lam=1e-3, lam2=0.1, pde_loss="FPE", ic_metric="L2",
                                   pde_metric="L1")
        else:
            x = torch.rand(B, 3, generator=g) * 2 - 1
            ys = torch.from_numpy(np.load(os.path.join(OUT, "data_scat.npz"))["y_test"])
            y = ys[torch.arange(B) % ys.shape[0]]
            sp = lambda xx, yy: -R.snf.energy_grad(xx, lambda v: R.scat.get_log_posterior(v, fm, a_s, b_s, yy, lbd))[0]
            lf = R.losses.PINNLoss(sp, lam=0.01, lam2=0.001, pde_loss="FPE", ic_metric="L2", pde_metric="L1")
            out["scat_ic_target"] = sp(x.clone(), y).detach().numpy()
        t = (1e-4 + torch.rand(B, 1, generator=g) * (1 - 1e-4)).requires_grad_(True)
        eps = torch.randn(B, xd, generator=g)
        sde = m.sde.base_sde
        std = sde.var(t) ** 0.5
        x_t = eps * std + sde.mean_weight(t) * x
        gg = sde.g(t, x_t)
        loss, info = lf(m.sde, x, y, x_t, t, eps, std, gg)
        loss.backward()
        out.update({f"{tag}_x": x.detach().numpy(), f"{tag}_y": y.numpy(), f"{tag}_t": t.detach().numpy(),
                    f"{tag}_eps": eps.numpy(), f"{tag}_seed": seed, f"{tag}_loss": float(loss)})
        for k, v in info.items():
            out[f"{tag}_{k.replace(' ', '_').replace('-', '_')}"] = float(v)
        for k, prm in m.sde.a.named_parameters():
            out[f"{tag}_grad_{k.replace('.', '_')}"] = prm.grad.numpy().copy()
        print("G11", tag, float(loss), {k: float(v) for k, v in info.items()})
    np.savez(os.path.join(OUT, "pinn_ref_configs.npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="all")
    ap.add_argument("--minutes-lin", type=float, default=4.0)
    ap.add_argument("--minutes-scat", type=float, default=12.0)
    ap.add_argument("--minutes-prior", type=float, default=6.0)
    a = ap.parse_args()
    R = import_reference()
    w = a.what
    if w in ("all", "schedule"):
        gen_schedule(R)
    if w in ("all", "mlp"):
        gen_mlp(R)
    if w in ("all", "data"):
        gen_data(R)
    if w in ("all", "train", "train_lin"):
        train_ckpt(R, "lin", a.minutes_lin)
    if w in ("all", "train", "train_scat"):
        train_ckpt(R, "scat", a.minutes_scat)
    if w in ("all", "traj"):
        gen_traj(R)
    if w in ("all", "pinn"):
        gen_pinn(R)
    if w in ("all", "samples"):
        gen_samples(R)
    if w in ("all", "posterior_loss"):
        gen_posterior_loss(R)
    if w in ("all", "pinn_ref"):
        gen_pinn_ref_configs(R)
    if w in ("all", "surrogate"):
        gen_surrogate(R)
    if w in ("all", "prior"):
        train_prior(R, a.minutes_prior)
    if w in ("all", "cdiffe_dsm"):
        gen_cdiffe_dsm(R)


if __name__ == "__main__":
    main()
