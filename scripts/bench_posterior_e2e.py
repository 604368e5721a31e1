"""Scatterometry end to end on one MI355X: train the reference's learned estimators on the device and
score their posteriors against the fused MCMC ground truth (the reference's own pipeline,
main_diffusion_scatterometry.py train + evaluate, with generate_scatterometry_ground_truth.py's MH).

  * PosteriorDiffusionEstimator [W]^3 trained with PosteriorLoss (lam from config_scatterometry.yml,
    the fused exact-f32 dmip_posterior_loss_grad: prior DSM + likelihood target through the surrogate),
    sampled with the fused two-network sampler -- BASELINE config 4's reference method;
  * CDE [W]^3 trained with the reference config's PINNLoss (lam 0.01, lam2 0.001, FPE/L1, IC L2 with the
    -energy_grad initial condition, main_diffusion_scatterometry.py:142-145) on the exact-f32 engine;
  * CDiffE [W]^3 on the joint z = (x, y) trained with DSMLoss (the only loss the reference's joint
    training accepts; the fused exact-f32 joint DSM), sampled predictor-only and with the Langevin
    predictor-corrector (BASELINE config 3: 1 corrector step per step, snr 0.16);
  * for comparison: DPS guided by the same surrogate (fixture prior) and two independent MH runs (the
    KL2 noise floor at this sample size).
Data: the reference's own generator (inverse-CDF prior samples pushed through the surrogate with its
noise model, datasets.py:26-34), fresh each epoch; y = the reference's seeded y_test[i].
Prints one JSON line: training steps / time / samples per second, and KL2 (75^3 bins on [-1.2, 1.2]^3,
the reference metric) and per-dimension W1 against the MH ground truth.
    python scripts/bench_posterior_e2e.py [--width 256] [--epochs 400] [--batch 8192]
Recipes (CDE only, --save-cde writes the trained weights for scripts/bench_evaluate_pipeline.py --ckpt):
  --recipe reference  config_scatterometry.yml as main_diffusion_scatterometry.py trains it: CDE [512]^3,
                      PINNLoss (lam 0.01, lam2 0.001, FPE / L1, IC L2 against -energy_grad), Adam lr 1e-4 (no
                      schedule), batch 1000, 20,000 epochs of 8 batches (datasets.py:26-34), debiased t;
  --recipe fixture    the CPU fixture's recipe (tests/golden/make_golden.py train_ckpt): CDE [256]^3, DSMLoss,
                      uniform t, batch 1000, Adam from lr 1e-3 on the cosine with floor 0.05, 18,560 epochs
                      (its train_log) -- the control for the device-trained quality."""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=256)
    ap.add_argument("--epochs", type=int, default=400, help="epochs of 8 batches (datasets.py:26-34)")
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--n", type=int, default=30000, help="posterior samples / MH chains")
    ap.add_argument("--steps", type=int, default=1000, help="SDE steps")
    ap.add_argument("--y-index", type=int, default=0)
    ap.add_argument("--no-cde", action="store_true")
    ap.add_argument("--no-posterior", action="store_true")
    ap.add_argument("--no-cdiffe", action="store_true")
    ap.add_argument("--snr", type=float, default=0.16, help="corrector signal-to-noise ratio (config 3)")
    ap.add_argument("--snr-sweep", default="", help="comma-separated corrector snr values to score as well")
    ap.add_argument("--load-cdiffe", default="", help="sample a CDiffE checkpoint written by --save-cdiffe")
    ap.add_argument("--save-cdiffe", default="", help="write the trained CDiffE's state_dict here (.npz)")
    ap.add_argument("--recipe", default="", choices=["", "reference", "fixture"])
    ap.add_argument("--save-cde", default="", help="write the trained CDE's state_dict here (.npz)")
    ap.add_argument("--no-dps", action="store_true")
    a = ap.parse_args()
    if a.recipe:  # CDE only, at the recipe's own sizes
        a.no_posterior = a.no_cdiffe = a.no_dps = True
        a.batch = 1000
        if a.recipe == "reference":
            a.width, a.lr, a.epochs = 512, 1e-4, a.epochs if a.epochs != 400 else 20000
        else:
            a.width, a.lr, a.epochs = 256, 1e-3, a.epochs if a.epochs != 400 else 18560
    pkg = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
    ev = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.evaluate")
    pr = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.problems")
    dev = torch.device("cuda:0")
    gold = os.path.join(ROOT, "tests", "golden")
    fm, prm = pkg.load_forward_model(gold)
    fm = fm.to(dev)
    y = torch.from_numpy(np.load(os.path.join(gold, "data_scat.npz"))["y_test"][a.y_index]).to(dev)
    torch.manual_seed(0)
    np.random.seed(0)

    gt = pkg.mh_sample(fm, prm, y[None], a.n, 1000, 0.5, seed=99)[0]
    gt2 = pkg.mh_sample(fm, prm, y[None], a.n, 1000, 0.5, seed=98)[0]
    h_gt = ev.histograms(gt, 75, (-1.2, 1.2))[0]

    def score(x):
        x = x.reshape(-1, 3)[:a.n]
        kl, _ = ev.hist_kl(h_gt, ev.histograms(x, 75, (-1.2, 1.2))[0])
        w1 = [float((torch.sort(x[:, k])[0] - torch.sort(gt[:, k])[0]).abs().mean()) for k in range(3)]
        return {"KL2_vs_mcmc": kl, "W1_vs_mcmc": w1, "mean": x.mean(0).tolist(), "std": x.std(0).tolist()}

    def train(model, loss_fn, tag):
        opt = torch.optim.Adam(model.sde.a.parameters(), lr=a.lr)
        sched = None if a.recipe else torch.optim.lr_scheduler.CosineAnnealingLR(opt, a.epochs)
        losses = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for ep in range(a.epochs):
            if a.recipe == "fixture":  # make_golden.py train_ckpt: cosine over the run, floor 0.05
                for gr in opt.param_groups:
                    gr["lr"] = a.lr * (0.05 + 0.95 * 0.5 * (1 + np.cos(np.pi * ep / a.epochs)))
            loader = pr.get_dataloader_scatterometry(a.batch, fm, prm["a"], prm["b"], prm["lambd_bd"])
            loss, _ = model.train_epoch(opt, loss_fn, loader)
            if sched is not None:
                sched.step()
            if ep % max(1, a.epochs // (40 if a.recipe else 8)) == 0 or ep == a.epochs - 1:
                losses.append(float(loss))
                print(f"[{tag}] epoch {ep}: loss {losses[-1]:.4g}", file=sys.stderr, flush=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        n_steps = 8 * a.epochs
        return {"model": tag, "width": a.width, "optimizer_steps": n_steps, "batch": a.batch, "lr": a.lr,
                "recipe": a.recipe or "device default (cosine lr)",
                "train_s": el, "train_samples_per_s": n_steps * a.batch / el, "loss_trace": losses}

    out = {"metric": "scatterometry estimators trained and sampled on one GPU, quality vs MCMC",
           "y_index": a.y_index, "n": a.n, "sde_steps": a.steps,
           "mcmc_floor": {"KL2_mcmc_vs_mcmc": ev.hist_kl(h_gt, ev.histograms(gt2, 75, (-1.2, 1.2))[0])[0]}}

    if not a.no_posterior:
        post = pkg.PosteriorDiffusionEstimator(3, 23, [a.width] * 3)
        post.sde.a.to(dev)
        plf = pkg.PosteriorLoss(fm, prm["a"], prm["b"], 0.01)  # config_scatterometry.yml lam
        n0 = pkg._lib.calls.get("posterior_loss_grad", 0)
        r = train(post, plf, "PosteriorDiffusionEstimator + PosteriorLoss")
        r["fused_steps"] = pkg._lib.calls.get("posterior_loss_grad", 0) - n0
        x = post.sample_device(y, a.n, a.steps, seed=7)
        r["quality"] = score(x)
        out["posterior"] = r

    if not a.no_cde:
        cde = pkg.CDE(3, 23, [a.width] * 3)
        cde.sde.a.to(dev)
        if a.recipe == "fixture":
            cde.sde.debias = False  # uniform t (the fixture: sdeflow-light's debiased sampler is not vendored)
            lf, tag = pkg.DSMLoss(), "CDE + DSMLoss (the CPU fixture's recipe)"
        else:
            sp = lambda xx, yy: -pkg.energy_grad(xx, lambda v: pkg.get_log_posterior(v, fm, prm["a"], prm["b"], yy,
                                                                                      prm["lambd_bd"]))[0]
            lf = pkg.PINNLoss(sp, lam=0.01, lam2=0.001, pde_loss="FPE", ic_metric="L2", pde_metric="L1")
            tag = "CDE + PINNLoss (reference config losses, -energy_grad IC)"
        n0 = pkg._lib.calls.get("loss_grad_f32", 0)
        r = train(cde, lf, tag)
        r["fused_steps"] = pkg._lib.calls.get("loss_grad_f32", 0) - n0
        x = cde.sample_device(y, a.n, a.steps, seed=8)
        r["quality"] = score(x)
        out["cde_" + (a.recipe or "pinn")] = r
        if a.save_cde:
            sd = {k.replace(".", "_"): v.detach().cpu().numpy() for k, v in cde.sde.a.state_dict().items()}
            np.savez(a.save_cde, **sd)

    if not a.no_cdiffe:
        cd = pkg.CDiffE(3, 23, [a.width] * 3)
        if a.load_cdiffe:  # a checkpoint this script wrote (--save-cdiffe): sampling only
            z = np.load(a.load_cdiffe)
            cd.sde.a.load_state_dict({k.replace("_", "."): torch.from_numpy(z[k]) for k in z.files
                                      if k.split("_")[0].isdigit()})
            cd.sde.a.to(dev)
            r = {"model": "CDiffE + DSMLoss on the joint z = (x, y)", "width": a.width, "weights": a.load_cdiffe}
        else:
            cd.sde.a.to(dev)
            n0 = pkg._lib.calls.get("loss_grad_f32", 0)
            r = train(cd, pkg.DSMLoss(), "CDiffE + DSMLoss on the joint z = (x, y)")
            r["fused_steps"] = pkg._lib.calls.get("loss_grad_f32", 0) - n0
        r["quality_predictor_only"] = score(cd.sample_device(y, a.n, a.steps, seed=10))
        r["quality_predictor_corrector"] = score(cd.sample_device(y, a.n, a.steps, seed=11, corrector_steps=1,
                                                                  snr=a.snr))
        r["corrector"] = {"steps_per_sde_step": 1, "snr": a.snr}
        if a.snr_sweep:  # the corrector's step-size rule at other signal-to-noise ratios
            r["snr_sweep"] = {v: score(cd.sample_device(y, a.n, a.steps, seed=12, corrector_steps=1, snr=float(v)))
                              for v in a.snr_sweep.split(",")}
        out["cdiffe"] = r
        if a.save_cdiffe and not a.load_cdiffe:
            sd = {k.replace(".", "_"): v.detach().cpu().numpy() for k, v in cd.sde.a.state_dict().items()}
            np.savez(a.save_cdiffe, **sd)

    if a.no_dps:
        print(json.dumps(out), flush=True)
        return
    dps = pkg.DPS(3, 23, [256] * 3, fm, prm)
    ck = os.path.join(gold, "ckpt_prior_scat.npz")
    z = np.load(ck)
    dps.prior_net.load_state_dict({k.replace("_", "."): torch.from_numpy(z[k]) for k in z.files
                                   if k.split("_")[0].isdigit()})
    dps.prior_net.to(dev)
    out["dps_fixture_prior"] = {"quality": score(dps.sample_device(y, a.n, a.steps, seed=9))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
