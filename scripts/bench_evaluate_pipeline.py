"""The reference's scatterometry evaluation pipeline at its own sizes, on one MI355X:
generate_scatterometry_ground_truth.py (30k MH chains x 1000 steps for each of the 100 test ys and 10
repeats: 3e10 chain-steps, one fused launch) followed by main_diffusion_scatterometry.py `evaluate`
(per y: 10 repeats x 30k posterior samples at the default 200 SDE steps, 75^3 histograms + KL2 /
reverse KL, NLL of the MCMC and diffusion samples through the surrogate, the score MSE at t = 0 against
-energy_grad), all through the package's reference-API functions. Prints one JSON line with the wall
times and the metric means.
Model: the fixture-trained CDE [256]^3 (tests/golden/ckpt_scat.npz), or --ckpt a CDE state_dict (.npz, e.g. one
scripts/bench_posterior_e2e.py --recipe reference --save-cde wrote) of hidden width --width.
    python scripts/bench_evaluate_pipeline.py [--n-y 100] [--n 30000] [--repeats 10] [--ckpt PATH --width 512]
                                              [--gt-precision fp32x3]"""
import argparse
import importlib
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-y", type=int, default=100)
    ap.add_argument("--n", type=int, default=30000)
    ap.add_argument("--repeats", type=int, default=10)
    ap.add_argument("--steps", type=int, default=200, help="SDE steps (the reference's default)")
    ap.add_argument("--metr-steps", type=int, default=1000)
    ap.add_argument("--ckpt", default="", help="CDE state_dict (.npz) instead of the fixture")
    ap.add_argument("--width", type=int, default=256)
    ap.add_argument("--gt-precision", default="fp32", choices=["fp32", "fp32x3"],
                    help="MH kernel of the ground truth (problems.mh_sample precision)")
    a = ap.parse_args()
    pkg = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
    ev = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.evaluate")
    pr = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.problems")
    from conftest import state_from_npz
    dev = torch.device("cuda:0")
    gold = os.path.join(ROOT, "tests", "golden")
    fm, prm = pkg.load_forward_model(gold)
    fm = fm.to(dev)
    _, ys = pr.generate_dataset_scatterometry(fm, prm["a"], prm["b"], size=100)
    ys = ys[:a.n_y].to(dev)
    m = pkg.CDE(3, 23, [a.width] * 3)
    ck = a.ckpt or os.path.join(gold, "ckpt_scat.npz")
    m.sde.a.load_state_dict(state_from_npz(np.load(ck)))
    m.sde.a.to(dev)
    # warm-up (kernel images, handles)
    pkg.generate_gt_samples(fm, prm, ys[:1], None, 256, 1, 10, 0.5, seed=1, precision=a.gt_precision)
    m.sample_device(ys[0], 256, 10)
    torch.cuda.synchronize()

    t0 = time.perf_counter()
    gt = pkg.generate_gt_samples(fm, prm, ys, None, a.n, a.repeats, a.metr_steps, 0.5, seed=2,
                                 precision=a.gt_precision)
    torch.cuda.synchronize()
    t_gt = time.perf_counter() - t0

    sp = lambda x, y: -pkg.energy_grad(x, lambda v: pkg.get_log_posterior(v, fm, prm["a"], prm["b"], y,
                                                                           prm["lambd_bd"]))[0]
    with tempfile.TemporaryDirectory() as td:
        torch.manual_seed(0)
        t0 = time.perf_counter()
        kl, nlpd, mse = ev.evaluate_scatterometry(m, ys, fm, td, [], a.n, sp, prm["a"], prm["b"], prm["lambd_bd"],
                                                  None, n_repeats=a.repeats, gt_loader=lambda i, j: gt[i, j],
                                                  num_steps=a.steps)
        torch.cuda.synchronize()
        t_ev = time.perf_counter() - t0
    chain_steps_gt = a.n_y * a.repeats * a.n * a.metr_steps
    samples = a.n_y * a.repeats * a.n
    print(json.dumps({
        "metric": "reference scatterometry evaluation pipeline (ground truth + evaluate) wall time, one GPU",
        "n_y": a.n_y, "n_samples_x": a.n, "n_repeats": a.repeats, "sde_steps": a.steps, "metr_steps": a.metr_steps,
        "ground_truth_precision": a.gt_precision, "ground_truth_s": t_gt, "ground_truth_chain_steps_per_s": chain_steps_gt / t_gt,
        "evaluate_s": t_ev, "evaluate_posterior_samples_per_s": samples / t_ev,
        "KL2_mean": float(kl), "NLPD_mean": float(nlpd), "MSE_mean": float(mse),
        "model": f"CDE [{a.width}]^3 from {os.path.relpath(ck, ROOT)}"}), flush=True)


if __name__ == "__main__":
    main()
