"""Evaluation drivers with the reference's signatures and metrics:
`evaluate_scatterometry` = main_diffusion_scatterometry.py:40-124 `evaluate`, `evaluate_linear` =
main_diffusion_linear.py:53-137 `evaluate`.

Same metrics and `results.csv` columns as the reference (KL2 / KL_reverse from 75-bin histograms with
epsilon smoothing and `rel_entr`, NLL, score MSE at t = 0), computed on the device:
  * all `n_repeats` draws of one y are one fused-sampler launch (`sample_device` with the y row
    repeated: repeat j is y-row j, its own RNG stream), instead of n_repeats host round trips;
  * histograms are `dmip_histogram` (numpy.histogramdd-exact binning, csrc/dmip_eval.hip), KL in
    float64 on the device.
Under torch.distributed (world_size > 1) the ys are sharded over the ranks (parallel.map_sharded:
each rank samples and scores its contiguous range of ys; one all_gather of the per-y metric rows;
rank 0 writes results.csv). Deliberate difference: the reference returns `mse_score_vals.mean()` on a Python list
(AttributeError at :124 / :137); here the mean is taken.
"""
import os

import numpy as np
import torch

from . import _lib, parallel
from .problems import get_gt_samples_scatterometry, get_log_posterior


def histograms(samples, nbins, xlim):
    """(n_hist, n, d) samples -> (n_hist, nbins**d) int32 counts, numpy.histogramdd binning."""
    x = samples.to(dtype=torch.float32).contiguous()
    if x.ndim == 2:
        x = x[None]
    counts = torch.zeros(x.shape[0], nbins ** x.shape[2], dtype=torch.int32, device=x.device)
    _lib.histogram(x, nbins, xlim[0], xlim[1], counts)
    return counts


def hist_kl(counts_true, counts_model, epsilon=1e-10):
    """KL2 and reverse KL of two count histograms exactly as the reference drivers compute them
    (normalise, + epsilon, renormalise, sum rel_entr) -- float64 on the device."""
    p = counts_true.to(torch.float64)
    q = counts_model.to(torch.float64)
    p = p / p.sum()
    q = q / q.sum()
    p = p + epsilon
    q = q + epsilon
    p = p / p.sum()
    q = q / q.sum()
    kl = torch.sum(p * torch.log(p / q))
    klr = torch.sum(q * torch.log(q / p))
    return float(kl), float(klr)


def _is_root():
    return parallel.world()[0] == 0


def _write_results(out_dir, columns):
    import pandas as pd
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        pd.DataFrame(columns).to_csv(os.path.join(out_dir, 'results.csv'))


def _plot(x, nbins, xlim, fname, **kw):
    try:
        from .refapi.utils import plot_density
    except Exception:  # plotting is optional (matplotlib)
        return
    plot_density(x, nbins, limits=xlim, fname=fname, **kw)


def evaluate_scatterometry(model, ys, forward_model, out_dir, plot_ys, n_samples_x, score_posterior, a, b,
                           lambd_bd, gt_dir, n_repeats=10, epsilon=1e-10, xlim=(-1.2, 1.2), nbins=75,
                           figsize=(12, 12), labelsize=30, gt_loader=None, num_steps=200):
    """main_diffusion_scatterometry.py:40-124. `gt_loader(i, j)` overrides the MCMC ground-truth
    files (`gt_dir/<i>/<j>.npy`, generate_scatterometry_ground_truth.py)."""
    dev = model._exec_device(ys)
    ys = torch.as_tensor(ys).to(device=dev, dtype=torch.float32)
    load = gt_loader or (lambda i, j: get_gt_samples_scatterometry(gt_dir, i, j))

    def one_y(i):
        y = ys[i]
        # (R, N, 3); the default precision's fp16-range guard (parallel.sample_checked) -- this rank's own y
        x_pred = parallel.sample_checked(model, y.expand(n_repeats, -1), n_samples_x, num_steps, 0, 1)
        x_true = torch.stack([torch.as_tensor(load(i, j)).to(device=dev, dtype=torch.float32)
                              for j in range(n_repeats)])
        inflated = y[None, :].expand(x_true.shape[1], -1)
        nll_t = nll_d = mse = 0.0
        for j in range(n_repeats):
            xt = x_true[j]
            t0 = torch.zeros(xt.shape[0], 1, device=dev)
            with torch.no_grad():
                s_pred = model.sde.a(xt, inflated, t0) / model.sde.base_sde.g(t0, xt)
            s_true = score_posterior(xt, inflated)
            mse += float(torch.mean(torch.sum((s_pred - s_true) ** 2, dim=1)))
            with torch.no_grad():
                nll_t += float(get_log_posterior(xt, forward_model, a, b, inflated, lambd_bd).sum()) / n_samples_x
                nll_d += float(get_log_posterior(x_pred[j], forward_model, a, b,
                                                 y[None, :].expand(x_pred.shape[1], -1), lambd_bd).sum()) / n_samples_x
        ht = histograms(x_true.reshape(1, -1, 3), nbins, xlim)[0]
        hd = histograms(x_pred.reshape(1, -1, 3), nbins, xlim)[0]
        kl, klr = hist_kl(ht, hd, epsilon)
        if i in plot_ys and out_dir:
            _plot(x_true[-1].cpu().numpy(), nbins, xlim, os.path.join(out_dir, 'posterior-mcmc-%d.svg' % i),
                  xticks=[-1, 0, 1], size=figsize, labelsize=labelsize)
            _plot(x_pred[-1].cpu().numpy(), nbins, xlim, os.path.join(out_dir, 'posterior-diffusion-%d.svg' % i),
                  xticks=[-1, 0, 1], size=figsize, labelsize=labelsize)
        return kl, klr, nll_t / n_repeats, nll_d / n_repeats, mse / n_repeats

    kl2_vals, kl2_rev, nll_mcmc, nll_diff, mse_vals = parallel.map_sharded(ys.shape[0], one_y, 5).T
    nlpd = np.abs(nll_diff - nll_mcmc)
    if _is_root():
        _write_results(out_dir, {'KL2': kl2_vals, 'KL_reverse': kl2_rev, 'NLL_mcmc': nll_mcmc,
                                 'NLL_diffusion': nll_diff, 'MSE': mse_vals})
        print('KL2:', kl2_vals.mean(), '+-', np.mean((kl2_vals - kl2_vals.mean()) ** 2))
    return kl2_vals.mean(), nlpd.mean(), float(np.mean(mse_vals))


def evaluate_linear(model, ys, forward_model, out_dir, plot_ys, n_samples_x=5000, n_repeats=10, epsilon=1e-10,
                    xlim=(-3.5, 3.5), nbins=75, figsize=(12, 12), labelsize=30, num_steps=200):
    """main_diffusion_linear.py:53-137, against the analytic Gaussian posterior."""
    dev = model._exec_device(ys)
    ys = torch.as_tensor(ys).to(device=dev, dtype=torch.float32)
    model.sde.eval()

    def one_y(i):
        y = ys[i]
        posterior = forward_model.get_posterior(y.cpu(), device='cpu')
        x_pred = parallel.sample_checked(model, y.expand(n_repeats, -1), n_samples_x, num_steps, 0, 1)  # (R, N, 2)
        x_true = posterior.sample((n_repeats, n_samples_x)).to(device=dev, dtype=torch.float32)
        nll_t = nll_d = mse = 0.0
        for j in range(n_repeats):
            xt = x_true[j]
            t0 = torch.zeros(xt.shape[0], 1, device=dev)
            inflated = torch.ones_like(xt) * y
            with torch.no_grad():
                s_pred = model.sde.a(xt, inflated, t0) / model.sde.base_sde.g(t0, xt)
            s_true = forward_model.score_posterior(xt, inflated)
            mse += float(torch.mean(torch.sum((s_pred - s_true) ** 2, dim=1)))
            nll_t -= float(torch.mean(posterior.log_prob(xt.cpu())))
            nll_d -= float(torch.mean(posterior.log_prob(x_pred[j].cpu())))
        ht = histograms(x_true.reshape(1, -1, 2), nbins, xlim)[0]
        hd = histograms(x_pred.reshape(1, -1, 2), nbins, xlim)[0]
        kl, _ = hist_kl(ht, hd, epsilon)
        if i in plot_ys and out_dir:
            _plot(x_true[-1].cpu().numpy(), nbins, xlim, os.path.join(out_dir, 'posterior-true-%d.svg' % i),
                  xticks=xlim, size=figsize, labelsize=labelsize, show_mean=True)
            _plot(x_pred[-1].cpu().numpy(), nbins, xlim, os.path.join(out_dir, 'posterior-diffusion-%d.svg' % i),
                  xticks=xlim, size=figsize, labelsize=labelsize, show_mean=True)
        return kl, nll_t / n_repeats, nll_d / n_repeats, mse / n_repeats

    kl2_vals, nll_true, nll_diff, mse_vals = parallel.map_sharded(ys.shape[0], one_y, 4).T
    nlpd = np.abs(nll_true - nll_diff)
    if _is_root():
        _write_results(out_dir, {'KL2': kl2_vals, 'NLL_true': nll_true, 'NLL_diffusion': nll_diff,
                                 'MSE': mse_vals})
        print('KL2:', kl2_vals.mean(), '+-', np.mean((kl2_vals - kl2_vals.mean()) ** 2))
    return kl2_vals.mean(), nlpd.mean(), float(np.mean(mse_vals))
