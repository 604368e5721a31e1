"""Training losses with the reference's API (losses.py:7-386).

DSM, ScoreFPE (exact divergence + the total time-derivative of the score by autograd), the
conditional ScoreFPE, DSM_PDE, PINN and Posterior losses as PyTorch autograd graphs (the reference's
own arithmetic, on any device), checked against the reference's values and parameter gradients
(tests/golden/pinn_linear.npz). On a HIP device, CDE.train_epoch replaces the loss + backward of
the supported (network, loss) pairs with the fused HIP loss-and-gradient kernel (csrc/dmip_train.hip,
training.py); these classes stay the API and the reference for every other case.
"""
import torch
from torch import nn


def divergence(y, x):
    """sum_i d y_i / d x_i by one VJP per output dimension, graph kept (losses.py:14-18)."""
    div = 0.
    for i in range(y.shape[-1]):
        vjp = torch.autograd.grad(y[..., i], x, torch.ones_like(y[..., i]), create_graph=True, retain_graph=True)[0]
        div = div + vjp[..., i:i + 1]
    return div


def batch_gradient(y, x):
    """Column i = d y_i / d x for a per-row scalar x (losses.py:20-26): with x = t this is the TOTAL
    derivative of the score through x_t(t) and g(t) as well as the explicit time input."""
    cols = []
    for i in range(y.shape[1]):
        cols.append(torch.autograd.grad(y[:, i].sum(), x, retain_graph=True, create_graph=True)[0].view(-1))
    return torch.zeros_like(y) + torch.stack(cols, dim=1)


def div_estimator(s, x, num_samples=1, rademacher=True):
    """Hutchinson divergence estimate (losses.py:28-40)."""
    div = torch.zeros(s.shape[0], 1, device=s.device)
    for _ in range(num_samples):
        if rademacher:
            v = torch.randint(0, 2, s.shape, device=s.device).to(s.dtype) * 2 - 1
        else:
            v = torch.randn_like(s)
        vjp = torch.autograd.grad(s, x, grad_outputs=v, create_graph=True, retain_graph=True)[0]
        div = div + (vjp * v).sum(dim=1, keepdim=True)
    return div / num_samples


class DSMLoss(nn.Module):
    """0.5 ||s std + eps||^2 per row (losses.py:42-52)."""

    def __init__(self):
        super().__init__()
        self.name = 'DSMLoss'

    def forward(self, s, std, target):
        return ((s * std + target) ** 2).view(s.shape[0], -1).sum(1, keepdim=False) / 2


class ScoreFPELoss(nn.Module):
    """Residual of the score Fokker-Planck equation (losses.py:55-98):
    mean_k | ds_k/dt - 0.5 beta d/dx_k [div s + ||s||^2 + x.s] |  (L1) or squared (L2).
    The x-gradient is taken without create_graph, i.e. it is a constant for the parameter
    gradients -- exactly as in the reference."""

    def __init__(self, metric='L1'):
        super().__init__()
        self.name = 'FPELoss'
        self.metric = metric

    def forward(self, s, x_t, t, beta, divergence_method='exact'):
        if s.shape != x_t.shape:
            raise ValueError(f"score shape {tuple(s.shape)} differs from x_t shape {tuple(x_t.shape)}")
        n = x_t.shape[0]
        if divergence_method == 'exact':
            div = divergence(s, x_t)
        elif divergence_method in ['hutchinson', 'approx', 'approximate']:
            div = div_estimator(s, x_t)
        else:
            raise ValueError(f"unknown divergence method {divergence_method!r} "
                             "(one of 'exact', 'hutchinson', 'approx', 'approximate')")
        ds_dt = batch_gradient(s, t)
        potential = div + torch.sum(s ** 2, dim=1).view(-1, 1) + (x_t[:, None, :] @ s[:, :, None]).view(-1, 1)
        grad_x = torch.autograd.grad(potential, x_t, grad_outputs=torch.ones_like(div), retain_graph=True)[0]
        r = ds_dt - .5 * beta * grad_x
        if self.metric == 'L1':
            return torch.mean(torch.abs(r), dim=1).view(n, 1)
        if self.metric == 'L2':
            return torch.mean(r ** 2, dim=1).view(n, 1)
        raise ValueError(f"metric must be 'L1' or 'L2', got {self.metric!r}")


class ConditionalScoreFPELoss(nn.Module):
    """sum_k (std^3 ds_k/dt - 0.5 eps_k beta alpha^2)^2 (L2) or |.| (L1) (losses.py:100-124)."""

    def __init__(self, metric='L2'):
        super().__init__()
        self.name = 'cScoreFPELoss'
        self.metric = metric

    def forward(self, s, t, alpha, beta, target, std):
        ds_dt = batch_gradient(s, t)
        u = .5 * target * beta * alpha ** 2
        r = std ** 3 * ds_dt - u
        if self.metric == 'L2':
            return torch.sum(r ** 2, dim=1)
        if self.metric == 'L1':
            return torch.sum(torch.abs(r), dim=1)
        raise ValueError(f"metric must be 'L1' or 'L2', got {self.metric!r}")


def _score_and_cond(model, x, y, diffused_samples, t, g):
    cond = y if diffused_samples.shape[1] == x.shape[1] else torch.Tensor([]).to(x)
    return model.a(diffused_samples, cond, t) / g


def _pde_term(pde_loss, lam, model, score, diffused_samples, t, beta, target, std):
    if pde_loss.name == 'cScoreFPELoss':
        return lam * pde_loss(score, t, model.base_sde.mean_weight(t), beta, target, std)
    return lam * pde_loss(score, diffused_samples, t, beta)


class DSM_PDELoss(nn.Module):
    """DSM + lam * PDE residual, Lai et al. 2023 (losses.py:126-164)."""

    def __init__(self, lam=1., pde_loss='FPE', pde_metric='L1'):
        super().__init__()
        self.lam = lam
        self.dsm_loss = DSMLoss()
        self.pde_loss = ScoreFPELoss(pde_metric) if pde_loss == 'FPE' else ConditionalScoreFPELoss(pde_metric)
        self.name = 'DSM_PDELoss'

    def forward(self, model, x, y, diffused_samples, t, target, std, g):
        score = _score_and_cond(model, x, y, diffused_samples, t, g)
        beta = model.base_sde.beta(t)
        dsm = self.dsm_loss(score, std, target)
        pde = _pde_term(self.pde_loss, self.lam, model, score, diffused_samples, t, beta, target, std)
        return torch.mean(dsm + pde), {'PDE-Loss': pde.mean(), 'DSM-Loss': dsm.mean()}


def _initial_condition(metric, lam2, s0, ic_target, n):
    if metric == 'L2':
        return lam2 * torch.mean((s0 - ic_target) ** 2, dim=1).view(n, 1)
    if metric == 'L1':
        return lam2 * torch.mean(torch.abs(s0 - ic_target), dim=1).view(n, 1)
    raise ValueError('ic_metric must be "L1" or "L2", got {}'.format(metric))


class PINNLoss(nn.Module):
    """DSM + initial-condition (score at t=0 vs the known posterior score) + PDE residual,
    Raissi et al. 2019 (losses.py:168-242)."""

    def __init__(self, initial_condition, lam=1., lam2=1., pde_loss='FPE', ic_metric='L1', pde_metric='L1'):
        super().__init__()
        self.lam = lam
        self.lam2 = lam2
        self.initial_condition = initial_condition
        self.pde_loss = ConditionalScoreFPELoss(pde_metric) if pde_loss == 'cScoreFPE' else ScoreFPELoss(pde_metric)
        self.dsm_loss = DSMLoss()
        self.name = 'PINNLoss'
        self.ic_metric = ic_metric

    def forward(self, model, x, y, diffused_samples, t, target, std, g):
        n, xdim = x.shape
        t0 = torch.zeros_like(t)
        s0 = model.a(x, y, t0) / model.base_sde.g(t0, diffused_samples)
        score = _score_and_cond(model, x, y, diffused_samples, t, g)
        beta = model.base_sde.beta(t)
        ic = _initial_condition(self.ic_metric, self.lam2, s0[:, :xdim], self.initial_condition(x, y), n)
        dsm = self.dsm_loss(score, std, target)
        pde = _pde_term(self.pde_loss, self.lam, model, score, diffused_samples, t, beta, target, std)
        loss = torch.mean(dsm + ic + pde)
        return loss, {'PDE-Loss': pde.mean(), 'Initial Condition': ic.mean(), 'DSM-Loss': dsm.mean()}


class PINNLoss2(nn.Module):
    """PINN loss without the DSM term (losses.py:245-291). The reference never sets
    `self.ic_metric` (AttributeError on first call); here it is a constructor argument."""

    def __init__(self, initial_condition, lam=1., lam2=1., pde_loss='FPE', pde_metric='L1', ic_metric='L2'):
        super().__init__()
        self.lam = lam
        self.lam2 = lam2
        self.initial_condition = initial_condition
        self.pde_loss = ScoreFPELoss(pde_metric) if pde_loss == 'FPE' else ConditionalScoreFPELoss(pde_metric)
        self.eval_metric = DSMLoss()
        self.name = 'PINNLoss2'
        self.ic_metric = ic_metric

    def forward(self, model, x, y, diffused_samples, t, target, std, g):
        n, xdim = x.shape
        t0 = torch.zeros_like(t)
        s0 = model.a(x, y, t0) / model.base_sde.g(t0, diffused_samples)
        score = _score_and_cond(model, x, y, diffused_samples, t, g)
        beta = model.base_sde.beta(t)
        ic = _initial_condition(self.ic_metric, self.lam2, s0[:, :xdim], self.initial_condition(x, y), n)
        pde = _pde_term(self.pde_loss, self.lam, model, score, diffused_samples, t, beta, target, std)
        return torch.mean(ic + pde), {'PDE-Loss': pde.mean(), 'Initial Condition': ic.mean(),
                                      'DSM_eval': self.eval_metric(score, std, target).mean()}


class PosteriorLoss(nn.Module):
    """Prior DSM + lam ||alpha s_lik - grad log p(y | x0_hat)||^2 with the Tweedie estimate
    x0_hat = (x_t + std^2 s_prior) / alpha, Chung & Kim 2023 (losses.py:293-386)."""

    def __init__(self, forward_model, a, b, lam):
        super().__init__()
        self.name = 'PosteriorLoss'
        self.dsm_loss = DSMLoss()
        self.forward_model = forward_model
        self.a = a
        self.b = b
        self.lam = lam

    def likelihood_target(self, x_0, y, x_t, s, sigma):
        f_x = self.forward_model(x_0)
        pref = (self.a * f_x) ** 2 + self.b ** 2
        vs = (f_x / pref, (y - f_x) / pref, (y - f_x) ** 2 * f_x / pref)
        vjp = [torch.autograd.grad(f_x, x_0, v, retain_graph=True)[0] for v in vs]
        vhp = [torch.autograd.grad(s, x_t, u, retain_graph=True)[0] for u in vjp]
        return -self.a ** 2 * (sigma ** 2 * vhp[0] + vjp[0]) + sigma ** 2 * vhp[1] + vjp[1] + \
            self.a ** 2 * (sigma ** 2 * vhp[2] + vjp[2])

    def forward(self, model, x, y, t):
        x_t, target, std, g = model.base_sde.sample(t, x, return_noise=True)
        s_prior = model.a.prior_net(x_t, t)
        s_lik = model.a.likelihood_net(x_t, y, t)
        alpha = model.base_sde.mean_weight(t)
        prior_loss = self.dsm_loss(s_prior, std, target)
        x_0 = 1 / model.base_sde.mean_weight(t) * (x_t + std ** 2 * s_prior)
        lik = torch.sum((alpha * s_lik - self.likelihood_target(x_0, y, x_t, s_prior, std)) ** 2, dim=1)
        loss = torch.mean(prior_loss + self.lam * lik)
        return loss, {'PriorLoss': prior_loss.mean(), 'LikelihoodLoss': self.lam * lik.mean()}
