"""VP-SDE and plug-in reverse SDE with the reference's API (sdes.py:9-126).

These objects carry the SDE coefficients for the host side (losses, training, evaluate) and the
parameters the fused HIP sampler consumes; the sampling loop itself never runs here -- it is one
kernel launch (estimators.BaseClassDiffusionModel.forward -> libdmip dmip_em_sample).
"""
import math

import torch


class VariancePreservingSDE(torch.nn.Module):
    """Song et al. VP-SDE, eq. 32-33 (sdes.py:9-57): beta(t) = beta_min + (beta_max-beta_min) t."""

    def __init__(self, beta_min=0.1, beta_max=20.0, T=1.0, t_epsilon=0.001):
        super().__init__()
        self.beta_min = beta_min
        self.beta_max = beta_max
        self.T = T
        self.t_epsilon = t_epsilon

    def beta(self, t):
        return self.beta_min + (self.beta_max - self.beta_min) * t

    def mean_weight(self, t):
        return torch.exp(-0.25 * t ** 2 * (self.beta_max - self.beta_min) - 0.5 * t * self.beta_min)

    def var(self, t):
        return 1. - torch.exp(-0.5 * t ** 2 * (self.beta_max - self.beta_min) - t * self.beta_min)

    def f(self, t, y):
        return -0.5 * self.beta(t) * y

    def g(self, t, y):
        return torch.ones_like(y) * self.beta(t) ** 0.5

    def sample(self, t, y0, return_noise=False):
        """y_t | y0 ~ N(alpha(t) y0, var(t)) (sdes.py:37-49); optionally (y_t, eps, std, g(t, y_t))."""
        mu = self.mean_weight(t) * y0
        std = self.var(t) ** 0.5
        eps = torch.randn_like(y0)
        yt = eps * std + mu
        if not return_noise:
            return yt
        return yt, eps, std, self.g(t, yt)

    def sample_debiasing_t(self, shape):
        """Importance-sampled training times, pdf proportional to g^2/std^2 = beta/var on
        [t_eps, T] and flat below t_eps (sdes.py:51-57 -> sdeflow-light sample_vp_truncated_q, not
        vendored in the reference; restated from its math, see sample_vp_truncated_q)."""
        return sample_vp_truncated_q(shape, self.beta_min, self.beta_max, self.t_epsilon, self.T)


def _integral_beta(t, bmin, bmax):
    return 0.5 * t ** 2 * (bmax - bmin) + t * bmin


def sample_vp_truncated_q(shape, beta_min, beta_max, t_epsilon, T, u=None):
    """Inverse-CDF sampler of q(t) ~ r(max(t, t_eps)), r(t) = beta(t)/var(t), on [0, T].

    With B(t) = int_0^t beta, the antiderivative of r is A(t) = log(e^{B(t)} - 1); the CDF is
    linear below t_eps (slope r(t_eps)) and A(t) - A(t_eps) + t_eps r(t_eps) above. Inverting the
    upper branch: B = log(1 + exp(Z u + A(t_eps) - t_eps r(t_eps))) and t = (-b + sqrt(b^2 + 2aB))/a
    with a = beta_max - beta_min, b = beta_min. (sdeflow-light is absent from the reference, so this
    restatement is parity-unpinned; tests check its density.)
    """
    a = float(beta_max - beta_min)
    b = float(beta_min)
    te = float(t_epsilon)
    B_te = 0.5 * a * te * te + b * te
    r_te = (b + a * te) / (1.0 - math.exp(-B_te))
    A_te = math.log(math.expm1(B_te))
    B_T = 0.5 * a * float(T) ** 2 + b * float(T)
    Z = te * r_te + math.log(math.expm1(B_T)) - A_te
    if u is None:
        u = torch.rand(*shape)
    lower = u <= te * r_te / Z
    Bu = torch.nn.functional.softplus(Z * u + A_te - te * r_te)
    t_hi = (-b + torch.sqrt(b * b + 2.0 * a * Bu)) / a
    t_lo = Z / r_te * u
    return torch.where(lower, t_lo, t_hi)


class PluginReverseSDE(torch.nn.Module):
    """Reverse-time SDE from a base SDE and a learned drift `a` (sdes.py:60-87):
    mu(t, x, cond) = (1 - lmbd/2) g(T-t) a(x, cond, T-t) - f(T-t, x);  sigma = sqrt(1-lmbd) g(T-t)."""

    def __init__(self, base_sde, drift_a, T, vtype='rademacher', debias=False):
        super().__init__()
        self.base_sde = base_sde
        self.a = drift_a
        self.T = T
        self.vtype = vtype
        self.debias = debias

    def mu(self, t, x, cond, lmbd=0.):
        return (1. - 0.5 * lmbd) * self.base_sde.g(self.T - t, x) * self.a(x, cond, self.T - t) - \
            self.base_sde.f(self.T - t, x)

    def sigma(self, t, y, lmbd=0.):
        return (1. - lmbd) ** 0.5 * self.base_sde.g(self.T - t, y)
