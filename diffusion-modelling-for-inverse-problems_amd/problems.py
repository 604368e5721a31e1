"""Workload definitions of the two inverse problems (SURVEY.md §2 rows "Linear problem",
"Scatterometry problem", "Datasets"), with the reference's function names so the drivers keep
working: linear_problem.py:5-65, utils_scatterometry.py:8-52, datasets.py:8-54, models/SNF.py:234-237.

These are host-side data producers (a few small torch ops per call); the hot path consumes their
outputs (y observations, training pairs) on the device.
"""
import os

import numpy as np
import torch
from torch import nn
from torch.distributions import MultivariateNormal

device = 'cuda' if torch.cuda.is_available() else 'cpu'


# ---------------------------------------------------------------------------- linear problem
class LinearForwardProblem:
    """y = A x + b + N(0, 0.3 I), x ~ N(0, I): a shear by 0.5 plus a translation (0.3, 0.5)
    (linear_problem.py:5-65). Gaussian posterior in closed form."""

    def __init__(self):
        self.epsilon = 1e-6
        self.xdim = 2
        self.ydim = 2
        self.A = torch.Tensor([[1, 0.5], [0, 1]])
        self.b = torch.Tensor([0.3, 0.5])
        self.scale = .3
        self.Sigma = self.scale * torch.eye(self.ydim)
        self.Lam = torch.eye(self.xdim)
        self.Sigma_inv = 1 / self.scale * torch.eye(self.ydim)
        self.Sigma_y_inv = torch.linalg.inv(self.Sigma + self.A @ self.Lam @ self.A.T + self.epsilon * torch.eye(self.ydim))
        self.mu = torch.zeros(self.xdim)

    def __call__(self, *args, **kwargs):
        return self.forward(args[0])

    def forward(self, x):
        return (self.A @ x.T).T + self.b

    def get_likelihood(self, x):
        return MultivariateNormal(self.A.to(x) @ x + self.b.to(x), self.Sigma)

    def get_evidence(self):
        return MultivariateNormal(self.A @ self.mu + self.b, self.Sigma + self.A @ self.Lam @ self.A.T)

    def get_posterior(self, y, device=device):
        y_res = y.cpu() - (self.A @ self.mu + self.b)
        mean = self.Lam @ self.A.T @ self.Sigma_y_inv @ y_res
        cov = self.Lam - self.Lam @ self.A.T @ self.Sigma_y_inv @ self.A @ self.Lam
        return MultivariateNormal(mean.to(device), cov.to(device))

    def log_posterior(self, xs, ys, epsilon=1e-6):
        mean = (ys - (self.A @ self.mu + self.b)) @ (self.A.T @ self.Sigma_y_inv)
        x_res = xs - mean
        cov = self.Lam - self.A.T @ self.Sigma_y_inv @ self.A
        cov_inv = torch.linalg.inv(cov + epsilon * torch.eye(self.xdim))
        return ((.5 * x_res @ cov_inv)[:, None, :] @ x_res[:, :, None]).view(-1, 1)

    def score_posterior(self, x, y):
        """-x + ((y - (A x + b)) Sigma^-1) A: the PINN initial condition (linear_problem.py:61-65)."""
        A, b, S = self.A.to(x), self.b.to(x), self.Sigma_inv.to(x)
        return -x + ((y - (x @ A.T + b)) @ S.T) @ A


# ---------------------------------------------------------------------- scatterometry problem
SCAT_PARAMS = {'a': 0.2, 'b': 0.01, 'lambd_bd': 1000, 'xdim': 3, 'ydim': 23}


def load_forward_model(src_dir):
    """Frozen 3 -> 256 -> 256 -> 256 -> 23 ReLU surrogate (utils_scatterometry.py:8-25). Reads the
    reference's `surrogate.pt` with weights_only=True, or a `surrogate.npz` of the same keys."""
    fm = nn.Sequential(nn.Linear(3, 256), nn.ReLU(), nn.Linear(256, 256), nn.ReLU(),
                       nn.Linear(256, 256), nn.ReLU(), nn.Linear(256, 23)).to(device)
    pt = os.path.join(src_dir, 'surrogate.pt')
    if os.path.exists(pt):
        sd = torch.load(pt, map_location=torch.device(device), weights_only=True)
    else:
        z = np.load(os.path.join(src_dir, 'surrogate.npz'))
        sd = {k.replace('_', '.'): torch.from_numpy(z[k]) for k in z.files}
    fm.load_state_dict(sd)
    for p in fm.parameters():
        p.requires_grad = False
    return fm, dict(SCAT_PARAMS)


def get_log_posterior(samples, forward_model, a, b, ys, lambd_bd):
    """Negative log posterior: heteroscedastic Gaussian likelihood + boundary-penalty prior
    (utils_scatterometry.py:30-38)."""
    f = forward_model(samples)
    pref = (a * f) ** 2 + b ** 2
    p = .5 * torch.sum(torch.log(pref), dim=1)
    p2 = 0.5 * torch.sum((ys - f) ** 2 / pref, dim=1)
    p3 = lambd_bd * torch.sum(torch.relu(samples - 1) + torch.relu(-1 - samples), dim=1)
    return p + p2 + p3


def inverse_cdf_prior(x, lambd_bd):
    """Samples of the boundary-penalty prior by inverse CDF (utils_scatterometry.py:42-52)."""
    x = x * ((2 * lambd_bd + 2) / lambd_bd)
    y = np.zeros_like(x)
    left = x < 1 / lambd_bd
    y[left] = np.log(x[left] * lambd_bd) - 1
    middle = np.logical_and(x >= 1 / lambd_bd, x < 2 + 1 / lambd_bd)
    y[middle] = x[middle] - 1 / lambd_bd - 1
    right = x >= 2 + 1 / lambd_bd
    y[right] = -np.log(((2 + 2 / lambd_bd) - x[right]) * lambd_bd) + 1
    return y


def energy_grad(x, energy):
    """d energy / dx and the energy (models/SNF.py:234-237): the scatterometry score is -grad."""
    x = x.requires_grad_(True)
    e = energy(x)
    return torch.autograd.grad(e.sum(), x, create_graph=True)[0], e


# ---------------------------------------------------------------------------------- datasets
def generate_dataset_scatterometry(forward_model, a, b, size=100):
    """Seeded test set: x ~ U[-1,1]^3 (seed 13), y = f(x) + b eps1 + a f(x) eps2 (seed 14)
    (datasets.py:8-17)."""
    gen = torch.manual_seed(13)
    xs = torch.rand(size, 3, generator=gen).to(device) * 2 - 1
    ys = forward_model(xs)
    ys = ys + b * torch.randn(ys.shape, generator=gen).to(device) + \
        ys * a * torch.randn(ys.shape, generator=torch.manual_seed(14)).to(device)
    return xs, ys


def get_gt_samples_scatterometry(src_dir, y, i):
    with open(os.path.join(src_dir, str(y), '%d.npy' % i), 'rb') as f:
        return np.load(f)


def get_dataloader_scatterometry(batch_size, forward_model, a, b, lambd_bd):
    """8 batches of prior samples pushed through the surrogate plus noise (datasets.py:26-34)."""
    x = torch.tensor(inverse_cdf_prior(np.random.uniform(size=(8 * batch_size, 3)), lambd_bd),
                     dtype=torch.float, device=device)
    y = forward_model(x)
    y += torch.randn_like(y) * b + torch.randn_like(y) * a * y

    def epoch_data_loader():
        for i in range(0, 8 * batch_size, batch_size):
            yield x[i:i + batch_size].clone(), y[i:i + batch_size].clone()
    return epoch_data_loader


def generate_dataset_linear(xdim, f, n_samples, random_state=7):
    gen = torch.random.manual_seed(random_state)
    x = torch.randn(n_samples, xdim, generator=gen).to(device)
    return x, f(x)


def get_dataloader_linear(x_train, y_train, sigma, batch_size):
    """Shuffled epoch with fresh observation noise (datasets.py:44-54)."""
    perm = torch.randperm(len(x_train))
    x = x_train[perm]
    y = y_train[perm]
    y += sigma * torch.randn_like(y)

    def epoch_data_loader():
        for i in range(0, len(x), batch_size):
            yield x[i:i + batch_size].to(device), y[i:i + batch_size].to(device)
    return epoch_data_loader
