"""Workload definitions of the two inverse problems (SURVEY.md §2 rows "Linear problem",
"Scatterometry problem", "Datasets"), with the reference's function names so the drivers keep
working: linear_problem.py:5-65, utils_scatterometry.py:8-52, datasets.py:8-54, models/SNF.py:234-237.

The data producers are host-side torch ops; the hot path consumes their outputs (y observations,
training pairs) on the device. The scatterometry posterior itself (get_log_posterior, energy_grad)
and the Metropolis-Hastings ground-truth sampler (anneal_to_energy) run on the device as fused
exact-f32 MFMA kernels (libdmip dmip_log_posterior / dmip_mh_sample, csrc/dmip_surrogate.hip)
whenever the samples are on a HIP device and the forward model is the reference's surrogate shape.
"""
import os
import warnings

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


_SUR_SHAPES = [(256, 3), (256, 256), (256, 256), (23, 256)]


def _surrogate_layers(forward_model):
    """[(weight, bias)] if forward_model is the reference surrogate (Linear/ReLU x3/Linear,
    3 -> 256 -> 256 -> 256 -> 23, utils_scatterometry.py:9-12), else None."""
    if not isinstance(forward_model, nn.Sequential) or len(forward_model) != 7:
        return None
    mods = list(forward_model)
    if not all(isinstance(mods[i], nn.ReLU) for i in (1, 3, 5)):
        return None
    lin = [mods[i] for i in (0, 2, 4, 6)]
    if not all(isinstance(m, nn.Linear) and m.bias is not None for m in lin):
        return None
    if [tuple(m.weight.shape) for m in lin] != _SUR_SHAPES:
        return None
    return [(m.weight, m.bias) for m in lin]


def surrogate_handle(forward_model, device):
    """Packed device images of the frozen surrogate (dmip_surrogate_create), cached on the module
    per parameter snapshot; None if the module is not the compiled surrogate shape."""
    from . import _lib
    layers = _surrogate_layers(forward_model)
    if layers is None:
        return None
    key = (str(device),) + tuple((p.data_ptr(), p._version) for p in forward_model.parameters())
    cached = getattr(forward_model, "_dmip_surrogate", None)
    if cached is None or cached[0] != key:
        cached = (key, _lib.SurrogateHandle(layers, device))
        forward_model._dmip_surrogate = cached
    return cached[1]


class _FusedLogPosterior(torch.autograd.Function):
    """get_log_posterior on the device: E and (when samples need a gradient) dE/dx from one launch of
    the fused kernel; backward scales the stored gradient (first order, as energy_grad uses it)."""

    @staticmethod
    def forward(ctx, samples, handle, noise, ys, y_stride):
        from . import _lib
        x = samples.detach().to(torch.float32).contiguous()
        e = torch.empty(x.shape[0], device=x.device, dtype=torch.float32)
        g = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        _lib.log_posterior(handle, noise, x, ys, y_stride, e, g)
        ctx.save_for_backward(g if g is not None else e)
        ctx.has_grad = g is not None
        return e

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, ge):
        (g,) = ctx.saved_tensors
        return (ge[:, None] * g if ctx.has_grad else None), None, None, None, None


def get_log_posterior(samples, forward_model, a, b, ys, lambd_bd):
    """Negative log posterior: heteroscedastic Gaussian likelihood + boundary-penalty prior
    (utils_scatterometry.py:30-38). On a HIP device with the reference surrogate: the fused exact-f32
    kernel (differentiable w.r.t. samples, first order); otherwise the reference's torch ops."""
    if isinstance(samples, torch.Tensor) and samples.is_cuda:
        h = surrogate_handle(forward_model, samples.device)
        if h is not None and samples.ndim == 2 and samples.shape[1] == 3:
            from . import _lib
            y = torch.as_tensor(ys).to(device=samples.device, dtype=torch.float32)
            if y.ndim == 1 or y.shape[0] == 1:
                y, stride = y.reshape(1, -1).contiguous(), 0
            else:
                y = y.expand(samples.shape[0], -1).contiguous()
                stride = y.shape[1]
            return _FusedLogPosterior.apply(samples, h, _lib.scat_noise(a, b, lambd_bd), y, stride)
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


# ------------------------------------------------------- Metropolis-Hastings ground truth (F3)
class ScatterometryEnergy:
    """energy(x) = get_log_posterior(x, forward_model, a, b, y, lambd_bd) for one observation y -- the
    `mcmc_energy` of generate_scatterometry_ground_truth.py:61 as an object anneal_to_energy can fuse."""

    def __init__(self, forward_model, a, b, y, lambd_bd):
        self.forward_model, self.a, self.b, self.lambd_bd = forward_model, a, b, lambd_bd
        self.y = torch.as_tensor(y, dtype=torch.float32).reshape(-1)

    def __call__(self, x):
        return get_log_posterior(x, self.forward_model, self.a, self.b, self.y.to(x.device)[None, :], self.lambd_bd)


def mh_sample(forward_model, params, ys, n_chains, num_steps, noise_std, seed=None, chain_offset=0, x_init=None,
              noise=None, unif=None, return_ediff=False, precision="fp32", agree=None):
    """Fused random-walk MH (dmip_mh_sample_ex) for every row of ys (n_y, 23): device tensor
    (n_y, n_chains, 3). x_init (n_y, n_chains, 3) or None for x0 ~ U[-1, 1]^3 from the chain RNG;
    noise (S, n_y, n_chains, 3) / unif (S, n_y, n_chains) replay captured draws (exact f32 only).
    precision "fp32": the exact-f32 kernel; "fp32x3": the surrogate's products as three-term fp16 splits (same
    RNG stream and acceptance test per chain) -- a weight, proposal or activation beyond fp16's range resamples
    every chain with "fp32" (RuntimeWarning); `agree` (parallel.any_rank) makes that decision, and any other failure,
    collective (parallel.guarded)."""
    from . import _lib
    ys = torch.as_tensor(ys)
    if not torch.cuda.is_available():
        raise RuntimeError("dmip: MH sampling needs a HIP device (fused kernel; there is no CPU path)")
    dev = ys.device if ys.is_cuda else torch.device("cuda", torch.cuda.current_device())
    ys = ys.to(device=dev, dtype=torch.float32).reshape(-1, 23).contiguous()
    h = surrogate_handle(forward_model, dev)
    if h is None:
        raise ValueError("mh_sample: forward_model is not the scatterometry surrogate shape (3 -> 256^3 -> 23)")
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    out = torch.empty(ys.shape[0], int(n_chains), 3, device=dev, dtype=torch.float32)
    ed = torch.empty(ys.shape[0], int(n_chains), device=dev, dtype=torch.float32) if return_ediff else None
    prep = lambda t: None if t is None else t.to(device=dev, dtype=torch.float32).contiguous()
    if precision not in ("fp32", "fp32x3"):
        raise ValueError(f"mh_sample: precision {precision!r} (\"fp32\" or \"fp32x3\")")
    if precision == "fp32x3" and (noise is not None or unif is not None):
        raise ValueError("mh_sample: injected draws replay the exact-f32 kernel (precision=\"fp32\")")
    nz = _lib.scat_noise(params['a'], params['b'], params['lambd_bd'])
    x0 = prep(x_init)
    from . import parallel

    def run(prec):
        def launch():
            if prec == "fp32x3":
                _lib.mh_sample(h, nz, ys, n_chains, chain_offset, num_steps, noise_std, seed, out, x0, None, None, ed,
                               precision="fp32x3")
            else:
                _lib.mh_sample(h, nz, ys, n_chains, chain_offset, num_steps, noise_std, seed, out, x0, prep(noise),
                               prep(unif), ed)
            return (out, ed) if return_ediff else out
        return launch

    # the status word is read after the launch either way; a fp32x3 range report resamples every chain in exact f32,
    # decided by all ranks together under `agree` (parallel.guarded)
    return parallel.guarded(dev, run(precision), run("fp32") if precision == "fp32x3" else None, agree)


def anneal_to_energy(x_curr, energy, metr_steps_per_block, noise_std=0.1, langevin_prop=False, lang_steps=None,
                     stepsize=None):
    """models/SNF.py:250-275 (random-walk proposals). Returns (x, E(x) - E(x0)). With a
    ScatterometryEnergy and device samples: one fused launch for all steps; any other energy
    callable: the reference's loop (its energy evaluations still go to the device kernel when the
    callable is get_log_posterior on device samples)."""
    if langevin_prop:
        raise NotImplementedError("Langevin proposals belong to the SNF baseline (out of scope, SURVEY.md §2)")
    if isinstance(energy, ScatterometryEnergy) and x_curr.is_cuda:
        x0 = x_curr.detach().to(torch.float32).reshape(1, -1, 3).contiguous()
        x, ed = mh_sample(energy.forward_model, {'a': energy.a, 'b': energy.b, 'lambd_bd': energy.lambd_bd},
                          energy.y.to(x_curr.device)[None, :], x0.shape[1], metr_steps_per_block, noise_std,
                          x_init=x0, return_ediff=True)
        return x[0], ed[0]
    e0 = energy(x_curr)
    e_curr = e0
    for _ in range(metr_steps_per_block):
        x_prop = x_curr + noise_std * torch.randn_like(x_curr)
        e_prop = energy(x_prop)
        e_curr = energy(x_curr)
        acc = (torch.rand_like(e_prop) < torch.exp(-e_prop + e_curr)).float().view(len(x_prop), 1)
        x_curr = (1. - acc) * x_curr + acc * x_prop
        e_curr = (1. - acc.view(-1)) * e_curr + acc.view(-1) * e_prop
    return x_curr, e_curr.view(-1) - e0.view(-1)


def generate_gt_samples(forward_model, params, ys, out_dir=None, n_samples_x=30000, n_repeats=10, metr_steps=1000,
                        noise_std=0.5, seed=None, precision="fp32"):
    """generate_scatterometry_ground_truth.py:26-63 on the device: for every y and repeat j,
    n_samples_x MH chains from U[-1, 1]^3 for metr_steps steps (NOISE_STD_MCMC, METR_STEPS of
    config_scatterometry.yml), all in one launch (precision as mh_sample); under torch.distributed the chains
    are sharded over the ranks (parallel.chains_sharded: every rank gets the whole, bit-identical to one GPU; rank 0
    writes the files); optionally written as out_dir/<i>/<j>.npy. Returns a device tensor (n_y, n_repeats, n_samples_x, 3)."""
    from . import parallel
    ys = torch.as_tensor(ys, dtype=torch.float32).reshape(-1, 23)
    rows = ys.repeat_interleave(n_repeats, dim=0)
    if not torch.cuda.is_available():
        raise RuntimeError("dmip: MH sampling needs a HIP device (fused kernel; there is no CPU path)")
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    dev = ys.device if ys.is_cuda else torch.device("cuda", torch.cuda.current_device())
    run = lambda n, off, s, agree: mh_sample(forward_model, params, rows, n, metr_steps, noise_std, seed=s,
                                             chain_offset=off, precision=precision, agree=agree)
    x = parallel.chains_sharded(n_samples_x, run, seed, dev)  # one process: a single launch of all chains
    x = x.reshape(ys.shape[0], n_repeats, n_samples_x, 3)
    rank, ws = parallel.world()
    if out_dir and rank == 0:
        xh = x.cpu().numpy()
        for i in range(ys.shape[0]):
            d = os.path.join(out_dir, str(i))
            os.makedirs(d, exist_ok=True)
            for j in range(n_repeats):
                with open(os.path.join(d, '%d.npy' % j), 'wb') as fh:
                    np.save(fh, xh[i, j])
    if out_dir and ws > 1:
        import torch.distributed as dist
        dist.barrier()  # no rank returns (and reads gt_dir) before rank 0's files are complete
    return x


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
