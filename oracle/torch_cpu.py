"""Reference-order CPU sampler on torch-CPU -- TEST / BASELINE INFRASTRUCTURE ONLY.

The reference's sampling path IS PyTorch eager on the CPU (models/diffusion.py:27-46 with
nets.py:17-35 and sdes.py:77-87). This restates that loop op for op on torch-CPU tensors so that
bench.py's `cpu_baseline` times the same arithmetic the reference runs (MKL sgemm, vectorised
tanh, one randn per step), on the GPU box's host cores. It is never imported by the product.
"""
import torch


def build_mlp(params):
    """nn.Sequential with the reference's chain: Linear, Tanh, Tanh, [Linear, Tanh]*, Linear."""
    layers = []
    for i, (W, b) in enumerate(params):
        lin = torch.nn.Linear(W.shape[1], W.shape[0])
        with torch.no_grad():
            lin.weight.copy_(torch.as_tensor(W))
            lin.bias.copy_(torch.as_tensor(b))
        layers.append(lin)
        if i < len(params) - 1:
            layers.append(torch.nn.Tanh())
            if i == 0:
                layers.append(torch.nn.Tanh())
    return torch.nn.Sequential(*layers)


@torch.no_grad()
def cde_sample(net, y, num_samples, num_steps, xdim, T=1.0, beta_min=0.1, beta_max=20.0, seed=0):
    """models/diffusion.py:27-46 for CDE on the CPU; returns (num_samples, xdim) float32."""
    gen = torch.Generator().manual_seed(seed)
    y = torch.as_tensor(y, dtype=torch.float32)
    ys = torch.zeros(num_samples, y.shape[-1]) + y
    delta = T / num_steps
    x = torch.randn(num_samples, xdim, generator=gen)
    ts = torch.linspace(0, 1, num_steps + 1) * T
    ones = torch.ones(num_samples, 1)
    for i in range(num_steps):
        tau = T - ones * ts[i]
        beta = beta_min + (beta_max - beta_min) * tau
        g = torch.ones_like(x) * beta ** 0.5
        a = net(torch.cat([x, ys, tau], dim=1))
        mu = g * a - (-0.5 * beta * x)
        x = x + delta * mu + delta ** 0.5 * g * torch.randn(x.shape, generator=gen)
    return x
