"""CDE / CDiffE / PosteriorDiffusionEstimator with the reference's construct-and-sample API
(models/diffusion.py:14-229).

Sampling is the hot path and runs on the HIP device only: one launch of the fused persistent
reverse-SDE kernel for all num_steps, the chain state never leaving the registers --
  * CDE: dmip_em_sample;
  * PosteriorDiffusionEstimator: dmip_em_sample_posterior (prior + likelihood networks in one kernel);
  * CDiffE (repaired sampler): dmip_em_sample_cdiffe;
  * DPS (BASELINE config 4, prior score net + forward-model guidance): dmip_dps_sample.
Precision (`model.precision`, or `precision=` per call; default from $DMIP_PRECISION, else "fp32x3"):
  "fp32x3" -- the reference's fp32 arithmetic at the fp16 matrix rate: every product as three fp16 MFMAs
             (W_hi h_hi + W_hi h_lo + W_lo h_hi, fp32 accumulation; csrc/dmip_x3.h), tanh by exp2 + rcp.
             Error per product 2^-23 of sum |w h|, as an fp32 fmaf chain. The default.
  "fp32"   -- exact f32 (v_mfma_f32_16x16x4_f32, an fmaf chain, libm tanh): the bit-level parity mode.
  "fp16"   -- 16-bit MFMA operands (fp16 hidden and output layers, split-bf16 layer 1): the fastest
             mode, ~1e-3 relative per network evaluation. ("bf16" is its deprecated name.)
A shape without a fused kernel in the requested precision runs the next more accurate one that has one
(fp16 -> fp32x3 -> fp32). Shapes with no fused kernel at all step through per-step launches of the
network kernel (dmip_mlp_forward, exact f32) with the SDE update as device tensor ops and the kernels'
chain-keyed RNG (so sharding stays bit-identical there too).
There is no CPU sampling path: without a HIP device the samplers raise.

RNG: the reference draws x0 and the per-step noise from torch's global generator. Here every chain
has its own counter-keyed stream (seed, global chain index, y index); the seed itself is drawn from
torch's global generator, so torch.manual_seed(s) still makes a sampling call reproducible, and the
samples of a chain do not depend on how chains are split over workgroups or GPUs.
"""
import os

import numpy as np
import torch
from torch import nn

from . import _lib
from . import sdes
from .losses import PosteriorLoss
from .nets import MLP, MLP2, PosteriorScore

device = 'cuda' if torch.cuda.is_available() else 'cpu'


class _FusedStep:
    """A batch whose loss and parameter gradients came from the fused kernel (training.py)."""

    def __init__(self, loss, info, stepped=False):
        self.loss, self.info, self.stepped = loss, info, stepped  # stepped: the optimizer update ran too


def _draw_seed():
    return int(torch.randint(0, 2 ** 62, (1,)).item())


def canonical_precision(precision):
    """The sampler precision's name: "bf16" is the deprecated name of "fp16" (the 16-bit engine computes its
    hidden and output layers in fp16)."""
    return "fp16" if precision == "bf16" else precision


def default_precision():
    return canonical_precision(os.environ.get("DMIP_PRECISION", "fp32x3"))


# a precision whose fused kernel is missing for a shape falls back to a more accurate one, never a less
# accurate one: fp16 -> fp32x3 -> fp32
_MORE_ACCURATE = {"fp16": ("fp32x3", "fp32"), "fp32x3": ("fp32",), "fp32": ()}


def _fused_precision(precision, mode, width, n_hidden, xdim, ydim, acts=(_lib.DMIP_ACT_TANH_TWICE_FIRST,)):
    """The precision a fused kernel runs this shape in: the requested one, else the next more accurate
    one that is compiled (_MORE_ACCURATE); None when none is (per-step loop). `acts`: the networks' activation
    chains -- a SiLU network has the exact-f32 CDE sampler only (include/dmip.h dmip_act)."""
    _lib.precision_code(precision)
    precision = canonical_precision(precision)
    if any(a != _lib.DMIP_ACT_TANH_TWICE_FIRST for a in acts):
        ok = mode == _lib.DMIP_SAMPLER_CDE and _lib.sampler_supported(width, n_hidden, xdim, ydim, mode, "fp32")
        return "fp32" if ok else None
    for prec in (precision,) + _MORE_ACCURATE[precision]:
        if _lib.sampler_supported(width, n_hidden, xdim, ydim, mode, prec):
            return prec
    return None


class BaseClassDiffusionModel:
    """models/diffusion.py:14-58."""

    def __init__(self, xdim, ydim):
        self.xdim = xdim
        self.ydim = ydim
        self.sde = None
        self.precision = default_precision()  # "fp32x3" | "fp32" | "fp16": arithmetic of the sampler's networks

    def __call__(self, *args, **kwargs):
        return self.forward(*args, **kwargs)

    # ----------------------------------------------------------------- sampling API
    def forward(self, y, num_samples=2000, num_steps=200, mean=0, std=1, precision=None):
        """Posterior samples for one observation y (ydim,): np.ndarray (num_samples, xdim) float32
        (models/diffusion.py:27-46). Under torch.distributed with world_size > 1 the chains are
        sharded over the ranks and every rank returns all num_samples (parallel.sample_sharded).
        `precision` overrides self.precision for this call."""
        from . import parallel
        # (sample_sharded's launch is guarded: the device status word was read after it, so an asynchronous kernel
        # failure has raised already rather than coming back as silent NaNs)
        x = parallel.sample_sharded(self, y, num_samples, num_steps, mean, std, precision=precision)
        return x.cpu().numpy()

    def sample_trajectory(self, y, num_samples=2000, num_steps=200, snapshot_every=10, mean=0, std=1, seed=None,
                          chain_offset=0, precision=None, corrector_steps=0, snr=0.16):
        """The fused sampler with trajectory snapshots (dmip_em_sample_snapshots): returns device tensors
        (x (n_y, num_samples, xdim), snaps (num_steps // snapshot_every, n_y, num_samples, xdim)), snaps[k]
        = the chains after step (k + 1) * snapshot_every of the loop of models/diffusion.py:27-46 (the
        reference returns only the final state). Same chains, RNG and sharding as sample_device."""
        if isinstance(self, PosteriorDiffusionEstimator):
            score = self.sde.a
            nets, mode = [score.prior_net, score.likelihood_net], _lib.DMIP_SAMPLER_POSTERIOR
        elif isinstance(self, (CDE, CDiffE)):
            nets = [self.sde.a]
            mode = _lib.DMIP_SAMPLER_CDIFFE if isinstance(self, CDiffE) else _lib.DMIP_SAMPLER_CDE
        else:
            raise NotImplementedError(f"{type(self).__name__}: no fused trajectory sampler")
        if corrector_steps and mode != _lib.DMIP_SAMPLER_CDIFFE:
            raise ValueError("corrector steps: CDiffE only")
        dev, ys, sde, out = self._prepare(y, num_samples, num_steps, nets)
        handles = [n.dmip_handle(dev, self.xdim) for n in nets]
        net, prior = handles[-1], (handles[0] if len(handles) > 1 else None)
        if prior is not None and (prior.width, prior.n_hidden) != (net.width, net.n_hidden):
            raise ValueError("prior and likelihood networks must have the same hidden layers")
        prec = _fused_precision(precision or self.precision, mode, net.width, net.n_hidden, self.xdim, self.ydim,
                                [h.act for h in handles])
        if prec is None:
            raise ValueError("no fused sampler for this network shape / activation")
        snaps = torch.empty(int(num_steps) // int(snapshot_every), ys.shape[0], int(num_samples), self.xdim,
                            device=dev, dtype=torch.float32)
        seed = _draw_seed() if seed is None else seed
        _lib.em_sample_snapshots(mode, net, prior, sde, ys, num_samples, chain_offset, num_steps, mean, std, seed,
                                 snapshot_every, snaps, out, corrector_steps, snr, prec)
        return out, snaps

    def _exec_device(self, y):
        if isinstance(y, torch.Tensor) and y.is_cuda:
            return y.device
        p = next(self.sde.a.parameters())
        if p.is_cuda:
            return p.device
        if torch.cuda.is_available():
            return torch.device('cuda', torch.cuda.current_device())
        raise RuntimeError("dmip: sampling needs a HIP device (the reverse-SDE sampler is a HIP kernel; "
                           "there is no CPU sampling path)")

    def _ys(self, y, dev):
        ys = torch.as_tensor(y).to(device=dev, dtype=torch.float32)
        return ys.reshape(-1, self.ydim).contiguous()

    def sample_device(self, y, num_samples, num_steps=200, mean=0, std=1, seed=None, chain_offset=0,
                      noise=None, precision=None):
        """Device-resident samples (n_y, num_samples, xdim) for ys (n_y, ydim) -- no host copy.
        `chain_offset` selects a shard of a larger run; `noise` injects standard normals
        (num_steps + 1, n_y, num_samples, xdim) (slot 0 -> x0) in place of the internal RNG;
        `precision` ("fp32x3" | "fp32" | "fp16") overrides self.precision."""
        raise NotImplementedError

    def _prepare(self, y, num_samples, num_steps, nets):
        dev = self._exec_device(y)
        ys = self._ys(y, dev)
        for net in nets:
            pdev = next(net.parameters()).device
            if pdev != dev:
                raise RuntimeError(f"dmip: score network is on {pdev}, y on {dev}")
        base = self.sde.base_sde
        if float(base.T) != float(self.sde.T):
            raise ValueError("PluginReverseSDE.T must equal the base SDE's T")
        out = torch.empty(ys.shape[0], int(num_samples), self.xdim, device=dev, dtype=torch.float32)
        return dev, ys, _lib.vpsde(base.beta_min, base.beta_max, self.sde.T), out

    def sample_t(self, x, eps=1e-4):
        """Training times (models/diffusion.py:48-58)."""
        if self.sde.debias:
            t_ = self.sde.base_sde.sample_debiasing_t([x.size(0), ] + [1 for _ in range(x.ndim - 1)]) + eps
            t_ = t_.to(x)
            t_[torch.where(t_ > self.sde.T)] -= eps
            t_.requires_grad = True
        else:
            t_ = eps + torch.rand([x.size(0), ] + [1 for _ in range(x.ndim - 1)], requires_grad=True).to(x) * self.sde.T
            t_[torch.where(t_ > self.sde.T)] = self.sde.T - eps
        return t_

    # ----------------------------------------------------------------- training API
    @staticmethod
    def _accumulate(logger_info, k, loss):
        if isinstance(loss, tuple):
            loss, info = loss
            for key, value in info.items():
                prev = logger_info.get(key, 0.0)
                logger_info[key] = prev * k / (k + 1) + value.item() / (k + 1)
        return loss

    def _train_loop(self, optimizer, epoch_data_loader, batch_loss):
        mean_loss = 0
        logger_info = {}
        for k, (x, y) in enumerate(epoch_data_loader()):
            out = batch_loss(x, y)
            if isinstance(out, _FusedStep):  # gradients already written by the fused kernel
                loss = self._accumulate(logger_info, k, (out.loss, out.info))
            else:
                loss = self._accumulate(logger_info, k, out)
                optimizer.zero_grad()
                loss.backward()
            if not (isinstance(out, _FusedStep) and out.stepped):
                optimizer.step()
            mean_loss = mean_loss * k / (k + 1) + loss / (k + 1)
        return mean_loss, logger_info


class CDE(BaseClassDiffusionModel):
    """Conditional diffusion estimator: score net a(x_t, y, t) (models/diffusion.py:60-105)."""

    def __init__(self, xdim, ydim, hidden_layers):
        super().__init__(xdim, ydim)
        score_net = MLP(xdim + ydim + 1, xdim, hidden_layers, nn.Tanh()).to(device)
        self.sde = sdes.PluginReverseSDE(sdes.VariancePreservingSDE(), score_net, T=1, debias=True)

    def sample_device(self, y, num_samples, num_steps=200, mean=0, std=1, seed=None, chain_offset=0,
                      noise=None, precision=None):
        net = self.sde.a
        dev, ys, sde, out = self._prepare(y, num_samples, num_steps, [net])
        handle = net.dmip_handle(dev, self.xdim)
        seed = _draw_seed() if seed is None else seed
        prec = _fused_precision(precision or self.precision, _lib.DMIP_SAMPLER_CDE, handle.width, handle.n_hidden,
                                self.xdim, self.ydim, [handle.act])
        if noise is not None:
            noise = noise.to(device=dev, dtype=torch.float32).contiguous()
            if tuple(noise.shape) != (int(num_steps) + 1, ys.shape[0], int(num_samples), self.xdim):
                raise ValueError("noise must have shape (num_steps+1, n_y, num_samples, xdim)")
        if prec is None:
            if noise is not None:
                raise ValueError("noise injection needs a fused CDE kernel for this shape")
            base = self.sde.base_sde

            def drift(x, y, tvec):
                return base.g(tvec, x) * self.sde.a(x, y, tvec) - base.f(tvec, x)

            return _em_device_loop(self, ys, int(num_samples), int(num_steps), mean, std, seed, chain_offset,
                                   drift, self.xdim, self.xdim)
        _lib.em_sample(handle, sde, ys, num_samples, chain_offset, num_steps, mean, std, seed, out, noise, prec)
        return out

    def train_epoch(self, optimizer, loss_fn, epoch_data_loader):
        from .training import DeviceTrainStep, _plain_adam, device_step_enabled, device_step_ok, fused_config, \
            fused_loss_grad, loss_info
        cfg = fused_config(self, loss_fn)
        # $DMIP_TRAIN_DEVICE_STEP=1: t, eps and Adam on the device too (training.DeviceTrainStep)
        dstep = DeviceTrainStep(self, loss_fn, optimizer) \
            if cfg is not None and device_step_enabled() and _plain_adam(optimizer) is not None \
            and device_step_ok(self) else None

        def batch_loss(x, y):
            if dstep is not None:
                return _FusedStep(*loss_info(cfg.kind, dstep(x, y)), stepped=True)
            t = self.sample_t(x)
            if cfg is not None:
                # same draws as base_sde.sample (sdes.py:37-49): eps = randn_like(x)
                eps = torch.randn_like(x)
                optimizer.zero_grad()
                return _FusedStep(*fused_loss_grad(self, loss_fn, cfg, x, y, t, eps))
            x_t, target, std, g = self.sde.base_sde.sample(t, x, return_noise=True)
            if loss_fn.name == 'DSMLoss':
                return loss_fn(self.sde.a(x_t, y, t) / g, std, target).mean()
            return loss_fn(self.sde, x, y, x_t, t, target, std, g)
        return self._train_loop(optimizer, epoch_data_loader, batch_loss)


_LOOP_STREAM = 1 << 62  # RNG stream ids of the per-step loop (disjoint from the fused kernels' y indices)


def _loop_normals(seed, chain_offset, stream_id, n, d, dev):
    """(n, d) normals of the kernels' chain-keyed generator for chains [chain_offset, chain_offset + n)."""
    out = torch.empty(n, 2 * ((d + 1) // 2), device=dev, dtype=torch.float32)
    _lib.rng_normals(seed, chain_offset, stream_id, n, (d + 1) // 2, out)
    return out[:, :d]


def _em_device_loop(model, ys, num_samples, num_steps, mean, std, seed, chain_offset, drift, zdim,
                    keep, y_resample=None):
    """Reverse-SDE EM loop on device tensors for shapes without a compiled fused sampler: the
    network evaluations are dmip_mlp_forward launches in the networks' own forward precision
    (nets.MLP.dmip_precision, exact f32 unless set otherwise), the update follows
    models/diffusion.py:40-42 (same rounding order as the fused kernel). Noise comes from the
    kernels' counter-keyed generator, keyed by (seed, global chain index, stream = (y index, step)),
    so a shard of a run draws exactly the chains of the full run (bit-identical union)."""
    dev = ys.device
    base = model.sde.base_sde
    T = float(model.sde.T)
    n_y = ys.shape[0]
    outs = []
    ts = torch.linspace(0, 1, num_steps + 1) * T
    delta = T / num_steps
    off = int(chain_offset)
    with torch.no_grad():
        for k in range(n_y):
            y = ys[k]
            sid = _LOOP_STREAM + (k << 40)
            x = _loop_normals(seed, off, sid, num_samples, zdim, dev) * std + mean
            for i in range(num_steps):
                tau = (T - ts[i]).item()
                tvec = torch.full((num_samples, 1), tau, device=dev)
                eps_y = None
                if y_resample is not None:
                    eps_y = _loop_normals(seed, off, sid + (1 << 39) + i, num_samples, model.ydim, dev)
                z_in = x if y_resample is None else y_resample(x, y, tau, eps_y)
                mu = drift(z_in, y, tvec)
                sigma = base.g(tvec, z_in)
                xi = _loop_normals(seed, off, sid + 1 + i, num_samples, z_in.shape[1], dev)
                z = z_in + delta * mu + delta ** 0.5 * sigma * xi
                x = z[:, :keep] if keep < z.shape[1] else z
            outs.append(x[:, :keep])
    return torch.stack(outs)


class CDiffE(BaseClassDiffusionModel):
    """Conditional diffusion over the joint z = (x, y) (models/diffusion.py:109-180).

    The reference sampler (models/diffusion.py:158-180) raises TypeError (`sde.mu` without `cond`).
    Repaired semantics, consistent with its training (models/diffusion.py:129-137): each step
    re-diffuses the observation, y_t ~ q(y_t | y) at forward time T - t_i, evaluates the joint score
    net a(x_t, y_t, T - t_i) (output xdim + ydim), takes the EM step on z_t = [x_t, y_t] and keeps x.
    """

    def __init__(self, xdim, ydim, hidden_layers):
        super().__init__(xdim, ydim)
        score_net = MLP(xdim + ydim + 1, xdim + ydim, hidden_layers, nn.Tanh()).to(device)
        self.sde = sdes.PluginReverseSDE(sdes.VariancePreservingSDE(), score_net, T=1, debias=True)

    def forward(self, y, num_samples=2000, num_steps=200, mean=0, std=1, corrector_steps=0, snr=0.16,
                precision=None):
        """As BaseClassDiffusionModel.forward; `corrector_steps` > 0 adds Langevin corrector steps
        before every predictor step (predictor-corrector sampling, BASELINE config 3; see
        dmip_em_sample_cdiffe in include/dmip.h for the definition). The step size takes the norms at
        their expected values, eps = 2 alpha snr^2 var(T - t): `snr` is not score_sde's measured-norm snr
        (that one measures |s| on the batch; for a trained score with |s| != sqrt(d)/std the same value
        gives a different step)."""
        from . import parallel
        x = parallel.sample_sharded(self, y, num_samples, num_steps, mean, std,
                                    corrector_steps=corrector_steps, snr=snr, precision=precision)
        return x.cpu().numpy()  # (the guarded launch read the device status word)

    def sample_device(self, y, num_samples, num_steps=200, mean=0, std=1, seed=None, chain_offset=0,
                      noise=None, corrector_steps=0, snr=0.16, precision=None):
        if noise is not None:
            raise ValueError("noise injection is only implemented for the fused CDE sampler")
        net = self.sde.a
        dev, ys, sde, out = self._prepare(y, num_samples, num_steps, [net])
        seed = _draw_seed() if seed is None else seed
        handle = net.dmip_handle(dev, self.xdim)
        prec = _fused_precision(precision or self.precision, _lib.DMIP_SAMPLER_CDIFFE, handle.width,
                                handle.n_hidden, self.xdim, self.ydim, [handle.act])
        if prec is not None:
            _lib.em_sample_cdiffe(handle, sde, ys, num_samples, chain_offset, num_steps, mean, std, seed, out,
                                  corrector_steps, snr, prec)
            return out
        if corrector_steps:
            raise ValueError("the predictor-corrector sampler needs a compiled fused CDiffE kernel for this shape")
        base = self.sde.base_sde
        xd = self.xdim

        def y_resample(x, y, tau, eps):
            tt = torch.full((x.shape[0], 1), tau, device=x.device)
            y_t = base.mean_weight(tt) * y + base.var(tt) ** 0.5 * eps
            return torch.cat([x[:, :xd], y_t], dim=1)

        def drift(z, y, tvec):
            a = self.sde.a(z[:, :xd].contiguous(), z[:, xd:].contiguous(), tvec)
            return base.g(tvec, z) * a - base.f(tvec, z)

        return _em_device_loop(self, ys, int(num_samples), int(num_steps), mean, std, seed, chain_offset,
                               drift, xd, xd, y_resample)

    def train_epoch(self, optimizer, loss_fn, epoch_data_loader):
        """models/diffusion.py:123-156. On a HIP device DSMLoss on the joint z = (x, y) runs through the
        exact-f32 fused loss + gradient engine (training.joint_fused_config); otherwise autograd."""
        from .training import fused_loss_grad, joint_fused_config
        cfg = joint_fused_config(self, loss_fn)

        def batch_loss(x, y):
            z = torch.concat([x, y], dim=1)
            t = self.sample_t(z)
            if cfg is not None:
                eps = torch.randn_like(z)  # base_sde.sample's draw (sdes.py:37-49)
                optimizer.zero_grad()
                return _FusedStep(*fused_loss_grad(self, loss_fn, cfg, z, None, t, eps))
            diffused, target, std, g = self.sde.base_sde.sample(t, z, return_noise=True)
            x_t, y_t = diffused[:, :self.xdim], diffused[:, self.xdim:]
            if loss_fn.name == 'DSMLoss':
                return loss_fn(self.sde.a(x_t, y_t, t) / g, std, target).mean()
            return loss_fn(self.sde, x, y, diffused, t, target, std, g)
        return self._train_loop(optimizer, epoch_data_loader, batch_loss)


class PosteriorDiffusionEstimator(BaseClassDiffusionModel):
    """Prior score + likelihood score, score = g (prior(x,t) + lik(x,y,t)) (models/diffusion.py:182-229)."""

    def __init__(self, xdim, ydim, hidden_layers):
        super().__init__(xdim, ydim)
        forward_process = sdes.VariancePreservingSDE()
        prior_net = MLP2(xdim + 1, xdim, hidden_layers, nn.Tanh()).to(device)
        likelihood_net = MLP(xdim + ydim + 1, xdim, hidden_layers, nn.Tanh()).to(device)
        score_net = PosteriorScore(prior_net, likelihood_net, forward_process)
        self.sde = sdes.PluginReverseSDE(forward_process, score_net, T=1, debias=True)
        self.loss_fn = PosteriorLoss

    def sample_device(self, y, num_samples, num_steps=200, mean=0, std=1, seed=None, chain_offset=0,
                      noise=None, precision=None):
        if noise is not None:
            raise ValueError("noise injection is only implemented for the fused CDE sampler")
        score = self.sde.a
        dev, ys, sde, out = self._prepare(y, num_samples, num_steps, [score.prior_net, score.likelihood_net])
        seed = _draw_seed() if seed is None else seed
        prior = score.prior_net.dmip_handle(dev, self.xdim)
        lik = score.likelihood_net.dmip_handle(dev, self.xdim)
        prec = None
        if (prior.width, prior.n_hidden) == (lik.width, lik.n_hidden):
            prec = _fused_precision(precision or self.precision, _lib.DMIP_SAMPLER_POSTERIOR, lik.width,
                                    lik.n_hidden, self.xdim, self.ydim, [prior.act, lik.act])
        if prec is not None:
            _lib.em_sample_posterior(prior, lik, sde, ys, num_samples, chain_offset, num_steps, mean, std, seed,
                                     out, prec)
            return out
        base = self.sde.base_sde

        def drift(x, y, tvec):
            return base.g(tvec, x) * self.sde.a(x, y, tvec) - base.f(tvec, x)

        return _em_device_loop(self, ys, int(num_samples), int(num_steps), mean, std, seed, chain_offset,
                               drift, self.xdim, self.xdim)

    def train_epoch(self, optimizer, loss_fn, epoch_data_loader):
        """models/diffusion.py:204-229. On a HIP device with PosteriorLoss on the scatterometry surrogate,
        each batch's loss and both networks' gradients come from dmip_posterior_loss_grad (exact f32,
        training.posterior_loss_grad); otherwise the autograd graph of losses.PosteriorLoss."""
        from .training import posterior_fused_ok, posterior_loss_grad
        fused = posterior_fused_ok(self, loss_fn)

        def batch_loss(x, y):
            t = self.sample_t(x)
            if fused:
                eps = torch.randn_like(x)  # base_sde.sample's draw (sdes.py:37-49)
                optimizer.zero_grad()
                return _FusedStep(*posterior_loss_grad(self, loss_fn, x, y, t, eps))
            return loss_fn(self.sde, x, y, t)
        return self._train_loop(optimizer, epoch_data_loader, batch_loss)


class _PriorDrift(nn.Module):
    """a(x, y, t) = g(t) prior(x, t): the unconditional drift of a prior score network (the prior half of
    PosteriorScore, nets.py:155-157); y is ignored."""

    def __init__(self, prior_net, forward_process):
        super().__init__()
        self.prior_net = prior_net
        self.forward_sde = forward_process

    def forward(self, x, y, t):
        return self.forward_sde.g(t, x) * self.prior_net(x, t)


class DPS(BaseClassDiffusionModel):
    """Diffusion posterior sampling (Chung et al. 2023; BASELINE config 4) for the scatterometry problem:
    a prior score network MLP2(x, t) (the PosteriorDiffusionEstimator's prior, trained with DSM as
    PosteriorLoss trains it, losses.py:373-377) guided at every EM step by the gradient of the
    measurement likelihood through the surrogate forward model at the Tweedie estimate
    x0_hat = (x + var s) / mean_weight -- the quantity PosteriorLoss.likelihood_target (losses.py:349-371)
    trains the reference's likelihood network towards, here computed exactly on the fly.
    Fused kernel: dmip_dps_sample_ex (include/dmip.h), one launch for all steps: fp32x3 by default (the split-fp16
    engine, J^T by a reverse pass through the prior), exact f32 with precision="fp32".

    forward_model: the surrogate nn.Sequential (load_forward_model); params: {'a', 'b', 'lambd_bd'};
    guidance: 'norm' (default; Chung et al.'s zeta / ||y - F(x0_hat)|| step on ||y - F(x0_hat)||^2) or 'nll'
    (score + zeta grad log p(y | x0_hat), the reference PosteriorLoss target; unstable for zeta >~ 0.01 on
    scatterometry because of the 1/mean_weight amplification at large diffusion times). Measured quality
    against the fused MH ground truth: DESIGN.md §4c."""

    def __init__(self, xdim, ydim, hidden_layers, forward_model=None, params=None, zeta=0.005, guidance='norm'):
        super().__init__(xdim, ydim)
        forward_process = sdes.VariancePreservingSDE()
        prior_net = MLP2(xdim + 1, xdim, hidden_layers, nn.Tanh()).to(device)
        self.sde = sdes.PluginReverseSDE(forward_process, _PriorDrift(prior_net, forward_process), T=1, debias=True)
        self.forward_model = forward_model
        self.params = dict(params or {'a': 0.2, 'b': 0.01, 'lambd_bd': 1000})
        self.zeta = float(zeta)
        if guidance not in ('nll', 'norm'):
            raise ValueError("guidance must be 'nll' or 'norm'")
        self.guidance = guidance

    @property
    def prior_net(self):
        return self.sde.a.prior_net

    @classmethod
    def from_posterior(cls, model, forward_model, params=None, zeta=0.005, guidance='norm'):
        """A DPS sampler on the prior network of a trained PosteriorDiffusionEstimator."""
        pn = model.sde.a.prior_net
        m = cls(model.xdim, model.ydim, pn.hidden_layers, forward_model, params, zeta, guidance)
        m.sde.a.prior_net.load_state_dict(pn.state_dict())
        m.sde.a.prior_net.to(next(pn.parameters()).device)
        return m

    def sample_device(self, y, num_samples, num_steps=200, mean=0, std=1, seed=None, chain_offset=0, noise=None,
                      precision=None):
        """dmip_dps_sample_ex at `precision` (default self.precision): "fp32x3" (the reference's fp32 accuracy at
        the fp16 matrix rate, dmip_dps_x3.hip; also what "fp16" runs: there is no 16-bit DPS) or "fp32" (exact f32,
        forward tangents). At the default precision a chain outside fp16's range resamples in exact f32
        (parallel.sample_checked)."""
        if noise is not None:
            raise ValueError("noise injection is only implemented for the fused CDE sampler")
        from .problems import surrogate_handle
        pn = self.sde.a.prior_net
        dev, ys, sde, out = self._prepare(y, num_samples, num_steps, [pn])
        if self.forward_model is None:
            raise ValueError("DPS needs the forward model (load_forward_model) for its guidance")
        sur = surrogate_handle(self.forward_model, dev)
        if sur is None:
            raise ValueError("DPS: forward_model is not the scatterometry surrogate shape (3 -> 256^3 -> 23)")
        seed = _draw_seed() if seed is None else seed
        prior = pn.dmip_handle(dev, self.xdim)
        p = self.params
        prec = canonical_precision(precision or self.precision)
        _lib.dps_sample(prior, sur, _lib.scat_noise(p['a'], p['b'], p['lambd_bd']), sde, ys, num_samples,
                        chain_offset, num_steps, mean, std, seed,
                        _lib.DMIP_DPS_NLL if self.guidance == 'nll' else _lib.DMIP_DPS_NORM, self.zeta, out,
                        precision="fp32" if prec == "fp32" else "fp32x3")
        return out

    def train_epoch(self, optimizer, loss_fn, epoch_data_loader):
        """Prior DSM epoch (the prior half of PosteriorLoss, losses.py:373-377): score = prior(x_t, t)."""
        def batch_loss(x, y):
            t = self.sample_t(x)
            x_t, target, std, g = self.sde.base_sde.sample(t, x, return_noise=True)
            return loss_fn(self.sde.a.prior_net(x_t, t), std, target).mean()
        return self._train_loop(optimizer, epoch_data_loader, batch_loss)
