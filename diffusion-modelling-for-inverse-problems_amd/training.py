"""Fused training step on the HIP device (§8a A6, A13-A18).

`fused_loss_grad(model, loss_fn, cfg, x, y, t, eps)` computes the loss value, its components and the
parameter gradients of DSMLoss / DSM_PDELoss / PINNLoss / PINNLoss2 (losses.py:42-290 with the
ScoreFPE or conditional ScoreFPE residual), writing the gradients into the parameters' `.grad` (set,
not accumulated). Two device paths:
  * "fp32" (default): dmip_loss_grad_f32 -- exact f32 at any width (the reference configs' [512]*3
    included) and any initial-condition target (the linear problem's analytic score, the
    scatterometry -energy_grad, ...): forward-mode jets as stacked-stream MFMA GEMMs;
  * "bf16": dmip_loss_grad -- the persistent bf16-MFMA kernel of BASELINE config 5 (the linear
    problem's width-64 CDE with its analytic IC target), selected with $DMIP_TRAIN_PRECISION=bf16.
It is what CDE.train_epoch runs on a HIP device when `fused_config` accepts the network and loss;
CDiffE.train_epoch runs its DSMLoss (the only loss the reference's joint training accepts) through the
same f32 engine on z = (x, y) (`joint_fused_config`); everything else (CPU tensors, other shapes)
takes the autograd path of losses.py.
"""
import os

import torch

from . import _lib
from .losses import DSMLoss, DSM_PDELoss, PINNLoss, PINNLoss2, ScoreFPELoss
from .problems import LinearForwardProblem


def _metric(m):
    return _lib.DMIP_METRIC_L1 if m == 'L1' else _lib.DMIP_METRIC_L2


def train_precision():
    return os.environ.get("DMIP_TRAIN_PRECISION", "fp32")


def _linear_ic(loss_fn):
    prob = getattr(loss_fn.initial_condition, "__self__", None)
    if isinstance(prob, LinearForwardProblem) and \
            getattr(loss_fn.initial_condition, "__func__", None) is LinearForwardProblem.score_posterior:
        return prob
    return None


def _tanh_chain(net):
    """The fused loss + gradient engines differentiate the reference's tanh chain only (their jets hold tanh
    derivatives): a network with another activation (nets.MLP dmip_act) trains through autograd."""
    return getattr(net, "dmip_act", None) == _lib.DMIP_ACT_TANH_TWICE_FIRST


def fused_config(model, loss_fn):
    """dmip_loss_cfg for (model, loss_fn), or None when no fused path covers them."""
    if os.environ.get("DMIP_TRAIN_FUSED", "1") == "0":
        return None
    net = model.sde.a
    if not hasattr(net, "linear_layers") or not _tanh_chain(net):
        return None
    layers = net.linear_layers()
    p0 = layers[0][0]
    if not p0.is_cuda or p0.dtype != torch.float32:
        return None
    if net.output_dim != model.xdim or model.xdim > 4 or len(layers) - 1 > 8:  # CDE only (CDiffE trains on z)
        return None
    cfg = _lib.DmipLossCfg()
    if type(loss_fn) is DSMLoss:
        cfg.kind, cfg.pde = _lib.DMIP_LOSS_DSM, _lib.DMIP_PDE_NONE
        return cfg
    kinds = {DSM_PDELoss: _lib.DMIP_LOSS_DSM_PDE, PINNLoss: _lib.DMIP_LOSS_PINN, PINNLoss2: _lib.DMIP_LOSS_PINN2}
    if type(loss_fn) not in kinds:
        return None
    cfg.kind = kinds[type(loss_fn)]
    cfg.pde = _lib.DMIP_PDE_FPE if isinstance(loss_fn.pde_loss, ScoreFPELoss) else _lib.DMIP_PDE_CFPE
    cfg.pde_metric = _metric(loss_fn.pde_loss.metric)
    cfg.lam = float(loss_fn.lam)
    if cfg.kind in (_lib.DMIP_LOSS_PINN, _lib.DMIP_LOSS_PINN2):
        cfg.ic_metric = _metric(loss_fn.ic_metric)
        cfg.lam2 = float(loss_fn.lam2)
        prob = _linear_ic(loss_fn)
        if prob is not None:
            cfg.ic_A[:] = [float(v) for v in prob.A.reshape(-1)]
            cfg.ic_b[:] = [float(v) for v in prob.b.reshape(-1)]
            cfg.ic_Sinv[:] = [float(v) for v in prob.Sigma_inv.reshape(-1)]
        elif not callable(loss_fn.initial_condition):
            return None
    return cfg


def joint_fused_config(model, loss_fn):
    """dmip_loss_cfg for CDiffE's joint training (models/diffusion.py:123-156), or None. The reference
    trains CDiffE with DSMLoss only: its other losses call sde.a(x_t, y, t) with the joint x_t and fail
    on the input width. DSM on z = (x, y) is the engine's DSM with state z and no condition (ydim 0)."""
    if os.environ.get("DMIP_TRAIN_FUSED", "1") == "0" or type(loss_fn) is not DSMLoss:
        return None
    net = model.sde.a
    if not hasattr(net, "linear_layers") or not _tanh_chain(net):
        return None
    layers = net.linear_layers()
    p0 = layers[0][0]
    zdim = model.xdim + model.ydim
    if not p0.is_cuda or p0.dtype != torch.float32 or net.output_dim != zdim or net.input_dim != zdim + 1 \
            or zdim > 64 or len(layers) - 1 > 8:
        return None
    cfg = _lib.DmipLossCfg()
    cfg.kind, cfg.pde = _lib.DMIP_LOSS_DSM, _lib.DMIP_PDE_NONE
    return cfg


def fused_loss_grad(model, loss_fn, cfg, x, y, t, eps, precision=None):
    """One fused loss + gradient evaluation. Returns (loss, info) like the reference loss objects:
    a 0-d tensor and {component name: 0-d tensor}. precision: "fp32" (dmip_loss_grad_f32, default) or
    "bf16" (dmip_loss_grad, where compiled: the linear problem's width-64 CDE, analytic IC).
    y=None: joint training (CDiffE), x is the state z = (x, y) and the network has no condition input."""
    net = model.sde.a
    layers = [(w.detach(), b.detach()) for w, b in net.linear_layers()]
    dev = layers[0][0].device
    f32 = dict(device=dev, dtype=torch.float32)
    x = x.detach().to(**f32).contiguous()
    if y is None:  # ydim 0: the pointer is never read
        t = t.detach().to(**f32).reshape(-1).contiguous()
        eps = eps.detach().to(**f32).contiguous()
        params = list(net.parameters())
        flat = torch.empty(sum(p.numel() for p in params), **f32)
        out = torch.empty(4, **f32)
        base = model.sde.base_sde
        sde = _lib.vpsde(base.beta_min, base.beta_max, 1.0)
        _lib.loss_grad_f32(layers, net.input_dim, net.output_dim, x.shape[1], sde, cfg, x, x, t, eps, flat, out)
        _set_grads(params, flat)
        return loss_info(cfg.kind, out)
    y = y.detach().to(**f32).contiguous()
    t = t.detach().to(**f32).reshape(-1).contiguous()
    eps = eps.detach().to(**f32).contiguous()
    params = list(net.parameters())
    flat = torch.empty(sum(p.numel() for p in params), **f32)
    out = torch.empty(4, **f32)
    base = model.sde.base_sde
    sde = _lib.vpsde(base.beta_min, base.beta_max, 1.0)
    has_ic = cfg.kind in (_lib.DMIP_LOSS_PINN, _lib.DMIP_LOSS_PINN2)
    precision = precision or train_precision()
    widths = [int(w.shape[0]) for w, _ in layers[:-1]]
    bf16_ok = _lib.loss_grad_supported(net.input_dim, net.output_dim, widths, model.xdim) and \
        (not has_ic or _linear_ic(loss_fn) is not None)
    if precision == "bf16" and bf16_ok:
        _lib.loss_grad(layers, net.input_dim, net.output_dim, model.xdim, sde, cfg, x, y, t, eps, flat, out)
    else:
        ic = None
        if has_ic and _linear_ic(loss_fn) is None:
            # the reference's initial_condition(x, y) is a constant target (losses.py:223-226)
            with torch.enable_grad():
                ic = loss_fn.initial_condition(x, y)
            ic = ic.detach().to(**f32)[:, :model.xdim].contiguous()
        _lib.loss_grad_f32(layers, net.input_dim, net.output_dim, model.xdim, sde, cfg, x, y, t, eps, flat, out, ic)
    _set_grads(params, flat)
    return loss_info(cfg.kind, out)


def _set_grads(params, flat):
    off = 0
    for p in params:
        p.grad = flat[off:off + p.numel()].view_as(p)
        off += p.numel()


def loss_info(kind, out):
    """(loss, {component: value}) from the [4] loss tensor (loss, PDE, IC, DSM), keyed like the
    reference's loss objects."""
    loss, pde, ic, dsm = out[0], out[1], out[2], out[3]
    if kind == _lib.DMIP_LOSS_DSM:
        return loss, {}
    if kind == _lib.DMIP_LOSS_DSM_PDE:
        return loss, {'PDE-Loss': pde, 'DSM-Loss': dsm}
    if kind == _lib.DMIP_LOSS_PINN:
        return loss, {'PDE-Loss': pde, 'Initial Condition': ic, 'DSM-Loss': dsm}
    return loss, {'PDE-Loss': pde, 'Initial Condition': ic, 'DSM_eval': dsm}


# ------------------------------------------------------------- the whole step on the device
def _plain_adam(optimizer):
    """torch.optim.Adam with the options dmip_adam_step implements (amsgrad off, no weight decay,
    not maximizing), else None."""
    if type(optimizer) is not torch.optim.Adam or len(optimizer.param_groups) != 1:
        return None
    g = optimizer.param_groups[0]
    if g.get("amsgrad") or g.get("weight_decay", 0) != 0 or g.get("maximize") or g.get("differentiable") \
            or g.get("fused") or g.get("capturable"):
        return None
    return optimizer


def device_step_enabled():
    return os.environ.get("DMIP_TRAIN_DEVICE_STEP", "0") == "1"


def graph_step_enabled():
    return os.environ.get("DMIP_TRAIN_GRAPH", "1") != "0"


class _TrainPlan:
    """Owns a dmip_train_plan: one captured hipGraph of a DeviceTrainStep at a fixed batch size."""

    def __init__(self, ds, B):
        import ctypes
        self.lib, self.B = ds.lib, B
        f32 = dict(device=ds.dev, dtype=torch.float32)
        self.t = torch.empty(B, **f32)
        self.eps = torch.empty(B, ds.model.xdim, **f32)
        self.out = torch.empty(4, **f32)
        g0 = ds.opt.param_groups[0]
        b1, b2 = g0["betas"]
        d = _lib.DmipTrainPlanDesc()
        d.in_dim, d.out_dim, d.n_hidden = ds.net.input_dim, ds.net.output_dim, ds.L
        d.widths = ctypes.cast(ds.widths, ctypes.c_void_p)
        d.xdim = ds.model.xdim
        d.weights_dev, d.biases_dev = ctypes.cast(ds.wp, ctypes.c_void_p), ctypes.cast(ds.bp, ctypes.c_void_p)
        d.sde, d.cfg = ds.sde, ds.cfg
        d.precision = _lib.DMIP_PREC_BF16 if ds.bf16 else _lib.DMIP_PREC_F32
        d.batch, d.seed, d.first_draw = B, ds.seed, 0
        d.debias, d.t_epsilon, d.t_add = int(ds.debias), ds.t_eps, 1e-4
        d.n_tensors = ds.n
        d.params, d.grads = ctypes.cast(ds.a_p, ctypes.c_void_p), ctypes.cast(ds.a_g, ctypes.c_void_p)
        d.exp_avg, d.exp_avg_sq = ctypes.cast(ds.a_m, ctypes.c_void_p), ctypes.cast(ds.a_v, ctypes.c_void_p)
        d.numel = ctypes.cast(ds.a_n, ctypes.c_void_p)
        d.lr, d.beta1, d.beta2, d.eps = float(g0["lr"]), float(b1), float(b2), float(g0["eps"])
        d.step0 = 0
        d.t_dev, d.eps_dev, d.loss_dev = self.t.data_ptr(), self.eps.data_ptr(), self.out.data_ptr()
        self.hyper = (d.lr, d.beta1, d.beta2, d.eps)
        h = ctypes.c_void_p()
        with torch.cuda.device(ds.dev):  # the plan's buffers and capture stream on the parameters' device
            _lib.check(self.lib.dmip_train_plan_create(ctypes.byref(d), ctypes.byref(h)))
        self.h = h
        self.k, self.step = None, None  # the device counters' values (unknown until set)

    def __del__(self):
        h, self.h = getattr(self, "h", None), None
        if h:
            try:
                self.lib.dmip_train_plan_destroy(h)
            except Exception:  # noqa: BLE001 -- interpreter shutdown: the runtime may already be gone
                pass


ADAM_MAX_TENSORS = 16  # dmip_adam_step / dmip_train_plan (csrc dmip_internal.h kAdamMaxTensors)


def device_step_ok(model):
    """The whole-step device path handles this network (at most ADAM_MAX_TENSORS parameter tensors, i.e. up
    to 7 hidden layers); otherwise train_epoch keeps the fused loss + torch Adam path."""
    return len(list(model.sde.a.parameters())) <= ADAM_MAX_TENSORS


class DeviceTrainStep:
    """One CDE training step with no host work between launches (verdict r1 item 4): the batch's t and
    eps (dmip_train_draws: sample_t's debiased sampler and base_sde.sample's noise, from the chain-keyed
    generator), the fused loss + gradients (dmip_loss_grad_f32, or the bf16 kernel), and Adam on the
    optimizer's own state (dmip_adam_step) -- pointers, buffers and ctypes arrays built once.
    Opt-in ($DMIP_TRAIN_DEVICE_STEP=1 in CDE.train_epoch, or directly): its t / eps come from the
    device generator (seeded from torch's), not from torch's global stream as in the reference."""

    def __init__(self, model, loss_fn, optimizer, precision=None):
        import ctypes
        self.model, self.loss_fn, self.opt = model, loss_fn, _plain_adam(optimizer)
        if self.opt is None:
            raise ValueError("DeviceTrainStep needs a plain torch.optim.Adam")
        self.cfg = fused_config(model, loss_fn)
        if self.cfg is None:
            raise ValueError("no fused loss path for this network / loss")
        net = model.sde.a
        self.params = list(net.parameters())
        if len(self.params) > ADAM_MAX_TENSORS:
            raise ValueError(f"DeviceTrainStep: dmip_adam_step takes at most {ADAM_MAX_TENSORS} parameter tensors "
                             f"(this network has {len(self.params)})")
        if {id(p) for p in self.opt.param_groups[0]["params"]} != {id(p) for p in self.params}:
            raise ValueError("DeviceTrainStep: the optimizer must hold exactly the score network's parameters")
        p0 = self.params[0]
        self.dev = p0.device
        f32 = dict(device=self.dev, dtype=torch.float32)
        self.cap = 0
        self.flat = torch.empty(sum(p.numel() for p in self.params), **f32)
        self.out = torch.empty(4, **f32)
        off, self.grads = 0, []
        for p in self.params:
            self.grads.append(self.flat[off:off + p.numel()].view_as(p))
            off += p.numel()
        for p, g in zip(self.params, self.grads):
            p.grad = g
            st = self.opt.state[p]
            if len(st) == 0:  # torch.optim.Adam's lazy state (step on the host, moments like the param)
                st["step"] = torch.tensor(0.0, dtype=torch.float32)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        layers = net.linear_layers()
        L = len(layers) - 1
        self.L = L
        self.widths = (_lib._i32 * L)(*[int(layers[i][0].shape[0]) for i in range(L)])
        self.wp = (ctypes.c_void_p * (L + 1))(*[w.data_ptr() for w, _ in layers])
        self.bp = (ctypes.c_void_p * (L + 1))(*[b.data_ptr() for _, b in layers])
        base = model.sde.base_sde
        self.sde = _lib.vpsde(base.beta_min, base.beta_max, 1.0)
        self.t_eps = float(getattr(base, "t_epsilon", 1e-3))
        self.debias = bool(model.sde.debias)
        widths = [int(w.shape[0]) for w, _ in layers[:-1]]
        has_ic = self.cfg.kind in (_lib.DMIP_LOSS_PINN, _lib.DMIP_LOSS_PINN2)
        prec = precision or train_precision()
        self.bf16 = prec == "bf16" and _lib.loss_grad_supported(net.input_dim, net.output_dim, widths, model.xdim) \
            and (not has_ic or _linear_ic(loss_fn) is not None)
        self.ic_fn = loss_fn.initial_condition if has_ic and _linear_ic(loss_fn) is None else None
        n = len(self.params)
        vp = lambda ts: (ctypes.c_void_p * n)(*[x.data_ptr() for x in ts])
        self.a_p = vp(self.params)
        self.a_g = vp(self.grads)
        self.a_m = vp([self.opt.state[p]["exp_avg"] for p in self.params])
        self.a_v = vp([self.opt.state[p]["exp_avg_sq"] for p in self.params])
        self.a_n = (_lib._i64 * n)(*[p.numel() for p in self.params])
        self.n = n
        self.seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self.k = 0
        self.ptr = _lib.ptr
        self.stream = _lib.stream_of(self.dev)
        self.lib = _lib.lib()
        self.net = net
        # whole step as one captured graph per batch size (dmip_train_plan; $DMIP_TRAIN_GRAPH=0 disables),
        # for the built-in initial condition (a Python initial_condition callable cannot be captured)
        self.graph = graph_step_enabled() and self.ic_fn is None and hasattr(self.lib, "dmip_train_plan_create")
        self.plans = {}

    def __call__(self, x, y):
        """One step on a batch (x, y) (device fp32): returns the [4] loss tensor (loss, PDE, IC, DSM)
        without synchronising; the parameters and the optimizer state are updated in place. Runs with the
        parameters' device current (the launches and the captured plan belong to it)."""
        with torch.cuda.device(self.dev):
            return self._step(x, y)

    def _step(self, x, y):
        import ctypes
        L, P, lib = self.L, self.ptr, self.lib
        B = int(x.shape[0])
        if self.graph:
            return self._graph_step(x, y, B)
        if B > self.cap:
            f32 = dict(device=self.dev, dtype=torch.float32)
            self.cap = B
            self._t = torch.empty(B, **f32)
            self._eps = torch.empty(B, self.model.xdim, **f32)
        self.t, self.eps = self._t[:B], self._eps[:B]
        x = x.detach().to(device=self.dev, dtype=torch.float32).contiguous()
        y = y.detach().to(device=self.dev, dtype=torch.float32).contiguous()
        _lib.check(lib.dmip_train_draws(ctypes.c_uint64(self.seed), ctypes.c_uint64(self.k), B, self.model.xdim,
                                        int(self.debias), ctypes.byref(self.sde), self.t_eps, 1e-4, P(self.t),
                                        P(self.eps), self.stream))
        self.k += 1
        if self.bf16:
            _lib.calls["loss_grad"] += 1
            _lib.check(lib.dmip_loss_grad(self.net.input_dim, self.net.output_dim, L, self.widths, self.model.xdim,
                                          self.wp, self.bp, ctypes.byref(self.sde), ctypes.byref(self.cfg), P(x), P(y),
                                          P(self.t), P(self.eps), B, P(self.flat), P(self.out), self.stream))
        else:
            ic = None
            if self.ic_fn is not None:
                with torch.enable_grad():
                    ic = self.ic_fn(x.clone(), y).detach()[:, :self.model.xdim].contiguous()
            _lib.calls["loss_grad_f32"] = _lib.calls.get("loss_grad_f32", 0) + 1
            _lib.check(lib.dmip_loss_grad_f32(self.net.input_dim, self.net.output_dim, L, self.widths,
                                              self.model.xdim, self.wp, self.bp, ctypes.byref(self.sde),
                                              ctypes.byref(self.cfg), P(x), P(y), P(self.t), P(self.eps), P(ic),
                                              B, P(self.flat), P(self.out), self.stream))
        # Adam: torch increments each parameter's step before its update
        g0 = self.opt.param_groups[0]
        step = None
        for p in self.params:
            st = self.opt.state[p]["step"]
            st += 1
            step = int(st.item()) if step is None else step
        b1, b2 = g0["betas"]
        _lib.check(lib.dmip_adam_step(self.n, self.a_p, self.a_g, self.a_m, self.a_v, self.a_n, float(g0["lr"]),
                                      float(b1), float(b2), float(g0["eps"]), step, self.stream))
        return self.out

    def _graph_step(self, x, y, B):
        """The same step as one hipGraphLaunch of the batch size's captured plan (draw stream id and Adam
        step from the plan's device counters, re-set only when they drift from this object's)."""
        plan = self.plans.get(B)
        g0 = self.opt.param_groups[0]
        hyper = (float(g0["lr"]), float(g0["betas"][0]), float(g0["betas"][1]), float(g0["eps"]))
        if plan is None or plan.hyper != hyper:  # (a changed lr is baked into the graph: recapture)
            plan = self.plans[B] = _TrainPlan(self, B)
        step = None
        for p in self.params:
            st = self.opt.state[p]["step"]
            step = int(st.item()) if step is None else step
            st += 1
        if (plan.k, plan.step) != (self.k, step):
            _lib.check(self.lib.dmip_train_plan_set_counters(plan.h, self.k, step, self.stream))
        x = x.detach().to(device=self.dev, dtype=torch.float32).contiguous()
        y = y.detach().to(device=self.dev, dtype=torch.float32).contiguous()
        _lib.calls["train_plan_step"] = _lib.calls.get("train_plan_step", 0) + 1
        _lib.check(self.lib.dmip_train_plan_step(plan.h, self.ptr(x), self.ptr(y), self.stream))
        self.k += 1
        plan.k, plan.step = self.k, step + 1
        self.t, self.eps = plan.t, plan.eps
        return plan.out


# ------------------------------------------------------------------ training drivers
class _Log:
    """torch SummaryWriter when tensorboard is installed, else JSON lines in log_dir/train_log.jsonl
    (same scalar tags: 'Train/Loss', 'Train/<component>')."""

    def __init__(self, log_dir):
        self.w, self.f = None, None
        try:
            from torch.utils.tensorboard import SummaryWriter
            self.w = SummaryWriter(log_dir)
        except Exception:
            if log_dir:
                os.makedirs(log_dir, exist_ok=True)
                self.f = open(os.path.join(log_dir, 'train_log.jsonl'), 'a')

    def add_scalar(self, tag, value, step):
        value = float(value)
        if self.w is not None:
            self.w.add_scalar(tag, value, step)
        elif self.f is not None:
            import json
            self.f.write(json.dumps({"tag": tag, "value": value, "step": int(step)}) + "\n")

    def close(self):
        if self.f is not None:
            self.f.close()


def _epochs(model, optim, loss_fn, loader_fn, num_epochs, log, step_offset=0):
    for i in range(num_epochs):
        loss, logger_info = model.train_epoch(optim, loss_fn, loader_fn())
        log.add_scalar('Train/Loss', loss, i + step_offset)
        for key, value in logger_info.items():
            log.add_scalar('Train/' + key, value, i + step_offset)


def train_linear(model, optim, loss_fn, forward_model_params, save_dir, log_dir, num_epochs, batch_size, xs, ys,
                 resume_training=False):
    """main_diffusion_linear.py:19-51 `train`: per epoch a shuffled loader with fresh observation noise
    (datasets.py:44-54), `model.train_epoch`, scalar logging (steps offset by 5000 when resuming, as the
    reference logs them); the state_dict goes to save_dir/current_model.pt."""
    from .problems import get_dataloader_linear
    model.sde.train()
    log = _Log(log_dir)
    _epochs(model, optim, loss_fn,
            lambda: get_dataloader_linear(xs, ys, forward_model_params['scale'], batch_size),
            num_epochs, log, 5000 if resume_training else 0)
    log.close()
    os.makedirs(save_dir, exist_ok=True)
    torch.save(model.sde.a.state_dict(), os.path.join(save_dir, 'current_model.pt'))
    return model


def train_scatterometry(model, optimizer, loss_fn, forward_model_params, save_dir, log_dir, num_epochs, batch_size,
                        forward_model):
    """main_diffusion_scatterometry.py:19-38 `train`: per epoch 8 batches of prior samples pushed
    through the surrogate with fresh noise (datasets.py:26-34); the state_dict goes to
    save_dir/diffusion.pt."""
    from .problems import get_dataloader_scatterometry
    log = _Log(log_dir)
    _epochs(model, optimizer, loss_fn,
            lambda: get_dataloader_scatterometry(batch_size, forward_model, forward_model_params['a'],
                                                 forward_model_params['b'], forward_model_params['lambd_bd']),
            num_epochs, log)
    log.close()
    os.makedirs(save_dir, exist_ok=True)
    torch.save(model.sde.a.state_dict(), os.path.join(save_dir, 'diffusion.pt'))
    return model


# ------------------------------------------------------------------ A18: PosteriorLoss on the device
def posterior_fused_ok(model, loss_fn):
    """True when PosteriorDiffusionEstimator.train_epoch can take dmip_posterior_loss_grad: a PosteriorLoss on
    the scatterometry surrogate, both networks fp32 on a HIP device with equal hidden layers."""
    from .losses import PosteriorLoss
    from .problems import surrogate_handle
    if os.environ.get("DMIP_TRAIN_FUSED", "1") == "0" or not isinstance(loss_fn, PosteriorLoss):
        return False
    prior, lik = model.sde.a.prior_net, model.sde.a.likelihood_net
    if not (_tanh_chain(prior) and _tanh_chain(lik)):
        return False
    p0 = prior.linear_layers()[0][0]
    if not p0.is_cuda or p0.dtype != torch.float32 or (model.xdim, model.ydim) != (3, 23):
        return False
    if [int(w.shape[0]) for w, _ in prior.linear_layers()] != [int(w.shape[0]) for w, _ in lik.linear_layers()]:
        return False
    return loss_fn.forward_model is not None and surrogate_handle(loss_fn.forward_model, p0.device) is not None


def posterior_loss_grad(model, loss_fn, x, y, t, eps, want_target=False):
    """One fused PosteriorLoss evaluation (dmip_posterior_loss_grad): gradients written into both networks'
    .grad (set, not accumulated); returns (loss, info[, target]) like the reference loss object."""
    from .problems import surrogate_handle
    prior, lik = model.sde.a.prior_net, model.sde.a.likelihood_net
    pl = [(w.detach(), b.detach()) for w, b in prior.linear_layers()]
    ll = [(w.detach(), b.detach()) for w, b in lik.linear_layers()]
    dev = pl[0][0].device
    f32 = dict(device=dev, dtype=torch.float32)
    x = x.detach().to(**f32).contiguous()
    y = y.detach().to(**f32).contiguous()
    t = t.detach().to(**f32).reshape(-1).contiguous()
    eps = eps.detach().to(**f32).contiguous()
    pp, lp = list(prior.parameters()), list(lik.parameters())
    gp = torch.empty(sum(p.numel() for p in pp), **f32)
    gl = torch.empty(sum(p.numel() for p in lp), **f32)
    out = torch.empty(3, **f32)
    tgt = torch.empty_like(x) if want_target else None
    base = model.sde.base_sde
    sur = surrogate_handle(loss_fn.forward_model, dev)
    _lib.posterior_loss_grad(pl, ll, sur, _lib.scat_noise(loss_fn.a, loss_fn.b, 0.0), loss_fn.lam,
                             _lib.vpsde(base.beta_min, base.beta_max, 1.0), x, y, t, eps, gp, gl, out, tgt)
    for params, flat in ((pp, gp), (lp, gl)):
        off = 0
        for p in params:
            n = p.numel()
            p.grad = flat[off:off + n].view_as(p).clone()
            off += n
    info = {'PriorLoss': out[1], 'LikelihoodLoss': out[2]}
    return (out[0], info, tgt) if want_target else (out[0], info)
