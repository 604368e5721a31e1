"""Score networks with the reference's module layout (nets.py:17-57, 143-157).

`MLP` / `MLP2` keep the exact parameter naming of the reference (`0.*, 3.*, 5.*, 7.*` for three
hidden layers) so reference checkpoints load unchanged, including the quirk that makes the first
hidden layer apply tanh twice: the reference stores its activation module a second time as
`self.act` on the nn.Sequential (nets.py:26), which registers it as an extra child between layer 0
and the next Linear and shifts the numbering.

Evaluation on a HIP device with autograd off goes to the fused MFMA kernel
(libdmip dmip_mlp_forward) -- in exact f32 by default (`dmip_precision = "fp32"`, the reference's own
arithmetic, e.g. for the evaluate drivers' score MSE), or with 16-bit operands (`"fp16"`: split-bf16 layer 1,
fp16 hidden and output layers; `"bf16"` is its deprecated name); the weights
are packed once per parameter snapshot. Autograd (the training losses) uses the eager module chain.
The activation is the reference's constructor argument: nn.Tanh runs on every engine, nn.SiLU on the exact-f32
forward and CDE sampler (`dmip_act`); any other activation has no HIP kernel: its forward is the module chain (as the
reference's, on the device), and the fused samplers refuse it.
"""
import collections

import torch
from torch import nn

from . import _lib


class _TanhChainMLP(nn.Sequential):
    input_layout = _lib.DMIP_INPUT_X_Y_T

    def __init__(self, input_dim, output_dim, hidden_layers, activation):
        self.input_dim = input_dim
        self.output_dim = output_dim
        self.hidden_layers = list(hidden_layers)
        w = [input_dim] + self.hidden_layers + [output_dim]
        # the activation is one module object registered under several names, as in the reference
        mods = [("0", nn.Linear(w[0], w[1])), ("1", activation), ("act", activation)]
        for i in range(1, len(self.hidden_layers)):
            mods += [(str(2 * i + 1), nn.Linear(w[i], w[i + 1])), (str(2 * i + 2), activation)]
        mods.append((str(2 * len(self.hidden_layers) + 1), nn.Linear(w[-2], w[-1])))
        super().__init__(collections.OrderedDict(mods))
        self.act = activation
        self._dmip = None
        self.dmip_precision = "fp32"  # arithmetic of the HIP forward (dmip_mlp_forward): "fp32" or "fp16"

    # -------------------------------------------------------------- packed HIP weights
    @property
    def dmip_act(self):
        """The compiled activation chain of this network (include/dmip.h dmip_act): nn.Tanh -> the reference's
        chain, nn.SiLU -> the SiLU chain (exact-f32 forward and CDE sampler only); None for any other activation,
        which has no HIP kernel (the HIP paths raise NotImplementedError rather than compute another function)."""
        if isinstance(self.act, nn.Tanh):
            return _lib.DMIP_ACT_TANH_TWICE_FIRST
        if isinstance(self.act, nn.SiLU):
            return _lib.DMIP_ACT_SILU_TWICE_FIRST
        return None

    def require_dmip_act(self):
        act = self.dmip_act
        if act is None:
            raise NotImplementedError(f"{type(self.act).__name__} has no HIP kernel: the compiled activation chains "
                                      "are nn.Tanh (every engine) and nn.SiLU (exact f32)")
        return act

    def linear_layers(self):
        return [(m.weight, m.bias) for m in self if isinstance(m, nn.Linear)]

    def _snapshot_key(self, device):
        return (str(device),) + tuple((p.data_ptr(), p._version) for p in self.parameters())

    def dmip_handle(self, device, xdim):
        act = self.require_dmip_act()
        key = self._snapshot_key(device) + (xdim, act)
        if self._dmip is None or self._dmip[0] != key:
            handle = _lib.MlpHandle(self.linear_layers(), self.input_dim, self.output_dim, xdim,
                                    self.input_layout, device, act)
            self._dmip = (key, handle)
        return self._dmip[1]

    def _wants_autograd(self, *tensors):
        if not torch.is_grad_enabled():
            return False
        return any(t.requires_grad for t in tensors) or any(p.requires_grad for p in self.parameters())

    def _hip_forward(self, x, y, t, xdim):
        n = x.shape[0]
        dev = x.device
        h = self.dmip_handle(dev, xdim)
        xc = x.detach().to(torch.float32).contiguous()
        tt = t.detach().to(device=dev, dtype=torch.float32).reshape(-1).contiguous()
        t_stride = 1 if tt.numel() == n else 0
        if t_stride == 0 and tt.numel() != 1:
            raise ValueError("t must have one entry per row or a single entry")
        yc, y_stride = None, 0
        if y is not None:
            yc = y.detach().to(device=dev, dtype=torch.float32)
            if yc.ndim == 1:
                yc = yc.reshape(1, -1)
            y_stride = yc.shape[1] if yc.shape[0] == n and n != 1 else 0
            yc = yc.contiguous()
        out = torch.empty(n, self.output_dim, device=dev, dtype=torch.float32)
        prec = getattr(self, "dmip_precision", "fp32")
        if h.act != _lib.DMIP_ACT_TANH_TWICE_FIRST:
            prec = "fp32"  # the SiLU chain's forward is compiled in exact f32 only
        _lib.mlp_forward(h, xc, yc, tt, out, y_stride, t_stride, prec)
        return out


class MLP(_TanhChainMLP):
    """Score network a(x, y, t) on cat[x, y, t] (nets.py:17-35)."""

    def forward(self, x, y, t):
        if x.is_cuda and self.dmip_act is not None and not self._wants_autograd(x, y, t):
            return self._hip_forward(x, y, t, x.shape[1])
        inp = torch.cat([x, y, t.view(len(x), 1)], dim=1)
        assert inp.ndim == 2, 'Input Tensor is expected to be 2D with shape (batch_size, ydim+ydim+embeddim)'
        return super().forward(inp)


class MLP2(_TanhChainMLP):
    """Prior score network a(x, t) on cat[x, t] (nets.py:37-57)."""
    input_layout = _lib.DMIP_INPUT_X_T

    def forward(self, x, t):
        if x.is_cuda and self.dmip_act is not None and not self._wants_autograd(x, t):
            return self._hip_forward(x, None, t, x.shape[1])
        inp = torch.cat([x, t.view(len(x), 1)], dim=1)
        assert inp.ndim == 2, 'Input Tensor is expected to be 2D with shape (batch_size, ydim+ydim+embeddim)'
        return super().forward(inp)


class PosteriorScore(nn.Module):
    """g(t) * (prior(x, t) + likelihood(x, y, t)) (nets.py:143-157)."""

    def __init__(self, prior_net, likelihood_net, forward_process):
        super().__init__()
        self.prior_net = prior_net
        self.likelihood_net = likelihood_net
        self.forward_sde = forward_process

    def forward(self, x, y, t):
        return self.forward_sde.g(t, x) * (self.prior_net(x, t) + self.likelihood_net(x, y, t))
