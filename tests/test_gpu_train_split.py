"""The config-5 training kernel's builds: the forward / reverse split (default; loss_grad_kernel<NL, 1> and the
record reverse <NL, 3>, which reads the forward half's per-layer records instead of recomputing the forward), the
split with the recomputing reverse <NL, 2> (DMIP_TRAIN_REC=0) and the one-kernel fused build (DMIP_TRAIN_SPLIT=0).
The build is chosen once per process (the training plan's workspace is sized by it), so the fused build
runs in one child process. Both are held to the oracle's float64 loss and gradients at the bounds of
tests/test_gpu_parity.py (ragged batch: loss 3e-5, gradients 8e-3) and to each other. Needs an MI355X."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# computes the fused bf16 loss and gradients of a seeded net on a seeded ragged batch; prints JSON
_CHILD = r"""
import importlib, json, sys
import numpy as np, torch
sys.path.insert(0, sys.argv[1])
dmip = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
tr = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.training")
NL, n = int(sys.argv[2]), int(sys.argv[3])
torch.manual_seed(NL)
m = dmip.CDE(2, 2, [64] * NL)
g = np.random.default_rng(11)
x = g.normal(size=(n, 2)).astype(np.float32)
y = (x @ np.array([[1, 0.5], [0, 1]], np.float32).T + np.array([0.3, 0.5], np.float32)
     + 0.3 * g.normal(size=(n, 2))).astype(np.float32)
t = (1e-4 + g.uniform(size=(n, 1)) * (1 - 1e-4)).astype(np.float32)
eps = g.normal(size=(n, 2)).astype(np.float32)
sp = dmip.LinearForwardProblem().score_posterior
lf = dmip.PINNLoss(sp, lam=1e-3, lam2=0.1, pde_loss="FPE", ic_metric="L2", pde_metric="L1")
cfg = tr.fused_config(m, lf)
loss, _ = tr.fused_loss_grad(m, lf, cfg, *[torch.from_numpy(a).to("cuda:0") for a in (x, y, t, eps)], precision="bf16")
grads = [p.grad.detach().cpu().numpy().ravel().tolist() for p in m.sde.a.parameters()]
params = [(l.weight.detach().cpu().numpy().tolist(), l.bias.detach().cpu().numpy().tolist())
          for l in m.sde.a if isinstance(l, torch.nn.Linear)]
print(json.dumps({"loss": float(loss), "grads": grads, "params": params, "batch": [x.tolist(), y.tolist(), t.tolist(), eps.tolist()]}))
"""


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _run(split, NL, n, rec=1):
    env = dict(os.environ, DMIP_TRAIN_SPLIT=str(split), DMIP_TRAIN_REC=str(rec), HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = subprocess.run([sys.executable, "-c", _CHILD, ROOT, str(NL), str(n)], env=env, capture_output=True,
                         text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(1e-30, np.linalg.norm(b)))


@pytest.mark.parametrize("NL", [2, 3])
def test_split_and_fused_builds_agree_with_the_oracle(NL):
    n = 5003  # ragged: not a multiple of the 16-sample tile nor of the waves
    fused = _run(0, NL, n)
    split = _run(1, NL, n)
    recompute = _run(1, NL, n, rec=0)
    params = [(np.asarray(w, np.float32), np.asarray(b, np.float32)) for w, b in split["params"]]
    x, y, t, eps = (np.asarray(a, np.float32) for a in split["batch"])
    ref_loss, _, ref = O.loss_grad(params, x, y, t, eps, lam=1e-3, lam2=0.1, pde="FPE", ic_metric="L2",
                                   pde_metric="L1", ic_A=[[1, 0.5], [0, 1]], ic_b=[0.3, 0.5],
                                   ic_Sinv=np.eye(2) / 0.3)
    flat_ref = [a.ravel() for wb in ref for a in wb]
    for tag, r in (("fused", fused), ("split", split), ("split, recomputing reverse", recompute)):
        lrel = abs(r["loss"] - ref_loss) / abs(ref_loss)
        errs = [_rel(gk, rk) for gk, rk in zip(r["grads"], flat_ref)]
        print(f"\n[train {tag}] NL={NL}: loss rel {lrel:.2e}, max grad rel L2 {max(errs):.2e}")
        assert lrel < 3e-5, (tag, lrel)
        assert max(errs) < 8e-3, (tag, errs)
    # the two builds sum the same bf16 products in different orders
    assert abs(fused["loss"] - split["loss"]) / abs(ref_loss) < 3e-5
    assert max(_rel(a, b) for a, b in zip(fused["grads"], split["grads"])) < 8e-3
    # the record reverse rounds its three derivative coefficients to 16 bits; the
    # activations it reads are the recompute's own bf16 values
    assert abs(recompute["loss"] - split["loss"]) / abs(ref_loss) < 3e-5
    assert max(_rel(a, b) for a, b in zip(recompute["grads"], split["grads"])) < 8e-3
