# Width-512 one-tile fp32x3 CDE against the oracle (NL 1..3, xdim 2 / 3, 1 / 2 / 6 steps): which chains are wrong.
# Debug aid of round 6 (scripts/archive/gpu_r6_x3dbg.sh); prints one line per case.
import importlib, os, sys

import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import oracle as O
dmip = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
DEV = "cuda:0"
for NL in (1, 2, 3):
    for xd, yd in ((2, 2), (3, 23)):
        torch.manual_seed(512 + NL + xd)
        m = dmip.CDE(xd, yd, [512] * NL)
        params = [(l.weight.detach().cpu().numpy(), l.bias.detach().cpu().numpy()) for l in m.sde.a if isinstance(l, torch.nn.Linear)]
        y = np.random.default_rng(5).uniform(0, 1, yd).astype(np.float32)
        for S in (1, 2, 6):
            x = m.sample_device(torch.from_numpy(y).to(DEV), 700, S, seed=99, precision="fp32x3")[0].cpu().numpy()
            ref = O.cde_sample(params, y, 700, S, 99)
            e = np.abs(x - ref).max(1)
            bad = np.where(~(e < 1e-3))[0]
            print(f"NL={NL} xd={xd} S={S}: max {np.nanmax(e) if np.isfinite(e).any() else 'nan'} bad {len(bad)} first {bad[:8]} nan {np.isnan(x).any(1).sum()}", flush=True)
