# x3s (width-64 latency engine) kernel time by HIP events: 1000 chains x 200 steps of the linear [64]^3 fixture,
# device y, 60 back-to-back launches after warmup; prints the median per launch (round-6 A/B aid).
import importlib, json, os, sys

import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
zl = np.load(os.path.join(ROOT, "tests", "golden", "ckpt_lin.npz"))
ml = pkg.CDE(2, 2, [64] * 3)
ml.sde.a.load_state_dict({k.replace("_", "."): torch.from_numpy(zl[k]) for k in zl.files if k.split("_")[0].isdigit()})
ml.sde.a.to("cuda:0")
y = torch.tensor([0.5, 1.0], device="cuda:0")
for _ in range(10):
    ml.sample_device(y, 1000, 200, seed=1)
ts = []
for _ in range(60):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    ml.sample_device(y, 1000, 200, seed=1)
    b.record()
    b.synchronize()
    ts.append(a.elapsed_time(b))
print(json.dumps({"ms_median": float(np.median(ts)), "ms_min": float(np.min(ts))}), flush=True)
