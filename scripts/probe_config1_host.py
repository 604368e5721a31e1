# Config-1 host-cost probe (round 6): where the fixed ~0.17 ms of model(y, num_samples=1000, num_steps=S) goes at S = 1
# (median of 50 calls per phase, after warmup): the whole call; sample_device + synchronize; device_status;
# the D2H copy; the y upload; the seeded launch path without the status read.
import importlib, json, os, sys, time

import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
L = importlib.import_module("diffusion-modelling-for-inverse-problems_amd._lib")
dev = "cuda:0"
zl = np.load(os.path.join(ROOT, "tests", "golden", "ckpt_lin.npz"))
ml = pkg.CDE(2, 2, [64] * 3)
ml.sde.a.load_state_dict({k.replace("_", "."): torch.from_numpy(zl[k]) for k in zl.files if k.split("_")[0].isdigit()})
ml.sde.a.to(dev)
yl = torch.tensor([0.5, 1.0])
yd = yl.to(dev)


def med(fn, reps=50):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


S = int(sys.argv[1]) if len(sys.argv) > 1 else 1
x = ml.sample_device(yd, 1000, S, seed=1)
out = {
    "call_us": med(lambda: ml(yl, num_samples=1000, num_steps=S)),
    "sample_device_sync_us": med(lambda: (ml.sample_device(yd, 1000, S, seed=1), torch.cuda.synchronize())),
    "sample_device_host_y_sync_us": med(lambda: (ml.sample_device(yl, 1000, S, seed=1), torch.cuda.synchronize())),
    "device_status_us": med(lambda: L.device_status(x.device)),
    "d2h_us": med(lambda: x.cpu().numpy()),
    "y_upload_us": med(lambda: yl.to(dev)),
    "empty_sync_us": med(lambda: torch.cuda.synchronize()),
}
print(json.dumps(out), flush=True)
