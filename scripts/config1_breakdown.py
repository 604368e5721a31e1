"""Where the time of BASELINE configs[0]'s call goes: model(y, num_samples=1000, num_steps=200) on the linear [64]^3
fixture (main_diffusion_linear.py:74), end to end (host ndarray returned) against its parts: sample_device +
synchronize, the sampler kernels alone (HIP events on the stream), and a rocprof-free host overhead estimate.
    python scripts/config1_breakdown.py"""
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    pkg = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
    par = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.parallel")
    dev = torch.device("cuda", 0)
    z = np.load(os.path.join(ROOT, "tests", "golden", "ckpt_lin.npz"))
    m = pkg.CDE(2, 2, [64] * 3)
    m.sde.a.load_state_dict({k.replace("_", "."): torch.from_numpy(z[k]) for k in z.files if k.split("_")[0].isdigit()})
    m.sde.a.to(dev)
    y = torch.tensor([0.5, 1.0])
    yd = y.to(dev)
    out = {}

    def med(fn, n=15):
        ts = []
        for _ in range(n):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts[3:])) * 1e3

    out["model_call_ms"] = med(lambda: m(y, num_samples=1000, num_steps=200))
    out["sample_checked_ms"] = med(lambda: (par.sample_checked(m, yd, 1000, 200, 0, 1), torch.cuda.synchronize()))
    out["sample_device_ms"] = med(lambda: (m.sample_device(yd, 1000, 200, seed=1), torch.cuda.synchronize()))
    st = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ks = []
    for _ in range(12):
        e0.record(st)
        m.sample_device(yd, 1000, 200, seed=1)
        e1.record(st)
        torch.cuda.synchronize()
        ks.append(e0.elapsed_time(e1))
    out["device_ms_events"] = float(np.median(ks[3:]))
    x = torch.empty(1000, 2, device=dev)
    out["d2h_12kb_ms"] = med(lambda: x.cpu().numpy())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
