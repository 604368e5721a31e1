"""The exact-f32 engine (dmip_f32.h) bench rows, timed by HIP events: CDE / Posterior / CDiffE predictor-
corrector at the reference width [512]^3 (100k chains) and CDiffE-PC at [256]^3 (config 3's per-GPU share, 125k
chains), 1000 steps, random-init weights. One JSON line of launch milliseconds (median of --reps).
    python scripts/bench_f32_rows.py [--reps 3]"""
import argparse
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=1000)
    a = ap.parse_args()
    pkg = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
    dev = torch.device("cuda:0")
    y = torch.rand(23, device=dev)
    rows = {"cde256": (pkg.CDE, 256, 100000, {}), "post256": (pkg.PosteriorDiffusionEstimator, 256, 100000, {}), "cdiffe256": (pkg.CDiffE, 256, 100000, {"corrector_steps": 1}),
            
            }
    out = {}
    st = torch.cuda.current_stream(dev)
    for name, (cls, W, n, kw) in rows.items():
        torch.manual_seed(0)
        m = cls(3, 23, [W] * 3)
        m.sde.a.to(dev)
        m.sample_device(y, n, a.steps, seed=1, precision="fp32", **kw)
        ts = []
        for r in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            x = m.sample_device(y, n, a.steps, seed=2 + r, precision="fp32", **kw)
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        out[name] = {"ms": float(np.median(ts)), "finite": bool(torch.isfinite(x).all())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
