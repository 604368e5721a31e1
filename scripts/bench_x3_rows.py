"""The one-tile fp32x3 engine's (dmip_x3.h) bench rows, timed by HIP events: CDE / Posterior / CDiffE predictor-
corrector at the reference width [512]^3 (100k chains) and CDiffE-PC at [256]^3 (config 3's per-GPU share, 125k
chains), 1000 steps, random-init weights. One JSON line of launch milliseconds (median of --reps).
    python scripts/bench_x3_rows.py [--reps 3]"""
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
    ap.add_argument("--rows", default="", help="comma-separated subset of cde512,post512,cdiffe_pc512,cdiffe_pc256")
    a = ap.parse_args()
    pkg = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
    dev = torch.device("cuda:0")
    y = torch.rand(23, device=dev)
    rows = {"cde512": (pkg.CDE, 512, 100000, {}), "post512": (pkg.PosteriorDiffusionEstimator, 512, 100000, {}),
            "cdiffe_pc512": (pkg.CDiffE, 512, 100000, {"corrector_steps": 1}),
            "cdiffe_pc256": (pkg.CDiffE, 256, 125000, {"corrector_steps": 1})}
    if a.rows:
        rows = {k: rows[k] for k in a.rows.split(",")}
    out = {}
    st = torch.cuda.current_stream(dev)
    for name, (cls, W, n, kw) in rows.items():
        torch.manual_seed(0)
        m = cls(3, 23, [W] * 3)
        m.sde.a.to(dev)
        m.sample_device(y, n, a.steps, seed=1, precision="fp32x3", **kw)
        ts = []
        for r in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            x = m.sample_device(y, n, a.steps, seed=2 + r, precision="fp32x3", **kw)
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        out[name] = {"ms": float(np.median(ts)), "finite": bool(torch.isfinite(x).all())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
