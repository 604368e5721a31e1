"""The three estimators' fused 16-bit samplers at the reference configs' width [512]*3 (random-init
weights, scatterometry shapes, 1000 steps, one y): samples/s and algorithmic TFLOP/s per launch (HIP
events), beside the exact-f32 engine on the same shape. One JSON line.
    python scripts/bench_width512.py [--chains 100000]"""
import argparse
import importlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def F(i, w, o, nh=3):
    return 2 * (i * w + (nh - 1) * w * w + w * o)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=100000)
    ap.add_argument("--steps", type=int, default=1000)
    a = ap.parse_args()
    pkg = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
    dev = torch.device("cuda:0")
    y = torch.rand(23, device=dev)
    W, out = 512, {}
    rows = {"CDE": (pkg.CDE, F(27, W, 3), {}),
            "PosteriorDiffusionEstimator": (pkg.PosteriorDiffusionEstimator, F(27, W, 3) + F(4, W, 3), {}),
            "CDiffE": (pkg.CDiffE, F(27, W, 26), {}),
            "CDiffE_pc1": (pkg.CDiffE, 2 * F(27, W, 26), {"corrector_steps": 1})}
    for name, (cls, flops, kw) in rows.items():
        torch.manual_seed(0)
        m = cls(3, 23, [W] * 3)
        for prec, peak in (("bf16", 2500.0), ("fp32", 157.3)):
            n = a.chains if prec == "bf16" else a.chains // 10
            m.sample_device(y, 4096, 10, seed=1, precision=prec, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            x = m.sample_device(y, n, a.steps, seed=2, precision=prec, **kw)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            tf = flops * a.steps * n / (ms * 1e-3) / 1e12
            out[f"{name}_{prec}"] = {"chains": n, "ms": ms, "samples_per_s": n / (ms * 1e-3), "tflops": tf,
                                     "frac": tf / peak, "finite": bool(torch.isfinite(x).all())}
    print(json.dumps({"workload": "fused samplers at hidden_layers [512]*3, scatterometry shapes, 1000 steps",
                      "weights": "random-init", "rows": out}))


if __name__ == "__main__":
    main()
