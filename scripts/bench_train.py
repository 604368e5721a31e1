"""BASELINE config 5: PINNLoss training step of the linear CDE ([64]*3, batch 65,536) on one MI355X.

Times (HIP events on the launching stream) the fused loss+gradient kernel (dmip_loss_grad), the whole
fused train step (sample_t + randn + kernel + Adam), the same step through torch autograd on the GPU
(DMIP_TRAIN_FUSED=0), and the torch autograd step on the host CPU on a bounded batch. Prints one
JSON line. Algorithmic flops per sample: 16.94 F, F = 17,280 (SURVEY.md §8a A14, W = 64).
    python scripts/bench_train.py [--batch 65536] [--steps 20] [--cpu-batch 4096]"""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu-batch", type=int, default=4096)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    pkg = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
    tr = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.training")
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    prob = pkg.LinearForwardProblem()
    lf = pkg.PINNLoss(prob.score_posterior, lam=1e-3, lam2=0.1, pde_loss="FPE", ic_metric="L2", pde_metric="L1")
    m = pkg.CDE(2, 2, [64] * 3)
    B = a.batch
    x = torch.randn(B, 2, device=dev)
    y = x @ prob.A.to(dev).T + prob.b.to(dev) + 0.3 * torch.randn(B, 2, device=dev)
    t = m.sample_t(x).detach()
    eps = torch.randn_like(x)
    cfg = tr.fused_config(m, lf)
    assert cfg is not None
    st = torch.cuda.current_stream()

    def timed(fn, k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(st)
        for _ in range(k):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k

    kern = lambda: tr.fused_loss_grad(m, lf, cfg, x, y, t, eps)
    for _ in range(a.warmup):
        kern()
    ms_kernel = timed(kern, a.steps)

    opt = torch.optim.Adam(m.sde.a.parameters(), lr=1e-4)

    def loader():
        yield x, y
    step = lambda: m.train_epoch(opt, lf, loader)
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    ms_step = (time.perf_counter() - t0) * 1e3 / a.steps

    os.environ["DMIP_TRAIN_FUSED"] = "0"
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    k_ag = max(3, a.steps // 4)
    for _ in range(k_ag):
        step()
    torch.cuda.synchronize()
    ms_autograd = (time.perf_counter() - t0) * 1e3 / k_ag
    os.environ["DMIP_TRAIN_FUSED"] = "1"

    cpu = None
    if not a.no_cpu:
        mc = pkg.CDE(2, 2, [64] * 3)
        mc.sde.a.to("cpu")
        optc = torch.optim.Adam(mc.sde.a.parameters(), lr=1e-4)
        xc, yc = x[:a.cpu_batch].cpu(), y[:a.cpu_batch].cpu()

        def loader_c():
            yield xc, yc
        mc.train_epoch(optc, lf, loader_c)
        t0 = time.perf_counter()
        n_c = 3
        for _ in range(n_c):
            mc.train_epoch(optc, lf, loader_c)
        s = (time.perf_counter() - t0) / n_c
        cpu = {"value": a.cpu_batch / s, "unit": "samples/s", "cores": torch.get_num_threads(), "kind": "port",
               "sample": f"torch autograd PINNLoss step on the host CPU, batch {a.cpu_batch}, {n_c} steps"}

    F = 2 * (5 * 64 + 2 * 64 * 64 + 64 * 2)
    flops = 16.94 * F * B
    tflops = flops / (ms_kernel * 1e-3) / 1e12
    print(json.dumps({
        "metric": "PINNLoss train-step samples/sec (linear CDE [64]*3, BASELINE configs[4])",
        "value": B / (ms_step * 1e-3), "unit": "samples/s", "n_gpus": 1, "steps": a.steps,
        "ms_per_step": ms_step, "ms_loss_grad_kernel": ms_kernel, "ms_per_step_torch_autograd_gpu": ms_autograd,
        "higher_is_better": True, "dtype": "bf16 (split-bf16 primal streams)", "data": "synthetic",
        "config": {"workload": "PINNLoss(FPE, L1; IC L2, lam 1e-3, lam2 0.1) train step", "batch": B,
                   "hidden_layers": [64, 64, 64]},
        "roofline": {"bound": "mfma", "achieved": tflops, "peak": 2500.0, "unit": "TFLOP/s",
                     "frac": tflops / 2500.0, "flops_per_step": flops,
                     "note": "algorithmic 16.94 F per sample (SURVEY A14); the kernel is latency-bound at this size"},
        "cpu_baseline": cpu,
    }))


if __name__ == "__main__":
    main()
