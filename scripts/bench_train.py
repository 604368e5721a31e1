"""BASELINE config 5: PINNLoss training step of the linear CDE ([64]*3, batch 65,536) on one MI355X,
plus the exact-f32 engine at the reference configs' hidden_layers [512]*3.

For each (width, precision) it times with HIP events on the launching stream:
  * ms_loss_grad   the fused loss + gradient launch sequence alone (dmip_loss_grad / _f32),
  * ms_device_step the whole step on the device as one captured hipGraph (training.DeviceTrainStep ->
                   dmip_train_plan; ms_device_step_no_graph: launch by launch: dmip_train_draws ->
                   loss + gradients -> dmip_adam_step, no host synchronisation),
  * ms_epoch_step  CDE.train_epoch's step (host t / eps draws, torch Adam, the reference's per-batch
                   loss.item()), host-timed,
and once, the same step through torch autograd on the GPU and on the host CPU (bounded batch); plus
PosteriorLoss (A18, dmip_posterior_loss_grad) at widths 256 and 512 on scatterometry-shaped data.
Algorithmic flops per sample: 16.94 F, F = 2 (5 W + 2 W^2 + 2 W). One JSON line.
    python scripts/bench_train.py [--batch 65536] [--steps 20] [--cpu-batch 4096]"""
import argparse
import importlib
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK = {"bf16": 2500.0, "fp32": 157.3}  # dense TFLOP/s (MI355X_MICROARCH.md)


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
    B = a.batch
    x = torch.randn(B, 2, device=dev)
    y = x @ prob.A.to(dev).T + prob.b.to(dev) + 0.3 * torch.randn(B, 2, device=dev)
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

    def loader():
        yield x, y

    rows = {}
    for width, prec in ((64, "bf16"), (64, "fp32"), (512, "fp32")):
        os.environ["DMIP_TRAIN_PRECISION"] = prec
        m = pkg.CDE(2, 2, [width] * 3)
        cfg = tr.fused_config(m, lf)
        assert cfg is not None
        t = m.sample_t(x).detach()
        eps = torch.randn_like(x)
        kern = lambda: tr.fused_loss_grad(m, lf, cfg, x, y, t, eps, precision=prec)
        for _ in range(a.warmup):
            kern()
        ms_kernel = timed(kern, a.steps)
        opt = torch.optim.Adam(m.sde.a.parameters(), lr=1e-4)
        ms_dev_modes = {}
        for graph in ("0", "1"):  # launch by launch, then the captured hipGraph (dmip_train_plan)
            os.environ["DMIP_TRAIN_GRAPH"] = graph
            dstep = tr.DeviceTrainStep(m, lf, opt, precision=prec)
            run = lambda: dstep(x, y)
            for _ in range(a.warmup):
                run()
            ms_dev_modes[graph] = timed(run, a.steps)
        ms_dev = ms_dev_modes["1"]
        step = lambda: m.train_epoch(opt, lf, loader)
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        ms_epoch = (time.perf_counter() - t0) * 1e3 / a.steps
        F = 2 * (5 * width + 2 * width * width + width * 2)
        tf = 16.94 * F * B / (ms_kernel * 1e-3) / 1e12
        rows[f"w{width}_{prec}"] = {"ms_loss_grad": ms_kernel, "ms_device_step": ms_dev,
                                    "ms_device_step_no_graph": ms_dev_modes["0"], "ms_epoch_step": ms_epoch,
                                    "device_step_samples_per_s": B / (ms_dev * 1e-3),
                                    "loss_grad_tflops": tf, "frac_of_dense_peak": tf / PEAK[prec]}
    os.environ.pop("DMIP_TRAIN_PRECISION", None)

    # A18: PosteriorLoss (prior DSM + likelihood target through the surrogate), exact f32, the fused
    # dmip_posterior_loss_grad on scatterometry-shaped data
    gold = os.path.join(ROOT, "tests", "golden")
    fm, prm = pkg.load_forward_model(gold)
    fm = fm.to(dev)
    xs = torch.rand(B, 3, device=dev) * 2 - 1
    with torch.no_grad():
        ysc = fm(xs)
    ysc = ysc + (prm["a"] * ysc.abs() + prm["b"]) * torch.randn_like(ysc)
    for width in (256, 512):
        mp = pkg.PosteriorDiffusionEstimator(3, 23, [width] * 3)
        mp.sde.a.to(dev)
        plf = pkg.PosteriorLoss(fm, prm["a"], prm["b"], 0.01)
        tp = mp.sample_t(xs).detach()
        ep = torch.randn_like(xs)
        run = lambda: tr.posterior_loss_grad(mp, plf, xs, ysc, tp, ep)
        for _ in range(a.warmup):
            run()
        ms = timed(run, a.steps)
        rows[f"posterior_loss_w{width}_fp32"] = {"ms_loss_grad": ms, "samples_per_s": B / (ms * 1e-3)}

    m = pkg.CDE(2, 2, [64] * 3)
    opt = torch.optim.Adam(m.sde.a.parameters(), lr=1e-4)
    step = lambda: m.train_epoch(opt, lf, loader)
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
               "sample": f"torch autograd PINNLoss step ([64]*3) on the host CPU, batch {a.cpu_batch}, {n_c} steps"}
    os.environ.pop("DMIP_TRAIN_FUSED", None)

    head = rows["w64_bf16"]
    print(json.dumps({
        "metric": "PINNLoss train-step samples/sec (linear CDE [64]*3, BASELINE configs[4])",
        "value": head["device_step_samples_per_s"], "unit": "samples/s", "n_gpus": 1, "steps": a.steps,
        "ms_per_step": head["ms_device_step"], "ms_per_step_torch_autograd_gpu": ms_autograd,
        "higher_is_better": True, "dtype": "bf16 (split-bf16 primal streams)", "data": "synthetic",
        "config": {"workload": "PINNLoss(FPE, L1; IC L2, lam 1e-3, lam2 0.1) train step: draws + loss/grad + Adam",
                   "batch": B, "hidden_layers": [64, 64, 64]},
        "roofline": {"bound": "mfma", "achieved": head["loss_grad_tflops"], "peak": PEAK["bf16"], "unit": "TFLOP/s",
                     "frac": head["frac_of_dense_peak"], "traffic": None,
                     "note": "algorithmic 16.94 F per sample (SURVEY A14) over the loss+grad launches"},
        "per_config": rows,
        "cpu_baseline": cpu,
    }))


if __name__ == "__main__":
    main()
