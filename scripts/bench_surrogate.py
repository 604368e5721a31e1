"""Scatterometry forward-model kernels on one MI355X.

  * MH ground truth (generate_scatterometry_ground_truth.py settings: 30,000 chains per (y, repeat),
    METR_STEPS = 1000, NOISE_STD_MCMC = 0.5), --rows (y, repeat) rows in one fused launch: chain-steps/s
    and the f32-MFMA roofline of dmip_mh_sample (one surrogate evaluation per chain-step);
  * get_log_posterior + energy_grad (dmip_log_posterior with gradient) on --eval-n rows: rows/s;
  * the reference's torch-CPU anneal_to_energy loop (restated with the same torch ops:
    problems.anneal_to_energy's generic path, which calls the surrogate twice per step like
    models/SNF.py:258-261) on a bounded sample, on the host cores.
Algorithmic flops per surrogate evaluation: 2 (3*256 + 2*256^2 + 256*23) = 275,456 (the energy terms
are O(23) VALU and not counted); with the gradient (reverse pass) 2x.
Prints one JSON line.   python scripts/bench_surrogate.py [--rows 10] [--chains 30000] [--steps 1000]"""
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
FLOPS_EVAL = 2 * (3 * 256 + 2 * 256 * 256 + 256 * 23)
PEAK_F32_MFMA = 157.3  # TFLOP/s, MI355X dense f32-input MFMA (MI355X_MICROARCH.md)
PEAK_FP16_MFMA = 2500.0  # TFLOP/s, dense fp16 MFMA (the same guide; bench.py PEAK_BF16_TFLOPS)


def surrogate(dev):
    z = np.load(os.path.join(ROOT, "tests", "golden", "surrogate.npz"))
    fm = torch.nn.Sequential(torch.nn.Linear(3, 256), torch.nn.ReLU(), torch.nn.Linear(256, 256), torch.nn.ReLU(),
                             torch.nn.Linear(256, 256), torch.nn.ReLU(), torch.nn.Linear(256, 23))
    fm.load_state_dict({k.replace("_", "."): torch.from_numpy(z[k]) for k in z.files})
    for p in fm.parameters():
        p.requires_grad = False
    return fm.to(dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10, help="(y, repeat) rows per MH launch")
    ap.add_argument("--chains", type=int, default=30000)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--eval-n", type=int, default=1 << 20)
    ap.add_argument("--cpu-chains", type=int, default=4000)
    ap.add_argument("--cpu-steps", type=int, default=200)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    pr = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.problems")
    dev = torch.device("cuda:0")
    fm = surrogate(dev)
    prm = {"a": 0.2, "b": 0.01, "lambd_bd": 1000}
    ys = torch.from_numpy(np.load(os.path.join(ROOT, "tests", "golden", "data_scat.npz"))["y_test"])
    rows = ys[torch.arange(a.rows) % ys.shape[0]].to(dev)
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

    mh = lambda: pr.mh_sample(fm, prm, rows, a.chains, a.steps, 0.5, seed=1)
    mh()
    ms_mh = timed(mh, a.reps)
    chain_steps = a.rows * a.chains * a.steps
    mh_tf = chain_steps * FLOPS_EVAL / (ms_mh * 1e-3) / 1e12
    # the fp32x3 kernel (dmip_dps_x3.hip mh_x3_kernel): 3 fp16 MFMA products per algorithmic one
    mh3 = lambda: pr.mh_sample(fm, prm, rows, a.chains, a.steps, 0.5, seed=1, precision="fp32x3")
    mh3()
    ms_mh3 = timed(mh3, a.reps)
    mh3_tf = chain_steps * FLOPS_EVAL / (ms_mh3 * 1e-3) / 1e12

    x = (torch.rand(a.eval_n, 3, device=dev) * 2.2 - 1.1)
    y = rows[:1].contiguous()
    h = pr.surrogate_handle(fm, dev)
    from importlib import import_module
    L = import_module("diffusion-modelling-for-inverse-problems_amd._lib")
    e = torch.empty(a.eval_n, device=dev)
    g = torch.empty_like(x)
    nz = L.scat_noise(0.2, 0.01, 1000)
    ev = lambda: L.log_posterior(h, nz, x, y, 0, e, g)
    ev()
    ms_ev = timed(ev, 5)
    ev_tf = a.eval_n * 2 * FLOPS_EVAL / (ms_ev * 1e-3) / 1e12
    ev0 = lambda: L.log_posterior(h, nz, x, y, 0, e, None)
    ev0()
    ms_ev0 = timed(ev0, 5)

    out = {
        "metric": "MH ground-truth chain-steps/s (scatterometry surrogate, fused)",
        "value": chain_steps / (ms_mh * 1e-3), "unit": "chain-steps/s",
        "config": {"rows": a.rows, "chains_per_row": a.chains, "mh_steps": a.steps, "noise_std": 0.5},
        "mh_ms_per_launch": ms_mh,
        "roofline": {"bound": "mfma", "achieved": mh_tf, "peak": PEAK_F32_MFMA, "unit": "TFLOP/s",
                     "frac": mh_tf / PEAK_F32_MFMA, "dtype": "f32 (v_mfma_f32_16x16x4_f32)",
                     "flops_per_chain_step": FLOPS_EVAL},
        "mh_fp32x3": {"ms_per_launch": ms_mh3, "chain_steps_per_s": chain_steps / (ms_mh3 * 1e-3),
                      "algorithmic_tflops": mh3_tf, "executed_fp16_tflops": 3 * mh3_tf,
                      "frac_fp16_peak_executed": 3 * mh3_tf / PEAK_FP16_MFMA, "speedup_vs_f32": ms_mh / ms_mh3},
        "log_posterior_grad": {"rows": a.eval_n, "ms": ms_ev, "rows_per_s": a.eval_n / (ms_ev * 1e-3),
                               "tflops": ev_tf, "frac": ev_tf / PEAK_F32_MFMA},
        "log_posterior": {"rows": a.eval_n, "ms": ms_ev0, "rows_per_s": a.eval_n / (ms_ev0 * 1e-3),
                          "tflops": a.eval_n * FLOPS_EVAL / (ms_ev0 * 1e-3) / 1e12},
    }
    if not a.no_cpu:
        fc = surrogate("cpu")
        en = pr.ScatterometryEnergy(fc, 0.2, 0.01, ys[0], 1000)
        torch.manual_seed(0)
        x0 = torch.rand(a.cpu_chains, 3) * 2 - 1
        t0 = time.perf_counter()
        with torch.no_grad():
            pr.anneal_to_energy(x0, en, a.cpu_steps, noise_std=0.5)
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": a.cpu_chains * a.cpu_steps / dt, "unit": "chain-steps/s",
                               "cores": torch.get_num_threads(), "kind": "port",
                               "sample": f"{a.cpu_chains} chains x {a.cpu_steps} steps, reference-order torch-CPU "
                                         f"anneal_to_energy (2 surrogate evaluations per step), {dt:.1f} s"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
