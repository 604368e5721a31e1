"""BASELINE config 4: scatterometry DPS (prior score network + surrogate-likelihood guidance every step),
1000 SDE steps, 256k posterior samples (sharded over the ranks under torchrun; weak scaling with
--per-gpu). Reports samples/s over all ranks, the f32-MFMA roofline of the fused kernel on rank 0, and
the sample quality against the fused MH ground truth of the same y (KL2 on 75^3 bins over [-1.2, 1.2]^3,
the reference's metric, main_diffusion_scatterometry.py:71-102).

Weights: the fixture-trained prior (tests/golden/ckpt_prior_scat.npz, DSM on inverse_cdf_prior
samples) or random init. Algorithmic flops per chain-step: prior forward + input VJP (2 F_prior,
F_prior = 2 (4*256 + 2*256^2 + 256*3)) + surrogate forward + VJP (2 F_sur, F_sur = 275,456); the kernel
executes 4 F_prior for the prior (primal + 3 forward tangents).
    python scripts/bench_dps.py [--samples 262144] [--steps 1000] [--zeta 0.005] [--guidance norm] [--precision fp32x3]
    torchrun --nproc-per-node 4 scripts/bench_dps.py"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
F_PRIOR = 2 * (4 * 256 + 2 * 256 * 256 + 256 * 3)
F_SUR = 2 * (3 * 256 + 2 * 256 * 256 + 256 * 23)
PEAK_F32_MFMA = 157.3
PEAK_F16_MFMA = 2500.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=262144, help="total samples (all ranks)")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--zeta", type=float, default=0.005)
    ap.add_argument("--guidance", default="norm")
    ap.add_argument("--y-index", type=int, default=0)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--gt-chains", type=int, default=30000)
    ap.add_argument("--precision", default="fp32x3", choices=["fp32x3", "fp32"])
    ap.add_argument("--compare-cde", action="store_true", help="also score the fixture-trained CDE on the same y")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    pkg = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
    par = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.parallel")
    ev = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.evaluate")
    gold = os.path.join(ROOT, "tests", "golden")
    fm, prm = pkg.load_forward_model(gold)  # reads surrogate.npz (the reference's surrogate.pt, converted)
    fm = fm.to(dev)
    m = pkg.DPS(3, 23, [256] * 3, fm, prm, zeta=a.zeta, guidance=a.guidance)
    weights = "random-init"
    ck = os.path.join(gold, "ckpt_prior_scat.npz")
    if os.path.exists(ck):
        z = np.load(ck)
        m.prior_net.load_state_dict({k.replace("_", "."): torch.from_numpy(z[k]) for k in z.files
                                     if k.split("_")[0].isdigit()})
        weights = "fixture-trained prior (tests/golden/ckpt_prior_scat.npz)"
    m.prior_net.to(dev)
    y = torch.from_numpy(np.load(os.path.join(gold, "data_scat.npz"))["y_test"][a.y_index]).to(dev)

    lo, hi = par.shard_range(a.samples, rank, world)
    run = lambda s: par.gather_shards(m.sample_device(y, hi - lo, a.steps, seed=s, chain_offset=lo,
                                                     precision=a.precision), a.samples, dev)
    x = run(1)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    e0.record(st)
    for r in range(a.reps):
        x = run(2 + r)
    e1.record(st)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    launch_ms = e0.elapsed_time(e1) / a.reps
    alg = (2 * F_PRIOR + 2 * F_SUR) * a.steps * (hi - lo)
    # fp32 engine: primal + 3 forward tangents through the prior; fp32x3: every product as three fp16 MFMAs
    exe_cs = 4 * F_PRIOR + 2 * F_SUR if a.precision == "fp32" else 3 * (2 * F_PRIOR + 2 * F_SUR)
    exe = exe_cs * a.steps * (hi - lo)
    peak = PEAK_F32_MFMA if a.precision == "fp32" else PEAK_F16_MFMA
    out = {"metric": "DPS posterior samples/s (1000-step reverse SDE + surrogate guidance)",
           "value": a.samples * a.reps / el, "unit": "samples/s", "n_gpus": world, "samples": a.samples,
           "sde_steps": a.steps, "zeta": a.zeta, "guidance": a.guidance, "weights": weights, "precision": a.precision,
           "ms_per_call": el / a.reps * 1e3, "rank0_launch_ms": launch_ms,
           "roofline": {"bound": "mfma", "achieved": alg / (launch_ms * 1e-3) / 1e12, "peak": peak,
                        "unit": "TFLOP/s", "frac": alg / (launch_ms * 1e-3) / 1e12 / peak,
                        "executed_tflops": exe / (launch_ms * 1e-3) / 1e12,
                        "executed_frac": exe / (launch_ms * 1e-3) / 1e12 / peak,
                        "flops_per_chain_step_alg": 2 * F_PRIOR + 2 * F_SUR,
                        "flops_per_chain_step_executed": exe_cs}}
    if rank == 0 and a.gt_chains > 0:  # --gt-chains 0: timing only (A/B runs)
        gt = pkg.mh_sample(fm, prm, y[None], a.gt_chains, 1000, 0.5, seed=99)[0]
        xs = x[:a.gt_chains] if x.ndim == 2 else x[0, :a.gt_chains]
        kl, klr = ev.hist_kl(ev.histograms(gt, 75, (-1.2, 1.2))[0], ev.histograms(xs, 75, (-1.2, 1.2))[0])
        # two independent MH runs: the histogram-noise floor of KL2 at this sample size
        gt2 = pkg.mh_sample(fm, prm, y[None], a.gt_chains, 1000, 0.5, seed=98)[0]
        kl0, _ = ev.hist_kl(ev.histograms(gt, 75, (-1.2, 1.2))[0], ev.histograms(gt2, 75, (-1.2, 1.2))[0])
        def w1(u, v):  # per-dimension 1-D Wasserstein distance on equal-size samples
            return [float((torch.sort(u[:, k])[0] - torch.sort(v[:, k])[0]).abs().mean()) for k in range(3)]
        out["quality"] = {"KL2_vs_mcmc": kl, "KL_reverse": klr, "KL2_mcmc_vs_mcmc": kl0, "n": a.gt_chains,
                          "y_index": a.y_index, "W1_vs_mcmc": w1(xs, gt), "W1_mcmc_vs_mcmc": w1(gt2, gt),
                          "mean": xs.mean(0).tolist(), "mcmc_mean": gt.mean(0).tolist(),
                          "std": xs.std(0).tolist(), "mcmc_std": gt.std(0).tolist()}
        if a.compare_cde:
            cde = pkg.CDE(3, 23, [256] * 3)
            zc = np.load(os.path.join(gold, "ckpt_scat.npz"))
            cde.sde.a.load_state_dict({k.replace("_", "."): torch.from_numpy(zc[k]) for k in zc.files
                                       if k.split("_")[0].isdigit()})
            cde.sde.a.to(dev)
            xc = cde.sample_device(y, a.gt_chains, a.steps, seed=5)[0]
            klc, _ = ev.hist_kl(ev.histograms(gt, 75, (-1.2, 1.2))[0], ev.histograms(xc, 75, (-1.2, 1.2))[0])
            out["quality_cde"] = {"KL2_vs_mcmc": klc, "W1_vs_mcmc": w1(xc, gt), "mean": xc.mean(0).tolist(),
                                  "std": xc.std(0).tolist()}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
