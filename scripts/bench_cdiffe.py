"""BASELINE config 3: scatterometry CDiffE with a Langevin predictor-corrector, 1000 SDE steps,
1M posterior samples sharded over the ranks (torchrun; 125k per GPU at 8 GPUs), RCCL all_gather of
the shards at the end. On one GPU: the per-GPU share of the 8-GPU job (--samples 125000).

CDiffE's joint net is 27 -> [256]*3 -> 26 (x and y outputs, models/diffusion.py:111-121); each SDE
step evaluates it once for the predictor and once per corrector step, so the algorithmic work per
chain-step is (1 + corrector_steps) * F(27, 26), F(in, out) = 2 (in W + 2 W^2 + W out) = 289,280
flop at W = 256. The fused kernel draws y_t ~ q(y_t | y) in-kernel every step.

Weights: random init (no CDiffE checkpoint exists; the reference's CDiffE sampler raises TypeError,
SURVEY §0 D4) -- the kernel's time does not depend on the weights.
    python scripts/bench_cdiffe.py [--samples 125000] [--corrector-steps 1]
    torchrun --nproc-per-node 8 scripts/bench_cdiffe.py --samples 1000000"""
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
W, XDIM, YDIM = 256, 3, 23
F_JOINT = 2 * ((XDIM + YDIM + 1) * W + 2 * W * W + W * (XDIM + YDIM))
PEAK_BF16 = 2500.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=125000, help="total samples (all ranks)")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--corrector-steps", type=int, default=1)
    ap.add_argument("--snr", type=float, default=0.16)
    ap.add_argument("--reps", type=int, default=3)
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
    lib = importlib.import_module("diffusion-modelling-for-inverse-problems_amd._lib")
    torch.manual_seed(0)
    m = pkg.CDiffE(XDIM, YDIM, [W] * 3)
    m.sde.a.to(dev)
    y = torch.from_numpy(np.load(os.path.join(ROOT, "tests", "golden", "data_scat.npz"))["y_test"][0]).to(dev)

    lo, hi = par.shard_range(a.samples, rank, world)
    kw = dict(corrector_steps=a.corrector_steps, snr=a.snr)

    def run(s):
        return par.gather_shards(m.sample_device(y, hi - lo, a.steps, seed=s, chain_offset=lo, **kw), a.samples, dev)

    calls0 = lib.calls["em_sample_cdiffe"]
    x = run(1)
    torch.cuda.synchronize()
    assert lib.calls["em_sample_cdiffe"] == calls0 + 1, "the fused CDiffE kernel did not run"
    st = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(a.reps):
        ev[r][0].record(st)
        x = run(2 + r)
        ev[r][1].record(st)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    launch_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in ev]))
    evals = 1 + a.corrector_steps
    alg = evals * F_JOINT * a.steps * (hi - lo)
    out = {"metric": "CDiffE predictor-corrector posterior samples/s (1000-step reverse SDE)",
           "value": a.samples * a.reps / el, "unit": "samples/s", "n_gpus": world, "samples": a.samples,
           "sde_steps": a.steps, "corrector_steps": a.corrector_steps, "snr": a.snr,
           "weights": "random init (timing only)", "finite_fraction": float(torch.isfinite(x).float().mean()),
           "ms_per_call": el / a.reps * 1e3, "rank0_launch_ms": launch_ms,
           "roofline": {"bound": "mfma", "achieved": alg / (launch_ms * 1e-3) / 1e12, "peak": PEAK_BF16,
                        "unit": "TFLOP/s", "frac": alg / (launch_ms * 1e-3) / 1e12 / PEAK_BF16,
                        "flops_per_chain_step": evals * F_JOINT, "net_evals_per_step": evals}}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
