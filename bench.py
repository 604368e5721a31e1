"""Benchmark: posterior samples/s of the fused reverse-SDE sampler (BASELINE.json metric).

Workload (BASELINE.json configs[1]): scatterometry CDE, MLP 27 -> [256]*3 -> 3 (tanh, double tanh
on layer 1), 1000 Euler-Maruyama steps, 100,000 chains per GPU for one y (y_test[0] of the
reference's seeded test set, tests/golden/data_scat.npz), weights = the fixture-trained checkpoint
(tests/golden/ckpt_scat.npz; random init if absent -- timing does not depend on the weights).
One "step" = one full sampling call (x0 draw + 1000 SDE steps + output in HBM). With --gpus N the
chains are sharded by global chain index (weak scaling: 100k chains per GPU) and the shards are
gathered to every rank with one RCCL all_gather inside the timed region.

Prints ONE JSON line on rank 0 (driver contract) with `roofline` (MFMA-bound; algorithmic flops per
launch / HIP-event-timed average launch) and `cpu_baseline` (reference-order torch-CPU sampler on a
bounded sample, rank 0, N=1 only).
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "diffusion-modelling-for-inverse-problems_amd"

XDIM, YDIM, WIDTH, NH = 3, 23, 256, 3
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, no sparsity)


def flops_per_sample_step(in_dim=XDIM + YDIM + 1, w=WIDTH, nh=NH, out=XDIM):
    return 2 * (in_dim * w + (nh - 1) * w * w + w * out)


def load_model(pkg, dev):
    model = pkg.CDE(XDIM, YDIM, [WIDTH] * NH)
    ck = os.path.join(ROOT, "tests", "golden", "ckpt_scat.npz")
    weights = "random-init"
    if os.path.exists(ck):
        z = np.load(ck)
        model.sde.a.load_state_dict({k.replace("_", "."): torch.from_numpy(z[k]) for k in z.files
                                     if k.split("_")[0].isdigit()})
        weights = "fixture-trained (tests/golden/ckpt_scat.npz)"
    model.sde.a.to(dev)
    return model, weights


def synthetic_y():
    p = os.path.join(ROOT, "tests", "golden", "data_scat.npz")
    if os.path.exists(p):
        return np.load(p)["y_test"][0].astype(np.float32)
    return np.abs(np.random.default_rng(13).normal(0.3, 0.4, YDIM)).astype(np.float32)


def pmc_traffic(kernel_match="em_sampler"):
    """HBM bytes per launch of the sampler kernel from the committed rocprofv3 PMC summary
    (profiles/pmc_summary_latest.json, written by scripts/pmc_summary.py from separate --pmc
    passes on the same workload), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_summary_latest.json")
    if not os.path.exists(p):
        return None
    z = json.load(open(p))
    if kernel_match not in z.get("kernel_match", "") or "hbm_bytes_per_launch" not in z:
        return None
    return z["hbm_bytes_per_launch"]


def ks_vs_reference(x, num_steps, weights):
    """Per-dimension two-sample KS statistic of the timed run's samples against the reference
    sampler's own stored draws (tests/golden/samples_scat.npz: 20k of a 100k-chain run of the
    reference's models/diffusion.py:27-46 loop, same y and the same fixture weights), with the
    alpha = 0.01 critical value. The 'KS vs ref' half of BASELINE.json's metric; computed after
    the timed region. None when the weights or the step count differ from the fixture's."""
    p = os.path.join(ROOT, "tests", "golden", "samples_scat.npz")
    if not os.path.exists(p) or not weights.startswith("fixture"):
        return None
    z = np.load(p)
    if int(z["num_steps"]) != num_steps:
        return None
    ref = np.sort(z["samples"].astype(np.float64), axis=0)
    x = np.sort(np.asarray(x, np.float64), axis=0)
    stats = []
    for k in range(ref.shape[1]):
        both = np.concatenate([x[:, k], ref[:, k]])
        ca = np.searchsorted(x[:, k], both, side="right") / x.shape[0]
        cb = np.searchsorted(ref[:, k], both, side="right") / ref.shape[0]
        stats.append(float(np.max(np.abs(ca - cb))))
    n1, n2 = x.shape[0], ref.shape[0]
    crit = 1.63 * float(np.sqrt((n1 + n2) / (n1 * n2)))
    return {"stat": stats, "crit_alpha_0.01": crit, "pass": bool(max(stats) < crit),
            "n_samples": n1, "n_ref": n2,
            "ref": "reference sampler's own draws (tests/golden/samples_scat.npz, same y, same weights)"}


def cpu_baseline(num_steps, n_chains):
    """Reference-order torch-CPU sampler (oracle/torch_cpu.py) on a bounded sample."""
    from oracle import torch_cpu
    threads = torch.get_num_threads()
    gen = torch.Generator().manual_seed(0)
    params = []
    dims = [XDIM + YDIM + 1] + [WIDTH] * NH + [XDIM]
    for i in range(len(dims) - 1):
        bound = 1.0 / np.sqrt(dims[i])
        params.append(((torch.rand(dims[i + 1], dims[i], generator=gen) * 2 - 1) * bound,
                       (torch.rand(dims[i + 1], generator=gen) * 2 - 1) * bound))
    ck = os.path.join(ROOT, "tests", "golden", "ckpt_scat.npz")
    if os.path.exists(ck):
        z = np.load(ck)
        idx = sorted({int(k.split("_")[0]) for k in z.files if k.split("_")[0].isdigit()})
        params = [(z[f"{i}_weight"], z[f"{i}_bias"]) for i in idx]
    net = torch_cpu.build_mlp(params)
    y = synthetic_y()
    torch_cpu.cde_sample(net, y, n_chains, 2, XDIM)  # warm-up
    t0 = time.perf_counter()
    torch_cpu.cde_sample(net, y, n_chains, num_steps, XDIM)
    dt = time.perf_counter() - t0
    return {"value": n_chains / dt, "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"{n_chains} chains x {num_steps} steps, reference-order torch-CPU sampler "
                      f"(oracle/torch_cpu.py), {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--chains", type=int, default=100000, help="chains per GPU")
    ap.add_argument("--num-steps", type=int, default=1000, help="SDE steps per sample")
    ap.add_argument("--cpu-chains", type=int, default=16384)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    pkg = importlib.import_module(PKG)
    from importlib import import_module
    parallel = import_module(PKG + ".parallel")

    model, weights = load_model(pkg, dev)
    y = torch.from_numpy(synthetic_y()).to(dev)
    n_local, S = args.chains, args.num_steps
    n_total = n_local * world
    lo = rank * n_local

    def one_step(seed):
        x = model.sample_device(y, n_local, S, seed=seed, chain_offset=lo)
        if world > 1:
            x = parallel.gather_shards(x, n_total, dev)
        return x

    for i in range(args.warmup):
        one_step(1000 + i)
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    x_last = None
    for i in range(args.steps):
        ev[i][0].record(stream)
        x_last = model.sample_device(y, n_local, S, seed=i, chain_offset=lo) if world == 1 else one_step(i)
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    launch_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    ms_per_step = elapsed / args.steps * 1e3
    value = n_total * args.steps / elapsed
    flops_launch = flops_per_sample_step() * S * n_local
    achieved = flops_launch / (launch_ms * 1e-3) / 1e12
    line = {
        "metric": "posterior samples/sec (1000-step reverse SDE)",
        "value": value,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": f"synthetic y (reference seeded y_test[0]); weights {weights}",
        "config": {"workload": "scatterometry CDE posterior sampling (BASELINE configs[1])",
                   "xdim": XDIM, "ydim": YDIM, "hidden_layers": [WIDTH] * NH, "sde_steps": S,
                   "chains_per_gpu": n_local, "chains_total": n_total,
                   "parallelism": f"sample-parallel x{world}" + (" + RCCL all_gather" if world > 1 else ""),
                   "arith": "bf16 MFMA operands, fp32 accumulate; fp32 chain state / SDE update"},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / PEAK_BF16_TFLOPS, "traffic": pmc_traffic(),
                     "kernel": "em_sampler_kernel<256,3,3,8,4> (+a1_prep, inside the events)",
                     "launch_ms": launch_ms, "flops_per_launch": flops_launch},
    }
    if rank == 0:
        line["ks_vs_ref"] = ks_vs_reference(x_last.reshape(-1, XDIM).cpu().numpy(), S, weights)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(S, args.cpu_chains)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
