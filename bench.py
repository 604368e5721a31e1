"""Benchmark: posterior samples/s of the fused reverse-SDE sampler (BASELINE.json metric).

Default workload (BASELINE.json configs[1]): scatterometry CDE, MLP 27 -> [256]*3 -> 3 (tanh, double
tanh on layer 1), 1000 Euler-Maruyama steps, 100,000 chains per GPU for one y (y_test[0] of the
reference's seeded test set, tests/golden/data_scat.npz), weights = the fixture-trained checkpoint
(tests/golden/ckpt_scat.npz; random init if absent -- timing does not depend on the weights).
Headline arithmetic: the reference's fp32 (models/diffusion.py:38-42, nets.py:32-35), computed by the
fp32x3 engine (every product as three fp16 MFMAs, W_hi h_hi + W_hi h_lo + W_lo h_hi, fp32 accumulation;
at this shape the k-major multi-tile kernel of csrc/dmip_x3k.h). One "step" = one full sampling call (x0 draw + 1000 SDE steps + output in HBM). With
--gpus N the chains are sharded by global chain index (weak scaling: 100k chains per GPU) and the shards
are gathered to every rank with one RCCL all_gather inside the timed region.

Launch: `python bench.py --gpus N` starts N rank processes itself (one per GPU, RCCL over xGMI) when
it is not already running under torch.distributed.run; the parent never touches the GPU, polls its
children and terminates the others as soon as one fails.

Prints ONE JSON line on rank 0 (driver contract) with
  * `roofline`: MFMA-bound; algorithmic flops per launch / HIP-event-timed average launch, against the
    matrix pipe the kernel runs on (fp16 for fp32x3 -- `executed_frac` counts its three products);
  * `cpu_baseline`: reference-order torch-CPU sampler on a bounded sample (rank 0, N = 1 only);
  * `ks_vs_ref` / `w1_vs_ref` / `parity`: the timed run's samples against the reference sampler's own
    draws (tests/golden/samples_scat.npz: 20k draws and the 1001 quantiles of its 100k-chain run, same
    y and weights): per-dimension KS (alpha = 0.01), per-dimension and sliced W1 with their null levels;
  * `fast_mode`: the same workload on the 16-bit engine (fp16 hidden layers), `fp32_mode`: on the
    exact-f32 engine (v_mfma_f32_16x16x4_f32) -- each timed after the headline with its own parity report;
  * `dist`: the world size torch.distributed reports after init and every rank's device (PCI bus id).
Other workloads (not the headline): --workload cdiffe-pc (BASELINE config 3: CDiffE + 1 Langevin
corrector step, --chains-total 1000000 sharded over the ranks: strong scaling) and --workload dps
(config 4: DPS with surrogate guidance, --chains-total 262144; fp32x3 by default, --precision fp32 for the
exact-f32 kernel).
"""
import argparse
import datetime
import importlib
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "diffusion-modelling-for-inverse-problems_amd"

XDIM, YDIM, WIDTH, NH = 3, 23, 256, 3
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 / fp16 MFMA (MI355X_MICROARCH.md, no sparsity)
PEAK_F32_TFLOPS = 157.3    # MI355X f32 MFMA (= the f32 vector rate)


def flops_per_sample_step(in_dim=XDIM + YDIM + 1, w=WIDTH, nh=NH, out=XDIM):
    return 2 * (in_dim * w + (nh - 1) * w * w + w * out)


F_PRIOR = flops_per_sample_step(XDIM + 1, WIDTH, NH, XDIM)

# the headline workload's sampler kernel per precision (+ its per-y prep kernel, inside the HIP events)
KERNELS = {"fp32x3": "x3k_sampler_kernel<3,3,false> (+x3_bias_prep)",
           "fp16": "em_sampler_kernel<0,256,3,3,0,8,4,false> (+a1_prep)",
           "fp32": "f32_sampler_kernel<0,256,3,0,false> (+f32_l1_prep)"}
KERNEL_MATCH = {"fp32x3": "x3k_sampler_kernel", "fp16": "em_sampler_kernel", "fp32": "f32_sampler_kernel"}
ARITH = {
    "fp32x3": "fp32-accurate: every product as three fp16 MFMAs W_hi h_hi + W_hi h_lo + W_lo h_hi "
              "(v_mfma_f32_16x16x32_f16, fp32 accumulation; 2^-23.2 of sum|w h| per product vs 2^-23.0 for an fp32 "
              "fmaf chain, profiles/r3_mfma_f16_check.txt), tanh by exp2 + rcp (~1 ulp); fp32 chain state / SDE update",
    "fp16": "16-bit MFMA operands (layer 1: bf16 over split hi+lo inputs, ~fp32; hidden and output layers: fp16 "
            "weights and activations), fp32 accumulate; fp32 chain state / SDE update",
    "fp32": "exact f32 MFMA (v_mfma_f32_16x16x4_f32, an fmaf chain), libm tanh; fp32 chain state / SDE update"}
DTYPE = {"fp32x3": "fp32", "fp16": "fp16", "fp32": "fp32"}


def executed_flops_per_sample_step(precision, in_dim=XDIM + YDIM + 1, w=WIDTH, nh=NH, out=XDIM):
    """MFMA work the kernel issues per chain-step: fp32x3 runs every hidden/output product three times
    (layer 1 carries its split in the k-slots: 3 slots per input); the other engines one."""
    if precision != "fp32x3":
        return flops_per_sample_step(in_dim, w, nh, out)
    return 2 * (3 * (XDIM + 1) * w + 3 * ((nh - 1) * w * w + w * out))
F_SUR = 2 * (3 * 256 + 2 * 256 * 256 + 256 * 23)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="cde", choices=["cde", "cdiffe-pc", "dps"])
    ap.add_argument("--precision", default="fp32x3", choices=["fp32x3", "fp16", "bf16", "fp32"],
                    help="headline arithmetic (default: fp32x3, the reference's fp32 at the fp16 matrix rate)")
    ap.add_argument("--chains", type=int, default=100000, help="chains per GPU (weak scaling)")
    ap.add_argument("--chains-total", type=int, default=0, help="total chains over all GPUs (strong scaling)")
    ap.add_argument("--num-steps", type=int, default=1000, help="SDE steps per sample")
    ap.add_argument("--cpu-chains", type=int, default=16384)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fp32", action="store_true", help="skip the exact-f32 run beside the headline")
    ap.add_argument("--fp32-steps", type=int, default=2)
    ap.add_argument("--no-fast", action="store_true", help="skip the 16-bit engine run beside the headline")
    ap.add_argument("--fast-steps", type=int, default=3)
    ap.add_argument("--dist-timeout", type=float, default=900.0,
                    help="seconds before a blocked collective (a dead rank) fails the job")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="skip the one-GPU runs of BASELINE configs 3-5 and the reference width reported beside the headline")
    ap.add_argument("--master-port", type=int, default=29511)
    ap.add_argument("--stub", action="store_true", help=argparse.SUPPRESS)  # CPU/gloo launcher test only
    ap.add_argument("--stub-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)  # launcher fail-fast test
    a = ap.parse_args()
    if a.precision == "bf16":  # deprecated alias of the 16-bit sampler engine (its hidden layers are fp16)
        a.precision = "fp16"
    return a


# ------------------------------------------------------------------------------ launcher
def launch_ranks(args, poll_s=0.2):
    """Start args.gpus rank processes (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in their environment) and
    wait for them, polling: the first rank to exit non-zero gets its siblings terminated (they would
    otherwise block in a collective until the timeout). The parent initialises no GPU state. Exit
    status: the first failure's, else 0."""
    env0 = dict(os.environ)
    env0.setdefault("MASTER_ADDR", "127.0.0.1")
    env0.setdefault("MASTER_PORT", str(args.master_port))
    env0.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = []
    for r in range(args.gpus):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                sys.stderr.write(f"bench.py: rank {procs.index(p)} exited with {code}; terminating the other ranks\n")
                for q in live:
                    q.terminate()
                deadline = time.time() + 10
                for q in live:
                    try:
                        q.wait(timeout=max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                live = []
                break
        if live:
            time.sleep(poll_s)
    return rc


def init_dist(backend, dev, timeout_s):
    """init_process_group with a timeout (a dead rank fails the others instead of hanging them); the world
    size torch.distributed reports must equal WORLD_SIZE."""
    import torch.distributed as dist
    kw = {"timeout": datetime.timedelta(seconds=timeout_s)}
    if dev is not None:
        kw["device_id"] = dev
    dist.init_process_group(backend, **kw)
    world = dist.get_world_size()
    if world != int(os.environ["WORLD_SIZE"]):
        raise RuntimeError(f"torch.distributed world size {world} != WORLD_SIZE {os.environ['WORLD_SIZE']}")
    return world


def rank_devices(dist, world, dev):
    """Every rank's device as 'rank:pci_domain:bus:device name' (gathered), so the line records which
    GPUs ran the job."""
    import torch
    if dev is None:
        mine = f"{dist.get_rank() if world > 1 else 0}:cpu"
    else:
        pr = torch.cuda.get_device_properties(dev)
        mine = (f"{dist.get_rank() if world > 1 else 0}:{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:"
                f"{pr.pci_device_id:02x} {pr.name} {pr.gcnArchName}")
    if world == 1:
        return [mine]
    out = [None] * world
    dist.all_gather_object(out, mine)
    return out


# ------------------------------------------------------------------------------ workloads
def load_model(pkg, dev):
    import torch
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


def pmc_traffic(kernel_family="x3k_sampler_kernel"):
    """HBM bytes per launch of a sampler kernel family on this workload from the committed rocprofv3 PMC
    passes (profiles/pmc_traffic.json, written by scripts/pmc_traffic.py from separate FETCH_SIZE and
    WRITE_SIZE passes over this bench line, corrected per MI355X_MICROARCH.md §HBM), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    z = json.load(open(p)).get(kernel_family)
    return z["hbm_bytes_per_launch"] if z else None


def parity_vs_reference(metrics, x, num_steps, weights):
    """The timed run's samples against the reference sampler's own stored draws (tests/golden/
    samples_scat.npz: 20k draws of a 100k-chain run of the reference's models/diffusion.py:27-46 loop
    and that run's 1001 quantiles, same y and the same fixture weights). None when the weights or the
    step count differ from the fixture's."""
    p = os.path.join(ROOT, "tests", "golden", "samples_scat.npz")
    if not os.path.exists(p) or not weights.startswith("fixture"):
        return None
    z = np.load(p)
    if int(z["num_steps"]) != num_steps:
        return None
    return metrics.parity_report(x, z["samples"], z["quantiles"], int(z["n_total"]))


def ks_field(rep):
    if rep is None:
        return None
    k = rep["ks_draws"]
    return {"stat": k["stat"], "crit_alpha_0.01": k["crit"], "pass": bool(max(k["stat"]) < k["crit"]),
            "n_samples": rep["n"], "n_ref": rep["n_ref"],
            "vs_100k_quantiles": rep.get("ks_quantiles"),
            "ref": "reference sampler's own draws (tests/golden/samples_scat.npz, same y, same weights)"}


def w1_field(rep):
    if rep is None:
        return None
    return {"per_dim": rep["w1_draws"]["stat"], "per_dim_null": rep["w1_draws"]["null"],
            "sliced": rep["sliced_w1_draws"]["stat"], "sliced_null": rep["sliced_w1_draws"]["null"],
            "vs_100k_quantiles": rep.get("w1_quantiles"),
            "bound": "3x the expected W1 of two same-distribution samples of these sizes (metrics.w1_null)"}


def cpu_baseline(num_steps, n_chains):
    """Reference-order torch-CPU sampler (oracle/torch_cpu.py) on a bounded sample."""
    import torch
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


class Workload:
    """One sampling call per step on this rank's chain range [lo, hi) of n_total (+ the gather)."""

    def __init__(self, args, pkg, dev, rank, world):
        import torch
        par = importlib.import_module(PKG + ".parallel")
        self.args, self.dev, self.world = args, dev, world
        S = args.num_steps
        gold = os.path.join(ROOT, "tests", "golden")
        self.y = torch.from_numpy(synthetic_y()).to(dev)
        if args.chains_total > 0:
            self.n_total, self.scaling = args.chains_total, "strong"
        else:
            self.n_total, self.scaling = args.chains * world, "weak"
        self.lo, self.hi = par.shard_range(self.n_total, rank, world)
        self.n_local = self.hi - self.lo
        self.weights = "random-init"
        self.kw = {}
        if args.workload == "cde":
            self.model, self.weights = load_model(pkg, dev)
            self.flops_sample_step = flops_per_sample_step()
            self.peak = PEAK_F32_TFLOPS if args.precision == "fp32" else PEAK_BF16_TFLOPS
            self.kernel = KERNELS[args.precision]
            self.workload = "scatterometry CDE posterior sampling (BASELINE configs[1])"
            self.kw = {"precision": args.precision}
        elif args.workload == "cdiffe-pc":
            torch.manual_seed(0)
            self.model = pkg.CDiffE(XDIM, YDIM, [WIDTH] * NH)
            ck = os.path.join(gold, "ckpt_cdiffe_scat.npz")
            if os.path.exists(ck):  # trained by scripts/bench_posterior_e2e.py (joint DSM, fused), scored vs MCMC
                z = np.load(ck)
                self.model.sde.a.load_state_dict({k.replace("_", "."): torch.from_numpy(z[k]) for k in z.files
                                                  if k.split("_")[0].isdigit()})
                self.weights = "trained (tests/golden/ckpt_cdiffe_scat.npz: joint DSM on the device, profiles/r3_e2e_cdiffe_pc.json)"
            self.model.sde.a.to(dev)
            self.kw = {"corrector_steps": 1, "snr": 0.16, "precision": args.precision}
            self.flops_sample_step = 2 * flops_per_sample_step(XDIM + YDIM + 1, WIDTH, NH, XDIM + YDIM)
            self.peak = PEAK_F32_TFLOPS if args.precision == "fp32" else PEAK_BF16_TFLOPS
            self.kernel = {"fp32x3": "x3_sampler_kernel<2,256,3,23,false>", "fp16": "em_sampler_kernel<2,256,3,3,23,8,4,false>",
                           "fp32": "f32_sampler_kernel<2,256,3,23,false>"}[args.precision] + " (CDiffE + Langevin corrector)"
            self.workload = "scatterometry CDiffE predictor-corrector (BASELINE configs[2])"
        else:  # dps
            fm, prm = pkg.load_forward_model(gold)
            self.model = pkg.DPS(XDIM, YDIM, [WIDTH] * NH, fm.to(dev), prm)
            ck = os.path.join(gold, "ckpt_prior_scat.npz")
            if os.path.exists(ck):
                z = np.load(ck)
                self.model.prior_net.load_state_dict({k.replace("_", "."): torch.from_numpy(z[k]) for k in z.files
                                                      if k.split("_")[0].isdigit()})
                self.weights = "fixture-trained prior (tests/golden/ckpt_prior_scat.npz)"
            self.model.prior_net.to(dev)
            self.flops_sample_step = 2 * F_PRIOR + 2 * F_SUR
            dprec = "fp32" if args.precision == "fp32" else "fp32x3"
            self.kw = {"precision": dprec}
            self.peak = PEAK_F32_TFLOPS if dprec == "fp32" else PEAK_BF16_TFLOPS
            self.kernel = {"fp32": "dps_kernel (exact f32, forward tangents)",
                           "fp32x3": "dps_x3_kernel (split-fp16, reverse-mode J^T)"}[dprec]
            self.workload = "scatterometry DPS, surrogate guidance (BASELINE configs[3])"
        self.par = par

    def sample_local(self, seed, **over):
        kw = dict(self.kw, **over)
        return self.model.sample_device(self.y, self.n_local, self.args.num_steps, seed=seed, chain_offset=self.lo,
                                        **kw)

    def step(self, seed, **over):
        x = self.sample_local(seed, **over)
        if self.world > 1:
            x = self.par.gather_shards(x, self.n_total, self.dev)
        return x


def timed(wl, steps, dist, world, dev, seed0=0, **over):
    """barrier + sync, K steps (HIP events around each sampling call on its stream), sync + barrier;
    (elapsed max over ranks, mean launch ms, last output)."""
    import torch
    gpu = dev.type == "cuda"  # the CPU launcher test (--stub) times the stand-in with the host clock
    sync = torch.cuda.synchronize if gpu else (lambda: None)
    if gpu:
        stream = torch.cuda.current_stream(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    else:
        ev = [[0.0, 0.0] for _ in range(steps)]
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    x = None
    for i in range(steps):
        if gpu:
            ev[i][0].record(stream)
        else:
            ev[i][0] = time.perf_counter()
        x = wl.sample_local(seed0 + i, **over)
        if gpu:
            ev[i][1].record(stream)
        else:
            ev[i][1] = time.perf_counter()
        if world > 1:
            x = wl.par.gather_shards(x, wl.n_total, dev)
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    launch_ms = float(np.mean([a.elapsed_time(b) if gpu else (b - a) * 1e3 for a, b in ev]))
    return elapsed, launch_ms, x


def other_configs(args, pkg, lib, dev):
    """The other BASELINE configurations on this GPU, timed beside the headline so the driver observes
    them (each: one warm-up launch, then timed launches with HIP events): configs[2] CDiffE
    predictor-corrector (the per-GPU share of 1M chains over 8 GPUs), configs[3] DPS (256k samples),
    configs[4] the PINNLoss training step (whole step on the device), and the reference configs'
    own width [512]*3 for the CDE, the two-network Posterior and the CDiffE predictor-corrector samplers. Not the headline; errors are reported, not raised."""
    import copy
    import torch
    out = {}

    fam = {"fp32x3": "x3_sampler_kernel", "fp16": "em_sampler_kernel", "fp32": "f32_sampler_kernel"}

    def sampler(name, workload, chains, reps, precision, **kw):
        try:
            a = copy.copy(args)
            a.workload, a.chains, a.chains_total, a.precision = workload, chains, 0, precision
            for k, v in kw.items():
                setattr(a, k, v)
            wl = Workload(a, pkg, dev, 0, 1)
            mode = {"cde": 0, "cdiffe-pc": 2}.get(workload)
            if workload == "cde" and kw.get("width"):
                torch.manual_seed(0)
                W = kw["width"]
                if kw.get("posterior"):  # two networks: likelihood (x, y, t) + prior (x, t)
                    wl.model = pkg.PosteriorDiffusionEstimator(XDIM, YDIM, [W] * NH)
                    wl.flops_sample_step = flops_per_sample_step(w=W) + flops_per_sample_step(XDIM + 1, W, NH, XDIM)
                    wl.workload, mode = "PosteriorDiffusionEstimator at the reference width", 1
                else:
                    wl.model = pkg.CDE(XDIM, YDIM, [W] * NH)
                    wl.flops_sample_step = flops_per_sample_step(w=W)
                    wl.workload = "CDE at the reference width"
                wl.model.sde.a.to(dev)
                wl.weights = "random-init"
            W = kw.get("width", WIDTH)
            if workload == "cdiffe-pc" and kw.get("width"):
                torch.manual_seed(0)
                wl.model = pkg.CDiffE(XDIM, YDIM, [W] * NH)
                wl.model.sde.a.to(dev)
                wl.flops_sample_step = 2 * flops_per_sample_step(XDIM + YDIM + 1, W, NH, XDIM + YDIM)
                wl.workload = "CDiffE predictor-corrector at the reference width"
                wl.weights = "random-init"
            if workload != "dps":
                wl.kernel = f"{fam[precision]}<{mode},{W},...>"
            wl.peak = PEAK_F32_TFLOPS if precision == "fp32" else PEAK_BF16_TFLOPS
            wl.step(3000)
            el, lm, x = timed(wl, reps, None, 1, dev, seed0=3100)
            lib.device_status(dev)
            ach = wl.flops_sample_step * a.num_steps * wl.n_local / (lm * 1e-3) / 1e12
            out[name] = {"workload": wl.workload, "chains": wl.n_local, "sde_steps": a.num_steps,
                         "precision": precision, "value": wl.n_local * reps / el,
                         "unit": "samples/s", "launch_ms": lm,
                         "roofline": {"achieved": ach, "peak": wl.peak, "unit": "TFLOP/s", "frac": ach / wl.peak},
                         "kernel": wl.kernel, "weights": wl.weights, "finite": bool(torch.isfinite(x).all())}
        except Exception as e:  # noqa: BLE001 -- reported in the line, never fatal to the headline
            out[name] = {"error": f"{type(e).__name__}: {e}"}

    try:  # configs[0]: the reference's own sampling call (main_diffusion_linear.py:74), host result included
        zl = np.load(os.path.join(ROOT, "tests", "golden", "ckpt_lin.npz"))
        ml = pkg.CDE(2, 2, [64] * 3)
        ml.sde.a.load_state_dict({k.replace("_", "."): torch.from_numpy(zl[k]) for k in zl.files
                                  if k.split("_")[0].isdigit()})
        ml.sde.a.to(dev)
        yl = torch.tensor([0.5, 1.0])
        ts = []
        for r in range(9):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            xs = ml(yl, num_samples=1000, num_steps=200)  # returns the host ndarray: D2H inside
            ts.append(time.perf_counter() - t0)
        med = float(np.median(ts[2:]))
        out["config1_linear"] = {
            "workload": "linear CDE [64]*3 (fixture weights), model(y, num_samples=1000, num_steps=200) -- "
                        "main_diffusion_linear.py:74, default precision fp32x3, host ndarray returned (D2H included)",
            "value": 1000 / med, "unit": "samples/s", "latency_ms_median_of_7": med * 1e3,
            "latency_ms_min": min(ts[2:]) * 1e3, "cpu_reference_samples_per_s": 13400.0,
            "cpu_reference": "BASELINE.md configs[0]: 0.075 s median of 5, 8-core Xeon, reference CPU torch",
            "vs_cpu_reference": (1000 / med) / 13400.0, "finite": bool(np.all(np.isfinite(xs)))}
    except Exception as e:  # noqa: BLE001
        out["config1_linear"] = {"error": f"{type(e).__name__}: {e}"}
    sampler("config3_cdiffe_pc_per_gpu", "cdiffe-pc", 125000, 2, "fp32x3")
    sampler("config3_cdiffe_pc_per_gpu_fast", "cdiffe-pc", 125000, 2, "fp16")
    sampler("config4_dps", "dps", 262144, 1, "fp32x3")
    sampler("config4_dps_exact_f32", "dps", 262144, 1, "fp32")
    sampler("cde_reference_width_512", "cde", 100000, 2, "fp32x3", width=512)
    sampler("posterior_reference_width_512", "cde", 100000, 1, "fp32x3", width=512, posterior=True)
    # CDiffE scatterometry at width 512: fp32x3 with its 96 KiB split layer 1 streamed through the ring (L1R)
    sampler("cdiffe_pc_reference_width_512", "cdiffe-pc", 100000, 1, "fp32x3", width=512)
    sampler("cdiffe_pc_reference_width_512_fast", "cdiffe-pc", 100000, 1, "fp16", width=512)
    try:
        tr = importlib.import_module(PKG + ".training")
        torch.manual_seed(0)
        prob = pkg.LinearForwardProblem()
        lf = pkg.PINNLoss(prob.score_posterior, lam=1e-3, lam2=0.1, pde_loss="FPE", ic_metric="L2", pde_metric="L1")
        m = pkg.CDE(2, 2, [64] * 3)
        B = 65536
        xb = torch.randn(B, 2, device=dev)
        yb = xb @ prob.A.to(dev).T + prob.b.to(dev) + 0.3 * torch.randn(B, 2, device=dev)
        opt = torch.optim.Adam(m.sde.a.parameters(), lr=1e-4)
        step = tr.DeviceTrainStep(m, lf, opt, precision="bf16")
        for _ in range(3):
            step(xb, yb)
        st = torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(st)
        K = 20
        for _ in range(K):
            out_loss = step(xb, yb)
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / K
        F = 2 * (5 * 64 + 2 * 64 * 64 + 64 * 2)
        ach = 16.94 * F * B / (ms * 1e-3) / 1e12
        out["config5_pinn_train_step"] = {
            "workload": "PINNLoss train step, linear CDE [64]*3, batch 65536: t/eps draws + fused loss/grad + Adam",
            "value": B / (ms * 1e-3), "unit": "samples/s", "ms_per_step": ms,
            "roofline": {"achieved": ach, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": ach / PEAK_BF16_TFLOPS},
            "loss_finite": bool(torch.isfinite(out_loss).all())}
        try:
            out["config5_pinn_train_step"]["loss_vs_ref"] = config5_loss_check(tr, m, lf, prob, B, dev)
        except Exception as e:  # noqa: BLE001
            out["config5_pinn_train_step"]["loss_vs_ref"] = {"error": f"{type(e).__name__}: {e}"}
    except Exception as e:  # noqa: BLE001
        out["config5_pinn_train_step"] = {"error": f"{type(e).__name__}: {e}"}
    return out


def config5_loss_check(tr, m, lf, prob, B, dev):
    """BASELINE configs[4]'s loss-vs-ref tolerance check at its own batch: on one seeded batch (x, y, t,
    eps of the timed shape) the timed bf16 kernel's PINNLoss value and all 8 gradient tensors against the
    exact-f32 engine (dmip_loss_grad_f32), which reproduces the reference's own loss and gradients
    (losses.py:214-242) to <= 3e-6 (tests/test_gpu_train_f32.py, fixtures G5/G11). Bounds: those of
    tests/test_gpu_parity.py::test_config5_loss_grad_at_batch_65536_vs_oracle (loss 2e-5, gradients 6e-3)."""
    import torch
    g = torch.Generator().manual_seed(2024)
    x = torch.randn(B, 2, generator=g)
    y = x @ prob.A.T + prob.b + 0.3 * torch.randn(B, 2, generator=g)
    t = 1e-4 + torch.rand(B, 1, generator=g) * (1 - 1e-4)
    eps = torch.randn(B, 2, generator=g)
    args = [a.to(dev) for a in (x, y, t, eps)]
    cfg = tr.fused_config(m, lf)
    res = {}
    for prec in ("bf16", "fp32"):
        loss, _ = tr.fused_loss_grad(m, lf, cfg, *args, precision=prec)
        res[prec] = (float(loss), [p.grad.detach().double().clone() for p in m.sde.a.parameters()])
    (lb, gb), (lr, gr) = res["bf16"], res["fp32"]
    lrel = abs(lb - lr) / max(abs(lr), 1e-30)
    grel = max(float((a - b).norm() / max(float(b.norm()), 1e-30)) for a, b in zip(gb, gr))
    return {"loss": lb, "loss_ref": lr, "loss_rel": lrel, "max_grad_rel_l2": grel,
            "bound": {"loss_rel": 2e-5, "grad_rel_l2": 6e-3}, "pass": lrel < 2e-5 and grel < 6e-3,
            "ref": "exact-f32 engine on the same batch (pinned to the reference's loss/gradients, G5/G11, <= 3e-6)"}


def side_mode(wl, args, dist, world, dev, lib, metrics, precision, steps, S, flops_launch):
    """The headline workload on another engine, timed beside the headline (not the headline)."""
    wl.step(2000, precision=precision)
    el, lm, x = timed(wl, steps, dist, world, dev, seed0=100, precision=precision)
    lib.device_status(dev)
    if dist is not None and world > 1 and dist.get_rank() != 0:
        return None
    peak = PEAK_F32_TFLOPS if precision == "fp32" else PEAK_BF16_TFLOPS
    a = flops_launch / (lm * 1e-3) / 1e12
    rep = parity_vs_reference(metrics, x.reshape(-1, XDIM).cpu().numpy(), S, wl.weights)
    return {"precision": precision, "dtype": DTYPE[precision], "arith": ARITH[precision],
            "value": wl.n_total * steps / el, "unit": "samples/s", "steps": steps,
            "ms_per_step": el / steps * 1e3, "launch_ms": lm, "kernel": KERNELS[precision],
            "roofline": {"bound": "mfma", "achieved": a, "peak": peak, "unit": "TFLOP/s", "frac": a / peak,
                         "traffic": pmc_traffic(KERNEL_MATCH[precision])},
            "ks_vs_ref": ks_field(rep), "w1_vs_ref": w1_field(rep), "parity": {"pass": rep["pass"]} if rep else None}


def main_worker(args):
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.stub:  # CPU / gloo launcher test: the real line with a chain-keyed stand-in for the sampler
        dev = torch.device("cpu")
        if world > 1:
            world = init_dist("gloo", None, args.dist_timeout)
        devices = rank_devices(dist, world, None)
        if rank == args.stub_fail_rank:
            sys.stderr.write(f"stub rank {rank}: failing on purpose\n")
            return 1
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if world > 1:
            world = init_dist("nccl", dev, args.dist_timeout)
        devices = rank_devices(dist, world, dev)
    pkg = importlib.import_module(PKG)
    lib = importlib.import_module(PKG + "._lib")
    metrics = importlib.import_module(PKG + ".metrics")
    wl = Workload(args, pkg, dev, rank, world)
    if args.stub:
        wl.sample_local = stub_sampler(wl)
    S = args.num_steps

    for i in range(args.warmup):
        wl.step(1000 + i)
    if not args.stub:
        torch.cuda.synchronize()
    elapsed, launch_ms, x_last = timed(wl, args.steps, dist, world, dev)
    if not args.stub:
        lib.device_status(dev)  # no asynchronous kernel failure in the timed region

    ms_per_step = elapsed / args.steps * 1e3
    value = wl.n_total * args.steps / elapsed
    flops_launch = wl.flops_sample_step * S * wl.n_local
    achieved = flops_launch / (launch_ms * 1e-3) / 1e12
    prec = args.precision if args.workload != "dps" else "fp32"
    dtype = DTYPE[prec]
    roof = {"bound": "mfma", "achieved": achieved, "peak": wl.peak, "unit": "TFLOP/s", "frac": achieved / wl.peak,
            "traffic": pmc_traffic(KERNEL_MATCH[prec]) if args.workload == "cde" else None,
            "kernel": wl.kernel, "launch_ms": launch_ms, "flops_per_launch": flops_launch}
    if args.workload == "cde" and prec == "fp32x3":
        ex = executed_flops_per_sample_step("fp32x3") * S * wl.n_local / (launch_ms * 1e-3) / 1e12
        roof.update({"pipe": "v_mfma_f32_16x16x32_f16 (2500 TFLOP/s dense); three products per fp32 product",
                     "executed_tflops": ex, "executed_frac": ex / wl.peak,
                     "vs_f32_mfma_peak": achieved / PEAK_F32_TFLOPS})
    line = {
        "metric": "posterior samples/sec (1000-step reverse SDE)",
        "value": value,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": wl.scaling,
        "vs_baseline": None,
        "dtype": dtype,
        "data": f"synthetic y (reference seeded y_test[0]); weights {wl.weights}",
        "config": {"workload": wl.workload, "xdim": XDIM, "ydim": YDIM, "hidden_layers": [WIDTH] * NH,
                   "sde_steps": S, "chains_per_gpu": wl.n_local, "chains_total": wl.n_total,
                   "parallelism": f"sample-parallel x{world}" + (" + RCCL all_gather" if world > 1 else ""),
                   "precision": prec, "arith": ARITH[prec]},
        "roofline": roof,
        "dist": {"world_size_observed": world, "backend": "nccl (RCCL)" if world > 1 else None,
                 "devices": devices},
    }
    if args.stub:
        line["stub"] = stub_check(wl, x_last)
        if world > 1:
            dist.barrier()
        if rank == 0:
            print(json.dumps(line), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return 0 if line["stub"]["gather_ok"] else 1
    rep = None
    if args.workload == "cde" and rank == 0:
        rep = parity_vs_reference(metrics, x_last.reshape(-1, XDIM).cpu().numpy(), S, wl.weights)
        line["ks_vs_ref"] = ks_field(rep)
        line["w1_vs_ref"] = w1_field(rep)
        line["parity"] = {"pass": rep["pass"]} if rep else None
    if args.workload == "cde" and prec != "fp16" and not args.no_fast:
        line["fast_mode"] = side_mode(wl, args, dist, world, dev, lib, metrics, "fp16", args.fast_steps, S, flops_launch)
    if args.workload == "cde" and prec != "fp32" and not args.no_fp32:
        line["fp32_mode"] = side_mode(wl, args, dist, world, dev, lib, metrics, "fp32", args.fp32_steps, S, flops_launch)
    if rank == 0 and world == 1 and args.workload == "cde" and not args.no_other_configs:
        line["other_configs"] = other_configs(args, pkg, lib, dev)
    if rank == 0 and world == 1 and args.workload == "cde" and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(S, args.cpu_chains)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def stub_sampler(wl):
    """The launcher test's stand-in for the fused sampler (--stub, CPU): x[c] = (c, seed mod 997, lo) for the rank's
    global chains c in [lo, hi) -- a pure function of (seed, global chain index), the property the HIP kernels keep
    (chain-keyed RNG), plus the producing rank's range start, so the gathered union shows who produced what."""
    import torch

    def sample_local(seed, **over):
        c = torch.arange(wl.lo, wl.hi, dtype=torch.float32)
        return torch.stack([c, c * 0 + float(seed % 997), c * 0 + float(wl.lo)], dim=1)[None].contiguous()
    return sample_local


def stub_check(wl, x):
    """Every chain exactly once, in global order, each from the rank whose shard_range holds it."""
    import torch
    n = wl.n_total
    lo_of = torch.tensor([float(wl.par.shard_range(n, r, wl.world)[0]) for r in range(wl.world)
                          for _ in range(*wl.par.shard_range(n, r, wl.world))])
    ok = (tuple(x.shape) == (1, n, XDIM) and torch.equal(x[0, :, 0], torch.arange(n, dtype=torch.float32))
          and torch.equal(x[0, :, 2], lo_of) and bool((x[0, :, 1] == x[0, 0, 1]).all()))
    return {"gathered_shape": list(x.shape), "gather_ok": bool(ok), "chains_total": n,
            "rank0_chains": wl.n_local}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; run it as `python bench.py --gpus N` "
                 "or under torch.distributed.run with --nproc-per-node N")
    sys.exit(main_worker(args))


if __name__ == "__main__":
    main()
