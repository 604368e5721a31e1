"""The fp32-accurate split-fp16 sampler (DMIP_PREC_F32X3, csrc/dmip_x3.h) -- the package's default
precision -- against the reference's own trajectories and draws, the oracle, and the exact-f32 engine.
Every test here needs an MI355X: run with `pytest -m gpu`.

The engine claims the reference's fp32 arithmetic, so it is held to the exact-f32 engine's gates
(test_gpu_f32.py), not the 16-bit engine's:
  * injected-noise trajectories (fixture G3, the reference's own x0 and per-step noise): final samples
    within 1e-3 max|x| after all steps (1e-4 for the short runs) -- the oracle's own bound;
  * product-RNG samplers vs the float32 oracle (same chains): 1e-4 max(1, |x|) after 6 steps;
  * posteriors at 100k samples vs the reference's draws: KS (alpha = 0.01) against the 20k draws and the
    100k-run quantiles, per-dimension and sliced W1 <= 3x the null level (metrics.parity_report);
  * against the exact-f32 engine on the same chains over 1000 steps: the two fp32 engines agree to
    within the G3 bound too.
Observed values are printed (pytest -s) and recorded in DESIGN.md §3c.
"""
import importlib

import numpy as np
import pytest
import torch

import oracle as O
from conftest import state_from_npz

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
PREC = "fp32x3"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _cde(dmip, tag, z):
    xd, yd, hl = {"lin": (2, 2, [64] * 3), "scat": (3, 23, [256] * 3)}[tag]
    m = dmip.CDE(xd, yd, hl)
    m.sde.a.load_state_dict(state_from_npz(z))
    return m


def _linear_params(net):
    return [(l.weight.detach().cpu().numpy(), l.bias.detach().cpu().numpy())
            for l in net if isinstance(l, torch.nn.Linear)]


def _rel(out, ref):
    return float(np.abs(out - ref).max() / max(1.0, np.abs(ref).max()))


def test_default_precision_is_fp32x3(dmip):
    m = dmip.CDE(3, 23, [256] * 3)
    assert m.precision == PREC
    assert dmip._lib.sampler_supported(256, 3, 3, 23, dmip._lib.DMIP_SAMPLER_CDE, PREC)


# ------------------------------------------------------------- injected-noise trajectories (A2)
@pytest.mark.parametrize("tag", ["lin", "scat"])
def test_x3_trajectory_injected_noise_matches_reference(dmip, golden, tag):
    """The reference's own x0 and per-step noise (G3) through the fused f32x3 sampler."""
    tr = golden(f"traj_{tag}.npz")
    m = _cde(dmip, tag, golden(f"ckpt_{tag}.npz"))
    S = int(tr["num_steps"])
    noise = np.concatenate([tr["x0"][None], tr["xi"]], 0)[:, None]
    n = tr["x0"].shape[0]
    before = dmip._lib.calls["em_sample"]
    out = m.sample_device(torch.from_numpy(tr["y"]).to(DEV), n, S, noise=torch.from_numpy(noise).to(DEV),
                          precision=PREC)[0].cpu().numpy()
    assert dmip._lib.calls["em_sample"] == before + 1
    ref = tr["x_final"]
    assert np.all(np.isfinite(out))
    err = _rel(out, ref)
    print(f"\n[x3] G3 {tag}: {S} steps, max err / max|x| = {err:.3e}")
    assert err < 1e-3, err
    Ss = int(tr["steps_short"])
    ns = np.concatenate([tr["x0_short"][None], tr["xi_short"]], 0)[:, None]
    out_s = m.sample_device(torch.from_numpy(tr["y"]).to(DEV), n, Ss, noise=torch.from_numpy(ns).to(DEV),
                            precision=PREC)[0].cpu().numpy()
    err_s = _rel(out_s, tr["x_final_short"])
    print(f"[x3] G3 {tag}: {Ss} steps, max err / max|x| = {err_s:.3e}")
    assert err_s < 1e-4, err_s


# ------------------------------------------------------------------- product-RNG samplers vs the oracle
@pytest.mark.parametrize("W", [64, 128, 256, 512])
@pytest.mark.parametrize("NL", [1, 2, 3])
@pytest.mark.parametrize("xd,yd", [(2, 2), (3, 23)])
def test_x3_cde_sampler_vs_oracle(dmip, W, NL, xd, yd):
    torch.manual_seed(W + NL + xd)
    m = dmip.CDE(xd, yd, [W] * NL)
    params = _linear_params(m.sde.a)
    y = np.random.default_rng(5).uniform(0, 1, yd).astype(np.float32)
    n, S, seed = 700, 6, 99
    x = m.sample_device(torch.from_numpy(y).to(DEV), n, S, seed=seed, precision=PREC)[0].cpu().numpy()
    ref = O.cde_sample(params, y, n, S, seed)
    err = _rel(x, ref)
    print(f"\n[x3] CDE W={W} L={NL} x{xd}: {err:.3e}")
    assert err < 1e-4, err


@pytest.mark.parametrize("W", [64, 256, 512])
@pytest.mark.parametrize("NL", [2, 3])
@pytest.mark.parametrize("xd,yd", [(2, 2), (3, 23)])
def test_x3_posterior_sampler_vs_oracle(dmip, W, NL, xd, yd):
    torch.manual_seed(W + xd + NL)
    m = dmip.PosteriorDiffusionEstimator(xd, yd, [W] * NL)
    prior, lik = _linear_params(m.sde.a.prior_net), _linear_params(m.sde.a.likelihood_net)
    y = np.random.default_rng(7).uniform(0, 1, yd).astype(np.float32)
    n, S, seed = 700, 6, 31
    before = dmip._lib.calls["em_sample_posterior"]
    x = m.sample_device(torch.from_numpy(y).to(DEV), n, S, seed=seed, precision=PREC)[0].cpu().numpy()
    assert dmip._lib.calls["em_sample_posterior"] == before + 1
    ref = O.posterior_sample(prior, lik, y, n, S, seed)
    err = _rel(x, ref)
    print(f"\n[x3] Posterior W={W} L={NL} x{xd}: {err:.3e}")
    assert err < 1e-4, err


@pytest.mark.parametrize("W,xd,yd", [(64, 2, 2), (256, 2, 2), (512, 2, 2), (64, 3, 23), (128, 3, 23), (256, 3, 23),
                                     (512, 3, 23)])
def test_x3_cdiffe_sampler_vs_oracle(dmip, W, xd, yd):
    torch.manual_seed(3 * W + xd)
    m = dmip.CDiffE(xd, yd, [W] * 3)
    params = _linear_params(m.sde.a)
    y = np.random.default_rng(8).uniform(0, 1, yd).astype(np.float32)
    n, S, seed = 700, 6, 57
    before = dmip._lib.calls["em_sample_cdiffe"]
    x = m.sample_device(torch.from_numpy(y).to(DEV), n, S, seed=seed, precision=PREC)[0].cpu().numpy()
    assert dmip._lib.calls["em_sample_cdiffe"] == before + 1
    ref = O.cdiffe_sample(params, y, n, S, seed)
    err = _rel(x, ref)
    print(f"\n[x3] CDiffE W={W} x{xd}: {err:.3e}")
    assert err < 1e-4, err


@pytest.mark.parametrize("W", [256, 512])
def test_x3_cdiffe_predictor_corrector_vs_oracle(dmip, W):
    torch.manual_seed(11)
    m = dmip.CDiffE(3, 23, [W] * 3)
    with torch.no_grad():
        last = [l for l in m.sde.a if isinstance(l, torch.nn.Linear)][-1]
        last.weight.mul_(0.05)
        last.bias.fill_(0.5)
    params = _linear_params(m.sde.a)
    y = np.random.default_rng(8).uniform(0, 1, 23).astype(np.float32)
    n, S, seed = 700, 5, 77
    x = m.sample_device(torch.from_numpy(y).to(DEV), n, S, seed=seed, corrector_steps=2, snr=0.16,
                        precision=PREC)[0].cpu().numpy()
    ref = O.cdiffe_sample(params, y, n, S, seed, corrector_steps=2, snr=0.16)
    x0 = O.cdiffe_sample(params, y, n, S, seed)
    assert np.abs(ref - x0).max() > 1e-2  # the corrector moves the chains
    err = _rel(x, ref)
    print(f"\n[x3] CDiffE PC W={W}: {err:.3e}")
    assert err < 1e-4, err


def test_x3_cdiffe_scat_width512_runs_fp32x3(dmip):
    """CDiffE scatterometry at the reference width 512: its 96 KiB split layer 1 streams through the weight ring
    (dmip_x3.h L1R), so a fp32x3 request runs the fp32x3 kernel (before round 4: the exact-f32 one)."""
    est = __import__("importlib").import_module("diffusion-modelling-for-inverse-problems_amd.estimators")
    assert dmip._lib.sampler_supported(512, 3, 3, 23, dmip._lib.DMIP_SAMPLER_CDIFFE, PREC)
    assert est._fused_precision(PREC, dmip._lib.DMIP_SAMPLER_CDIFFE, 512, 3, 3, 23) == PREC


# ------------------------------------------------------- the width-64 latency engine (dmip_x3s.h, round 6)
@pytest.mark.parametrize("NL", [1, 2, 3])
@pytest.mark.parametrize("xd,yd", [(2, 2), (3, 23)])
def test_x3_latency_engine_bit_identical_to_one_tile_engine(dmip, monkeypatch, NL, xd, yd):
    """Small CDE launches at width 64 run one tile per four-wave workgroup (dmip_x3s.h); every value is formed as in
    the one-tile engine, so the samples, a sharded run and the snapshots are bit-identical to it (DMIP_X3_SPLIT=0)."""
    torch.manual_seed(64 + NL + xd)
    m = dmip.CDE(xd, yd, [64] * NL)
    ys = torch.from_numpy(np.random.default_rng(NL).uniform(0, 1, (2, yd)).astype(np.float32)).to(DEV)
    n, S, seed = 1000, 40, 21
    a = m.sample_device(ys, n, S, seed=seed, precision=PREC)
    xa, sa = m.sample_trajectory(ys, 333, S, 8, seed=seed, chain_offset=101, precision=PREC)
    monkeypatch.setenv("DMIP_X3_SPLIT", "0")
    b = m.sample_device(ys, n, S, seed=seed, precision=PREC)
    xb, sb = m.sample_trajectory(ys, 333, S, 8, seed=seed, chain_offset=101, precision=PREC)
    monkeypatch.delenv("DMIP_X3_SPLIT")
    assert torch.isfinite(a).all()
    assert torch.equal(a, b)
    assert torch.equal(xa, xb) and torch.equal(sa, sb)
    assert torch.equal(xa, a[:, 101:434])


@pytest.mark.parametrize("n", [1, 17, 16 * 1024, 16 * 1024 + 1])
def test_x3_latency_engine_ragged_and_threshold_counts(dmip, monkeypatch, n):
    """Ragged tiles (1 and 17 chains) and the engine threshold (1,024 tiles run on the latency engine, one chain more
    on the one-tile engine): every count gives the one-tile engine's samples bit for bit."""
    torch.manual_seed(5)
    m = dmip.CDE(2, 2, [64] * 3)
    y = torch.tensor([0.3, 0.7], device=DEV)
    a = m.sample_device(y, n, 12, seed=3, precision=PREC)
    monkeypatch.setenv("DMIP_X3_SPLIT", "0")
    b = m.sample_device(y, n, 12, seed=3, precision=PREC)
    monkeypatch.delenv("DMIP_X3_SPLIT")
    assert torch.isfinite(a).all() and torch.equal(a, b)


def test_x3_latency_engine_injected_noise_bit_identical(dmip, golden, monkeypatch):
    """The reference's own x0 and per-step noise (G3, linear fixture) through both width-64 engines."""
    tr = golden("traj_lin.npz")
    m = _cde(dmip, "lin", golden("ckpt_lin.npz"))
    S = int(tr["num_steps"])
    noise = torch.from_numpy(np.concatenate([tr["x0"][None], tr["xi"]], 0)[:, None]).to(DEV)
    n = tr["x0"].shape[0]
    y = torch.from_numpy(tr["y"]).to(DEV)
    a = m.sample_device(y, n, S, noise=noise, precision=PREC)
    monkeypatch.setenv("DMIP_X3_SPLIT", "0")
    b = m.sample_device(y, n, S, noise=noise, precision=PREC)
    monkeypatch.delenv("DMIP_X3_SPLIT")
    assert torch.equal(a, b)
    print(f"\n[x3s] G3 lin through the latency engine: {n} chains, max err / max|x| = "
          f"{_rel(a[0].cpu().numpy(), tr['x_final']):.3e}")


# ------------------------------------------------------- the two fp32 engines over a long trajectory
@pytest.mark.parametrize("tag", ["lin", "scat"])
def test_x3_matches_exact_f32_engine_over_1000_steps(dmip, golden, tag):
    """Same chains (same RNG stream), 1000 steps, trained fixture weights: f32x3 vs exact f32."""
    m = _cde(dmip, tag, golden(f"ckpt_{tag}.npz"))
    y = torch.from_numpy(golden(f"samples_{tag}.npz")["y"]).to(DEV)
    a = m.sample_device(y, 20000, 1000, seed=123, precision=PREC)[0].cpu().numpy()
    b = m.sample_device(y, 20000, 1000, seed=123, precision="fp32")[0].cpu().numpy()
    err = _rel(a, b)
    q = np.quantile(np.abs(a - b).max(1), [0.5, 0.99])
    print(f"\n[x3] vs exact f32, {tag}, 1000 steps: max {err:.3e}, per-chain median {q[0]:.2e}, p99 {q[1]:.2e}")
    assert err < 1e-3, err


# ------------------------------------------------------------------- sharding / schedule / snapshots
@pytest.mark.parametrize("cls", ["CDE", "PosteriorDiffusionEstimator", "CDiffE"])
def test_x3_shards_and_batches_bit_identical(dmip, cls):
    torch.manual_seed(13)
    m = getattr(dmip, cls)(3, 23, [256] * 3)
    ys = torch.from_numpy(np.random.default_rng(9).uniform(0, 1, (3, 23)).astype(np.float32)).to(DEV)
    n, S, seed = 1000, 10, 5
    full = m.sample_device(ys, n, S, seed=seed, precision=PREC)
    shard = m.sample_device(ys, 300, S, seed=seed, chain_offset=500, precision=PREC)
    assert torch.equal(full[:, 500:800], shard)
    assert torch.equal(m.sample_device(ys, n, S, seed=seed, precision=PREC), full)
    assert not torch.equal(full[0], full[1])


@pytest.mark.parametrize("cls,W,n", [("CDE", 256, 70001), ("CDE", 512, 40001), ("PosteriorDiffusionEstimator", 256, 70001),
                                     ("CDiffE", 256, 70001), ("CDiffE", 512, 40001)])
def test_x3_balanced_schedule_matches_unsplit_runs(dmip, cls, W, n):
    """More chains than one GPU round: tiles split between waves through the balanced schedule; every
    chain equals a launch small enough to run each tile whole."""
    torch.manual_seed(W + n)
    m = getattr(dmip, cls)(3, 23, [W] * 3)
    y = torch.from_numpy(np.random.default_rng(5).uniform(0, 1, 23).astype(np.float32)).to(DEV)
    S = 6
    full = m.sample_device(y, n, S, seed=11, precision=PREC)[0]
    for lo in (0, n // 2 + 5, n - 333):
        part = m.sample_device(y, 333, S, seed=11, chain_offset=lo, precision=PREC)[0]
        assert torch.equal(full[lo:lo + 333], part), lo
    assert torch.isfinite(full).all()


def test_x3_handover_timeout_is_reported_not_silent(dmip, golden, monkeypatch):
    m = _cde(dmip, "scat", golden("ckpt_scat.npz"))
    y = torch.from_numpy(golden("data_scat.npz")["y_test"][0]).to(DEV)
    monkeypatch.setenv("DMIP_DEBUG_NO_HANDOVER", "1")
    # more jobs than the grid has waves (the paired engine's 64-chain jobs: > 65,536 chains), so tiles are handed over
    x = m.sample_device(y, 100000, 4, seed=1, precision=PREC)
    with pytest.raises(RuntimeError, match="hand-over"):
        dmip._lib.device_status(x.device)
    assert torch.isnan(x).any() and torch.isfinite(x).any()
    monkeypatch.delenv("DMIP_DEBUG_NO_HANDOVER")
    x = m.sample_device(y, 100000, 4, seed=1, precision=PREC)
    dmip._lib.device_status(x.device)
    assert torch.isfinite(x).all()


@pytest.mark.parametrize("cls", ["CDE", "PosteriorDiffusionEstimator", "CDiffE"])
def test_x3_snapshots(dmip, cls):
    """Trajectory snapshots through the balanced schedule: last snapshot = output = plain sampler, and a
    shard's snapshots are slices of the whole run's; CDE's snapshots against the oracle's loop states."""
    xd, yd = (3, 23) if cls != "CDiffE" else (2, 2)
    torch.manual_seed(1)
    m = getattr(dmip, cls)(xd, yd, [64] * 3)
    y = torch.from_numpy(np.random.default_rng(2).uniform(0, 1, (2, yd)).astype(np.float32)).to(DEV)
    n, S, every, seed = 90000, 40, 8, 7
    x, snaps = m.sample_trajectory(y, n, S, every, seed=seed, precision=PREC)
    assert tuple(snaps.shape) == (S // every, 2, n, xd)
    assert torch.equal(snaps[-1], x) and torch.isfinite(snaps).all()
    assert torch.equal(m.sample_device(y, n, S, seed=seed, precision=PREC), x)
    lo, hi = 30011, 61000
    xs, ss = m.sample_trajectory(y, hi - lo, S, every, seed=seed, chain_offset=lo, precision=PREC)
    assert torch.equal(ss, snaps[:, :, lo:hi]) and torch.equal(xs, x[:, lo:hi])
    if cls == "CDE":
        params = _linear_params(m.sde.a)
        yy = y[0].cpu().numpy()
        xs1, sn1 = m.sample_trajectory(y[:1], 700, 6, 2, seed=99, precision=PREC)
        _, ref_snaps = O.cde_sample(params, yy, 700, 6, 99, snapshots={2, 4, 6})
        for k in range(3):
            r = ref_snaps[(k + 1) * 2]
            assert _rel(sn1[k, 0].cpu().numpy(), r) < 1e-4


# ---------------------------------------------- distributional parity vs the reference (§8c)
@pytest.mark.parametrize("tag", ["lin", "scat"])
def test_x3_posterior_parity_fp32_gate(dmip, golden, tag):
    """100k samples against the reference sampler's draws on the same weights and y: the fp32 gate."""
    import importlib
    M = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.metrics")
    smp = golden(f"samples_{tag}.npz")
    m = _cde(dmip, tag, golden(f"ckpt_{tag}.npz"))
    S = int(smp["num_steps"])
    torch.manual_seed(0)
    x = m(torch.from_numpy(smp["y"]).to(DEV), num_samples=100000, num_steps=S)  # the default precision
    assert x.shape == (100000, smp["samples"].shape[1]) and np.all(np.isfinite(x))
    r = M.parity_report(x, smp["samples"], smp["quantiles"], int(smp["n_total"]))
    print(f"\n[x3] parity {tag}: {r}")
    assert r["pass"], r


# ------------------------------------------------------------- the split's fp16 range (include/dmip.h)
@pytest.mark.parametrize("engine", ["x3k", "x3"])
def test_x3_weight_outside_fp16_range_refused_default_falls_back(dmip, golden, engine, monkeypatch):
    """One hidden weight at 2e4 (x 4 log2(e) = 1.2e5 > 65504 in the split image): an explicit fp32x3 request is
    refused with a clear error; the default precision samples with the exact-f32 engine instead, equal to it chain
    by chain and to the float32 oracle."""
    if engine == "x3":
        monkeypatch.setenv("DMIP_X3K", "0")
    m = _cde(dmip, "scat", golden("ckpt_scat.npz"))
    with torch.no_grad():
        m.sde.a._modules["3"].weight[5, 7] = 2.0e4  # the first W x W layer (state_dict key 3)
    y = torch.from_numpy(golden("samples_scat.npz")["y"]).to(DEV)
    n, S = 600, 8
    with pytest.raises(ValueError, match="fp16 range"):
        m.sample_device(y, n, S, seed=3, precision=PREC)
    torch.manual_seed(5)
    with pytest.warns(RuntimeWarning, match="fp16 range"):
        x = m(y, num_samples=n, num_steps=S)
    torch.manual_seed(5)
    xf = m(y, num_samples=n, num_steps=S, precision="fp32")
    assert np.array_equal(x, xf)
    seed = 77
    xs = m.sample_device(y, n, S, seed=seed, precision="fp32")[0].cpu().numpy()
    ref = O.cde_sample(_linear_params(m.sde.a), y.cpu().numpy(), n, S, seed)
    e = _rel(xs, ref)
    print(f"\n[x3] {engine} weight 2e4: exact-f32 fallback vs oracle {e:.2e}")
    assert np.all(np.isfinite(x)) and e < 1e-4, e


@pytest.mark.parametrize("engine", ["x3k", "x3"])
def test_x3_trajectory_outside_fp16_range_reported_default_falls_back(dmip, golden, engine, monkeypatch):
    """An output bias of 1e6 drives every chain to |x| ~ 1e5-1e6 after one step (finite in fp32): the fp32x3
    kernel flags the layer-1 inputs beyond 65504 through the device status word; the default precision resamples
    with the exact-f32 engine, which matches the float32 oracle."""
    if engine == "x3":
        monkeypatch.setenv("DMIP_X3K", "0")
    m = _cde(dmip, "scat", golden("ckpt_scat.npz"))
    with torch.no_grad():
        m.sde.a._modules["7"].bias[:] = 1.0e6  # the output layer (state_dict key 7)
    y = torch.from_numpy(golden("samples_scat.npz")["y"]).to(DEV)
    n, S, seed = 600, 6, 91
    x3 = m.sample_device(y, n, S, seed=seed, precision=PREC)
    with pytest.raises(RuntimeError, match="fp16 range"):
        dmip._lib.device_status(x3.device)
    dmip._lib.device_status(x3.device)  # the status word was cleared
    torch.manual_seed(6)
    with pytest.warns(RuntimeWarning, match="fp16 range"):
        x = m(y, num_samples=n, num_steps=S)
    torch.manual_seed(6)
    xf = m(y, num_samples=n, num_steps=S, precision="fp32")
    assert np.array_equal(x, xf) and np.all(np.isfinite(x)) and np.abs(x).max() > 6.6e4
    xs = m.sample_device(y, n, S, seed=seed, precision="fp32")[0].cpu().numpy()
    ref = O.cde_sample(_linear_params(m.sde.a), y.cpu().numpy(), n, S, seed)
    e = _rel(xs, ref)
    print(f"\n[x3] {engine} |x| up to {np.abs(xs).max():.2e}: exact-f32 fallback vs oracle {e:.2e}")
    assert e < 1e-4, e


@pytest.mark.parametrize("engine", ["x3k", "x3"])
def test_x3_idle_waves_never_report_range(dmip, engine, monkeypatch):
    """the range flag covers returned chains only. 100 chains leave almost every wave of the grid an
    idle segment, which re-runs step 0 (beta = beta_max) on a dummy tile for all S steps: with x0 ~ N(0, 10^2) its
    |x| grows ~e^10 past 65504, while the real chains (an untrained net; growth ~e^5) stay inside. No range report
    may result, and the default path must not fall back."""
    if engine == "x3":
        monkeypatch.setenv("DMIP_X3K", "0")
    torch.manual_seed(12)
    m = dmip.CDE(3, 23, [256] * 3)
    y = torch.from_numpy(np.random.default_rng(3).uniform(0, 1, 23).astype(np.float32)).to(DEV)
    n, S = 100, 1000
    dmip._lib.clear_range_status(torch.device(DEV))
    x = m.sample_device(y, n, S, 0.0, 10.0, seed=4, precision=PREC)
    dmip._lib.device_status(x.device)  # raised "fp16 range" in round 4 (the idle waves' dummy tiles)
    xs = x[0].cpu().numpy()
    assert np.all(np.isfinite(xs)) and np.abs(xs).max() < 65504.0
    xf = m.sample_device(y, n, S, 0.0, 10.0, seed=4, precision="fp32")[0].cpu().numpy()
    e = _rel(xs, xf)
    print(f"\n[x3] {engine} idle waves: max |x| {np.abs(xs).max():.3g}, vs exact f32 {e:.2e}")
    assert e < 1e-3, e
    import warnings
    par = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.parallel")
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # no fallback warning
        xd = par.sample_checked(m, y, n, S, 0.0, 10.0, seed=4)
    assert torch.equal(xd, x)


def test_sample_checked_falls_back_for_evaluate(dmip, golden):
    """The evaluate drivers sample through parallel.sample_checked: a trajectory beyond the fp16 range
    at the default precision comes back from the exact-f32 engine, with a warning, chain for chain; a stale range
    report of an earlier, unread launch does not make a later in-range call fall back."""
    par = importlib.import_module("diffusion-modelling-for-inverse-problems_amd.parallel")
    m = _cde(dmip, "scat", golden("ckpt_scat.npz"))
    with torch.no_grad():
        m.sde.a._modules["7"].bias[:] = 1.0e6
    y = torch.from_numpy(golden("samples_scat.npz")["y"]).to(DEV)
    yy = y.expand(3, -1)
    n, S = 400, 5
    with pytest.warns(RuntimeWarning, match="fp16 range"):
        x = par.sample_checked(m, yy, n, S, 0, 1, seed=21)
    xf = m.sample_device(yy, n, S, seed=21, precision="fp32")
    assert torch.equal(x, xf)
    m.sample_device(yy, n, S, seed=22, precision=PREC)  # leaves an unread range report behind
    good = _cde(dmip, "scat", golden("ckpt_scat.npz"))
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        xg = par.sample_checked(good, yy, n, S, 0, 1, seed=23)
    assert torch.equal(xg, good.sample_device(yy, n, S, seed=23, precision=PREC))
