"""Pins the CPU oracle (oracle/dmip_oracle.py) to the reference's own outputs (golden fixtures
captured by tests/golden/make_golden.py). CPU only."""
import numpy as np
import pytest

import oracle as O


@pytest.mark.parametrize("S", [200, 1000])
def test_schedule_bit_exact(golden, S):
    z = golden("schedule.npz")
    ts, tau = O.schedule(S)
    assert np.array_equal(ts, z[f"ts_{S}"])
    assert np.array_equal(tau, z[f"tau_{S}"])
    assert np.array_equal(O.vp_beta(tau), z[f"beta_{S}"])
    # torch-CPU's vectorised sqrt is not correctly rounded on a handful of entries (1 ulp)
    ulp = np.abs(O.vp_g(tau).view(np.int32) - z[f"g_{S}"].view(np.int32))
    assert ulp.max() <= 1 and (ulp > 0).sum() <= 10
    np.testing.assert_allclose(O.vp_mean_weight(tau), z[f"mw_{S}"], rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(O.vp_var(tau), z[f"var_{S}"], rtol=2e-6, atol=1e-7)


def test_linspace_second_half_is_single_rounding(golden):
    # the branch the SURVEY probed: (S+1)//2 onwards ts[i] = 1 - (S-i)*step rounded once
    z = golden("schedule.npz")
    S = 1000
    step = np.float32(1.0) / np.float32(S)
    i = np.arange((S + 1) // 2, S + 1)
    two = (np.float32(1.0) - ((S - i).astype(np.float32) * step).astype(np.float32)).astype(np.float32)
    one = O.linspace_f32(S)[(S + 1) // 2:]
    assert np.array_equal(one, z["ts_1000"][(S + 1) // 2:])
    assert not np.array_equal(two, one)  # the double-rounded formula would not be bit-exact


@pytest.mark.parametrize("tag", ["lin", "scat"])
def test_mlp_forward(golden, tag):
    z = golden("mlp_io.npz")
    p = O.mlp_params_from_state(z, f"{tag}_")
    a = O.cde_a(p, z[f"{tag}_x"], z[f"{tag}_y"], z[f"{tag}_t"])
    np.testing.assert_allclose(a, z[f"{tag}_a"], rtol=1e-5, atol=1e-6)
    # the reference chain applies tanh twice on layer 1 (nets.py:26): a single tanh is far off
    single = O.mlp_forward(p, np.concatenate([z[f"{tag}_x"], z[f"{tag}_y"], z[f"{tag}_t"]], 1),
                           tanh_twice_first=False)
    assert np.abs(single - z[f"{tag}_a"]).max() > 1e-3


@pytest.mark.parametrize("tag", ["lin", "scat"])
def test_posterior_score(golden, tag):
    z = golden("mlp_io.npz")
    pp = O.mlp_params_from_state(z, f"{tag}_prior_")
    pl = O.mlp_params_from_state(z, f"{tag}_lik_")
    np.testing.assert_allclose(O.mlp2_a(pp, z[f"{tag}_x"], z[f"{tag}_t"]), z[f"{tag}_prior_out"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(O.posterior_a(pp, pl, z[f"{tag}_x"], z[f"{tag}_y"], z[f"{tag}_t"]),
                               z[f"{tag}_post_out"], rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("tag", ["lin", "scat"])
def test_em_trajectory_injected_noise(golden, tag):
    """The oracle, fed the reference's captured x0 and per-step noise, reproduces the reference's
    final samples to fp32 rounding (the only difference is the sgemm summation order)."""
    tr = golden(f"traj_{tag}.npz")
    ck = golden(f"ckpt_{tag}.npz")
    p = O.mlp_params_from_state(ck)
    for x0, xi, ref in [(tr["x0_short"], tr["xi_short"], tr["x_final_short"]),
                        (tr["x0"], tr["xi"], tr["x_final"])]:
        out = O.em_sample(lambda x, tau: O.cde_a(p, x, tr["y"], tau), x0, xi.shape[0], noise=xi)
        np.testing.assert_allclose(out, ref, rtol=1e-4, atol=1e-4 * max(1.0, np.abs(ref).max()))


def test_em_step_rounding_order_is_the_references():
    """One EM step with a = 0 and xi = 0 reduces to fl(x + fl(delta * fl(0.5 beta x)))."""
    x = np.array([[0.3, -1.7]], np.float32)
    tau = np.float32(0.75)
    out = O.em_step(x, np.zeros_like(x), tau, 1 / 200, xi=np.zeros_like(x))
    beta = O.vp_beta(tau)
    mu = (np.float32(0) - ((np.float32(-0.5) * beta).astype(np.float32) * x).astype(np.float32))
    ref = (x + (np.float32(1 / 200) * mu).astype(np.float32)).astype(np.float32)
    assert np.array_equal(out, ref)


def test_linear_score_posterior(golden):
    z = golden("linear_posterior.npz")
    y = z["y"]
    mean, cov = z["mean"], z["cov"]
    x = np.random.default_rng(0).normal(size=(64, 2)).astype(np.float32)
    # Gaussian posterior score: -cov^-1 (x - mean) (linear_problem.py:41-65)
    ref = -(x - mean) @ np.linalg.inv(cov).T
    np.testing.assert_allclose(O.linear_score_posterior(x, np.broadcast_to(y, x.shape)), ref, rtol=1e-3, atol=1e-3)


def test_rng_oracle_properties():
    s = O.rng_init(7, np.arange(50000))
    n = O.rng_normals(s, 3)
    assert n.shape == (50000, 3) and n.dtype == np.float32
    assert abs(n.mean()) < 0.01 and abs(n.std() - 1) < 0.01
    # keyed by the global chain index: chain 1000's stream is the same in any batch
    a = O.rng_uniform_words(7, np.arange(990, 1010), 5)
    b = O.rng_uniform_words(7, np.array([1000]), 5)
    assert np.array_equal(a[10], b[0])


def test_hist_kl_matches_reference_formula():
    rng = np.random.default_rng(1)
    a = rng.normal(size=(20000, 2)).astype(np.float32)
    b = rng.normal(size=(20000, 2)).astype(np.float32) * 1.1
    kl, klr = O.hist_kl(a, a, lim=(-3.5, 3.5))
    assert kl == pytest.approx(0.0, abs=1e-12) and klr == pytest.approx(0.0, abs=1e-12)
    kl, klr = O.hist_kl(a, b, lim=(-3.5, 3.5))
    assert kl > 0 and klr > 0


def test_reference_samples_fixture_consistent(golden):
    for tag in ("lin", "scat"):
        s = golden(f"samples_{tag}.npz")
        q = s["quantiles"]
        assert q.shape == (1001, s["samples"].shape[1])
        assert np.all(np.diff(q, axis=0) >= 0)
        # the stored 20k subset is drawn from the same run as the 100k quantiles
        for k in range(q.shape[1]):
            med = np.median(s["samples"][:, k])
            assert abs(med - q[500, k]) < 0.05 * (q[990, k] - q[10, k])


LOSS_CFGS = {
    "pinn": dict(kind="pinn", pde="FPE", pde_metric="L1", ic_metric="L2", lam=1e-3, lam2=0.1),
    "pinn_l1l2": dict(kind="pinn", pde="FPE", pde_metric="L2", ic_metric="L1", lam=0.5, lam2=0.3),
    "dsmpde": dict(kind="dsm_pde", pde="FPE", pde_metric="L1", lam=1e-2),
    "pinn_cfpe": dict(kind="pinn", pde="cFPE", pde_metric="L2", ic_metric="L2", lam=1e-3, lam2=0.1),
    "dsm": dict(kind="dsm"),
}
LIN_IC = dict(ic_A=[[1, 0.5], [0, 1]], ic_b=[0.3, 0.5], ic_Sinv=np.eye(2) / 0.3)


@pytest.mark.parametrize("name", list(LOSS_CFGS))
def test_loss_grad_jets_match_reference_autograd(golden, name):
    """The jet + hand-written-backward restatement (the fused training kernel's formulation) against
    the reference's autograd losses and parameter gradients (G5)."""
    z = golden("pinn_linear.npz")
    params = O.mlp_params_from_state(dict(golden("ckpt_lin.npz")))
    loss, comps, grads = O.loss_grad(params, z["x"], z["y"], z["t"], z["eps"], **LOSS_CFGS[name], **LIN_IC)
    if name != "dsm":
        assert loss == pytest.approx(float(z[f"{name}_loss"]), rel=5e-5)
        assert comps["PDE"] == pytest.approx(float(z[f"{name}_PDE_Loss"]), rel=5e-5)
    for (gW, gb), k in zip(grads, ["0", "3", "5", "7"]):
        rW, rb = z[f"{name}_grad_{k}_weight"], z[f"{name}_grad_{k}_bias"]
        assert np.abs(gW - rW).max() <= 1e-4 * np.abs(rW).max()
        assert np.abs(gb - rb).max() <= 1e-4 * np.abs(rb).max()
    if name == "dsmpde":
        np.testing.assert_allclose(comps["div"], z["fpe_div"], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(comps["pde_rows"].reshape(-1, 1), z["fpe_rows"], rtol=1e-3, atol=1e-4)


# ---------------------------------------------------------------- F2 / F3 scatterometry surrogate
def test_surrogate_oracle_matches_reference(golden):
    """surrogate forward, get_log_posterior and its autograd gradient (energy_grad) of the reference
    (fixture G8, 256 rows incl. points outside the prior box) against the float64 restatement."""
    z = golden("surrogate_io.npz")
    params = O.surrogate_params_from_npz(golden("surrogate.npz"))
    f = O.surrogate_forward(params, z["x"])
    assert np.abs(f - z["f"]).max() <= 2e-6 * np.abs(z["f"]).max()
    e, g = O.scat_log_posterior(params, z["x"], z["y"], float(z["a"]), float(z["b"]), float(z["lambd_bd"]), grad=True)
    np.testing.assert_allclose(e, z["energy"], rtol=1e-5, atol=1e-4)
    assert np.abs(g - z["grad"]).max() <= 1e-5 * np.abs(z["grad"]).max()
    assert (np.abs(z["x"]) > 1).any()  # the boundary penalty is exercised


def test_mh_oracle_replays_reference_trajectories(golden):
    """anneal_to_energy fed its own captured draws: every chain takes the reference's path."""
    z = golden("surrogate_io.npz")
    params = O.surrogate_params_from_npz(golden("surrogate.npz"))
    S = z["mh_xi"].shape[0]
    x, ed = O.mh_sample(params, z["mh_y"], S, float(z["mh_noise_std"]), x0=z["mh_x0"], noise=z["mh_xi"],
                        unif=z["mh_u"])
    assert np.array_equal(x, z["mh_x"])
    np.testing.assert_allclose(ed, z["mh_ediff"], rtol=1e-4, atol=1e-3)
    # some proposals were accepted and some rejected
    assert 0 < np.mean(np.any(x != z["mh_x0"], axis=1)) <= 1


def test_posterior_loss_oracle_matches_reference(golden):
    """oracle.posterior_loss_grad (float64, the likelihood target by linearity of the reference's
    detached VJPs / VHPs) against the reference's PosteriorLoss forward + backward (G10)."""
    z = golden("posterior_loss.npz")
    sur = O.surrogate_params_from_npz(golden("surrogate.npz"))
    pp, pl = O.mlp_params_from_state(z, "prior_"), O.mlp_params_from_state(z, "lik_")
    loss, info, gp, gl, T = O.posterior_loss_grad(pp, pl, sur, z["x"], z["y"], z["t"], z["eps"],
                                                  float(z["a"]), float(z["b"]), float(z["lam"]))
    assert abs(loss - float(z["loss"])) < 1e-5 * abs(float(z["loss"]))
    assert abs(info["PriorLoss"] - float(z["PriorLoss"])) < 1e-5 * float(z["PriorLoss"])
    assert abs(info["LikelihoodLoss"] - float(z["LikelihoodLoss"])) < 1e-5 * float(z["LikelihoodLoss"])
    assert np.abs(T - z["target"]).max() < 2e-4 * np.abs(z["target"]).max()
    for tag, grads in (("prior", gp), ("lik", gl)):
        for i, (dW, db) in zip([0, 3, 5, 7], grads):
            for got, ref in ((dW, z[f"{tag}_grad_{i}_weight"]), (db, z[f"{tag}_grad_{i}_bias"])):
                assert np.abs(got - ref).max() < 2e-5 * np.abs(ref).max()


@pytest.mark.parametrize("tag", ["lin", "scat"])
def test_loss_grad_oracle_matches_reference_at_reference_width(golden, tag):
    """oracle.loss_grad against the reference PINNLoss at hidden_layers [512]*3 with the configs' loss
    settings (G11); the scatterometry IC target is the reference's own -energy_grad values."""
    z = golden("pinn_ref_configs.npz")
    xd, yd = (2, 2) if tag == "lin" else (3, 23)
    params = O.reference_weights([xd + yd + 1, 512, 512, 512, xd], int(z[f"{tag}_seed"]))
    kw = dict(kind="pinn", pde="FPE", pde_metric="L1", ic_metric="L2")
    if tag == "lin":
        kw.update(lam=1e-3, lam2=0.1, ic_A=[[1, 0.5], [0, 1]], ic_b=[0.3, 0.5], ic_Sinv=np.eye(2) / 0.3)
    else:
        kw.update(lam=0.01, lam2=0.001, ic_target=z["scat_ic_target"])
    loss, comps, grads = O.loss_grad(params, z[f"{tag}_x"], z[f"{tag}_y"], z[f"{tag}_t"], z[f"{tag}_eps"], **kw)
    assert abs(loss - float(z[f"{tag}_loss"])) < 1e-4 * abs(float(z[f"{tag}_loss"]))
    assert abs(comps["PDE"] - float(z[f"{tag}_PDE_Loss"])) < 1e-3 * abs(float(z[f"{tag}_PDE_Loss"]))
    for li, (dW, db) in zip([0, 3, 5, 7], grads):
        for got, ref in ((dW, z[f"{tag}_grad_{li}_weight"]), (db, z[f"{tag}_grad_{li}_bias"])):
            assert np.linalg.norm(got - ref) < 1e-3 * np.linalg.norm(ref), (li, np.linalg.norm(got - ref) / np.linalg.norm(ref))


def _g12_params(z, tag):
    return [(z[f"{tag}_{k}_weight"], z[f"{tag}_{k}_bias"]) for k in (0, 3, 5, 7)]


@pytest.mark.parametrize("tag", ["lin", "scat"])
def test_cdiffe_joint_dsm_vs_reference(golden, tag):
    """G12: the oracle's DSM on the joint state z = (x, y) with no condition input (ydim 0) reproduces
    the reference's CDiffE training loss and every parameter gradient (models/diffusion.py:128-136)."""
    z = golden("cdiffe_dsm.npz")
    zz, t, eps = z[f"{tag}_z"], z[f"{tag}_t"], z[f"{tag}_eps"]
    loss, _, grads = O.loss_grad(_g12_params(z, tag), zz, np.zeros((zz.shape[0], 0), np.float32), t, eps, kind="dsm")
    assert loss == pytest.approx(float(z[f"{tag}_loss"]), rel=1e-5)
    for (dW, db), k in zip(grads, (0, 3, 5, 7)):
        for g, ref in ((dW, z[f"{tag}_grad_{k}_weight"]), (db, z[f"{tag}_grad_{k}_bias"])):
            assert np.linalg.norm(g - ref) <= 1e-4 * np.linalg.norm(ref) + 1e-7
