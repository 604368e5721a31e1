"""CPU oracle for the conditional score-diffusion posterior sampler -- TEST INFRASTRUCTURE.

Restates, in numpy float32 and in the reference's operation order, every function on the hot
path. Each function cites the reference file:line it follows. It is pinned
against golden vectors captured from the reference (tests/golden/make_golden.py) by
tests/test_oracle_golden.py; it is never called by the product path.

RNG note: the reference draws from torch's mt19937 (CPU) stream, which cannot be reproduced by a
counter-keyed parallel sampler. Two parity modes therefore exist:
  * injected noise -- the oracle/kernel consume a captured (x0, xi) sequence (fixture G3) and
    must match the reference trajectory to fp tolerance;
  * chain-keyed RNG -- the oracle restates the product RNG (splitmix64-seeded xoshiro128**,
    Box-Muller), so the kernel's integer stream is checked bit-exactly and its normals to ulps.
"""
import numpy as np

F32 = np.float32

# ------------------------------------------------------------------------------------------
# A1  schedule -- models/diffusion.py:31,34-35,40-41
# ------------------------------------------------------------------------------------------

def linspace_f32(num_steps):
    """torch.linspace(0, 1, S+1) in float32 (models/diffusion.py:34).

    Restates ATen's CPU linspace: step = fl32(1/S); the first (S+1)//2 points are fl32(i*step),
    the rest are 1 - (S-i)*step with a single rounding (fused multiply-add).
    """
    S = int(num_steps)
    n = S + 1
    step = F32(1.0) / F32(S)
    i = np.arange(n, dtype=np.int64)
    half = n // 2
    out = np.empty(n, dtype=F32)
    out[:half] = (i[:half].astype(F32) * step).astype(F32)
    # single-rounding 1 - (S-i)*step: evaluate exactly in float64, round once to float32
    k = (S - i[half:]).astype(np.float64)
    out[half:] = (1.0 - k * np.float64(step)).astype(F32)
    return out


def schedule(num_steps, T=1.0):
    """ts = linspace*T; the net and the coefficients see tau_i = T - ts[i] (sdes.py:78)."""
    ts = (linspace_f32(num_steps) * F32(T)).astype(F32)
    tau = (F32(T) - ts).astype(F32)
    return ts, tau


# ------------------------------------------------------------------------------------------
# A7  VariancePreservingSDE -- sdes.py:9-57
# ------------------------------------------------------------------------------------------
BETA_MIN = 0.1
BETA_MAX = 20.0


def vp_beta(t, beta_min=BETA_MIN, beta_max=BETA_MAX):
    """sdes.py:21-22: beta_min + (beta_max-beta_min)*t, python scalars rounded to fp32."""
    t = np.asarray(t, dtype=F32)
    return (F32(beta_min) + (F32(beta_max - beta_min) * t).astype(F32)).astype(F32)


def vp_g(t, beta_min=BETA_MIN, beta_max=BETA_MAX):
    """sdes.py:33-35: ones_like(y) * beta(t)**0.5 (pow 0.5 == correctly rounded sqrt)."""
    return np.sqrt(vp_beta(t, beta_min, beta_max)).astype(F32)


def vp_mean_weight(t, beta_min=BETA_MIN, beta_max=BETA_MAX):
    """sdes.py:24-25: exp(-0.25 t^2 (bmax-bmin) - 0.5 t bmin)."""
    t = np.asarray(t, dtype=F32)
    a = (F32(-0.25) * (t * t).astype(F32)).astype(F32) * F32(beta_max - beta_min)
    b = (F32(0.5) * t).astype(F32) * F32(beta_min)
    return np.exp((a.astype(F32) - b.astype(F32)).astype(F32)).astype(F32)


def vp_var(t, beta_min=BETA_MIN, beta_max=BETA_MAX):
    """sdes.py:27-28: 1 - exp(-0.5 t^2 (bmax-bmin) - t bmin)."""
    t = np.asarray(t, dtype=F32)
    a = (F32(-0.5) * (t * t).astype(F32)).astype(F32) * F32(beta_max - beta_min)
    b = (t * F32(beta_min)).astype(F32)
    return (F32(1.0) - np.exp((a.astype(F32) - b).astype(F32))).astype(F32)


# ------------------------------------------------------------------------------------------
# A9/A10  MLP / MLP2 / PosteriorScore -- nets.py:17-57,143-157
# ------------------------------------------------------------------------------------------

def mlp_params_from_state(state, prefix=""):
    """Ordered [(W, b), ...] from a reference MLP state_dict (keys 0,3,5,7 -- nets.py:21-30;
    the Tanh children '1', 'act', '4', '6' hold no parameters)."""
    idx = sorted({int(k[len(prefix):].split("_")[0]) for k in state.keys()
                  if k.startswith(prefix) and k[len(prefix):].split("_")[0].isdigit()
                  and k.endswith("weight")})
    return [(np.asarray(state[f"{prefix}{i}_weight"], F32), np.asarray(state[f"{prefix}{i}_bias"], F32))
            for i in idx]


def activation(h, act="tanh"):
    """The hidden activation of nets.py:17's `activation` argument: "tanh" (nn.Tanh, every diffusion net of the
    reference, models/diffusion.py:69,118,190,195) or "silu" (nn.SiLU: z sigmoid(z), evaluated in f64 and
    rounded once)."""
    if act == "tanh":
        return np.tanh(h).astype(F32)
    if act == "silu":
        z = np.asarray(h, np.float64)
        return (z / (1.0 + np.exp(-z))).astype(F32)
    raise ValueError(f"unknown activation {act!r}")


def mlp_forward(params, inp, tanh_twice_first=True, act="tanh"):
    """nets.py:17-35. Forward chain is Linear -> act -> act (the quirk of nets.py:26: the activation module is
    registered a second time as `act`) -> [Linear -> act] * (L-1) -> Linear."""
    h = np.asarray(inp, F32)
    L = len(params)
    for li, (W, b) in enumerate(params):
        h = (h @ W.T + b).astype(F32)
        if li < L - 1:
            h = activation(h, act)
            if li == 0 and tanh_twice_first:
                h = activation(h, act)
    return h


def cde_a(params, x, y, t, act="tanh"):
    """MLP.forward (nets.py:32-35): cat[x, y, t.view(N,1)]."""
    x = np.asarray(x, F32)
    n = x.shape[0]
    y = np.broadcast_to(np.asarray(y, F32), (n, np.asarray(y).shape[-1]))
    t = np.broadcast_to(np.asarray(t, F32).reshape(-1, 1), (n, 1))
    return mlp_forward(params, np.concatenate([x, y, t], axis=1), act=act)


def mlp2_a(params, x, t, act="tanh"):
    """MLP2.forward (nets.py:52-57): cat[x, t]."""
    x = np.asarray(x, F32)
    t = np.broadcast_to(np.asarray(t, F32).reshape(-1, 1), (x.shape[0], 1))
    return mlp_forward(params, np.concatenate([x, t], axis=1), act=act)


def posterior_a(prior_params, lik_params, x, y, t, act="tanh"):
    """PosteriorScore.forward (nets.py:155-157): g(t) * (prior(x,t) + lik(x,y,t))."""
    s = (mlp2_a(prior_params, x, t, act=act) + cde_a(lik_params, x, y, t, act=act)).astype(F32)
    tt = np.broadcast_to(np.asarray(t, F32).reshape(-1, 1), s.shape)
    return (vp_g(tt) * s).astype(F32)


# ------------------------------------------------------------------------------------------
# A19  LinearForwardProblem.score_posterior -- linear_problem.py:61-65
# ------------------------------------------------------------------------------------------
LIN_A = np.array([[1.0, 0.5], [0.0, 1.0]], F32)
LIN_B = np.array([0.3, 0.5], F32)
LIN_SCALE = F32(0.3)


def linear_score_posterior(x, y):
    x = np.asarray(x, F32)
    y = np.asarray(y, F32)
    y_res = (y - (x @ LIN_A.T + LIN_B)).astype(F32)
    sig_inv = (F32(1.0) / LIN_SCALE) * np.eye(2, dtype=F32)
    return (-x + (y_res @ sig_inv.T) @ LIN_A).astype(F32)


# ------------------------------------------------------------------------------------------
# product RNG restated: splitmix64-seeded xoshiro128** per chain + Box-Muller
# (the kernel's generator; see include/dmip.h dmip_rng_normals)
# ------------------------------------------------------------------------------------------
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
GOLDEN = np.uint64(0x9E3779B97F4A7C15)
CHAIN_MUL = np.uint64(0xD1B54A32D192ED03)
STREAM_MUL = np.uint64(0x8CB92BA72F3D8DD7)


def _splitmix_next(state):
    with np.errstate(over="ignore"):
        state = state + GOLDEN
        z = state.copy()
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return state, z


def rng_init(seed, chain_ids, stream=0):
    """Per-chain state: splitmix64 seeded with seed + chain*CHAIN_MUL + stream*STREAM_MUL.
    Keyed by the GLOBAL chain index, so a chain's draws do not depend on how the chains are
    sharded over workgroups or GPUs."""
    c = np.asarray(chain_ids, dtype=np.uint64)
    with np.errstate(over="ignore"):
        sm = np.uint64(seed) + c * CHAIN_MUL + np.uint64(stream) * STREAM_MUL
    sm, z0 = _splitmix_next(sm)
    sm, z1 = _splitmix_next(sm)
    s = np.stack([z0 & np.uint64(0xFFFFFFFF), z0 >> np.uint64(32),
                  z1 & np.uint64(0xFFFFFFFF), z1 >> np.uint64(32)]).astype(np.uint32)
    zero = (s == 0).all(axis=0)
    s[0, zero] = np.uint32(1)
    return s  # (4, n) uint32


def _rotl(x, k):
    return ((x << np.uint32(k)) | (x >> np.uint32(32 - k))).astype(np.uint32)


def rng_next(s):
    """xoshiro128** (Blackman & Vigna) on a (4, n) uint32 state, in place; returns n uint32."""
    with np.errstate(over="ignore"):
        result = (_rotl((s[1] * np.uint32(5)).astype(np.uint32), 7) * np.uint32(9)).astype(np.uint32)
    t = (s[1] << np.uint32(9)).astype(np.uint32)
    s[2] ^= s[0]
    s[3] ^= s[1]
    s[1] ^= s[2]
    s[0] ^= s[3]
    s[2] ^= t
    s[3] = _rotl(s[3], 11)
    return result


def rng_normals(s, d):
    """d normals per chain (ceil(d/2) Box-Muller pairs; the unused odd one is dropped).
    u1 = 1 - (r>>8)*2^-24 in (0,1], u2 = (r>>8)*2^-24; n = sqrt(-2 ln u1) * (cos, sin)(2 pi u2)."""
    n = s.shape[1]
    out = np.empty((n, 2 * ((d + 1) // 2)), F32)
    inv = F32(2.0 ** -24)
    for p in range((d + 1) // 2):
        r0 = rng_next(s)
        r1 = rng_next(s)
        u1 = (F32(1.0) - (r0 >> np.uint32(8)).astype(F32) * inv).astype(F32)
        u2 = ((r1 >> np.uint32(8)).astype(F32) * inv).astype(F32)
        rad = np.sqrt(F32(-2.0) * np.log(u1)).astype(F32)
        th = (F32(2.0 * np.pi) * u2).astype(F32)
        out[:, 2 * p] = rad * np.cos(th)
        out[:, 2 * p + 1] = rad * np.sin(th)
    return out[:, :d]


def rng_uniform_words(seed, chain_ids, n_words, stream=0):
    s = rng_init(seed, chain_ids, stream)
    return np.stack([rng_next(s) for _ in range(n_words)], axis=1)


# ------------------------------------------------------------------------------------------
# Training-time draws -- models/diffusion.py:48-58 (sample_t), sdes.py:37-57 (sample, sample_debiasing_t)
# ------------------------------------------------------------------------------------------
def vp_truncated_q(u, beta_min=0.1, beta_max=20.0, t_epsilon=1e-3, T=1.0):
    """Inverse CDF of q(t) ~ beta(t)/var(t) above t_epsilon, flat below (sdes.py:51-57 calls
    sdeflow-light's sample_vp_truncated_q, which the reference does not vendor: restated from its
    math in float64, parity unpinned). With B(t) = int_0^t beta: CDF(t) = t r(t_eps) below t_eps, and
    t_eps r(t_eps) + log(e^B(t) - 1) - log(e^B(t_eps) - 1) above; normalised by its value at T."""
    u = np.asarray(u, np.float64)
    a, b, te = beta_max - beta_min, beta_min, t_epsilon
    B = lambda t: 0.5 * a * t * t + b * t
    r_te = (b + a * te) / (1.0 - np.exp(-B(te)))
    A_te = np.log(np.expm1(B(te)))
    Z = te * r_te + np.log(np.expm1(B(T))) - A_te
    v = Z * u + A_te - te * r_te
    Bu = np.where(v > 30, v, np.log1p(np.exp(np.minimum(v, 30))))
    hi = (-b + np.sqrt(b * b + 2.0 * a * Bu)) / a
    return np.where(u <= te * r_te / Z, Z / r_te * u, hi)


def train_draws(seed, stream_id, batch, xdim, debias=True, beta_min=0.1, beta_max=20.0, t_epsilon=1e-3, T=1.0,
                t_add=1e-4):
    """dmip_train_draws restated: sample index b, generator (seed, b, stream_id); the first word gives
    u = (w >> 8) 2^-24 and t = sample_t's draw (models/diffusion.py:50-57: q(u) + t_add, minus t_add
    again above T; or t_add + u T, set to T - t_add above T); then two Box-Muller pairs give eps
    (base_sde.sample's randn_like, sdes.py:41), the first xdim of them kept. Returns (t[batch], eps)."""
    s = rng_init(seed, np.arange(batch, dtype=np.uint64), stream_id)
    u = (rng_next(s) >> np.uint32(8)).astype(np.float64) * 2.0 ** -24
    if debias:
        t = vp_truncated_q(u, beta_min, beta_max, t_epsilon, T) + t_add
        t = np.where(t > T, t - t_add, t)
    else:
        t = t_add + u * T
        t = np.where(t > T, T - t_add, t)
    eps = rng_normals(s, 4)[:, :xdim]
    return t, eps


# ------------------------------------------------------------------------------------------
# A2/A8  Euler-Maruyama reverse-SDE loop -- models/diffusion.py:27-46, sdes.py:77-87
# ------------------------------------------------------------------------------------------

def em_step(x, a, tau, delta, beta_min=BETA_MIN, beta_max=BETA_MAX, xi=None):
    """One EM update with the reference rounding order:
    mu = fl(g*a) - fl(fl(-0.5*beta)*x)     (sdes.py:77-79, lambda = 0)
    x <- fl(x + fl(delta*mu)) + fl(fl(sqrt(delta)*sigma)*xi), sigma = g (sdes.py:86-87)."""
    beta = vp_beta(tau, beta_min, beta_max)
    g = np.sqrt(beta).astype(F32)
    mu = ((g * a).astype(F32) - ((F32(-0.5) * beta).astype(F32) * x).astype(F32)).astype(F32)
    d32 = F32(delta)
    sd32 = F32(np.sqrt(np.float64(delta)))
    out = (x + (d32 * mu).astype(F32)).astype(F32)
    return (out + ((sd32 * g).astype(F32) * xi).astype(F32)).astype(F32)


def em_sample(a_fn, x0, num_steps, T=1.0, noise=None, rng_state=None, xdim=None,
              beta_min=BETA_MIN, beta_max=BETA_MAX, snapshots=None):
    """models/diffusion.py:27-46 with either an injected noise tensor (S, N, d) or the product
    RNG state (consumed in place). a_fn(x, tau_scalar) returns the net output (N, d)."""
    x = np.asarray(x0, F32).copy()
    ts, tau = schedule(num_steps, T)
    delta = float(T) / num_steps  # python double, rounded to fp32 inside em_step
    snaps = {}
    for i in range(num_steps):
        a = a_fn(x, tau[i])
        if noise is not None:
            xi = np.asarray(noise[i], F32)
        else:
            xi = rng_normals(rng_state, xdim or x.shape[1])
        x = em_step(x, a, tau[i], delta, beta_min, beta_max, xi)
        if snapshots is not None and (i + 1) in snapshots:
            snaps[i + 1] = x.copy()
    return (x, snaps) if snapshots is not None else x


def cde_sample(params, y, num_samples, num_steps, seed, mean=0.0, std=1.0, chain_offset=0,
               stream=0, T=1.0, snapshots=None, act="tanh"):
    """Product-RNG CDE sampler: x0 = normals*std + mean (models/diffusion.py:32-33), then EM."""
    xdim = params[-1][0].shape[0]
    st = rng_init(seed, np.arange(chain_offset, chain_offset + num_samples), stream)
    x0 = (rng_normals(st, xdim) * F32(std) + F32(mean)).astype(F32)
    y = np.asarray(y, F32)
    return em_sample(lambda x, tau: cde_a(params, x, y, tau, act=act), x0, num_steps, T=T,
                     rng_state=st, xdim=xdim, snapshots=snapshots)


def posterior_sample(prior_params, lik_params, y, num_samples, num_steps, seed, mean=0.0, std=1.0,
                     chain_offset=0, stream=0, T=1.0, act="tanh"):
    """Product-RNG PosteriorDiffusionEstimator sampler (models/diffusion.py:27-46 with the
    PosteriorScore drift a = g (prior + lik), nets.py:155-157): same RNG consumption as CDE."""
    xdim = lik_params[-1][0].shape[0]
    st = rng_init(seed, np.arange(chain_offset, chain_offset + num_samples), stream)
    x0 = (rng_normals(st, xdim) * F32(std) + F32(mean)).astype(F32)
    y = np.asarray(y, F32)
    return em_sample(lambda x, tau: posterior_a(prior_params, lik_params, x, y, tau, act=act), x0, num_steps, T=T,
                     rng_state=st, xdim=xdim)


def cdiffe_sample(params, y, num_samples, num_steps, seed, mean=0.0, std=1.0, chain_offset=0, stream=0,
                  T=1.0, beta_min=BETA_MIN, beta_max=BETA_MAX, corrector_steps=0, snr=0.16):
    """Product-RNG CDiffE sampler, repaired semantics of models/diffusion.py:158-180 (the reference
    loop raises TypeError at :174): per step y_t = eps std(T-t) + mean_weight(T-t) y
    (sdes.py:37-44, eps = ydim fresh normals), a = net(x, y_t, T-t)[:, :xdim], then the EM update of
    the x part with xdim fresh normals. x0 as CDE."""
    xdim = params[0][0].shape[1] - np.asarray(y).shape[-1] - 1
    ydim = np.asarray(y).shape[-1]
    st = rng_init(seed, np.arange(chain_offset, chain_offset + num_samples), stream)
    x = (rng_normals(st, xdim) * F32(std) + F32(mean)).astype(F32)
    y = np.asarray(y, F32).reshape(1, ydim)
    ts, tau = schedule(num_steps, T)
    delta = float(T) / num_steps
    for i in range(num_steps):
        mw = vp_mean_weight(tau[i], beta_min, beta_max)
        sd = np.sqrt(vp_var(tau[i], beta_min, beta_max)).astype(F32)
        eps = rng_normals(st, ydim)
        y_t = ((eps * sd).astype(F32) + (mw * y).astype(F32)).astype(F32)
        beta = vp_beta(tau[i], beta_min, beta_max)
        g = np.sqrt(beta).astype(F32)
        for _ in range(corrector_steps):
            # Langevin corrector (the build's definition, include/dmip.h dmip_em_sample_cdiffe; no
            # reference code): step 2 alpha (snr |z| / |s|)^2 at the norms' expected values for the
            # VP perturbation kernel, 2 alpha snr^2 var(T - t); alpha = exp(-beta delta)
            sc = (cde_a(params, x, y_t, tau[i])[:, :xdim] / g).astype(F32)
            z = rng_normals(st, xdim)
            alpha = np.exp(-beta * F32(delta)).astype(F32)
            es = (F32(2.0) * alpha * ((F32(snr) * F32(snr)) * (sd * sd))).astype(F32)
            x = (x + es * sc + np.sqrt(F32(2.0) * es) * z).astype(F32)
        a = cde_a(params, x, y_t, tau[i])[:, :xdim]
        xi = rng_normals(st, xdim)
        x = em_step(x, a, tau[i], delta, beta_min, beta_max, xi)
    return x


# ------------------------------------------------------------------------------------------
# A11  evaluation metric -- main_diffusion_scatterometry.py:71-102
# ------------------------------------------------------------------------------------------

def hist_kl(samples_true, samples_model, nbins=75, lim=(-1.2, 1.2), eps=1e-10):
    """KL2 = sum rel_entr(p_true+eps, p_model+eps) on a nbins^d histogram, renormalised."""
    from scipy.special import rel_entr
    d = samples_true.shape[1]
    rng = [lim] * d
    ht, _ = np.histogramdd(samples_true, bins=(nbins,) * d, range=rng)
    hm, _ = np.histogramdd(samples_model, bins=(nbins,) * d, range=rng)
    ht = ht / ht.sum() + eps
    hm = hm / hm.sum() + eps
    ht /= ht.sum()
    hm /= hm.sum()
    return float(np.sum(rel_entr(ht, hm))), float(np.sum(rel_entr(hm, ht)))


def ks_2samp_stat(a, b):
    """Two-sample Kolmogorov-Smirnov statistic (no p-value)."""
    a = np.sort(np.asarray(a, np.float64))
    b = np.sort(np.asarray(b, np.float64))
    z = np.concatenate([a, b])
    ca = np.searchsorted(a, z, side="right") / a.size
    cb = np.searchsorted(b, z, side="right") / b.size
    return float(np.max(np.abs(ca - cb)))


# ------------------------------------------------------------------------------------------
# A13-A17  DSM / ScoreFPE / PINN losses and their parameter gradients -- losses.py:42-242
# Restated with explicit forward-mode jets and a hand-written reverse pass (the formulation of the
# fused HIP training kernel), in float64. Pinned against the reference's autograd values and
# gradients (tests/golden/pinn_linear.npz, G5) by tests/test_oracle_golden.py.
# ------------------------------------------------------------------------------------------

def _vp_terms(t, beta_min=BETA_MIN, beta_max=BETA_MAX):
    """alpha, std, beta, g and their t-derivatives (sdes.py:21-35), float64."""
    d = beta_max - beta_min
    alpha = np.exp(-0.25 * t * t * d - 0.5 * t * beta_min)
    e = np.exp(-0.5 * t * t * d - t * beta_min)
    var = 1.0 - e
    std = np.sqrt(var)
    beta = beta_min + d * t
    g = np.sqrt(beta)
    dalpha = alpha * (-0.5 * t * d - 0.5 * beta_min)
    dstd = e * (t * d + beta_min) / (2.0 * std)
    dg = d / (2.0 * g)
    return alpha, std, beta, g, dalpha, dstd, dg


def loss_grad(params, x, y, t, eps, kind="pinn", pde="FPE", pde_metric="L1", ic_metric="L2", lam=1.0,
              lam2=1.0, ic_A=None, ic_b=None, ic_Sinv=None, beta_min=BETA_MIN, beta_max=BETA_MAX, ic_target=None):
    """Loss value, components and parameter gradients of the CDE training losses for one batch,
    with the reference's semantics (models/diffusion.py:80-89 -> losses.py):
      kind 'dsm'     DSMLoss(a/g, std, eps).mean()                        (losses.py:42-52)
      kind 'dsm_pde' DSM_PDELoss: mean(DSM + lam PDE)                      (losses.py:126-164)
      kind 'pinn'    PINNLoss: mean(DSM + IC) + mean(lam PDE)              (losses.py:168-242)
      kind 'pinn2'   PINNLoss2: mean(IC + lam PDE)                         (losses.py:245-290)
    PDE 'FPE' = ScoreFPELoss (exact divergence; ds/dt the total derivative through x_t(t) and g(t);
    grad_x detached), 'cFPE' = ConditionalScoreFPELoss. IC = lam2 * metric(a(x, y, 0)/g(0) - ic(x, y))
    with ic the linear problem's analytic posterior score (linear_problem.py:61-65), or the given
    ic_target (n, d) (e.g. the scatterometry -energy_grad, main_diffusion_scatterometry.py:142-145).
    Network: nets.py:17-35 with the double tanh on layer 1. Returns (loss, comps, grads) where
    grads = [(dW, db), ...] per linear layer."""
    P = [(np.asarray(W, np.float64), np.asarray(b, np.float64)) for W, b in params]
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    t = np.asarray(t, np.float64).reshape(-1, 1)
    eps = np.asarray(eps, np.float64)
    B, d = x.shape
    L = len(P)
    alpha, std, beta, g, dalpha, dstd, dg = _vp_terms(t, beta_min, beta_max)
    x_t = eps * std + alpha * x
    xdot = dalpha * x + dstd * eps

    def forward(u, udot_list, u2_list=None, with_bias=True):
        """Primal + first-order tangents (list of input directions) + optional second-order
        (pairs of tangent indices). Returns per-layer caches and outputs."""
        caches = []
        h = u
        hd = list(udot_list)
        h2 = {} if u2_list is None else {k: np.zeros_like(u) for k in u2_list}
        for li, (W, b) in enumerate(P):
            z = h @ W.T + (b if with_bias else 0.0)
            zd = [v @ W.T for v in hd]
            z2 = {k: v @ W.T for k, v in h2.items()}
            if li == L - 1:
                caches.append(dict(h_in=h, hd_in=hd))
                return z, zd, z2, caches
            if li == 0:
                p = np.tanh(z)
                hn = np.tanh(p)
                d1 = (1 - hn * hn) * (1 - p * p)
                d2 = -2 * (1 - p * p) * (hn * d1 + p * (1 - hn * hn))
            else:
                p = None
                hn = np.tanh(z)
                d1 = 1 - hn * hn
                d2 = -2 * hn * d1
            hdn = [d1 * v for v in zd]
            h2n = {(a, c): d1 * z2[(a, c)] + d2 * zd[a] * zd[c] for (a, c) in z2}
            caches.append(dict(h_in=h, hd_in=hd, z=z, zd=zd, d1=d1, d2=d2))
            h, hd, h2 = hn, hdn, h2n
        raise AssertionError

    inp = lambda xx, yy, tt: np.concatenate([xx, yy, np.broadcast_to(tt, (xx.shape[0], 1))], axis=1)
    u_P = inp(x_t, y, t)
    e = np.zeros((B, u_P.shape[1]))
    v_dir = e.copy()
    v_dir[:, :d] = xdot
    v_dir[:, -1] = 1.0
    dirs = [v_dir]
    if pde == "FPE":
        for a in range(d):
            ea = e.copy()
            ea[:, a] = 1.0
            dirs.append(ea)
        pairs = [(1 + a, 1 + c) for a in range(d) for c in range(a, d)]
    else:
        pairs = None
    aP, aT, a2, cache_P = forward(u_P, dirs, pairs)
    s = aP / g
    a_V = aT[0]
    ds_dt = a_V / g - aP * dg / (g * g)
    comps = {}
    # DSM (losses.py:50-52)
    r = s * std + eps
    dsm_rows = 0.5 * np.sum(r * r, axis=1)
    dL_ds = np.zeros_like(s)
    dL_dV = np.zeros_like(s)
    loss = 0.0
    has_dsm = kind in ("dsm", "dsm_pde", "pinn")
    has_pde = kind in ("dsm_pde", "pinn", "pinn2")
    has_ic = kind in ("pinn", "pinn2")
    comps["DSM"] = dsm_rows.mean()
    if has_dsm:
        loss += dsm_rows.mean()
        dL_ds += r * std / B
    if has_pde:
        if pde == "FPE":
            J = np.stack([aT[1 + a] / g for a in range(d)], axis=2)  # J[b, i, a] = ds_i/dx_a
            H = {k: v / g for k, v in a2.items()}
            div = sum(J[:, i, i] for i in range(d)).reshape(-1, 1)
            grad_x = np.zeros_like(s)
            for j in range(d):
                for i in range(d):
                    key = (1 + min(i, j), 1 + max(i, j))
                    grad_x[:, j] += H[key][:, i]
                    grad_x[:, j] += 2 * s[:, i] * J[:, i, j] + x_t[:, i] * J[:, i, j]
                grad_x[:, j] += s[:, j]
            u = ds_dt - 0.5 * beta * grad_x
            if pde_metric == "L1":
                rows = np.mean(np.abs(u), axis=1)
                du = np.sign(u) / d
            else:
                rows = np.mean(u * u, axis=1)
                du = 2 * u / d
            dds = du  # d rows / d ds_dt
            comps["div"] = div
        else:
            u = std ** 3 * ds_dt - 0.5 * eps * beta * alpha ** 2
            if pde_metric == "L2":
                rows = np.sum(u * u, axis=1)
                du = 2 * u
            else:
                rows = np.sum(np.abs(u), axis=1)
                du = np.sign(u)
            dds = du * std ** 3
        comps["ds_dt"] = ds_dt
        comps["PDE"] = lam * rows.mean()
        comps["pde_rows"] = rows
        loss += lam * rows.mean()
        dL_dV += lam * dds / B / g
        dL_ds += lam * dds / B * (-dg / g)  # through ds_dt's -a g'/g^2 term (times g below)
    dL_daP = dL_ds / g
    grads = [(np.zeros_like(W), np.zeros_like(b)) for W, b in P]

    def backward(cache, abar, adbar, u_in, with_bias=True):
        """Reverse through the primal and the first tangent stream (direction 0)."""
        zbar, zdbar = abar, adbar
        for li in range(L - 1, -1, -1):
            W, b = P[li]
            c = cache[li]
            hin = c["h_in"] if li > 0 else u_in
            hdin = c["hd_in"][0] if li > 0 else cache[0]["hd_in"][0]
            gW = zbar.T @ hin + (zdbar.T @ hdin if zdbar is not None else 0.0)
            gb = zbar.sum(0) if with_bias else 0.0
            grads[li] = (grads[li][0] + gW, grads[li][1] + gb)
            if li == 0:
                break
            hbar = zbar @ W
            hdbar = zdbar @ W if zdbar is not None else None
            cp = cache[li - 1]
            zbar_new = cp["d1"] * hbar
            zdbar_new = None
            if hdbar is not None:
                zdbar_new = cp["d1"] * hdbar
                zbar_new = zbar_new + cp["d2"] * cp["zd"][0] * hdbar
            zbar, zdbar = zbar_new, zdbar_new

    backward(cache_P, dL_daP, dL_dV, u_P)
    if has_ic:
        u_C = inp(x, y, np.zeros_like(t))
        aC, _, _, cache_C = forward(u_C, [e])  # dummy tangent (zero direction)
        g0 = np.sqrt(beta_min)
        s0 = aC / g0
        if ic_target is not None:
            ic = np.asarray(ic_target, np.float64)
        else:
            A = np.asarray(ic_A, np.float64)
            bb = np.asarray(ic_b, np.float64)
            S = np.asarray(ic_Sinv, np.float64)
            ic = -x + ((y - (x @ A.T + bb)) @ S.T) @ A
        dlt = s0[:, :d] - ic
        if ic_metric == "L2":
            rows = lam2 * np.mean(dlt * dlt, axis=1)
            dd = lam2 * 2 * dlt / d
        else:
            rows = lam2 * np.mean(np.abs(dlt), axis=1)
            dd = lam2 * np.sign(dlt) / d
        comps["IC"] = rows.mean()
        loss += rows.mean()
        abar = np.zeros_like(aC)
        abar[:, :d] = dd / B / g0
        backward(cache_C, abar, None, u_C)
    comps["loss"] = loss
    return loss, comps, grads


# ------------------------------------------------------------------------------------------
# F2  scatterometry surrogate, negative log posterior and its input gradient
#     utils_scatterometry.py:8-25 (model), :30-38 (get_log_posterior), models/SNF.py:234-237
#     (energy_grad by autograd; restated here as the explicit vector-Jacobian product)
# ------------------------------------------------------------------------------------------

def surrogate_params_from_npz(z, prefix=""):
    """[(W, b)] of nn.Sequential(Linear, ReLU, Linear, ReLU, Linear, ReLU, Linear): keys 0, 2, 4, 6."""
    return [(np.asarray(z[f"{prefix}{i}_weight"]), np.asarray(z[f"{prefix}{i}_bias"])) for i in (0, 2, 4, 6)]


def surrogate_forward(params, x, keep=False):
    """forward_model(x) in float64 (Linear -> ReLU x3 -> Linear)."""
    h = np.asarray(x, np.float64)
    pre = []
    for i, (W, b) in enumerate(params):
        z = h @ np.asarray(W, np.float64).T + np.asarray(b, np.float64)
        if i < len(params) - 1:
            pre.append(z)
            h = np.maximum(z, 0.0)
        else:
            h = z
    return (h, pre) if keep else h


def scat_log_posterior(params, x, y, a=0.2, b=0.01, lambd_bd=1000.0, grad=False):
    """Negative log posterior get_log_posterior (utils_scatterometry.py:30-38):
    E = 0.5 sum log((a f)^2 + b^2) + 0.5 sum (y - f)^2 / ((a f)^2 + b^2) + lambd_bd sum relu(x-1) + relu(-1-x).
    grad=True also returns dE/dx (energy_grad, models/SNF.py:234-237): the reverse pass through the
    surrogate with v = dE/df = a^2 f / pref - (y - f) / pref - a^2 f (y - f)^2 / pref^2, plus the
    boundary term lambd_bd ([x > 1] - [x < -1]) (torch's relu gradient is 0 at 0)."""
    x = np.asarray(x, np.float64)
    y = np.broadcast_to(np.asarray(y, np.float64), (x.shape[0], np.shape(y)[-1]))
    f, pre = surrogate_forward(params, x, keep=True)
    pref = (a * f) ** 2 + b ** 2
    res = y - f
    e = 0.5 * np.log(pref).sum(1) + 0.5 * (res ** 2 / pref).sum(1) + lambd_bd * (
        np.maximum(x - 1, 0) + np.maximum(-1 - x, 0)).sum(1)
    if not grad:
        return e
    v = a * a * f / pref - res / pref - a * a * f * res ** 2 / pref ** 2
    for i in range(len(params) - 1, -1, -1):
        W = np.asarray(params[i][0], np.float64)
        v = v @ W
        if i > 0:
            v = v * (pre[i - 1] > 0)
    g = v + lambd_bd * ((x > 1).astype(np.float64) - (x < -1).astype(np.float64))
    return e, g


# ------------------------------------------------------------------------------------------
# F3  random-walk Metropolis-Hastings ground truth -- models/SNF.py:250-275 (anneal_to_energy,
#     langevin_prop=False) as generate_scatterometry_ground_truth.py:26-28 drives it
# ------------------------------------------------------------------------------------------

def mh_sample(params, y, num_steps, noise_std, a=0.2, b=0.01, lambd_bd=1000.0, x0=None, noise=None, unif=None,
              seed=None, n_chains=None, chain_offset=0, stream=0):
    """x_prop = x + noise_std * xi; accept iff u < exp(-E(x_prop) + E(x)). Returns (x, E(x) - E(x0)).
    Draws: injected (x0 (n,3), noise (S,n,3), unif (S,n)) -- the reference's captured torch draws --
    or the product RNG keyed (seed, chain_offset + c, stream): x0 from three words
    ((w >> 8) 2^-24 * 2 - 1, float32) unless given, then per step rng_normals(3) (4 words) and one
    word for u = (w >> 8) 2^-24."""
    s = None
    if noise is None:
        s = rng_init(seed, np.arange(chain_offset, chain_offset + n_chains), stream)
    if x0 is None:
        inv = F32(2.0 ** -24)
        x0 = np.stack([((rng_next(s) >> np.uint32(8)).astype(F32) * inv * F32(2.0) - F32(1.0)).astype(F32)
                       for _ in range(3)], 1)
    x = np.asarray(x0, F32).copy()
    e_cur = scat_log_posterior(params, x, y, a, b, lambd_bd)
    e0 = e_cur.copy()
    for i in range(num_steps):
        if noise is None:
            xi = rng_normals(s, 3)
            u = ((rng_next(s) >> np.uint32(8)).astype(F32) * F32(2.0 ** -24)).astype(F32)
        else:
            xi, u = np.asarray(noise[i], F32), np.asarray(unif[i], F32)
        xp = (x + (F32(noise_std) * xi).astype(F32)).astype(F32)
        e_prop = scat_log_posterior(params, xp, y, a, b, lambd_bd)
        acc = u < np.exp(-e_prop + e_cur)
        x = np.where(acc[:, None], xp, x)
        e_cur = np.where(acc, e_prop, e_cur)
    return x, e_cur - e0


# ------------------------------------------------------------------------------------------
# config 4  DPS (Chung et al. 2023, Alg. 1) on the EM predictor -- no reference code (SURVEY.md
#           §0 D5); the build's definition (include/dmip.h dmip_dps_sample), restated here
# ------------------------------------------------------------------------------------------

def mlp2_jet(params, x, tau):
    """Prior score s = MLP2(cat[x, tau]) (nets.py:37-57, double tanh on layer 1) and its Jacobian
    J[n, i, k] = ds_i / dx_k by forward-mode tangents, float64."""
    x = np.asarray(x, np.float64)
    n, d = x.shape
    inp = np.concatenate([x, np.full((n, 1), np.float64(tau))], 1)
    W, b = [np.asarray(p[0], np.float64) for p in params], [np.asarray(p[1], np.float64) for p in params]
    z = inp @ W[0].T + b[0]
    t1 = np.tanh(z)
    h = np.tanh(t1)
    dh = ((1 - h * h) * (1 - t1 * t1))[:, :, None] * W[0][None, :, :d]  # (n, W, d)
    for l in range(1, len(W) - 1):
        z = h @ W[l].T + b[l]
        dz = np.einsum("ij,njk->nik", W[l], dh)
        h = np.tanh(z)
        dh = (1 - h * h)[:, :, None] * dz
    s = h @ W[-1].T + b[-1]
    J = np.einsum("ij,njk->nik", W[-1], dh)
    return s, J


def surrogate_residual_grad(sur_params, x, y, mode="norm", a=0.2, b=0.01):
    """L(x) and dL/dx through the ReLU surrogate (float64): mode "norm": L = ||y - F(x)||^2;
    mode "nll": L = 0.5 sum log pref + 0.5 sum (y - F)^2 / pref (the likelihood part of
    get_log_posterior, utils_scatterometry.py:33-35)."""
    f, pre = surrogate_forward(sur_params, x, keep=True)
    r = np.asarray(y, np.float64) - f
    if mode == "norm":
        L = (r * r).sum(1)
        v = -2.0 * r
    else:
        pref = (a * f) ** 2 + b ** 2
        L = 0.5 * np.log(pref).sum(1) + 0.5 * (r * r / pref).sum(1)
        v = a * a * f / pref - r / pref - a * a * f * r * r / pref ** 2
    for i in range(len(sur_params) - 1, -1, -1):
        v = v @ np.asarray(sur_params[i][0], np.float64)
        if i > 0:
            v = v * (pre[i - 1] > 0)
    return L, v


def dps_sample(prior_params, sur_params, y, num_samples, num_steps, seed, zeta=1.0, mode="nll", a=0.2, b=0.01,
               mean=0.0, std=1.0, chain_offset=0, stream=0, T=1.0, beta_min=BETA_MIN, beta_max=BETA_MAX):
    """DPS with the prior score network (include/dmip.h dmip_dps_sample): per step (tau = T - t_i)
      s, J = prior(x, tau), ds/dx;  x0_hat = (x + var(tau) s) / mean_weight(tau)   (Tweedie)
      G = (I + var J^T) (dL/dx0_hat) / mean_weight
      x <- EM(x, a = g s, xi) - lambda G
    mode "nll": L = likelihood NLL, lambda = zeta delta beta; "norm": L = ||y - F||^2,
    lambda = zeta / ||y - F(x0_hat)||. RNG as the CDE sampler (x0 then one 3-normal draw per step)."""
    st = rng_init(seed, np.arange(chain_offset, chain_offset + num_samples), stream)
    x = (rng_normals(st, 3) * F32(std) + F32(mean)).astype(F32)
    ts, tau = schedule(num_steps, T)
    delta = float(T) / num_steps
    y = np.asarray(y, np.float64).reshape(1, -1)
    for i in range(num_steps):
        s, J = mlp2_jet(prior_params, x, tau[i])
        mw = np.float64(vp_mean_weight(tau[i], beta_min, beta_max))
        var = np.float64(vp_var(tau[i], beta_min, beta_max))
        x0h = (x + var * s) / mw
        L, gx = surrogate_residual_grad(sur_params, x0h, y, mode, a, b)
        gt = (gx + var * np.einsum("nik,ni->nk", J, gx)) / mw
        xi = rng_normals(st, 3)
        beta = vp_beta(tau[i], beta_min, beta_max)
        g = np.sqrt(beta).astype(F32)
        if mode == "nll":
            lam = np.full(x.shape[0], np.float64(zeta) * np.float64(F32(delta)) * np.float64(beta))
        else:
            lam = np.float64(zeta) / np.sqrt(np.maximum(L, 1e-30))
        xe = em_step(x, (g * s.astype(F32)).astype(F32), tau[i], delta, beta_min, beta_max, xi)
        x = (xe - (lam[:, None] * gt).astype(F32)).astype(F32)
    return x


# ------------------------------------------------------------------------------------------
# A18  PosteriorLoss -- losses.py:293-386, driven by PosteriorDiffusionEstimator.train_epoch
#      (models/diffusion.py:204-229). Test infrastructure (the checker of the fused HIP path).
# ------------------------------------------------------------------------------------------

def _mlp_tape(params, inp):
    """Forward of the reference MLP chain (double tanh on layer 1) in float64, keeping what the
    reverse pass needs: per layer its input and the activation derivative."""
    W = [np.asarray(p[0], np.float64) for p in params]
    b = [np.asarray(p[1], np.float64) for p in params]
    h = np.asarray(inp, np.float64)
    tape = []
    for li in range(len(W)):
        z = h @ W[li].T + b[li]
        if li == len(W) - 1:
            tape.append((h, None))
            h = z
        elif li == 0:
            t1 = np.tanh(z)
            t2 = np.tanh(t1)
            tape.append((h, (1 - t2 * t2) * (1 - t1 * t1)))
            h = t2
        else:
            t = np.tanh(z)
            tape.append((h, 1 - t * t))
            h = t
    return h, tape, W


def _mlp_backprop(tape, W, adj):
    """Reverse pass from the output adjoint adj (n, out): per-layer (dW, db) and d/d(input)."""
    grads = [None] * len(W)
    d = np.asarray(adj, np.float64)
    for li in range(len(W) - 1, -1, -1):
        h_in, dact = tape[li]
        grads[li] = (d.T @ h_in, d.sum(0))
        d = d @ W[li]
        if li > 0:
            d = d * tape[li - 1][1]
    return grads, d


def reference_weights(dims, seed):
    """nn.Linear-range weights from a numpy seed (tests/golden/make_golden.py reference_weights, G11)."""
    g = np.random.default_rng(seed)
    out = []
    for i in range(len(dims) - 1):
        bd = 1.0 / np.sqrt(dims[i])
        out.append((g.uniform(-bd, bd, (dims[i + 1], dims[i])).astype(F32),
                    g.uniform(-bd, bd, dims[i + 1]).astype(F32)))
    return out


def posterior_loss_grad(prior_params, lik_params, sur_params, x, y, t, eps, a=0.2, b=0.01, lam=0.01,
                        beta_min=BETA_MIN, beta_max=BETA_MAX):
    """PosteriorLoss(forward_model, a, b, lam)(sde, x, y, t) and loss.backward(), float64.

    The reference's likelihood target takes every autograd.grad without create_graph (losses.py:
    358-365): it is a constant for the parameter gradients, which therefore come from the prior's DSM
    term (losses.py:376) and the likelihood net's regression term (losses.py:381) only. By linearity
    the three VJPs and three vector-Hessian (input-Jacobian) products collapse to
        target = (I + std^2 J_s^T) J_F^T (v2 + a^2 (v3 - v1)),
    J_s = d s_prior / d x_t, J_F = dF/dx0 at x0 = (x_t + std^2 s_prior) / alpha (losses.py:379-380).
    Returns (loss, {'PriorLoss', 'LikelihoodLoss'}, grads_prior [(dW, db)], grads_lik, target)."""
    x = np.asarray(x, np.float64)
    n, d = x.shape
    t = np.asarray(t, np.float64).reshape(-1, 1)
    eps = np.asarray(eps, np.float64)
    y = np.asarray(y, np.float64)
    bmin, bdiff = np.float64(beta_min), np.float64(beta_max - beta_min)
    alpha = np.exp(-0.25 * t * t * bdiff - 0.5 * t * bmin)
    std = np.sqrt(1.0 - np.exp(-0.5 * t * t * bdiff - t * bmin))
    x_t = eps * std + alpha * x
    s_p, tape_p, Wp = _mlp_tape(prior_params, np.concatenate([x_t, t], 1))
    s_l, tape_l, Wl = _mlp_tape(lik_params, np.concatenate([x_t, y, t], 1))
    x0 = (x_t + std ** 2 * s_p) / alpha
    f, pre = surrogate_forward(sur_params, x0, keep=True)
    pref = (a * f) ** 2 + b ** 2
    v1, v2, v3 = f / pref, (y - f) / pref, (y - f) ** 2 * f / pref
    u = v2 + a * a * (v3 - v1)
    for i in range(len(sur_params) - 1, -1, -1):
        u = u @ np.asarray(sur_params[i][0], np.float64)
        if i > 0:
            u = u * (pre[i - 1] > 0)
    _, jtu = _mlp_backprop(tape_p, Wp, u)  # J_s^T u: the input gradient of the prior at x_t
    target = u + std ** 2 * jtu[:, :d]
    prior_rows = 0.5 * ((s_p * std + eps) ** 2).sum(1)
    lik_rows = ((alpha * s_l - target) ** 2).sum(1)
    loss = float(np.mean(prior_rows + lam * lik_rows))
    gp, _ = _mlp_backprop(tape_p, Wp, (s_p * std + eps) * std / n)
    gl, _ = _mlp_backprop(tape_l, Wl, 2.0 * lam * alpha * (alpha * s_l - target) / n)
    info = {"PriorLoss": float(prior_rows.mean()), "LikelihoodLoss": float(lam * lik_rows.mean())}
    return loss, info, gp, gl, target
