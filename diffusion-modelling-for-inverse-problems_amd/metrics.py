"""Distributional parity metrics for posterior samples (per-dimension two-sample KS,
(sliced) Wasserstein-1, against the reference sampler's own stored draws).

The reference scores its posteriors with 75-bin KL (main_diffusion_scatterometry.py:71-102, see
evaluate.py); the parity gate between this sampler and the reference's CPU sampler uses these
sample-based distances, each with a stated null level:

* ks_2samp_stat / ks_crit: the two-sample Kolmogorov-Smirnov statistic and its alpha = 0.01 critical
  value 1.63 sqrt((n1 + n2) / (n1 n2)).
* ks_vs_quantiles: KS against a reference run stored as its 1001 quantiles (np.quantile at u = k/1000
  of n_ref samples): max_k |F_n(q_k) - k/1000|, which bounds the true statistic to within 1/1000;
  the critical value is ks_crit(n, n_ref) + 1/1000.
* w1_1d: exact 1-D W1 between two samples; w1_vs_quantiles: W1 to a quantile-stored reference.
* w1_null: the expected W1 between two independent samples of sizes n1, n2 of the same
  distribution, sqrt(2/pi) J sqrt(1/n1 + 1/n2) with J = int sqrt(F (1 - F)) dx (the Brownian-bridge
  limit of sqrt(n) (F_n - F)); J is computed from the reference's own quantiles / samples.
* sliced_w1: mean 1-D W1 over fixed random unit directions, with the matching null level.
Pure numpy; used by bench.py (reported beside the throughput) and the parity tests.
"""
import numpy as np


def ks_crit(n1, n2, c=1.63):
    return c * float(np.sqrt((n1 + n2) / (n1 * n2)))


def ks_2samp_stat(a, b):
    a = np.sort(np.asarray(a, np.float64))
    b = np.sort(np.asarray(b, np.float64))
    both = np.concatenate([a, b])
    ca = np.searchsorted(a, both, side="right") / a.size
    cb = np.searchsorted(b, both, side="right") / b.size
    return float(np.max(np.abs(ca - cb)))


def ks_vs_quantiles(x, q):
    """KS of samples x (n,) against a reference stored as quantiles q (K+1,) at u = k/K."""
    x = np.sort(np.asarray(x, np.float64))
    K = len(q) - 1
    u = np.arange(K + 1) / K
    fn = np.searchsorted(x, np.asarray(q, np.float64), side="right") / x.size
    return float(np.max(np.abs(fn - u)))


def w1_1d(a, b):
    """Exact W1 between the empirical distributions of a and b: int |F_a - F_b| dx."""
    a = np.sort(np.asarray(a, np.float64))
    b = np.sort(np.asarray(b, np.float64))
    both = np.sort(np.concatenate([a, b]))
    dx = np.diff(both)
    ca = np.searchsorted(a, both[:-1], side="right") / a.size
    cb = np.searchsorted(b, both[:-1], side="right") / b.size
    return float(np.sum(np.abs(ca - cb) * dx))


def w1_vs_quantiles(x, q):
    """W1 = int |Q_x(u) - Q_ref(u)| du on the reference's quantile grid over u in [1/K, 1 - 1/K]
    (trapezoid; the sample extremes at u = 0, 1 are left out)."""
    K = len(q) - 1
    u = np.arange(1, K) / K
    qx = np.quantile(np.asarray(x, np.float64), u)
    d = np.abs(qx - np.asarray(q, np.float64)[1:K])
    return float(np.sum(0.5 * (d[1:] + d[:-1])) / K)


def _j_from_quantiles(q):
    """J over the same interior u range as w1_vs_quantiles."""
    K = len(q) - 1
    um = (np.arange(1, K - 1) + 0.5) / K
    return float(np.sum(np.sqrt(um * (1.0 - um)) * np.diff(np.asarray(q, np.float64)[1:K])))


def _j_from_sample(s):
    s = np.sort(np.asarray(s, np.float64))
    u = np.arange(1, s.size) / s.size
    return float(np.sum(np.sqrt(u * (1.0 - u)) * np.diff(s)))


def w1_null(n1, n2, q=None, sample=None):
    """Expected W1 between independent samples (sizes n1, n2) of the reference distribution, whose
    spread is given by its quantiles q or a sample of it."""
    J = _j_from_quantiles(q) if q is not None else _j_from_sample(sample)
    return float(np.sqrt(2.0 / np.pi) * J * np.sqrt(1.0 / n1 + 1.0 / n2))


def directions(d, k=64, seed=1234):
    v = np.random.default_rng(seed).normal(size=(k, d))
    return v / np.linalg.norm(v, axis=1, keepdims=True)


def sliced_w1(x, ref, k=64, seed=1234):
    """(mean over k fixed directions of the 1-D W1 of the projections, its null level)."""
    x = np.asarray(x, np.float64)
    ref = np.asarray(ref, np.float64)
    V = directions(x.shape[1], k, seed)
    px, pr = x @ V.T, ref @ V.T
    w = [w1_1d(px[:, i], pr[:, i]) for i in range(k)]
    null = [w1_null(x.shape[0], ref.shape[0], sample=pr[:, i]) for i in range(k)]
    return float(np.mean(w)), float(np.mean(null))


def parity_report(x, ref_samples, ref_quantiles=None, n_ref_total=None, w1_factor=3.0):
    """Per-dimension KS and W1 of samples x (n, d) against the reference's stored draws (and, when
    given, the quantiles of its full run of n_ref_total samples), plus sliced W1; each with its
    stated bound. `pass` = every statistic below its bound (KS: alpha = 0.01; W1: w1_factor x the
    expected W1 of two same-distribution samples of these sizes)."""
    x = np.asarray(x, np.float64)
    ref = np.asarray(ref_samples, np.float64)
    n, d = x.shape
    rep = {"n": int(n), "n_ref": int(ref.shape[0])}
    ks = [ks_2samp_stat(x[:, k], ref[:, k]) for k in range(d)]
    rep["ks_draws"] = {"stat": ks, "crit": ks_crit(n, ref.shape[0])}
    w1 = [w1_1d(x[:, k], ref[:, k]) for k in range(d)]
    w1n = [w1_null(n, ref.shape[0], sample=ref[:, k]) for k in range(d)]
    rep["w1_draws"] = {"stat": w1, "null": w1n, "bound": [w1_factor * v for v in w1n]}
    sw, swn = sliced_w1(x, ref)
    rep["sliced_w1_draws"] = {"stat": sw, "null": swn, "bound": w1_factor * swn}
    ok = max(ks) < rep["ks_draws"]["crit"] and all(a <= b for a, b in zip(w1, rep["w1_draws"]["bound"])) \
        and sw <= rep["sliced_w1_draws"]["bound"]
    if ref_quantiles is not None:
        q = np.asarray(ref_quantiles, np.float64)
        nq = int(n_ref_total)
        ksq = [ks_vs_quantiles(x[:, k], q[:, k]) for k in range(d)]
        crit_q = ks_crit(n, nq) + 1.0 / (q.shape[0] - 1)
        w1q = [w1_vs_quantiles(x[:, k], q[:, k]) for k in range(d)]
        w1qn = [w1_null(n, nq, q=q[:, k]) for k in range(d)]
        rep["ks_quantiles"] = {"stat": ksq, "crit": crit_q, "n_ref_total": nq}
        rep["w1_quantiles"] = {"stat": w1q, "null": w1qn, "bound": [w1_factor * v for v in w1qn]}
        ok = ok and max(ksq) < crit_q and all(a <= b for a, b in zip(w1q, rep["w1_quantiles"]["bound"]))
    rep["pass"] = bool(ok)
    return rep
