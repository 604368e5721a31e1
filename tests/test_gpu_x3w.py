"""The 32x32-tile k-major fp32x3 CDE engine (csrc/dmip_x3w.h: one wave per SIMD with one 32-chain tile,
v_mfma_f32_32x32x16_f16, static weight ring, resident layer 1 and merged output layer) -- the default
path of `CDE.sample_device` at the headline shape (hidden_layers [256]*3). Needs an MI355X: `pytest -m gpu`.

Gates (the fp32 engines' own, test_gpu_x3.py): the float32 oracle on the same chains within 1e-4 of
max(1, |x|); the 16x16 k-major engine (DMIP_X3W=0: the same three-product arithmetic, its MFMAs summing
in another order) within 3e-5 after 1000 steps; chain results independent of sharding and of the
balanced schedule's hand-overs (bit-identical); snapshots; the reference's injected-noise trajectories
and draws through test_gpu_x3.py's gates (same entry point).
"""
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


def _params(net):
    return [(l.weight.detach().cpu().numpy(), l.bias.detach().cpu().numpy())
            for l in net if isinstance(l, torch.nn.Linear)]


def _rel(out, ref):
    return float(np.abs(out - ref).max() / max(1.0, np.abs(ref).max()))


def _seeded(dmip, xd, yd, seed):
    torch.manual_seed(seed)
    return dmip.CDE(xd, yd, [256] * 3)


def test_x3w_is_the_default_at_its_shape(dmip):
    """The headline shape runs the 32x32 engine (its launch counter), with no fallback."""
    m = _seeded(dmip, 3, 23, 1)
    y = torch.rand(23, device=DEV)
    before = dmip._lib.calls.get("em_sample", 0)
    x = m.sample_device(y, 100, 3, seed=1, precision=PREC)
    assert dmip._lib.calls.get("em_sample", 0) == before + 1
    assert torch.isfinite(x).all()


@pytest.mark.parametrize("xd,yd", [(2, 2), (3, 23)])
@pytest.mark.parametrize("n", [1, 31, 33, 63, 65, 1000])
def test_x3w_vs_oracle_ragged(dmip, xd, yd, n):
    """Chain counts that leave the last 32-chain job partial."""
    m = _seeded(dmip, xd, yd, 5 + n)
    y = np.random.default_rng(n).uniform(0, 1, yd).astype(np.float32)
    S, seed = 6, 43
    x = m.sample_device(torch.from_numpy(y).to(DEV), n, S, seed=seed, precision=PREC)[0].cpu().numpy()
    ref = O.cde_sample(_params(m.sde.a), y, n, S, seed)
    assert np.all(np.isfinite(x))
    e = _rel(x, ref)
    print(f"\n[x3w] oracle xd={xd} n={n}: {e:.3e}")
    assert e < 1e-4, e


@pytest.mark.parametrize("tag", ["scat", "lin256"])
def test_x3w_matches_x3k_over_1000_steps(dmip, golden, tag, monkeypatch):
    """Same chains through the 32x32 and the 16x16 k-major engines (same products, MFMA sums in another
    order), over 1000 contracting steps."""
    if tag == "scat":
        m = dmip.CDE(3, 23, [256] * 3)
        m.sde.a.load_state_dict(state_from_npz(golden("ckpt_scat.npz")))
        y = torch.from_numpy(golden("samples_scat.npz")["y"]).to(DEV)
    else:
        m = _seeded(dmip, 2, 2, 79)
        y = torch.tensor([0.5, 1.0], device=DEV)
    a = m.sample_device(y, 20000, 1000, seed=321, precision=PREC)[0].cpu().numpy()
    monkeypatch.setenv("DMIP_X3W", "0")
    b = m.sample_device(y, 20000, 1000, seed=321, precision=PREC)[0].cpu().numpy()
    monkeypatch.delenv("DMIP_X3W")
    assert np.all(np.isfinite(a))
    e = _rel(a, b)
    print(f"\n[x3w] vs x3k, {tag}, 1000 steps: {e:.3e}")
    assert e < 3e-5, e
    assert not np.array_equal(a, b)  # two engines ran


def test_x3w_injected_noise_matches_reference(dmip, golden):
    """The reference's own x0 and per-step noise (G3, scatterometry, 1000 steps) through the 32x32
    engine: within the fp32 gate 1e-3 max|x|."""
    tr = golden("traj_scat.npz")
    m = dmip.CDE(3, 23, [256] * 3)
    m.sde.a.load_state_dict(state_from_npz(golden("ckpt_scat.npz")))
    S = int(tr["num_steps"])
    noise = np.concatenate([tr["x0"][None], tr["xi"]], 0)[:, None]
    n = tr["x0"].shape[0]
    out = m.sample_device(torch.from_numpy(tr["y"]).to(DEV), n, S, noise=torch.from_numpy(noise).to(DEV),
                          precision=PREC)[0].cpu().numpy()
    ref = tr["x_final"]
    assert np.all(np.isfinite(out))
    e = _rel(out, ref)
    print(f"\n[x3w] G3 scat: {S} steps, max err / max|x| = {e:.3e}")
    assert e < 1e-3, e


def test_x3w_balanced_schedule_and_shards(dmip):
    """More jobs than waves (hand-overs) and two ys: every chain equals a launch small enough to run
    whole, and a chain_offset shard is a slice of the whole run."""
    m = _seeded(dmip, 3, 23, 6)
    ys = torch.from_numpy(np.random.default_rng(4).uniform(0, 1, (2, 23)).astype(np.float32)).to(DEV)
    n, S = 150001, 5
    full = m.sample_device(ys, n, S, seed=17, precision=PREC)
    for lo in (0, 49999, n - 777):
        part = m.sample_device(ys, 777, S, seed=17, chain_offset=lo, precision=PREC)
        assert torch.equal(full[:, lo:lo + 777], part), lo
    assert torch.isfinite(full).all()


def test_x3w_snapshots(dmip):
    """Trajectory snapshots: last = output, shard slices, the oracle's loop states."""
    m = _seeded(dmip, 3, 23, 8)
    y = torch.from_numpy(np.random.default_rng(6).uniform(0, 1, (2, 23)).astype(np.float32)).to(DEV)
    n, S, every, seed = 90000, 24, 6, 7
    x, snaps = m.sample_trajectory(y, n, S, every, seed=seed, precision=PREC)
    assert tuple(snaps.shape) == (S // every, 2, n, 3)
    assert torch.equal(snaps[-1], x) and torch.isfinite(snaps).all()
    assert torch.equal(m.sample_device(y, n, S, seed=seed, precision=PREC), x)
    lo, hi = 30011, 61000
    xs, ss = m.sample_trajectory(y, hi - lo, S, every, seed=seed, chain_offset=lo, precision=PREC)
    assert torch.equal(ss, snaps[:, :, lo:hi]) and torch.equal(xs, x[:, lo:hi])
    yy = y[0].cpu().numpy()
    _, sn1 = m.sample_trajectory(y[:1], 700, 6, 2, seed=99, precision=PREC)
    _, ref_snaps = O.cde_sample(_params(m.sde.a), yy, 700, 6, 99, snapshots={2, 4, 6})
    for k in range(3):
        assert _rel(sn1[k, 0].cpu().numpy(), ref_snaps[(k + 1) * 2]) < 1e-4
