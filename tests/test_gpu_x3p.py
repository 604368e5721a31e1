"""The paired-tile 32x32 fp32x3 CDE engine (csrc/dmip_x3p.h: one wave per SIMD with two 32-chain tiles in
ping-pong, layer 1 fused into hidden layer 1 (k-major), hidden layer 2 output-major into an exact-f32 output
layer). An A/B engine: it measured slower than the k-major engine (profiles/r4_ab_x3p_vs_x3k.json), so only
the A/B library (`make diag`, abv/diag/libdmip_diag.so) holds it, opt-in with DMIP_X3P=1. This module runs
in a child process on that library (tests/test_gpu_x3k.py::test_x3p_ab_engine_in_diag_library) and skips
when the loaded library is the product one. Needs an MI355X: `pytest -m gpu`.

Gates (the fp32 engines' own, test_gpu_x3.py): the float32 oracle on the same chains within 1e-4 of
max(1, |x|); the 16x16 k-major engine (DMIP_X3P=0; the same split hidden layers, its output layer split into
fp16 hi/lo where this one is exact f32) within 5e-5 after 1000 steps (the exact-f32 engine: test_gpu_x3.py); chain results independent of sharding,
of the balanced schedule's hand-overs (64-chain jobs whose two tiles run half a chunk apart) and of snapshots;
the reference's own injected-noise trajectories and draws through test_gpu_x3.py (same entry point).
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
def _need_gpu(dmip):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    if not hasattr(dmip._lib.lib(), "dmip_x3p_available"):
        pytest.skip("the paired engine is in the A/B library only (DMIP_LIB=abv/diag/libdmip_diag.so)")


@pytest.fixture(autouse=True)
def _x3p_engine(monkeypatch):
    monkeypatch.setenv("DMIP_X3P", "1")


def _params(net):
    return [(l.weight.detach().cpu().numpy(), l.bias.detach().cpu().numpy())
            for l in net if isinstance(l, torch.nn.Linear)]


def _rel(out, ref):
    return float(np.abs(out - ref).max() / max(1.0, np.abs(ref).max()))


def _seeded(dmip, xd, yd, seed):
    torch.manual_seed(seed)
    return dmip.CDE(xd, yd, [256] * 3)


@pytest.mark.parametrize("xd,yd", [(2, 2), (3, 23)])
@pytest.mark.parametrize("n", [1, 31, 33, 63, 65, 97, 1000])
def test_x3p_vs_oracle_ragged(dmip, xd, yd, n):
    """Chain counts that leave the last 64-chain job or one of its 32-chain tiles partial or empty."""
    m = _seeded(dmip, xd, yd, 3 + n)
    y = np.random.default_rng(n).uniform(0, 1, yd).astype(np.float32)
    S, seed = 6, 41
    before = dmip._lib.calls["em_sample"]
    x = m.sample_device(torch.from_numpy(y).to(DEV), n, S, seed=seed, precision=PREC)[0].cpu().numpy()
    assert dmip._lib.calls["em_sample"] == before + 1
    ref = O.cde_sample(_params(m.sde.a), y, n, S, seed)
    assert np.all(np.isfinite(x))
    e = _rel(x, ref)
    print(f"\n[x3p] oracle xd={xd} n={n}: {e:.3e}")
    assert e < 1e-4, e


@pytest.mark.parametrize("S", [1, 2, 17])
def test_x3p_step_counts_vs_oracle(dmip, S):
    """Tile B completes each step half a chunk after tile A (in the next loop iteration or the epilogue):
    one step, two steps and an odd count against the oracle."""
    m = _seeded(dmip, 3, 23, 100 + S)
    y = np.random.default_rng(S).uniform(0, 1, 23).astype(np.float32)
    x = m.sample_device(torch.from_numpy(y).to(DEV), 200, S, seed=8, precision=PREC)[0].cpu().numpy()
    ref = O.cde_sample(_params(m.sde.a), y, 200, S, 8)
    e = _rel(x, ref)
    print(f"\n[x3p] oracle S={S}: {e:.3e}")
    assert e < 1e-4, e


@pytest.mark.parametrize("tag", ["scat", "lin256"])
def test_x3p_matches_x3k_engine_over_1000_steps(dmip, golden, tag, monkeypatch):
    """Same chains through both multi-tile fp32x3 engines: the same split hidden layers (different MFMA shape
    and summation order), the output layer exact f32 here and split there, over 1000 contracting steps."""
    if tag == "scat":
        m = dmip.CDE(3, 23, [256] * 3)
        m.sde.a.load_state_dict(state_from_npz(golden("ckpt_scat.npz")))
        y = torch.from_numpy(golden("samples_scat.npz")["y"]).to(DEV)
    else:
        m = _seeded(dmip, 2, 2, 77)
        y = torch.tensor([0.5, 1.0], device=DEV)
    a = m.sample_device(y, 20000, 1000, seed=321, precision=PREC)[0].cpu().numpy()
    monkeypatch.setenv("DMIP_X3P", "0")
    b = m.sample_device(y, 20000, 1000, seed=321, precision=PREC)[0].cpu().numpy()
    monkeypatch.setenv("DMIP_X3P", "1")
    assert np.all(np.isfinite(a))
    e = _rel(a, b)
    print(f"\n[x3p] vs x3k engine, {tag}, 1000 steps: {e:.3e}")
    assert e < 5e-5, e  # measured 1.6e-5 (scat: the split output layer vs exact f32 over 1000 steps)
    assert not np.array_equal(a, b)  # two engines ran


def test_x3p_balanced_schedule_and_shards(dmip):
    """More jobs than waves (hand-overs of both tiles' state between waves) and two ys: every chain equals a
    launch small enough to run whole, and a chain_offset shard is a slice of the whole run."""
    m = _seeded(dmip, 3, 23, 6)
    ys = torch.from_numpy(np.random.default_rng(4).uniform(0, 1, (2, 23)).astype(np.float32)).to(DEV)
    n, S = 150001, 5
    full = m.sample_device(ys, n, S, seed=17, precision=PREC)
    for lo in (0, 49999, n - 777):
        part = m.sample_device(ys, 777, S, seed=17, chain_offset=lo, precision=PREC)
        assert torch.equal(full[:, lo:lo + 777], part), lo
    assert torch.isfinite(full).all()


def test_x3p_snapshots(dmip):
    """Trajectory snapshots through the paired engine (tile B's written one loop iteration late, or by the
    segment's epilogue): last = output, shard slices, the oracle's loop states."""
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


def test_x3p_trajectory_outside_fp16_range_reported(dmip, golden):
    """The paired engine's range guard (an output bias of 1e6: |x| ~ 1e5-1e6 after one step): the device status
    word reports it for an explicit fp32x3 request, and the default precision resamples in exact f32."""
    m = dmip.CDE(3, 23, [256] * 3)
    m.sde.a.load_state_dict(state_from_npz(golden("ckpt_scat.npz")))
    with torch.no_grad():
        m.sde.a._modules["7"].bias[:] = 1.0e6
    y = torch.from_numpy(golden("samples_scat.npz")["y"]).to(DEV)
    x3 = m.sample_device(y, 600, 6, seed=91, precision=PREC)
    with pytest.raises(RuntimeError, match="fp16 range"):
        dmip._lib.device_status(x3.device)
    torch.manual_seed(6)
    with pytest.warns(RuntimeWarning, match="fp16 range"):
        x = m(y, num_samples=600, num_steps=6)
    torch.manual_seed(6)
    assert np.array_equal(x, m(y, num_samples=600, num_steps=6, precision="fp32"))
