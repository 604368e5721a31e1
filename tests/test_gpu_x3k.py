"""The k-major multi-tile fp32x3 CDE engine (csrc/dmip_x3k.h: one wave per SIMD with 2 or 3 chain tiles,
static weight ring, resident merged output layer) -- the default path of `CDE.sample_device` at the
headline shape (hidden_layers [256]*3). Needs an MI355X: `pytest -m gpu`.

Gates (the fp32 engines' own, test_gpu_x3.py): the float32 oracle on the same chains within 1e-4 of
max(1, |x|); the one-tile fp32x3 engine (DMIP_X3K=0; identical hidden-layer arithmetic, the output
layer's three partial sums added in another order) within 1e-5 after 1000 steps; chain results
independent of the tiles per wave (bit-identical), of sharding and of the balanced schedule's
hand-overs; the reference's draws through test_gpu_x3.py's parity gate (same entry point).
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


@pytest.fixture(autouse=True)
def _x3k_engine(monkeypatch):
    """The k-major engine is the default at this shape; DMIP_X3P=0 keeps it so under the A/B library too, whose
    opt-in paired-tile engine (dmip_x3p.h) would take the shape with DMIP_X3P=1."""
    monkeypatch.setenv("DMIP_X3P", "0")


def test_x3p_ab_engine_in_diag_library():
    """The A/B paired-tile engine's own tests (tests/test_gpu_x3p.py) in ONE child process on the A/B library
    (the product library does not hold that engine; the library is chosen at import)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    diag = os.path.join(root, "abv", "diag", "libdmip_diag.so")
    if not os.path.exists(diag):
        pytest.skip("A/B library not built (make diag)")
    env = dict(os.environ, DMIP_LIB=diag)
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", os.path.join(root, "tests", "test_gpu_x3p.py"), "-x", "-q",
                        "-m", "gpu", "-p", "no:cacheprovider", "--timeout", "300", "--timeout-method", "thread"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=900)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert " passed" in r.stdout and "skipped" not in r.stdout.splitlines()[-1], r.stdout[-500:]


def _params(net):
    return [(l.weight.detach().cpu().numpy(), l.bias.detach().cpu().numpy())
            for l in net if isinstance(l, torch.nn.Linear)]


def _rel(out, ref):
    return float(np.abs(out - ref).max() / max(1.0, np.abs(ref).max()))


def _seeded(dmip, xd, yd, seed):
    torch.manual_seed(seed)
    return dmip.CDE(xd, yd, [256] * 3)


@pytest.mark.parametrize("xd,yd", [(2, 2), (3, 23)])
@pytest.mark.parametrize("n", [1, 15, 47, 49, 97, 1000])
def test_x3k_vs_oracle_ragged(dmip, xd, yd, n):
    """Chain counts that leave the last job (3 x 16 chains) partial or a tile partly empty."""
    m = _seeded(dmip, xd, yd, 3 + n)
    y = np.random.default_rng(n).uniform(0, 1, yd).astype(np.float32)
    S, seed = 6, 41
    x = m.sample_device(torch.from_numpy(y).to(DEV), n, S, seed=seed, precision=PREC)[0].cpu().numpy()
    ref = O.cde_sample(_params(m.sde.a), y, n, S, seed)
    assert np.all(np.isfinite(x))
    e = _rel(x, ref)
    print(f"\n[x3k] oracle xd={xd} n={n}: {e:.3e}")
    assert e < 1e-4, e


@pytest.mark.parametrize("tag", ["scat", "lin256"])
def test_x3k_matches_one_tile_engine_over_1000_steps(dmip, golden, tag, monkeypatch):
    """Same chains through both fp32x3 engines: the hidden layers are bit-identical, the output layer's
    partial sums are added in another order (~1 ulp per step), over 1000 contracting steps."""
    if tag == "scat":
        m = dmip.CDE(3, 23, [256] * 3)
        m.sde.a.load_state_dict(state_from_npz(golden("ckpt_scat.npz")))
        y = torch.from_numpy(golden("samples_scat.npz")["y"]).to(DEV)
    else:
        m = _seeded(dmip, 2, 2, 77)
        y = torch.tensor([0.5, 1.0], device=DEV)
    a = m.sample_device(y, 20000, 1000, seed=321, precision=PREC)[0].cpu().numpy()
    monkeypatch.setenv("DMIP_X3K", "0")
    b = m.sample_device(y, 20000, 1000, seed=321, precision=PREC)[0].cpu().numpy()
    monkeypatch.delenv("DMIP_X3K")
    assert np.all(np.isfinite(a))
    e = _rel(a, b)
    print(f"\n[x3k] vs one-tile engine, {tag}, 1000 steps: {e:.3e}")
    assert e < 1e-5, e
    assert not np.array_equal(a, b)  # two engines ran (the output layer's summation order differs)


@pytest.mark.parametrize("nt", ["1", "2"])
def test_x3k_tiles_per_wave_bit_identical(dmip, monkeypatch, nt):
    """1, 2 or 3 chain tiles per wave (NT = 1: two waves per SIMD): a chain's arithmetic does not depend on its
    neighbours."""
    m = _seeded(dmip, 3, 23, 5)
    ys = torch.from_numpy(np.random.default_rng(3).uniform(0, 1, (2, 23)).astype(np.float32)).to(DEV)
    monkeypatch.setenv("DMIP_X3K_NT", nt)
    a = m.sample_device(ys, 70001, 8, seed=9, precision=PREC)
    monkeypatch.setenv("DMIP_X3K_NT", "3")
    b = m.sample_device(ys, 70001, 8, seed=9, precision=PREC)
    assert torch.isfinite(a).all()
    assert torch.equal(a, b)


@pytest.mark.parametrize("nt", ["2", "3"])
def test_x3k_balanced_schedule_and_shards(dmip, monkeypatch, nt):
    """More jobs than waves (hand-overs of 2-3 tiles of state) and two ys: every chain equals a launch
    small enough to run whole, and a chain_offset shard is a slice of the whole run."""
    monkeypatch.setenv("DMIP_X3K_NT", nt)
    m = _seeded(dmip, 3, 23, 6)
    ys = torch.from_numpy(np.random.default_rng(4).uniform(0, 1, (2, 23)).astype(np.float32)).to(DEV)
    n, S = 150001, 5
    full = m.sample_device(ys, n, S, seed=17, precision=PREC)
    for lo in (0, 49999, n - 777):
        part = m.sample_device(ys, 777, S, seed=17, chain_offset=lo, precision=PREC)
        assert torch.equal(full[:, lo:lo + 777], part), lo
    assert torch.isfinite(full).all()


def test_x3k_snapshots(dmip):
    """Trajectory snapshots through the multi-tile engine: last = output, shard slices, the oracle's
    loop states."""
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
