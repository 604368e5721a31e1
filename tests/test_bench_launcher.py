"""bench.py's multi-GPU launcher on CPU: `python bench.py --gpus 2` (WORLD_SIZE unset) starts two rank
processes itself, each runs the sampler stand-in on its chain range over gloo, and rank 0 prints one
JSON line reporting 2 ranks and the full gathered shape (the RCCL path is the same code with the
nccl backend on the GPU box)."""
import json
import os
import socket
import subprocess
import sys
import time

from conftest import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["MASTER_ADDR"] = "127.0.0.1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--stub", "--master-port", str(_free_port())]
                       + args, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_launcher_spawns_ranks_weak_scaling():
    out = _run(["--gpus", "2", "--chains", "37"])
    assert out["n_gpus"] == 2 and out["chains_total"] == 74
    assert out["gathered_shape"] == [1, 74, 3] and out["gather_ok"]
    # the world size torch.distributed reports after init, and every rank's device (gathered)
    assert out["dist"]["world_size_observed"] == 2
    assert out["dist"]["devices"] == ["0:cpu", "1:cpu"]


def test_launcher_strong_scaling_ragged():
    out = _run(["--gpus", "3", "--chains-total", "100"])
    assert out["n_gpus"] == 3 and out["gathered_shape"] == [1, 100, 3] and out["gather_ok"]


def test_mismatched_world_size_is_an_error():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--stub", "--gpus", "2"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_launcher_fails_fast_when_a_rank_dies():
    """A rank that exits non-zero after init (the others blocked in the gather) makes the launcher
    terminate its siblings and return non-zero within seconds, not at the collective timeout."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["MASTER_ADDR"] = "127.0.0.1"
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--stub", "--gpus", "3", "--stub-fail-rank", "1",
                        "--dist-timeout", "600", "--master-port", str(_free_port())],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    dt = time.time() - t0
    assert r.returncode != 0
    assert "rank 1 exited with 1" in r.stderr, r.stderr[-2000:]
    assert dt < 120, dt
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
