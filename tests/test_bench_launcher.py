"""bench.py's multi-GPU launcher on CPU: `python bench.py --gpus 2` (WORLD_SIZE unset) starts two rank
processes itself, each runs the sampler stand-in on its chain range over gloo through bench.py's own
main_worker (the workload set-up, the timed region with the gather inside it, the max over ranks, the line),
and rank 0 prints one JSON line reporting the ranks and the full gathered shape (the RCCL path is the same
code with the nccl backend on the GPU box)."""
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
    out = _run(["--gpus", "2", "--chains", "37", "--steps", "2", "--warmup", "1"])
    assert out["n_gpus"] == 2 and out["config"]["chains_total"] == 74 and out["scaling"] == "weak"
    assert out["stub"]["gathered_shape"] == [1, 74, 3] and out["stub"]["gather_ok"]
    # the world size torch.distributed reports after init, and every rank's device (gathered)
    assert out["dist"]["world_size_observed"] == 2
    assert out["dist"]["devices"] == ["0:cpu", "1:cpu"]


def test_launcher_strong_scaling_ragged():
    out = _run(["--gpus", "3", "--chains-total", "100"])
    assert out["n_gpus"] == 3 and out["stub"]["gathered_shape"] == [1, 100, 3] and out["stub"]["gather_ok"]
    assert out["scaling"] == "strong" and out["config"]["chains_total"] == 100


def test_config3_strong_scaling_line_ragged():
    """BASELINE config 3's command shape (`bench.py --workload cdiffe-pc --chains-total 1000000 --gpus 8` on an
    8-GPU node; here 3 gloo ranks and a ragged total): one line with the observed world size, every rank's device,
    the roofline of the CDiffE predictor-corrector kernel, strong scaling, value = all chains / the max-over-ranks
    time, and the gather of the ragged shards (34 / 33 / 33) inside the timed region, each chain from its rank."""
    n = 100
    out = _run(["--gpus", "3", "--workload", "cdiffe-pc", "--chains-total", str(n), "--steps", "2", "--warmup", "1"])
    assert out["n_gpus"] == 3 and out["dist"]["world_size_observed"] == 3
    assert out["dist"]["devices"] == ["0:cpu", "1:cpu", "2:cpu"]
    assert out["scaling"] == "strong" and out["config"]["chains_total"] == n
    assert "CDiffE predictor-corrector" in out["config"]["workload"] and "all_gather" in out["config"]["parallelism"]
    assert out["config"]["chains_per_gpu"] == 34 == out["stub"]["rank0_chains"]  # rank 0's share of the ragged split
    r = out["roofline"]
    assert r["bound"] == "mfma" and "CDiffE + Langevin corrector" in r["kernel"] and r["unit"] == "TFLOP/s"
    assert r["flops_per_launch"] == 2 * 2 * (27 * 256 + 2 * 256 * 256 + 256 * 26) * 1000 * 34
    assert abs(out["value"] - n * out["steps"] / (out["ms_per_step"] * out["steps"] * 1e-3)) < 1e-6 * out["value"]
    assert out["stub"]["gathered_shape"] == [1, n, 3] and out["stub"]["gather_ok"]


def test_config4_dps_strong_scaling_line():
    """BASELINE config 4's command shape (`--workload dps --chains-total 262144 --gpus 4`), 2 gloo ranks."""
    out = _run(["--gpus", "2", "--workload", "dps", "--chains-total", "9", "--steps", "1", "--warmup", "0"])
    assert out["n_gpus"] == 2 and out["scaling"] == "strong" and out["config"]["chains_total"] == 9
    assert "DPS" in out["config"]["workload"] and "dps_x3_kernel" in out["roofline"]["kernel"]
    assert out["stub"]["gather_ok"] and out["config"]["chains_per_gpu"] == 5


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
