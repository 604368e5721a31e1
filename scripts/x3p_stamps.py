"""Per-chunk cycle stamps of the paired-tile fp32x3 sampler (diagnostic library only: make diag, then
DMIP_LIB=abv/diag/libdmip_diag.so python scripts/x3p_stamps.py): the headline workload (100k chains x 1000
steps, scatterometry CDE [256]^3), cycles per step and wave for each of the 16 ring chunks (0-7 hidden layer 1
with layer 1 fused, 8-15 hidden layer 2 with the output layer), the ring barrier waits. One JSON line."""
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    assert "diag" in os.environ.get("DMIP_LIB", ""), "needs the diagnostic library (DMIP_LIB)"
    os.environ["DMIP_X3P"] = "1"  # the paired-tile engine (opt-in while in development)
    pkg = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = pkg.CDE(3, 23, [256] * 3)
    m.sde.a.to(dev)
    y = torch.from_numpy(np.random.default_rng(1).uniform(0, 1, 23).astype(np.float32)).to(dev)
    n, S = 100000, 1000
    for _ in range(2):
        _, snaps = m.sample_trajectory(y, n, S, S, seed=1, precision="fp32x3")
    torch.cuda.synchronize()
    raw = snaps.reshape(-1).view(torch.int64).cpu().numpy()
    st = raw[: (raw.size // 18) * 18].reshape(-1, 18)
    st = st[(st[:, 17] > 0) & (st[:, 17] < 10 ** 6)]
    steps = st[:, 17].astype(np.float64)
    per = st[:, :17] / steps[:, None]
    chunks = per[:, :16].mean(0)
    out = {"waves": int(st.shape[0]), "steps_per_wave": float(steps.mean()),
           "cycles_per_step_total": float(per[:, :16].sum(1).mean()),
           "cycles_per_chunk": [round(float(c)) for c in chunks],
           "hidden1_chunks_0_7": float(chunks[:8].sum()), "hidden2_chunks_8_15": float(chunks[8:].sum()),
           "barrier_wait_per_step": float(per[:, 16].mean())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
