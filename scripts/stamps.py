"""Phase breakdown of one sampler step from the diagnostic stamped build (s_memtime sums per wave).
   python scripts/stamps.py [--chains 65536] [--steps 200]"""
import argparse
import ctypes
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    pkg = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
    L = pkg._lib
    from conftest import state_from_npz
    dev = torch.device("cuda:0")
    m = pkg.CDE(3, 23, [256] * 3)
    m.sde.a.load_state_dict(state_from_npz(np.load(os.path.join(ROOT, "tests/golden/ckpt_scat.npz"))))
    y = torch.from_numpy(np.load(os.path.join(ROOT, "tests/golden/data_scat.npz"))["y_test"][0]).to(dev).reshape(1, -1)
    h = m.sde.a.dmip_handle(dev, 3)
    n_wave = ((a.chains + 255) // 256) * 8
    st = torch.zeros(n_wave, 5, dtype=torch.int64, device=dev)
    out = torch.empty(1, a.chains, 3, device=dev)
    sde = L.vpsde(0.1, 20.0, 1.0)
    for _ in range(2):
        L.check(L.lib().dmip_em_sample_stamps(h.h, ctypes.byref(sde), L.ptr(y), 1, 23, 3, a.chains, a.steps, 1,
                                              L.ptr(out), L.ptr(st), L.stream_of(dev)))
    torch.cuda.synchronize()
    raw = st.cpu().numpy().astype(np.float64)
    s = raw[:, :3] / a.steps
    names = ["layer1+B1", "hidden+output", "rng+em"]
    res = {n: {"mean_cycles_per_step": float(s[:, i].mean()), "p10": float(np.percentile(s[:, i], 10)),
               "p90": float(np.percentile(s[:, i], 90))} for i, n in enumerate(names)}
    res["total_mean"] = float(s.sum(1).mean())
    res["shader_clock_GHz"] = float(np.median(raw[:, 3] / raw[:, 4] * 0.1))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
