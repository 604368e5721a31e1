"""Diagnostic: force the balanced sampler's hand-over timeout (DMIP_DEBUG_NO_HANDOVER=1) and print
what the host sees (NaN count, device status)."""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import state_from_npz  # noqa: E402

dmip = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
m = dmip.CDE(3, 23, [256] * 3)
m.sde.a.load_state_dict(state_from_npz(np.load(os.path.join(ROOT, "tests/golden/ckpt_scat.npz"))))
y = torch.from_numpy(np.load(os.path.join(ROOT, "tests/golden/data_scat.npz"))["y_test"][0]).cuda()
libc = ctypes.CDLL(None)
libc.getenv.restype = ctypes.c_char_p
for n, S in [(100000, 8), (100000, 20), (300000, 8)]:
    os.environ["DMIP_DEBUG_NO_HANDOVER"] = "1"
    print("getenv:", libc.getenv(b"DMIP_DEBUG_NO_HANDOVER"))
    x = m.sample_device(y, n, S, seed=1)
    torch.cuda.synchronize()
    print(n, S, "nan:", int(torch.isnan(x).sum()), "finite:", int(torch.isfinite(x).sum()))
    try:
        dmip._lib.device_status(x.device)
        print("status ok")
    except RuntimeError as e:
        print("status error:", e)
    del os.environ["DMIP_DEBUG_NO_HANDOVER"]
