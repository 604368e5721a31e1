"""reference `utils_scatterometry` -> MI355X package (utils_scatterometry.py:8-52)."""
import numpy as np  # noqa: F401
import torch  # noqa: F401
import os  # noqa: F401
from torch import nn  # noqa: F401
import os as _os, sys as _sys
_sys.path.insert(0, _os.path.dirname(_os.path.abspath(__file__)))
from _base import export  # noqa: E402
export(globals(), "problems", ["load_forward_model", "get_log_posterior", "inverse_cdf_prior"])
device = 'cuda' if torch.cuda.is_available() else 'cpu'
