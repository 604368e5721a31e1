"""reference `losses` -> MI355X package (losses.py:7-386)."""
import torch  # noqa: F401  (the drivers star-import these names)
from torch import nn  # noqa: F401
import os as _os, sys as _sys
_sys.path.insert(0, _os.path.dirname(_os.path.abspath(__file__)))
from _base import export  # noqa: E402
export(globals(), "losses")
device = 'cuda' if torch.cuda.is_available() else 'cpu'
