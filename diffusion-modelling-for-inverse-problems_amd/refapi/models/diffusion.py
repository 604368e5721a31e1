"""reference `models.diffusion` -> MI355X package (models/diffusion.py:14-229)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from torch import nn  # noqa: E402,F401
from _base import export  # noqa: E402
export(globals(), "estimators", ["BaseClassDiffusionModel", "CDE", "CDiffE", "PosteriorDiffusionEstimator"])
export(globals(), "losses", ["PosteriorLoss"])
device = 'cuda' if torch.cuda.is_available() else 'cpu'
