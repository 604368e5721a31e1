"""reference `models.SNF`: only `energy_grad` (models/SNF.py:234-237), which the scatterometry driver
imports for the posterior score. The SNF baseline itself is out of scope."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from _base import export  # noqa: E402
export(globals(), "problems", ["energy_grad"])
