"""reference `models.SNF`: `energy_grad` (models/SNF.py:234-237), which the scatterometry driver imports
for the posterior score, and `anneal_to_energy` (models/SNF.py:250-275), the random-walk MH that
generate_scatterometry_ground_truth.py imports (fused on the device for a ScatterometryEnergy). The SNF
baseline itself is out of scope."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from _base import export  # noqa: E402
export(globals(), "problems", ["energy_grad", "anneal_to_energy"])
