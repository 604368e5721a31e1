"""Reference-name shim: modules named exactly like the reference's flat modules (`utils`,
`models.diffusion`, `nets`, `sdes`, `losses`, `linear_problem`, `utils_scatterometry`, `datasets`,
`models.SNF.energy_grad`) that re-export this package. Put this directory first on sys.path (or use
scripts/run_reference_driver.py) and the reference's driver scripts import the MI355X framework
instead of the reference. See INTEGRATION.md."""
import importlib
import os
import sys

PKG = "diffusion-modelling-for-inverse-problems_amd"
_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _ROOT not in sys.path:
    sys.path.append(_ROOT)


def pkg(sub=None):
    return importlib.import_module(PKG if sub is None else f"{PKG}.{sub}")
