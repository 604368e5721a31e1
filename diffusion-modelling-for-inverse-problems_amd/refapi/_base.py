import importlib
import os
import sys

PKG = "diffusion-modelling-for-inverse-problems_amd"
_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _ROOT not in sys.path:
    sys.path.append(_ROOT)


def pkg(sub=None):
    return importlib.import_module(PKG if sub is None else f"{PKG}.{sub}")


def export(namespace, sub, names=None):
    m = pkg(sub)
    names = names or [n for n in dir(m) if not n.startswith("_")]
    for n in names:
        namespace[n] = getattr(m, n)
