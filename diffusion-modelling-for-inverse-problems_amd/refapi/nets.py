"""reference `nets` -> MI355X package (nets.py:17-57,143-157)."""
import os as _os, sys as _sys
_sys.path.insert(0, _os.path.dirname(_os.path.abspath(__file__)))
from _base import export  # noqa: E402
export(globals(), "nets", ["MLP", "MLP2", "PosteriorScore"])
