"""reference `linear_problem` -> MI355X package (linear_problem.py:5-65)."""
import os as _os, sys as _sys
_sys.path.insert(0, _os.path.dirname(_os.path.abspath(__file__)))
from _base import export  # noqa: E402
export(globals(), "problems", ["LinearForwardProblem"])
