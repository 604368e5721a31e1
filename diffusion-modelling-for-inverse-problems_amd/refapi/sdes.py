"""reference `sdes` -> MI355X package (sdes.py:9-87)."""
import os as _os, sys as _sys
_sys.path.insert(0, _os.path.dirname(_os.path.abspath(__file__)))
from _base import export  # noqa: E402
export(globals(), "sdes", ["VariancePreservingSDE", "PluginReverseSDE", "sample_vp_truncated_q"])
