"""reference `datasets` -> MI355X package (datasets.py:8-54)."""
import os as _os, sys as _sys
_sys.path.insert(0, _os.path.dirname(_os.path.abspath(__file__)))
from _base import export  # noqa: E402
export(globals(), "problems", ["generate_dataset_scatterometry", "get_gt_samples_scatterometry",
                               "get_dataloader_scatterometry", "generate_dataset_linear", "get_dataloader_linear"])
