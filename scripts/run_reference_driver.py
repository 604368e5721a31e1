"""Run one of the reference's driver scripts (main_diffusion_linear.py / main_diffusion_scatterometry.py,
unchanged) on this framework: the reference-name shim goes first on sys.path, the working directory
becomes the script's directory (the drivers read config/ relative to it), and `torch.utils.tensorboard`
gets a no-op SummaryWriter when tensorboard is not installed (it is not in this image).
   python scripts/run_reference_driver.py /path/to/reference_copy/main_diffusion_linear.py"""
import os
import runpy
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "diffusion-modelling-for-inverse-problems_amd", "refapi")


def install_tensorboard_stub():
    try:
        import torch.utils.tensorboard  # noqa: F401
    except Exception:
        mod = types.ModuleType("torch.utils.tensorboard")

        class SummaryWriter:
            def __init__(self, *a, **k):
                pass

            def add_scalar(self, *a, **k):
                pass

            def close(self):
                pass
        mod.SummaryWriter = SummaryWriter
        sys.modules["torch.utils.tensorboard"] = mod


def main():
    script = os.path.abspath(sys.argv[1])
    sys.path.insert(0, SHIM)
    install_tensorboard_stub()
    os.chdir(os.path.dirname(script))
    sys.argv = [script] + sys.argv[2:]
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
