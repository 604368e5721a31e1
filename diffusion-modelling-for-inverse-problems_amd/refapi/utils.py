"""reference `utils` (utils.py:14-205): the model factory from the MI355X package plus the small
host helpers the drivers call (directory setup, density plots -- matplotlib only, seaborn optional)."""
import itertools
import os
import shutil

import numpy as np
import torch  # noqa: F401
import os as _os, sys as _sys
_sys.path.insert(0, _os.path.dirname(_os.path.abspath(__file__)))
from _base import export  # noqa: E402

export(globals(), "factory", ["get_model_from_args"])
export(globals(), "losses")
device = 'cuda' if torch.cuda.is_available() else 'cpu'


def product_dict(**kwargs):
    keys = kwargs.keys()
    for inst in itertools.product(*kwargs.values()):
        yield dict(zip(keys, inst))


def set_directories(train_dir, out_dir, resume_training=False):
    """Same filesystem effects as utils.py:50-65 (removes stale output/log dirs unless resuming)."""
    if os.path.exists(out_dir) and not resume_training:
        shutil.rmtree(out_dir)
    os.makedirs(out_dir, exist_ok=True)
    log_dir = os.path.join(train_dir, 'logs')
    if os.path.exists(log_dir) and not resume_training:
        shutil.rmtree(log_dir)
    os.makedirs(log_dir, exist_ok=True)
    return log_dir


def plot_density(samples, nbins, size, fname, limits=None, xticks=None, labelsize=None, show_mean=False, **kw):
    """Pairwise 2-D histograms of the samples saved to fname (presentation only)."""
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        return
    samples = np.asarray(samples)
    d = samples.shape[1]
    fig, axes = plt.subplots(d, d, figsize=size, squeeze=False)
    rng = [limits] * 2 if limits is not None else None
    for i in range(d):
        for j in range(d):
            ax = axes[i][j]
            if i == j:
                ax.hist(samples[:, i], bins=nbins, range=limits)
            else:
                ax.hist2d(samples[:, j], samples[:, i], bins=nbins, range=rng)
            if show_mean:
                ax.axvline(samples[:, j].mean(), color="w", lw=0.5)
    fig.savefig(fname)
    plt.close(fig)
