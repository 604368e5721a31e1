"""dmip -- MI355X-native conditional score-diffusion posterior sampler.

Drop-in for the hot path of maffos/Diffusion-Modelling-for-inverse-problems: the reference's
construct-and-sample API (CDE / CDiffE / PosteriorDiffusionEstimator, get_model_from_args,
model(y, num_samples, num_steps)) on top of libdmip.so, whose hand-written gfx950 kernels run the
whole reverse-SDE loop. Import with importlib (the directory name is not an identifier):

    dmip = importlib.import_module("diffusion-modelling-for-inverse-problems_amd")
"""
from . import _lib
from .estimators import DPS, BaseClassDiffusionModel, CDE, CDiffE, PosteriorDiffusionEstimator
from .factory import get_model_from_args
from .losses import (ConditionalScoreFPELoss, DSM_PDELoss, DSMLoss, PINNLoss, PINNLoss2, PosteriorLoss,
                     ScoreFPELoss, batch_gradient, divergence)
from .nets import MLP, MLP2, PosteriorScore
from .problems import (LinearForwardProblem, ScatterometryEnergy, anneal_to_energy, energy_grad,
                       generate_gt_samples, get_log_posterior, load_forward_model, mh_sample)
from .sdes import PluginReverseSDE, VariancePreservingSDE, sample_vp_truncated_q

__all__ = [
    "BaseClassDiffusionModel", "CDE", "CDiffE", "PosteriorDiffusionEstimator", "DPS", "get_model_from_args",
    "ConditionalScoreFPELoss", "DSM_PDELoss", "DSMLoss", "PINNLoss", "PINNLoss2", "PosteriorLoss",
    "ScoreFPELoss", "batch_gradient", "divergence", "MLP", "MLP2", "PosteriorScore",
    "PluginReverseSDE", "VariancePreservingSDE", "sample_vp_truncated_q", "LinearForwardProblem",
    "ScatterometryEnergy", "anneal_to_energy", "energy_grad", "generate_gt_samples", "get_log_posterior",
    "load_forward_model", "mh_sample",
]


def hip_available():
    """True when libdmip.so is built and a HIP device is visible."""
    import os
    import torch
    return os.path.exists(_lib.LIB_PATH) and torch.cuda.is_available()
