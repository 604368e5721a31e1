"""Config -> (model, loss_fn) factory with the reference's dispatch (utils.py:22-48).

Extension (not in the reference): config['model'] == 'DPS' builds the guided sampler of BASELINE config 4
(estimators.DPS) on `forward_model`, with optional config keys 'zeta' (default 0.005) and 'guidance'
('norm' | 'nll', default 'norm'); its training loss is the prior DSM (DSMLoss)."""
from .estimators import CDE, DPS, CDiffE, PosteriorDiffusionEstimator
from .losses import DSM_PDELoss, DSMLoss, PINNLoss, PINNLoss2

_MODELS = {'CDE': CDE, 'CDiffE': CDiffE, 'Posterior': PosteriorDiffusionEstimator}


def get_model_from_args(config, forward_model_params, score_posterior, forward_model):
    if config['model'] == 'DPS':
        model = DPS(forward_model_params['xdim'], forward_model_params['ydim'], config['hidden_layers'], forward_model,
                    forward_model_params, zeta=config.get('zeta', 0.005), guidance=config.get('guidance', 'norm'))
        return model, DSMLoss()
    cls = _MODELS.get(config['model'])
    if cls is None:
        raise ValueError('No valid value for "model" passed. Has to be one of "CDE", "CDiffE" or "Posterior".')
    model = cls(forward_model_params['xdim'], forward_model_params['ydim'], config['hidden_layers'])

    name = config['loss_fn']
    if name == 'PINNLoss':
        loss_fn = PINNLoss(score_posterior, lam=config['lam'], lam2=config['lam2'], pde_loss=config['pde_loss'],
                           ic_metric=config['ic_metric'], pde_metric=config['pde_metric'])
    elif name == 'PINNLoss2':
        loss_fn = PINNLoss2(score_posterior, lam=config['lam'], pde_loss=config['pde_loss'],
                            pde_metric=config['pde_metric'])
    elif name == 'DSM_PDE':
        loss_fn = DSM_PDELoss(lam=config['lam'], pde_loss=config['pde_loss'], pde_metric=config['pde_metric'])
    elif name == 'DSM':
        loss_fn = DSMLoss()
    elif config['model'] == 'Posterior':
        loss_fn = model.loss_fn(forward_model, forward_model_params['a'], forward_model_params['b'], lam=config['lam'])
    else:
        raise ValueError('No valid loss_fn was specified. Options are: "PINNLoss","PINNLoss2","DSM" or "DSM_PDE".'
                         'When the model is PosteriorDiffusionEstimator, the PosteriorLoss is used as default.')
    return model, loss_fn
