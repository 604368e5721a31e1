"""ctypes binding of libdmip.so (include/dmip.h).

The library is built in-tree (Makefile / __graft_entry__.build()) next to this file. It must be
loaded AFTER `import torch` so that it binds to the HIP runtime torch already loaded (both carry
SONAME libamdhip64.so.7; the dynamic loader then reuses torch's copy and device pointers and
streams are shared). There is no fallback: if the library is missing, every device entry point
raises.
"""
import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DMIP_LIB", os.path.join(_HERE, "libdmip.so"))

DMIP_OK, DMIP_ERR_INVALID, DMIP_ERR_UNSUPPORTED, DMIP_ERR_HIP, DMIP_ERR_ALLOC = range(5)
DMIP_INPUT_X_Y_T, DMIP_INPUT_X_T = 0, 1
DMIP_ACT_TANH_TWICE_FIRST, DMIP_ACT_TANH, DMIP_ACT_SILU_TWICE_FIRST = 0, 1, 2
DMIP_PREC_FP16, DMIP_PREC_F32, DMIP_PREC_F32X3 = 0, 1, 2
# DMIP_PREC_BF16 (include/dmip.h): the same value -- the config-5 training kernel's split-bf16 arithmetic, and the
# samplers' deprecated name of DMIP_PREC_FP16 (their 16-bit engine computes its hidden and output layers in fp16)
DMIP_PREC_BF16 = DMIP_PREC_FP16
PRECISIONS = {"fp16": DMIP_PREC_FP16, "bf16": DMIP_PREC_BF16, "fp32": DMIP_PREC_F32, "fp32x3": DMIP_PREC_F32X3}
DMIP_SAMPLER_CDE, DMIP_SAMPLER_POSTERIOR, DMIP_SAMPLER_CDIFFE = 0, 1, 2
ABI_VERSION = 9
DMIP_LOSS_DSM, DMIP_LOSS_DSM_PDE, DMIP_LOSS_PINN, DMIP_LOSS_PINN2 = 0, 1, 2, 3
DMIP_PDE_NONE, DMIP_PDE_FPE, DMIP_PDE_CFPE = 0, 1, 2
DMIP_METRIC_L1, DMIP_METRIC_L2 = 0, 1

# every symbol include/dmip.h declares (checked by tests/test_capi.py)
EXPORTED = (
    "dmip_mlp_create", "dmip_mlp_destroy", "dmip_mlp_forward", "dmip_em_sample", "dmip_rng_words",
    "dmip_rng_normals", "dmip_schedule", "dmip_last_error", "dmip_abi_version", "dmip_sampler_supported",
    "dmip_em_sample_stamps", "dmip_em_sample_posterior", "dmip_em_sample_cdiffe", "dmip_loss_grad",
    "dmip_loss_grad_supported", "dmip_histogram", "dmip_surrogate_create", "dmip_surrogate_destroy",
    "dmip_surrogate_forward", "dmip_log_posterior", "dmip_mh_sample", "dmip_dps_sample", "dmip_device_status",
    "dmip_sampler_supported_f32", "dmip_posterior_loss_grad", "dmip_loss_grad_f32", "dmip_train_draws",
    "dmip_adam_step", "dmip_em_sample_snapshots", "dmip_train_plan_create", "dmip_train_plan_step",
    "dmip_train_plan_set_counters", "dmip_train_plan_destroy", "dmip_sampler_supported_precision",
    "dmip_dps_sample_ex", "dmip_mh_sample_ex",
)
DMIP_DPS_NLL, DMIP_DPS_NORM = 0, 1


class DmipVpsde(ctypes.Structure):
    _fields_ = [("beta_min", ctypes.c_double), ("beta_max", ctypes.c_double), ("T", ctypes.c_double)]


class DmipLossCfg(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("pde", ctypes.c_int), ("pde_metric", ctypes.c_int),
                ("ic_metric", ctypes.c_int), ("lam", ctypes.c_float), ("lam2", ctypes.c_float),
                ("ic_A", ctypes.c_float * 4), ("ic_b", ctypes.c_float * 2), ("ic_Sinv", ctypes.c_float * 4)]


class DmipTrainPlanDesc(ctypes.Structure):
    """dmip_train_plan_desc (include/dmip.h)."""
    _fields_ = [("in_dim", ctypes.c_int), ("out_dim", ctypes.c_int), ("n_hidden", ctypes.c_int),
                ("widths", ctypes.c_void_p), ("xdim", ctypes.c_int), ("weights_dev", ctypes.c_void_p),
                ("biases_dev", ctypes.c_void_p), ("sde", DmipVpsde), ("cfg", DmipLossCfg),
                ("precision", ctypes.c_int), ("batch", ctypes.c_int64), ("seed", ctypes.c_uint64),
                ("first_draw", ctypes.c_uint64), ("debias", ctypes.c_int), ("t_epsilon", ctypes.c_double),
                ("t_add", ctypes.c_float), ("n_tensors", ctypes.c_int), ("params", ctypes.c_void_p),
                ("grads", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p), ("exp_avg_sq", ctypes.c_void_p),
                ("numel", ctypes.c_void_p), ("lr", ctypes.c_double), ("beta1", ctypes.c_double),
                ("beta2", ctypes.c_double), ("eps", ctypes.c_double), ("step0", ctypes.c_int64),
                ("t_dev", ctypes.c_void_p), ("eps_dev", ctypes.c_void_p), ("loss_dev", ctypes.c_void_p)]


class DmipScatNoise(ctypes.Structure):
    _fields_ = [("a", ctypes.c_float), ("b", ctypes.c_float), ("lambd_bd", ctypes.c_float)]


_c_void_p = ctypes.c_void_p
_i32, _i64, _u64 = ctypes.c_int, ctypes.c_int64, ctypes.c_uint64
_f32 = ctypes.c_float

_lib = None
_lock = threading.Lock()
calls = {"em_sample": 0, "mlp_forward": 0, "em_sample_posterior": 0, "em_sample_cdiffe": 0, "loss_grad": 0}  # instrumentation: proves the HIP path ran


def _declare(lib):
    lib.dmip_last_error.restype = ctypes.c_char_p
    lib.dmip_abi_version.restype = _i32
    lib.dmip_sampler_supported.argtypes = [_i32, _i32, _i32, _i32, _i32]
    lib.dmip_sampler_supported_f32.argtypes = [_i32, _i32, _i32, _i32, _i32]
    lib.dmip_sampler_supported_precision.argtypes = [_i32, _i32, _i32, _i32, _i32, _i32]  # ABI >= 6 (EXPORTED)
    lib.dmip_sampler_supported_precision.restype = _i32
    lib.dmip_device_status.argtypes = [_c_void_p]
    lib.dmip_train_draws.argtypes = [_u64, _u64, _i64, _i32, _i32, ctypes.POINTER(DmipVpsde), ctypes.c_double, _f32,
                                     _c_void_p, _c_void_p, _c_void_p]
    lib.dmip_adam_step.argtypes = [_i32, ctypes.POINTER(_c_void_p), ctypes.POINTER(_c_void_p), ctypes.POINTER(_c_void_p),
                                   ctypes.POINTER(_c_void_p), ctypes.POINTER(_i64), ctypes.c_double, ctypes.c_double,
                                   ctypes.c_double, ctypes.c_double, _i64, _c_void_p]
    lib.dmip_loss_grad_f32.argtypes = [_i32, _i32, _i32, ctypes.POINTER(_i32), _i32, ctypes.POINTER(_c_void_p),
                                       ctypes.POINTER(_c_void_p), ctypes.POINTER(DmipVpsde), ctypes.POINTER(DmipLossCfg),
                                       _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p,
                                       _c_void_p, _c_void_p]
    _pp = ctypes.POINTER(_c_void_p)
    lib.dmip_posterior_loss_grad.argtypes = [_i32, _i32, _i32, ctypes.POINTER(_i32), _pp, _pp, _pp, _pp, _c_void_p,
                                             ctypes.POINTER(DmipScatNoise), _f32, ctypes.POINTER(DmipVpsde),
                                             _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p,
                                             _c_void_p, _c_void_p, _c_void_p]
    lib.dmip_mlp_create.argtypes = [_i32, _i32, _i32, ctypes.POINTER(_i32), _i32, _i32, _i32,
                                    ctypes.POINTER(_c_void_p), ctypes.POINTER(_c_void_p),
                                    ctypes.POINTER(_c_void_p)]
    lib.dmip_mlp_destroy.argtypes = [_c_void_p]
    lib.dmip_mlp_forward.argtypes = [_c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p, _i32, _i64,
                                     _c_void_p, _i32, _c_void_p]
    lib.dmip_em_sample.argtypes = [_c_void_p, ctypes.POINTER(DmipVpsde), _c_void_p, _i32, _i32, _i32,
                                   _i64, _i64, _i32, _f32, _f32, _u64, _i32, _c_void_p, _c_void_p,
                                   _c_void_p]
    lib.dmip_em_sample_posterior.argtypes = [_c_void_p, _c_void_p, ctypes.POINTER(DmipVpsde), _c_void_p, _i32,
                                             _i32, _i32, _i64, _i64, _i32, _f32, _f32, _u64, _i32, _c_void_p,
                                             _c_void_p]
    lib.dmip_em_sample_cdiffe.argtypes = [_c_void_p, ctypes.POINTER(DmipVpsde), _c_void_p, _i32, _i32, _i32,
                                          _i64, _i64, _i32, _f32, _f32, _u64, _i32, _i32, _f32, _c_void_p,
                                          _c_void_p]
    if hasattr(lib, "dmip_em_sample_snapshots"):  # (absent from older builds loaded by A/B timing scripts)
        lib.dmip_em_sample_snapshots.argtypes = [_i32, _c_void_p, _c_void_p, ctypes.POINTER(DmipVpsde), _c_void_p, _i32,
                                                 _i32, _i32, _i64, _i64, _i32, _f32, _f32, _u64, _i32, _i32, _f32,
                                                 _i32, _c_void_p, _c_void_p, _c_void_p]
    if hasattr(lib, "dmip_train_plan_create"):
        lib.dmip_train_plan_create.argtypes = [ctypes.POINTER(DmipTrainPlanDesc), ctypes.POINTER(_c_void_p)]
        lib.dmip_train_plan_step.argtypes = [_c_void_p, _c_void_p, _c_void_p, _c_void_p]
        lib.dmip_train_plan_set_counters.argtypes = [_c_void_p, _u64, _i64, _c_void_p]
        lib.dmip_train_plan_destroy.argtypes = [_c_void_p]
    lib.dmip_loss_grad.argtypes = [_i32, _i32, _i32, ctypes.POINTER(_i32), _i32, ctypes.POINTER(_c_void_p),
                                   ctypes.POINTER(_c_void_p), ctypes.POINTER(DmipVpsde), ctypes.POINTER(DmipLossCfg),
                                   _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p,
                                   _c_void_p]
    lib.dmip_histogram.argtypes = [_c_void_p, _i64, _i32, _i32, ctypes.c_double, ctypes.c_double, _i32, _c_void_p,
                                   _c_void_p]
    lib.dmip_loss_grad_supported.argtypes = [_i32, _i32, _i32, ctypes.POINTER(_i32), _i32]
    lib.dmip_em_sample_stamps.argtypes = [_c_void_p, ctypes.POINTER(DmipVpsde), _c_void_p, _i32, _i32, _i32,
                                          _i64, _i32, _u64, _c_void_p, _c_void_p, _c_void_p]
    lib.dmip_rng_words.argtypes = [_u64, _i64, _u64, _i64, _i32, _c_void_p, _c_void_p]
    lib.dmip_rng_normals.argtypes = [_u64, _i64, _u64, _i64, _i32, _c_void_p, _c_void_p]
    lib.dmip_schedule.argtypes = [_i32, ctypes.POINTER(DmipVpsde), _c_void_p, _c_void_p]
    lib.dmip_surrogate_create.argtypes = [_i32, _i32, _i32, ctypes.POINTER(_i32), ctypes.POINTER(_c_void_p),
                                          ctypes.POINTER(_c_void_p), ctypes.POINTER(_c_void_p)]
    lib.dmip_surrogate_destroy.argtypes = [_c_void_p]
    lib.dmip_surrogate_forward.argtypes = [_c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p]
    lib.dmip_log_posterior.argtypes = [_c_void_p, ctypes.POINTER(DmipScatNoise), _c_void_p, _c_void_p, _i64, _i64,
                                       _c_void_p, _c_void_p, _c_void_p]
    lib.dmip_mh_sample.argtypes = [_c_void_p, ctypes.POINTER(DmipScatNoise), _c_void_p, _i32, _i64, _i64, _i32, _f32,
                                   _u64, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p]
    lib.dmip_dps_sample.argtypes = [_c_void_p, _c_void_p, ctypes.POINTER(DmipScatNoise), ctypes.POINTER(DmipVpsde),
                                    _c_void_p, _i32, _i64, _i64, _i32, _f32, _f32, _u64, _i32, _f32, _c_void_p,
                                    _c_void_p]
    lib.dmip_dps_sample_ex.argtypes = [_c_void_p, _c_void_p, ctypes.POINTER(DmipScatNoise), ctypes.POINTER(DmipVpsde),
                                       _c_void_p, _i32, _i64, _i64, _i32, _f32, _f32, _u64, _i32, _f32, _i32,
                                       _c_void_p, _c_void_p]
    lib.dmip_dps_sample_ex.restype = _i32
    if hasattr(lib, "dmip_mh_sample_ex"):  # ABI >= 9
        lib.dmip_mh_sample_ex.argtypes = [_c_void_p, ctypes.POINTER(DmipScatNoise), _c_void_p, _i32, _i64, _i64, _i32,
                                          _f32, _u64, _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p,
                                          _c_void_p]
        lib.dmip_mh_sample_ex.restype = _i32
    for name in ("dmip_train_draws", "dmip_adam_step", "dmip_loss_grad_f32", "dmip_posterior_loss_grad", "dmip_device_status", "dmip_sampler_supported_f32", "dmip_dps_sample", "dmip_mlp_create", "dmip_mlp_destroy", "dmip_mlp_forward", "dmip_em_sample",
                 "dmip_rng_words", "dmip_rng_normals", "dmip_schedule", "dmip_sampler_supported",
                 "dmip_em_sample_stamps", "dmip_em_sample_posterior", "dmip_em_sample_cdiffe",
                 "dmip_loss_grad", "dmip_loss_grad_supported", "dmip_histogram", "dmip_surrogate_create",
                 "dmip_surrogate_destroy", "dmip_surrogate_forward", "dmip_log_posterior", "dmip_mh_sample"):
        getattr(lib, name).restype = _i32


class _OlderBuild:
    """An older build of the library loaded for a same-box timing A/B (DMIP_LIB=<path> DMIP_LIB_AB=1, scripts/): the
    entry points it lacks take their ctypes declarations and fail when called. Never the product path."""

    def __init__(self, handle):
        self._handle, self._absent = handle, {}

    def __getattr__(self, name):
        try:
            return getattr(self._handle, name)
        except AttributeError:
            return self._absent.setdefault(name, _Absent(name))


class _Absent:
    def __init__(self, name):
        self.name = name

    def __call__(self, *args):
        raise RuntimeError(f"dmip: {LIB_PATH} (A/B build) has no {self.name}")


def lib():
    """The loaded library; raises RuntimeError if it has not been built."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(
                        f"dmip: HIP library not found at {LIB_PATH}; build it with "
                        "`python -c 'import __graft_entry__ as g; g.build()'` or `make` at the repo root")
                handle = ctypes.CDLL(LIB_PATH)
                missing = [n for n in EXPORTED if not hasattr(handle, n)]
                ab = os.environ.get("DMIP_LIB_AB") == "1"
                if missing and ab:
                    handle = _OlderBuild(handle)
                elif missing:
                    raise RuntimeError(f"dmip: {LIB_PATH} is not ABI {ABI_VERSION}: missing {', '.join(missing)} "
                                       "(rebuild with `make` at the repo root)")
                elif not ab and handle.dmip_abi_version() != ABI_VERSION:
                    raise RuntimeError(f"dmip: {LIB_PATH} is ABI {handle.dmip_abi_version()}, this package needs "
                                       f"{ABI_VERSION} (rebuild with `make` at the repo root)")
                _declare(handle)
                _lib = handle
    return _lib


def check(rc):
    if rc == DMIP_OK:
        return
    msg = lib().dmip_last_error().decode(errors="replace")
    if rc in (DMIP_ERR_INVALID, DMIP_ERR_UNSUPPORTED):
        raise ValueError(f"dmip: {msg}")
    raise RuntimeError(f"dmip: {msg} (status {rc})")


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def stream_of(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device(t, what="tensor"):
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise RuntimeError(f"dmip: {what} must be on a HIP device (got {getattr(t, 'device', type(t))});"
                           " the dmip kernels have no CPU path")


def vpsde(beta_min, beta_max, T):
    return DmipVpsde(float(beta_min), float(beta_max), float(T))


class MlpHandle:
    """Owns a dmip_mlp* (packed device weights) for one snapshot of a network's parameters."""

    def __init__(self, layers, in_dim, out_dim, xdim, input_layout, device, act=DMIP_ACT_TANH_TWICE_FIRST):
        L = len(layers) - 1
        widths = (_i32 * L)(*[int(layers[i][0].shape[0]) for i in range(L)])
        with torch.cuda.device(device):
            ws = [w.detach().float().contiguous().cpu() for w, _ in layers]
            bs = [b.detach().float().contiguous().cpu() for _, b in layers]
            wp = (_c_void_p * (L + 1))(*[w.data_ptr() for w in ws])
            bp = (_c_void_p * (L + 1))(*[b.data_ptr() for b in bs])
            out = _c_void_p()
            check(lib().dmip_mlp_create(in_dim, out_dim, L, widths, act, input_layout, xdim, wp, bp,
                                        ctypes.byref(out)))
        self.h = out
        self.device = device
        self.width = int(layers[0][0].shape[0])
        self.n_hidden = L
        self.in_dim, self.out_dim, self.xdim = in_dim, out_dim, xdim
        self.act = act

    def __del__(self):
        h = getattr(self, "h", None)
        if h and _lib is not None:
            try:
                torch.cuda.synchronize(self.device)
            except Exception:
                pass
            _lib.dmip_mlp_destroy(h)
            self.h = None


def precision_code(precision):
    """'fp16' (16-bit MFMA operands, the fastest mode: split-bf16 layer 1, fp16 hidden and output layers; 'bf16' is
    its deprecated name), 'fp32x3' (fp32-accurate products as three fp16 MFMAs, the reference-precision throughput
    mode) or 'fp32' (exact f32 MFMA, bit-level parity mode)."""
    if precision not in PRECISIONS:
        raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, got {precision!r}")
    return PRECISIONS[precision]


def mlp_forward(handle, x, y, t, out, y_stride, t_stride, precision="fp32"):
    calls["mlp_forward"] += 1
    check(lib().dmip_mlp_forward(handle.h, ptr(x), ptr(y), y_stride, ptr(t), t_stride, x.shape[0],
                                 ptr(out), precision_code(precision), stream_of(x.device)))


def em_sample(handle, sde, y, n_chains, chain_offset, num_steps, mean, std, seed, out, noise=None,
              precision="fp16"):
    calls["em_sample"] += 1
    _status_pending.add(_dev_index(y.device))
    n_y, ydim = y.shape
    check(lib().dmip_em_sample(handle.h, ctypes.byref(sde), ptr(y), n_y, ydim, handle.xdim,
                               int(n_chains), int(chain_offset), int(num_steps), float(mean),
                               float(std), ctypes.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF),
                               precision_code(precision), ptr(noise), ptr(out), stream_of(y.device)))


def em_sample_posterior(prior, likelihood, sde, y, n_chains, chain_offset, num_steps, mean, std, seed, out,
                        precision="fp16"):
    calls["em_sample_posterior"] += 1
    _status_pending.add(_dev_index(y.device))
    n_y, ydim = y.shape
    check(lib().dmip_em_sample_posterior(prior.h, likelihood.h, ctypes.byref(sde), ptr(y), n_y, ydim,
                                         likelihood.xdim, int(n_chains), int(chain_offset), int(num_steps),
                                         float(mean), float(std), ctypes.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF),
                                         precision_code(precision), ptr(out), stream_of(y.device)))


def em_sample_cdiffe(handle, sde, y, n_chains, chain_offset, num_steps, mean, std, seed, out, corrector_steps=0,
                     snr=0.16, precision="fp16"):
    calls["em_sample_cdiffe"] += 1
    _status_pending.add(_dev_index(y.device))
    n_y, ydim = y.shape
    check(lib().dmip_em_sample_cdiffe(handle.h, ctypes.byref(sde), ptr(y), n_y, ydim, handle.xdim,
                                      int(n_chains), int(chain_offset), int(num_steps), float(mean), float(std),
                                      ctypes.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF), precision_code(precision),
                                      int(corrector_steps), float(snr), ptr(out), stream_of(y.device)))


def em_sample_snapshots(mode, net, prior, sde, y, n_chains, chain_offset, num_steps, mean, std, seed, snapshot_every,
                        snaps, out, corrector_steps=0, snr=0.16, precision="fp16"):
    """dmip_em_sample_snapshots: the fused sampler of `mode` that also writes x after every
    snapshot_every-th step into snaps [num_steps // snapshot_every][n_y][n_chains][xdim]."""
    calls["em_sample_snapshots"] = calls.get("em_sample_snapshots", 0) + 1
    _status_pending.add(_dev_index(y.device))
    n_y, ydim = y.shape
    check(lib().dmip_em_sample_snapshots(int(mode), net.h, prior.h if prior is not None else None, ctypes.byref(sde),
                                         ptr(y), n_y, ydim, net.xdim, int(n_chains), int(chain_offset),
                                         int(num_steps), float(mean), float(std),
                                         ctypes.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF), precision_code(precision),
                                         int(corrector_steps), float(snr), int(snapshot_every), ptr(snaps), ptr(out),
                                         stream_of(y.device)))


def sampler_supported(width, n_hidden, xdim, ydim=0, mode=DMIP_SAMPLER_CDE, precision="fp16"):
    return bool(lib().dmip_sampler_supported_precision(precision_code(precision), mode, width, n_hidden, xdim, ydim))


# devices with a launch of a status-writing kernel (the samplers, MH, DPS) whose status word has not been read since;
# clear_range_status skips the read (a stream synchronise and a copy) when there is none
_status_pending = set()


def _dev_index(device):
    d = torch.device(device)
    return d.index if d.index is not None else torch.cuda.current_device()


def device_status(device):
    """Synchronise the device's current stream and raise if a kernel reported an asynchronous failure
    (dmip_device_status: the balanced sampler's hand-over timeout, or an fp32x3 chain outside the fp16 range).
    Reading clears the status word."""
    try:
        check(lib().dmip_device_status(stream_of(device)))
    finally:
        _status_pending.discard(_dev_index(device))


def is_range_error(e):
    """The fp32x3 split's fp16-range refusal (pack time, ValueError) or report (device status, RuntimeError)."""
    return isinstance(e, (ValueError, RuntimeError)) and "fp16 range" in str(e)


def clear_range_status(device):
    """Read and clear the device status word before a launch whose range report will be read: a stale fp16-range
    report of an earlier launch (whose caller did not read it) is dropped; any other stale failure raises. Nothing to
    read (no status-writing launch of this process since the last read): returns at once."""
    if _dev_index(device) not in _status_pending:
        return
    try:
        device_status(device)
    except RuntimeError as e:
        if not is_range_error(e):
            raise


def rng_normals(seed, chain_offset, stream_id, n_chains, n_pairs, out):
    """(n_chains, 2 n_pairs) standard normals of the kernels' chain-keyed generator (dmip_rng_normals)."""
    check(lib().dmip_rng_normals(ctypes.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF), int(chain_offset),
                                 ctypes.c_uint64(int(stream_id) & 0xFFFFFFFFFFFFFFFF), int(n_chains), int(n_pairs),
                                 ptr(out), stream_of(out.device)))


def loss_grad_supported(in_dim, out_dim, widths, xdim):
    w = (_i32 * len(widths))(*widths)
    return bool(lib().dmip_loss_grad_supported(in_dim, out_dim, len(widths), w, xdim))


def loss_grad(layers, in_dim, out_dim, xdim, sde, cfg, x, y, t, eps, grad_out, loss_out):
    """layers: [(weight, bias), ...] device fp32 tensors (the torch parameters)."""
    calls["loss_grad"] += 1
    L = len(layers) - 1
    widths = (_i32 * L)(*[int(layers[i][0].shape[0]) for i in range(L)])
    wp = (_c_void_p * (L + 1))(*[w.data_ptr() for w, _ in layers])
    bp = (_c_void_p * (L + 1))(*[b.data_ptr() for _, b in layers])
    check(lib().dmip_loss_grad(in_dim, out_dim, L, widths, xdim, wp, bp, ctypes.byref(sde), ctypes.byref(cfg),
                               ptr(x), ptr(y), ptr(t), ptr(eps), int(x.shape[0]), ptr(grad_out), ptr(loss_out),
                               stream_of(x.device)))


def loss_grad_f32(layers, in_dim, out_dim, xdim, sde, cfg, x, y, t, eps, grad_out, loss_out, ic_target=None):
    """dmip_loss_grad_f32: the exact-f32 stacked-jet training step at any width."""
    calls["loss_grad_f32"] = calls.get("loss_grad_f32", 0) + 1
    L = len(layers) - 1
    widths = (_i32 * L)(*[int(layers[i][0].shape[0]) for i in range(L)])
    wp = (_c_void_p * (L + 1))(*[w.data_ptr() for w, _ in layers])
    bp = (_c_void_p * (L + 1))(*[b.data_ptr() for _, b in layers])
    check(lib().dmip_loss_grad_f32(in_dim, out_dim, L, widths, xdim, wp, bp, ctypes.byref(sde), ctypes.byref(cfg),
                                   ptr(x), ptr(y), ptr(t), ptr(eps), ptr(ic_target), int(x.shape[0]), ptr(grad_out),
                                   ptr(loss_out), stream_of(x.device)))


def histogram(x, nbins, lo, hi, counts):
    """x: (n_hist, n, d) fp32 device tensor; counts: (n_hist, nbins**d) int32 device tensor (accumulated)."""
    calls["histogram"] = calls.get("histogram", 0) + 1
    n_hist, n, d = x.shape
    check(lib().dmip_histogram(ptr(x), int(n), int(d), int(nbins), float(lo), float(hi), int(n_hist), ptr(counts),
                               stream_of(x.device)))


# ------------------------------------------------------------------------- scatterometry surrogate
class SurrogateHandle:
    """Owns a dmip_surrogate* (packed f32 MFMA images of the frozen forward model)."""

    def __init__(self, layers, device):
        widths = (_i32 * 3)(*[int(layers[i][0].shape[0]) for i in range(3)])
        with torch.cuda.device(device):
            ws = [w.detach().float().contiguous().cpu() for w, _ in layers]
            bs = [b.detach().float().contiguous().cpu() for _, b in layers]
            wp = (_c_void_p * 4)(*[w.data_ptr() for w in ws])
            bp = (_c_void_p * 4)(*[b.data_ptr() for b in bs])
            out = _c_void_p()
            check(lib().dmip_surrogate_create(int(layers[0][0].shape[1]), int(layers[-1][0].shape[0]), 3, widths,
                                              wp, bp, ctypes.byref(out)))
        self.h = out
        self.device = device

    def __del__(self):
        h = getattr(self, "h", None)
        if h and _lib is not None:
            try:
                torch.cuda.synchronize(self.device)
            except Exception:
                pass
            _lib.dmip_surrogate_destroy(h)
            self.h = None


def scat_noise(a, b, lambd_bd):
    return DmipScatNoise(float(a), float(b), float(lambd_bd))


def surrogate_forward(handle, x, out):
    calls["surrogate_forward"] = calls.get("surrogate_forward", 0) + 1
    check(lib().dmip_surrogate_forward(handle.h, ptr(x), int(x.shape[0]), ptr(out), stream_of(x.device)))


def log_posterior(handle, noise, x, y, y_stride, e_out, grad_out=None):
    calls["log_posterior"] = calls.get("log_posterior", 0) + 1
    check(lib().dmip_log_posterior(handle.h, ctypes.byref(noise), ptr(x), ptr(y), int(y_stride), int(x.shape[0]),
                                   ptr(e_out), ptr(grad_out), stream_of(x.device)))


def mh_sample(handle, noise, y, n_chains, chain_offset, num_steps, noise_std, seed, x_out, x_init=None,
              inj_noise=None, inj_unif=None, e_out=None, precision="fp32"):
    """dmip_mh_sample_ex: "fp32" the exact-f32 kernel, "fp32x3" the split-fp16 one (dmip_dps_x3.hip mh_x3_kernel)."""
    calls["mh_sample"] = calls.get("mh_sample", 0) + 1
    _status_pending.add(_dev_index(y.device))
    check(lib().dmip_mh_sample_ex(handle.h, ctypes.byref(noise), ptr(y), int(y.shape[0]), int(n_chains),
                                  int(chain_offset), int(num_steps), float(noise_std),
                                  ctypes.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF), ptr(x_init), ptr(inj_noise),
                                  ptr(inj_unif), precision_code(precision), ptr(x_out), ptr(e_out),
                                  stream_of(y.device)))


def dps_sample(prior, surrogate, noise, sde, y, n_chains, chain_offset, num_steps, mean, std, seed, mode, zeta, out,
               precision="fp32"):
    """dmip_dps_sample_ex: "fp32" the exact-f32 kernel, "fp32x3" the split-fp16 one (dmip_dps_x3.hip)."""
    calls["dps_sample"] = calls.get("dps_sample", 0) + 1
    _status_pending.add(_dev_index(y.device))
    check(lib().dmip_dps_sample_ex(prior.h, surrogate.h, ctypes.byref(noise), ctypes.byref(sde), ptr(y),
                                   int(y.shape[0]), int(n_chains), int(chain_offset), int(num_steps), float(mean),
                                   float(std), ctypes.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF), int(mode), float(zeta),
                                   precision_code(precision), ptr(out), stream_of(y.device)))


def posterior_loss_grad(prior_layers, lik_layers, surrogate, noise, lam, sde, x, y, t, eps, grad_prior, grad_lik,
                        loss_out, target_out=None):
    """dmip_posterior_loss_grad (A18): layers = [(weight, bias)] device fp32 tensors of the prior (MLP2) and
    likelihood (MLP) networks; writes the flat reference-order gradients, loss_out[3] and optionally the
    likelihood target."""
    calls["posterior_loss_grad"] = calls.get("posterior_loss_grad", 0) + 1
    L = len(prior_layers) - 1
    widths = (_i32 * L)(*[int(prior_layers[i][0].shape[0]) for i in range(L)])
    arr = lambda ts: (_c_void_p * (L + 1))(*[v.data_ptr() for v in ts])
    check(lib().dmip_posterior_loss_grad(
        int(x.shape[1]), int(y.shape[1]), L, widths, arr([w for w, _ in prior_layers]), arr([b for _, b in prior_layers]),
        arr([w for w, _ in lik_layers]), arr([b for _, b in lik_layers]), surrogate.h, ctypes.byref(noise),
        float(lam), ctypes.byref(sde), ptr(x), ptr(y), ptr(t), ptr(eps), int(x.shape[0]), ptr(grad_prior),
        ptr(grad_lik), ptr(loss_out), ptr(target_out), stream_of(x.device)))
