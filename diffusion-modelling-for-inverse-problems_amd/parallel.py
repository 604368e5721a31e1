"""Sample-parallel sharding over GPUs.

Posterior chains are independent given (weights, y), so a sampling call with N chains is split
into contiguous chain ranges, one per rank (one process per GPU, torch.distributed over RCCL).
Each rank runs the fused kernel on its range with `chain_offset` = the range start -- the RNG is
keyed by the global chain index, so the union of the shards is bit-identical to a single-GPU run
of all N chains. The only collective is one all_gather of the (N/G, xdim) fp32 shards at the end
(tens of microseconds over xGMI at these sizes); the per-step data path has no communication.
"""
import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_range(n, rank, world_size):
    """Contiguous chain range [lo, hi) of `rank`; the first n % world_size ranks take one extra."""
    base, rem = divmod(int(n), int(world_size))
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def common_seed(seed, device):
    """The same seed on every rank (rank 0's draw), so all shards belong to one logical run."""
    rank, ws = world()
    if ws == 1:
        return seed
    backend = dist.get_backend()
    dev = device if backend == "nccl" else torch.device("cpu")
    buf = torch.tensor([seed if rank == 0 else 0], dtype=torch.int64, device=dev)
    dist.broadcast(buf, src=0)
    return int(buf.item())


def gather_shards(local, n, device):
    """All ranks receive the (n_y, n, d) concatenation of the (n_y, hi-lo, d) shards."""
    rank, ws = world()
    if ws == 1:
        return local
    n_y, _, d = local.shape
    sizes = [shard_range(n, r, ws) for r in range(ws)]
    width = max(hi - lo for lo, hi in sizes)
    backend = dist.get_backend()
    dev = device if backend == "nccl" else torch.device("cpu")
    pad = torch.zeros(n_y, width, d, dtype=local.dtype, device=dev)
    pad[:, :local.shape[1]] = local.to(dev)
    out = torch.empty(ws * n_y, width, d, dtype=local.dtype, device=dev)
    dist.all_gather_into_tensor(out, pad)
    out = out.view(ws, n_y, width, d)
    parts = [out[r, :, :hi - lo] for r, (lo, hi) in enumerate(sizes)]
    return torch.cat(parts, dim=1).to(device)


def sample_sharded(model, y, num_samples, num_steps, mean, std, seed=None, **sampler_kwargs):
    """model(y, ...) over all ranks; returns the full (num_samples, xdim) device tensor.
    `sampler_kwargs` go to model.sample_device (e.g. CDiffE's corrector_steps / snr)."""
    from .estimators import _draw_seed
    rank, ws = world()
    dev = model._exec_device(y)
    seed = common_seed(_draw_seed() if seed is None else seed, dev)
    lo, hi = shard_range(num_samples, rank, ws)
    local = _sample_local(model, y, hi - lo, num_steps, mean, std, seed, lo, sampler_kwargs)
    full = gather_shards(local, num_samples, dev)
    return full[0] if torch.as_tensor(y).ndim == 1 else full


def _sample_local(model, y, n, num_steps, mean, std, seed, lo, kw):
    """This rank's shard (sample_checked, the fallback decided by all ranks together)."""
    return sample_checked(model, y, n, num_steps, mean, std, seed=seed, chain_offset=lo, agree=any_rank, **kw)


# per-rank outcome of a guarded launch; any_rank's MAX over ranks picks the worst
OK, RANGE, FAILED = 0, 1, 2


def any_rank(state):
    """The maximum of `state` (a bool or one of OK / RANGE / FAILED) over all ranks: one all_reduce MAX of a scalar,
    no-op at world size 1. As a flag: true on every rank when true on any rank."""
    _, ws = world()
    if ws == 1:
        return int(state)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    buf = torch.tensor([int(state)], dtype=torch.int32, device=dev)
    dist.all_reduce(buf, op=dist.ReduceOp.MAX)
    return int(buf.item())


def guarded(dev, launch, fallback=None, agree=None):
    """launch() with the device status word cleared before it and read after it, so an asynchronous failure of THIS
    launch surfaces here (a split-fp16 engine's fp16-range report, a hand-over timeout) and a stale report of an
    earlier launch is not taken for it. Each rank's outcome is OK, RANGE (the split's range refusal or report) or
    FAILED (any other error); `agree` (any_rank) makes it the maximum over all ranks, so the ranks leave together and
    none is left blocked in a collective another rank never reaches. RANGE with a `fallback` returns
    fallback() (the exact-f32 engine) on every rank; RANGE without one, or FAILED on any rank, raises on every rank."""
    import warnings
    from . import _lib
    err, state, res = None, OK, None
    try:
        _lib.clear_range_status(dev)
        res = launch()
        _lib.device_status(dev)
    except Exception as e:  # noqa: BLE001 -- every error takes part in the agreement, then is re-raised
        err, state = e, (RANGE if _lib.is_range_error(e) else FAILED)
    outcome = agree(state) if agree is not None else state
    if outcome == OK:
        return res
    if outcome == RANGE and fallback is not None:
        warnings.warn(f"{err or 'fp16 range (another rank)'}; sampled with the exact-f32 engine instead", RuntimeWarning)
        return fallback()
    if err is not None:
        raise err
    raise RuntimeError("dmip: another rank's launch failed (" + ("fp16 range" if outcome == RANGE else "error") +
                       "); this rank's shard is discarded")


def sample_checked(model, y, n, num_steps, mean, std, seed=None, chain_offset=0, agree=None, **kw):
    """model.sample_device(...) under `guarded`: the device status word is read after EVERY launch, whichever engine
    the request resolved to (a "fp16" request runs the split-fp16 fp32x3 engine for shapes without a 16-bit kernel,
    and DPS has no 16-bit engine at all).

    Without an explicit `precision` (the model's default: fp32x3, the reference's fp32 arithmetic from fp16 hi/lo
    splits, or fp16) a network or a trajectory outside the split's fp16 range -- a scaled weight, or a chain's
    layer-1 input, beyond 65504 -- is refused (at launch) or reported (device status word) by the library; the call
    is then sampled again with the exact-f32 engine, so the default path never returns the split's inf/NaN where
    the reference's fp32 stays finite. `agree(state)` makes the decision collective: under sample_sharded every rank
    resamples if any rank's shard left the range, so the gathered union is always one engine's chains (bit-identical
    to the 1-GPU run), and every rank raises if any rank failed otherwise. An explicit `precision` keeps the error."""
    from .estimators import canonical_precision
    explicit = kw.get("precision") is not None
    prec = canonical_precision(kw.get("precision") or getattr(model, "precision", "fp32x3"))
    if seed is None:  # one seed for both attempts: the fallback resamples the same chains
        from .estimators import _draw_seed
        seed = _draw_seed()
    dev = model._exec_device(y)

    def call(**over):
        return model.sample_device(y, n, num_steps, mean, std, seed=seed, chain_offset=chain_offset, **dict(kw, **over))

    fallback = None if explicit or prec == "fp32" else (lambda: call(precision="fp32"))
    return guarded(dev, call, fallback, agree)


def chains_sharded(n, run, seed, device):
    """A chain-keyed kernel launched over all ranks (the MH ground truth, problems.generate_gt_samples): rank r calls
    run(n_local, chain_offset, seed, agree) -> its (n_y, n_local, d) shard for its contiguous chain range, with the
    common seed; every rank receives the (n_y, n, d) union, bit-identical to one launch of all n chains. `agree` is
    any_rank, for a fallback decided by all ranks together (as sample_checked's)."""
    rank, ws = world()
    seed = common_seed(seed, device)
    lo, hi = shard_range(n, rank, ws)
    return gather_shards(run(hi - lo, lo, seed, any_rank), n, device)


def map_sharded(n, fn, width):
    """Evaluate-style multi-y runs (shard over (y, chain) pairs): rank r computes
    `fn(i)` -> `width` floats for its contiguous range of the n items (each item = one y with all
    its repeats in one sampler launch), and every rank receives the (n, width) float64 table in
    item order. One all_gather of n * width floats at the end; nothing per step."""
    import numpy as np
    rank, ws = world()
    lo, hi = shard_range(n, rank, ws)
    rows = [np.asarray(fn(i), dtype=np.float64).reshape(width) for i in range(lo, hi)]
    local = torch.from_numpy(np.stack(rows) if rows else np.zeros((0, width)))
    if ws == 1:
        return local.numpy()
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    return gather_shards(local[None].to(dev), n, dev)[0].cpu().numpy()
