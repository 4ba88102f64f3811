"""Sample diagnostics on the device.

Every statistic is computed by libmcmc355.so kernels (csrc/diag.h) on the
[C, S, D] sample buffer the samplers write; only per-element results (D
values) or a handful of order statistics come back to the host.

* ``compute_ess(samples)`` — the reference helper
  (examples/06_nuts_comparison.py:22-41) for one series: n / (1 + 2 sum rho_k)
  over lags 1 .. min(n//2, 100) - 1, stopping at (and including) the first
  rho < 0.05; n for a constant series.
* ``chain_diagnostics(samples)`` — per-series ESS (the same rule), ESS summed
  over chains and split R-hat (BDA3 eq. 11.4; the reference lists R-hat on its
  roadmap, README.md:214, without code) per element.  Under torch.distributed
  with chains sharded over ranks the reductions are two all-reduces of
  [2, D] f64 blocks — no sample leaves its GPU.
* ``summarize(samples, layout)`` — ``MCMC.summary`` (mcmc.py:191-227): pooled
  mean / std from per-series moments, median and percentiles from exact
  device order statistics, interpolated with numpy's own rule.

No CPU fallback: without the library these raise ``EngineUnavailable``.
"""
from __future__ import annotations

import ctypes
from typing import Dict

import numpy as np

from . import _lib

MAX_LAG = 100   # examples/06_nuts_comparison.py:33


def _as_device(samples):
    """[C, S, D] f32 contiguous device tensor from a tensor or array of
    shape [S], [S, D] (one chain) or [C, S, D]."""
    import torch

    dev = _lib.require_device()
    t = samples if isinstance(samples, torch.Tensor) else torch.from_numpy(
        np.array(samples, dtype=np.float32, copy=True))
    t = t.to(device=dev, dtype=torch.float32)
    if t.dim() == 1:
        t = t[None, :, None]
    elif t.dim() == 2:
        t = t[None]
    elif t.dim() != 3:
        raise ValueError("samples must be [S], [S, D] or [C, S, D]")
    return t.contiguous()


def series_stats(samples, max_lag: int = MAX_LAG):
    """mc_series_stats: [MC_ST_COUNT, C*D] f64 device tensor (fields in _lib.MC_ST_*)."""
    import torch

    x = _as_device(samples)
    C, S, D = x.shape
    st = torch.empty((_lib.MC_ST_COUNT, C * D), dtype=torch.float64, device=x.device)
    lib = _lib.load()
    _lib.check(lib.mc_series_stats(C, S, D, _lib.ptr(x), int(max_lag), _lib.ptr(st),
                                   _lib.stream_handle()))
    return st


def compute_ess(samples) -> float:
    """Reference ``compute_ess`` of one 1-D series, evaluated on the device."""
    x = np.asarray(samples)
    if x.ndim != 1:
        raise ValueError("compute_ess takes one 1-D series")
    if len(x) == 0:
        raise ValueError("empty series")
    return float(series_stats(x)[_lib.MC_ST_ESS, 0].item())


def ess(samples, max_lag: int = MAX_LAG):
    """Per-series ESS, [C, D] f64 numpy (reference rule for every chain and element)."""
    x = _as_device(samples)
    C, S, D = x.shape
    return series_stats(x, max_lag)[_lib.MC_ST_ESS].view(C, D).cpu().numpy()


def _all_reduce(t, group):
    import torch.distributed as dist

    if group is not False and dist.is_available() and dist.is_initialized() \
            and dist.get_world_size(group) > 1:
        if dist.get_backend(group) == "gloo" and t.is_cuda:
            # gloo (a CPU rehearsal of the RCCL path): reduce a host copy
            h = t.cpu()
            dist.all_reduce(h, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, group=group)
    return t


def chain_diagnostics(samples, max_lag: int = MAX_LAG, group=None) -> Dict[str, np.ndarray]:
    """ESS and split R-hat per element of a [C, S, D] buffer.

    Returns ``ess`` [C, D] (this rank's chains), ``ess_sum`` [D] (summed over
    every chain of every rank), ``rhat`` [D] (NaN unless S >= 4),
    ``n_constant`` (series of zero variance over all ranks) and
    ``n_nonpositive_ess`` (per-chain ESS values <= 0 over all ranks).  With an
    initialised process group (pass ``group=False`` to stay local) the chain
    sums are all-reduced over the ranks' shards.
    """
    import torch

    x = _as_device(samples)
    C, S, D = x.shape
    lib = _lib.load()
    stream = _lib.stream_handle()
    # a rank whose shard holds no chain (e.g. every one of its chains was
    # left out as frozen) still joins the all-reduces with zero blocks
    st = series_stats(x, max_lag) if C > 0 else torch.zeros(
        (_lib.MC_ST_COUNT, 0), dtype=torch.float64, device=x.device)
    red = torch.zeros((2, D), dtype=torch.float64, device=x.device)
    if C > 0:
        _lib.check(lib.mc_stats_reduce(C, S, D, _lib.ptr(st), None, 0, _lib.ptr(red), stream))
    # [split chains, constant series]: a constant series scores ESS = n by
    # the reference rule, so callers need to know how many there are
    # and non-positive per-chain ESS values (the reference rule on antithetic
    # draws): every rank's count, so every rank takes the same branch on them
    counts = torch.stack([torch.tensor(2.0 * C, dtype=torch.float64, device=x.device),
                          (st[_lib.MC_ST_M2] == 0).sum().to(torch.float64),
                          (st[_lib.MC_ST_ESS] <= 0).sum().to(torch.float64)])
    _all_reduce(red, group)
    _all_reduce(counts, group)
    ess_sum = red[1].clone()
    rhat = torch.full((D,), float("nan"), dtype=torch.float64, device=x.device)
    m_total, n_const, n_nonpos = (int(v) for v in counts.tolist())
    m = m_total
    if S >= 4 and m >= 2:
        center = red[0].contiguous()
        spread = torch.zeros((2, D), dtype=torch.float64, device=x.device)
        if C > 0:
            _lib.check(lib.mc_stats_reduce(C, S, D, _lib.ptr(st), _lib.ptr(center), m,
                                           _lib.ptr(spread), stream))
        _all_reduce(spread, group)
        _lib.check(lib.mc_rhat(D, m, S, _lib.ptr(spread), _lib.ptr(rhat), stream))
    return {"ess": st[_lib.MC_ST_ESS].view(C, D).cpu().numpy(),
            "ess_sum": ess_sum.cpu().numpy(), "rhat": rhat.cpu().numpy(),
            "n_constant": n_const, "n_nonpositive_ess": n_nonpos}


# ------------------------------------------------------------ summary -----
def order_statistics(x, off: int, length: int, ranks):
    """Exact k-th smallest pooled values of elements [off, off+length) of a
    device [C, S, D] buffer (mc_select), as float32; NaN if any value is NaN."""
    import torch

    C, S, D = x.shape
    ranks = [int(r) for r in ranks]
    lib = _lib.load()
    out = torch.empty(len(ranks), dtype=torch.float32, device=x.device)
    for i in range(0, len(ranks), 8):
        chunk = ranks[i:i + 8]
        nb = lib.mc_select_workspace_bytes(len(chunk))
        ws = torch.empty(nb, dtype=torch.uint8, device=x.device)
        karr = (ctypes.c_int64 * len(chunk))(*chunk)
        o = out[i:i + len(chunk)]
        _lib.check(lib.mc_select(C, S, D, _lib.ptr(x), off, length, len(chunk), karr,
                                 _lib.ptr(o), _lib.ptr(ws), nb, _lib.stream_handle()))
    return out.cpu().numpy()


def _percentile_ranks(n: int, q: float):
    """numpy's 'linear' percentile (np.percentile, numpy 2.x): the virtual
    index (n - 1) * (q / 100) is formed in the data dtype (float32 here)."""
    q32 = np.true_divide(np.asarray(q, np.float32), np.float32(100))
    vi = np.asarray((n - 1) * q32)
    if vi >= n - 1:      # _get_indexes: above the last index -> the maximum
        return n - 1, n - 1, np.asarray(0.0, vi.dtype)
    prev = np.floor(vi)
    gamma = np.asarray(vi - prev, dtype=vi.dtype)
    return int(prev), int(prev) + 1, gamma


def _lerp(a, b, t):
    """numpy's _lerp (numpy/lib/_function_base_impl.py) on float32 bounds."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    diff = np.subtract(b, a)
    r = np.add(a, diff * t)
    if t >= 0.5:
        r = np.subtract(b, diff * (1 - t))
    return r[()]


def quantiles_from_order_stats(n: int, lower_pct: float, upper_pct: float, fetch):
    """(median, lower, upper) exactly as np.median / np.percentile return them
    for n float32 values, given ``fetch(ranks) -> values`` of the sorted pool."""
    lo = _percentile_ranks(n, lower_pct)
    hi = _percentile_ranks(n, upper_pct)
    mid = [(n - 1) // 2, n // 2]
    ranks = sorted({lo[0], lo[1], hi[0], hi[1], *mid})
    vals = dict(zip(ranks, fetch(ranks)))
    a, b = np.float32(vals[mid[0]]), np.float32(vals[mid[1]])
    median = a if n % 2 else np.float32(np.float32(a + b) / 2)   # np.median: f32 mean of two
    return (median, _lerp(vals[lo[0]], vals[lo[1]], lo[2]),
            _lerp(vals[hi[0]], vals[hi[1]], hi[2]))


def summarize(samples, layout=None, credible_interval: float = 0.95) -> Dict[str, dict]:
    """``MCMC.summary`` (mcmc.py:191-227) from device statistics.

    ``samples``: a [C, S, D] device tensor with ``layout`` (names, shapes,
    offsets of the flattened elements), or a dict name -> array as
    ``MCMC.samples`` holds it.  Every value of a parameter (all chains, draws
    and vector elements) is pooled, exactly as np.mean(s) etc. pool them.
    """
    import torch

    alpha = 1 - credible_interval
    lower_pct = 100 * alpha / 2
    upper_pct = 100 * (1 - alpha / 2)
    if isinstance(samples, dict):
        # the pool is every value; its columns (last axis) become the series
        items = []
        for name, a in samples.items():
            a = np.asarray(a, np.float32)
            w = a.shape[-1] if a.ndim >= 2 else 1
            items.append((name, _as_device(a.reshape(1, -1, w)), 0, w))
    else:
        if layout is None:
            raise ValueError("a [C, S, D] buffer needs its layout")
        x = _as_device(samples)
        items = [(name, x, int(off), int(np.prod(shape)) if shape else 1)
                 for name, shape, off in zip(layout.names, layout.shapes, layout.offsets)]
    out: Dict[str, dict] = {}
    lib = _lib.load()
    for name, x, off, length in items:
        C, S, D = x.shape
        st = series_stats(x)
        mom = torch.empty(2, dtype=torch.float64, device=x.device)
        _lib.check(lib.mc_pool_moments(C, S, D, _lib.ptr(st), off, length, _lib.ptr(mom),
                                       _lib.stream_handle()))
        mean, std = mom.cpu().numpy().tolist()
        med, lo, hi = quantiles_from_order_stats(
            C * S * length, lower_pct, upper_pct,
            lambda ranks: order_statistics(x, off, length, ranks))
        out[name] = {
            'mean': float(mean),
            'std': float(std),
            'median': float(med),
            f'{lower_pct:.1f}%': float(lo),
            f'{upper_pct:.1f}%': float(hi),
        }
    return out
