"""Distributions on the sampling hot path: ``Distribution``, ``Normal``, ``HalfNormal``.

Same constructor arguments, ``log_prob(value)`` / ``sample(key, shape)``
contract and formulas as the reference (mlx_mcmc/distributions/base.py:6-54,
normal.py:8-80, halfnormal.py:8-86):

  Normal:      log p(x) = -0.5 log(2 pi) - log(scale) - 0.5 (x - loc)^2 / scale^2
  HalfNormal:  log p(x) = log 2 - 0.5 log(2 pi) - log(scale) - 0.5 x^2 / scale^2
               for x >= 0, -inf otherwise

Inside a traced ``log_prob(params)`` (any argument is a traced parameter),
``log_prob`` records a fused term for the HIP tape (see _trace.py).  On
concrete values it is evaluated elementwise on the GPU by the same device
code (``mc_dist_log_prob``) and returned as a float32 NumPy array; ``sample``
draws from the engine's Philox stream on the GPU.
"""
from __future__ import annotations

import numpy as np

from . import _lib, _trace
from .random import Key, _as_key


def _to_f32(x):
    return np.asarray(_trace._to_numpy(x), np.float32)


def _gpu_log_prob(dist: int, value, loc, scale) -> np.ndarray:
    import torch

    dev = _lib.require_device()
    v, s = _to_f32(value), _to_f32(scale)
    m = _to_f32(loc) if loc is not None else None
    shapes = [a.shape for a in (v, m, s) if a is not None]
    out_shape = np.broadcast_shapes(*shapes)
    n = int(np.prod(out_shape)) if out_shape else 1

    def dev_arr(a):
        if a is None:
            return None, 1
        if a.size == 1:
            return torch.from_numpy(a.reshape(1).copy()).to(dev), 1
        return torch.from_numpy(np.ascontiguousarray(
            np.broadcast_to(a, out_shape)).reshape(-1)).to(dev), 0

    tv, bv = dev_arr(v)
    tm, bm = dev_arr(m)
    ts, bs = dev_arr(s)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    lib = _lib.load()
    _lib.check(lib.mc_dist_log_prob(dist, n, _lib.ptr(tv), bv, _lib.ptr(tm), bm,
                                    _lib.ptr(ts), bs, _lib.ptr(out), _lib.stream_handle()))
    return out.cpu().numpy().reshape(out_shape)


class Distribution:
    """Base class: subclasses implement ``log_prob(value)`` and ``sample(key, shape)``
    (mlx_mcmc/distributions/base.py:6-54)."""

    def log_prob(self, value):
        raise NotImplementedError(f"{self.__class__.__name__} must implement log_prob()")

    def sample(self, key, shape=()):
        raise NotImplementedError(f"{self.__class__.__name__} must implement sample()")

    def __repr__(self):
        return f"{self.__class__.__name__}()"


def _scalar_repr(x):
    try:
        return f"{float(np.asarray(_trace._to_numpy(x)).reshape(())):.3f}"
    except Exception:
        return repr(x)


def _gpu_normals(key, shape) -> np.ndarray:
    """Standard normals from the engine's Philox stream (tag USER)."""
    import torch

    dev = _lib.require_device()
    k = _as_key(key)
    shape = tuple(shape) if isinstance(shape, (tuple, list)) else (int(shape),)
    n = int(np.prod(shape)) if shape else 1
    blocks = (n + 3) // 4
    out = torch.empty(max(1, blocks) * 4, dtype=torch.float32, device=dev)
    _lib.check(_lib.load().mc_rng_fill(k.seed, 0, 0, _lib.MC_RNG_TAG_USER, 0, 0, blocks, 2,
                                       _lib.ptr(out), _lib.stream_handle()))
    return out[:n].cpu().numpy().reshape(shape)


class Normal(Distribution):
    """Normal(loc, scale) (mlx_mcmc/distributions/normal.py:8-80)."""

    def __init__(self, loc, scale):
        self.loc = loc
        self.scale = scale

    def log_prob(self, value):
        if _trace.is_symbolic(value, self.loc, self.scale):
            return _trace.make_term(_lib.MC_DIST_NORMAL, "Normal", value, self.loc, self.scale)
        return _gpu_log_prob(_lib.MC_DIST_NORMAL, value, self.loc, self.scale)

    def sample(self, key, shape=()):
        z = _gpu_normals(key, shape)
        return (z * _to_f32(self.scale) + _to_f32(self.loc)).astype(np.float32)

    def __repr__(self):
        return f"Normal(loc={_scalar_repr(self.loc)}, scale={_scalar_repr(self.scale)})"


class HalfNormal(Distribution):
    """HalfNormal(scale) (mlx_mcmc/distributions/halfnormal.py:8-86)."""

    def __init__(self, scale):
        self.scale = scale

    def log_prob(self, value):
        if _trace.is_symbolic(value, self.scale):
            return _trace.make_term(_lib.MC_DIST_HALFNORMAL, "HalfNormal", value, None,
                                    self.scale)
        return _gpu_log_prob(_lib.MC_DIST_HALFNORMAL, value, None, self.scale)

    def sample(self, key, shape=()):
        z = _gpu_normals(key, shape)
        return np.abs(z * _to_f32(self.scale)).astype(np.float32)

    def __repr__(self):
        return f"HalfNormal(scale={_scalar_repr(self.scale)})"


__all__ = ["Distribution", "Normal", "HalfNormal", "Key"]
