"""Distributions of the tape: ``Distribution``, ``Normal``, ``HalfNormal``,
``Exponential``, ``Gamma``, ``Beta``.

Same constructor arguments, ``log_prob(value)`` / ``sample(key, shape)``
contract and formulas as the reference (mlx_mcmc/distributions/base.py:6-54,
normal.py:8-80, halfnormal.py:8-86, exponential.py:5-131, gamma.py:8-149,
beta.py:8-151):

  Normal:      log p(x) = -0.5 log(2 pi) - log(scale) - 0.5 (x - loc)^2 / scale^2
  HalfNormal:  log p(x) = log 2 - 0.5 log(2 pi) - log(scale) - 0.5 x^2 / scale^2
               for x >= 0, -inf otherwise
  Exponential: log p(x) = log(rate) - rate x for x >= 0, -inf otherwise
  Gamma:       log p(x) = alpha log(beta) - gammaln(alpha) + (alpha - 1) log x - beta x
               for x > 0, -inf otherwise
  Beta:        log p(x) = (alpha - 1) log x + (beta - 1) log(1 - x) - log B(alpha, beta)
               for 0 < x < 1, -inf otherwise
  (the gammaln normalisers are values without gradient, as the reference's
  host scipy gammaln)

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
        return torch.from_numpy(np.broadcast_to(a, out_shape).reshape(-1).copy()).to(dev), 0

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


def _gpu_uniforms(key, shape) -> np.ndarray:
    """Uniforms in (0, 1) from the engine's Philox stream (tag USER)."""
    import torch

    dev = _lib.require_device()
    k = _as_key(key)
    shape = tuple(shape) if isinstance(shape, (tuple, list)) else (int(shape),)
    n = int(np.prod(shape)) if shape else 1
    blocks = (n + 3) // 4
    out = torch.empty(max(1, blocks) * 4, dtype=torch.float32, device=dev)
    _lib.check(_lib.load().mc_rng_fill(k.seed, 0, 0, _lib.MC_RNG_TAG_USER, 1, 0, blocks, 1,
                                       _lib.ptr(out), _lib.stream_handle()))
    return out[:n].cpu().numpy().reshape(shape)


def _host_rng(key) -> np.random.Generator:
    """gamma.py:101-109 / beta.py: the reference draws Gamma and Beta samples with
    NumPy seeded from its key; here the seed is the key's Philox seed."""
    return np.random.default_rng(_as_key(key).seed & 0x7FFFFFFF)


class Exponential(Distribution):
    """Exponential(rate) (mlx_mcmc/distributions/exponential.py:5-131)."""

    def __init__(self, rate):
        self.rate = rate

    def log_prob(self, value):
        if _trace.is_symbolic(value, self.rate):
            return _trace.make_term(_lib.MC_DIST_EXPONENTIAL, "Exponential", value, None,
                                    self.rate)
        return _gpu_log_prob(_lib.MC_DIST_EXPONENTIAL, value, None, self.rate)

    def sample(self, key, shape=()):
        # inverse CDF as exponential.py:73-91: -log(1 - u) / rate
        u = _gpu_uniforms(key, shape)
        return (-np.log(np.float32(1) - u) / _to_f32(self.rate)).astype(np.float32)

    def mean(self):
        return np.float32(1.0) / _to_f32(self.rate)

    def variance(self):
        return np.float32(1.0) / (_to_f32(self.rate) ** 2)

    def mode(self):
        return np.zeros_like(_to_f32(self.rate))

    def __repr__(self):
        return f"Exponential(rate={_scalar_repr(self.rate)})"


class Gamma(Distribution):
    """Gamma(alpha, beta=1.0), shape-rate (mlx_mcmc/distributions/gamma.py:8-149)."""

    def __init__(self, alpha, beta=1.0):
        self.alpha = alpha
        self.beta = beta

    def log_prob(self, value):
        if _trace.is_symbolic(value, self.alpha, self.beta):
            return _trace.make_term(_lib.MC_DIST_GAMMA, "Gamma", value, self.alpha, self.beta)
        return _gpu_log_prob(_lib.MC_DIST_GAMMA, value, self.alpha, self.beta)

    def sample(self, key, shape=()):
        a, b = float(_to_f32(self.alpha)), float(_to_f32(self.beta))
        return _host_rng(key).gamma(a, scale=1.0 / b, size=shape).astype(np.float32)

    def mean(self):
        return _to_f32(self.alpha) / _to_f32(self.beta)

    def variance(self):
        return _to_f32(self.alpha) / (_to_f32(self.beta) ** 2)

    def mode(self):
        a, b = _to_f32(self.alpha), _to_f32(self.beta)
        return np.where(a >= 1, (a - 1) / b, np.float32(0)).astype(np.float32)

    def __repr__(self):
        return f"Gamma(alpha={_scalar_repr(self.alpha)}, beta={_scalar_repr(self.beta)})"


class Beta(Distribution):
    """Beta(alpha, beta) (mlx_mcmc/distributions/beta.py:8-151)."""

    def __init__(self, alpha, beta):
        self.alpha = alpha
        self.beta = beta

    def log_prob(self, value):
        if _trace.is_symbolic(value, self.alpha, self.beta):
            return _trace.make_term(_lib.MC_DIST_BETA, "Beta", value, self.alpha, self.beta)
        return _gpu_log_prob(_lib.MC_DIST_BETA, value, self.alpha, self.beta)

    def sample(self, key, shape=()):
        a, b = float(_to_f32(self.alpha)), float(_to_f32(self.beta))
        return _host_rng(key).beta(a, b, size=shape).astype(np.float32)

    def mean(self):
        a, b = _to_f32(self.alpha), _to_f32(self.beta)
        return a / (a + b)

    def variance(self):
        a, b = _to_f32(self.alpha), _to_f32(self.beta)
        return (a * b) / ((a + b) ** 2 * (a + b + 1))

    def mode(self):
        a, b = _to_f32(self.alpha), _to_f32(self.beta)
        return ((a - 1) / (a + b - 2)).astype(np.float32)

    def __repr__(self):
        return f"Beta(alpha={_scalar_repr(self.alpha)}, beta={_scalar_repr(self.beta)})"


__all__ = ["Distribution", "Normal", "HalfNormal", "Exponential", "Gamma", "Beta", "Key"]
