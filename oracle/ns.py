"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by mlx_mcmc_amd/).

An eager float32 namespace standing in for ``mlx.core`` + the reference's
distributions, on PyTorch CPU tensors, so that user models written against
the reference API run unchanged in the CPU restatement and are differentiated
by autograd exactly where the reference uses ``mx.grad``.

  Normal      restates mlx_mcmc/distributions/normal.py:27-56
  HalfNormal  restates mlx_mcmc/distributions/halfnormal.py:28-63
  Exponential restates mlx_mcmc/distributions/exponential.py:40-71
  Gamma       restates mlx_mcmc/distributions/gamma.py:40-88
  Beta        restates mlx_mcmc/distributions/beta.py:37-91
              (gammaln: host float64 value, no gradient, as the reference)
  sum/array/log/exp/sqrt/square/power/abs/log1p/tanh/sigmoid/where/pi/inf
              the mx.* calls those models use

Pinned by the reference's own known-answer tests (tests/test_oracle_pins.py
re-asserts tests/test_distributions.py:18-32,67-79 of the reference).
"""
from __future__ import annotations

import math

import numpy as np
import torch

pi = math.pi
inf = float("inf")
F32 = torch.float32


def _t(x):
    if isinstance(x, torch.Tensor):
        return x
    return torch.as_tensor(np.asarray(x, dtype=np.float32))


def array(x, dtype=None):
    if isinstance(x, (list, tuple)) and any(isinstance(v, torch.Tensor) for v in x):
        return torch.stack([_t(v).reshape(()) for v in x])
    return _t(x)


def sum(x, axis=None, keepdims=False):  # noqa: A001
    x = _t(x)
    return torch.sum(x) if axis is None else torch.sum(x, dim=axis, keepdim=keepdims)


def mean(x, axis=None, keepdims=False):
    """MLX's mean: the sum times the f32 reciprocal of the count."""
    x = _t(x)
    n = x.numel() if axis is None else int(np.prod([x.shape[a] for a in
                                                     (axis if isinstance(axis, (tuple, list)) else (axis,))]))
    r = float(np.float32(1.0) / np.float32(n))
    return (torch.sum(x) if axis is None else torch.sum(x, dim=axis, keepdim=keepdims)) * r


def log(x):
    return torch.log(_t(x))


def exp(x):
    return torch.exp(_t(x))


def sqrt(x):
    return torch.sqrt(_t(x))


def square(x):
    return torch.square(_t(x))


def power(a, b):
    return torch.pow(_t(a), _t(b))


def abs(x):  # noqa: A001
    return torch.abs(_t(x))


def log1p(x):
    return torch.log1p(_t(x))


def tanh(x):
    return torch.tanh(_t(x))


def sigmoid(x):
    return torch.sigmoid(_t(x))


def greater(a, b):
    return torch.gt(_t(a), _t(b))


def greater_equal(a, b):
    return torch.ge(_t(a), _t(b))


def less(a, b):
    return torch.lt(_t(a), _t(b))


def less_equal(a, b):
    return torch.le(_t(a), _t(b))


def where(c, a, b):
    c = _t(c)
    return torch.where(c if c.dtype == torch.bool else c != 0, _t(a), _t(b))


class Normal:
    """normal.py:27-56 — the formula and the f32 constants as the reference forms them."""

    def __init__(self, loc, scale):
        self.loc = _t(loc)
        self.scale = _t(scale)
        self._log_scale = torch.log(self.scale)
        self._log_norm = -0.5 * torch.log(_t(2 * math.pi))

    def log_prob(self, value):
        value = _t(value)
        var = self.scale ** 2
        return self._log_norm - self._log_scale - 0.5 * ((value - self.loc) ** 2) / var

    def sample(self, key, shape=()):
        raise NotImplementedError("oracle distributions do not sample")


class HalfNormal:
    """halfnormal.py:28-63."""

    def __init__(self, scale):
        self.scale = _t(scale)
        self._log_scale = torch.log(self.scale)
        self._log_norm = -0.5 * torch.log(_t(2 * math.pi))
        self._log2 = torch.log(_t(2.0))

    def log_prob(self, value):
        value = _t(value)
        var = self.scale ** 2
        log_prob_pos = self._log2 + self._log_norm - self._log_scale - 0.5 * (value ** 2) / var
        return torch.where(value >= 0, log_prob_pos, _t(-inf))


def _gammaln(x):
    """scipy.special.gammaln on the host, as gamma.py:48-59 / beta.py:45-57 call it:
    float64 of the current float32 value, a constant for autograd."""
    return torch.lgamma(_t(x).detach().double())


class Exponential:
    """exponential.py:40-71."""

    def __init__(self, rate):
        self.rate = _t(rate)

    def log_prob(self, value):
        value = _t(value)
        lp = torch.log(self.rate) - self.rate * value
        return torch.where(value >= 0, lp, _t(-inf))


class Gamma:
    """gamma.py:40-88 (shape alpha, rate beta)."""

    def __init__(self, alpha, beta=1.0):
        self.alpha = _t(alpha)
        self.beta = _t(beta)
        self._log_norm = self.alpha * torch.log(self.beta) - _gammaln(self.alpha).float()

    def log_prob(self, value):
        value = _t(value)
        lp = self._log_norm + (self.alpha - 1) * torch.log(value) - self.beta * value
        return torch.where(value > 0, lp, _t(-inf))


class Beta:
    """beta.py:37-91."""

    def __init__(self, alpha, beta):
        self.alpha = _t(alpha)
        self.beta = _t(beta)
        a, b = _gammaln(self.alpha), _gammaln(self.beta)
        ab = torch.lgamma(self.alpha.detach().double() + self.beta.detach().double())
        self._log_beta_const = (a + b - ab).float()

    def log_prob(self, value):
        value = _t(value)
        lp = ((self.alpha - 1) * torch.log(value) + (self.beta - 1) * torch.log(1 - value)
              - self._log_beta_const)
        return torch.where((value > 0) & (value < 1), lp, _t(-inf))
