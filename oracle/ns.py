"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by mlx_mcmc_amd/).

An eager float32 namespace standing in for ``mlx.core`` + the reference's
distributions, on PyTorch CPU tensors, so that user models written against
the reference API run unchanged in the CPU restatement and are differentiated
by autograd exactly where the reference uses ``mx.grad``.

  Normal      restates mlx_mcmc/distributions/normal.py:27-56
  HalfNormal  restates mlx_mcmc/distributions/halfnormal.py:28-63
  sum/array/log/exp/where/pi/inf  the mx.* calls those models use

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


def sum(x, axis=None):  # noqa: A001
    x = _t(x)
    return torch.sum(x) if axis is None else torch.sum(x, dim=axis)


def log(x):
    return torch.log(_t(x))


def exp(x):
    return torch.exp(_t(x))


def where(c, a, b):
    return torch.where(_t(c).bool() if not isinstance(c, torch.Tensor) else c, _t(a), _t(b))


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
