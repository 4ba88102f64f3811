"""``mx``-compatible array namespace for user models: ``import mlx_mcmc_amd.core as mx``.

Models written for the reference (``import mlx.core as mx``) use a handful of
``mx`` calls inside ``log_prob`` — ``mx.sum``, ``mx.array`` — and a few more on
the returned samples (``mx.mean``, ``mx.std``, ``mx.all``, ``mx.allclose``) and
``mx.random.key``.  Inside a traced ``log_prob`` these build the term program
(_trace.py); on concrete arrays they are ordinary NumPy float32 operations on
the host (post-processing only: sampling itself runs in the HIP kernels).
"""
from __future__ import annotations

import math

import numpy as np

from . import _trace
from . import random  # noqa: F401  (mx.random.key / split)

pi = math.pi
inf = float("inf")
nan = float("nan")
float32 = np.float32
int32 = np.int32


def array(x, dtype=None):
    if isinstance(x, (list, tuple)) and any(isinstance(v, _trace.LogProbExpr) for v in x):
        return _trace.stack(list(x))
    if isinstance(x, (_trace.LogProbExpr, _trace.Param, _trace.Affine)):
        return x
    a = np.asarray(_trace._to_numpy(x))
    if dtype is not None:
        return a.astype(dtype)
    if a.dtype.kind in "iu":
        return a.astype(np.int32)
    if a.dtype == np.bool_:
        return a
    return a.astype(np.float32)


def sum(x, axis=None, keepdims=False):  # noqa: A001 - mirrors mx.sum
    if isinstance(x, _trace.LogProbExpr):
        return x.sum(axis)
    if isinstance(x, (_trace.Param, _trace.Affine)):
        # a parameter expression summed into a log density (`mx.sum(log_x)`,
        # the Jacobian of a vector reparameterisation): identity terms
        return _trace.identity_expr(x).sum(axis)
    return np.sum(np.asarray(x), axis=axis, keepdims=keepdims)


def _concrete(name, fn):
    def f(x, *a, **k):
        if _trace.is_symbolic(x, *a):
            raise _trace.TraceError(f"mx.{name} of a traced value: " + _trace._UNSUPPORTED)
        return fn(np.asarray(_trace._to_numpy(x)), *a, **k)

    f.__name__ = name
    return f


def _transform(name, xf, fn):
    """mx.exp / mx.log: of a traced parameter (or view) a transformed parameter
    operand (mc_transform_kind); of concrete arrays the NumPy f32 value."""
    def f(x, *a, **k):
        if isinstance(x, _trace.Param) and not a and not k:
            return x.transformed(xf, name)
        if _trace.is_symbolic(x, *a):
            raise _trace.TraceError(f"mx.{name} of a traced expression (only of a parameter or "
                                    "a view of one): " + _trace._UNSUPPORTED)
        return fn(np.asarray(_trace._to_numpy(x)), *a, **k)

    f.__name__ = name
    return f


log = _transform("log", 2, np.log)
exp = _transform("exp", 1, np.exp)
sqrt = _concrete("sqrt", np.sqrt)
abs = _concrete("abs", np.abs)  # noqa: A001
mean = _concrete("mean", np.mean)
std = _concrete("std", np.std)
var = _concrete("var", np.var)
median = _concrete("median", np.median)
all = _concrete("all", np.all)  # noqa: A001
any = _concrete("any", np.any)  # noqa: A001
isnan = _concrete("isnan", np.isnan)
isinf = _concrete("isinf", np.isinf)


def where(cond, a, b):
    if _trace.is_symbolic(cond, a, b):
        raise _trace.TraceError("mx.where of traced values: " + _trace._UNSUPPORTED)
    return np.where(cond, a, b)


def allclose(a, b, rtol=1e-5, atol=1e-8, equal_nan=False):
    return bool(np.allclose(np.asarray(a), np.asarray(b), rtol=rtol, atol=atol,
                            equal_nan=equal_nan))


def eval(*args):  # noqa: A001 - mx.eval is a no-op here (results are eager)
    return None
