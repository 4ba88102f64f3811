"""``mx``-compatible array namespace for user models: ``import mlx_mcmc_amd.core as mx``.

Models written for the reference (``import mlx.core as mx``) use ``mx`` calls
inside ``log_prob`` — ``mx.sum``, ``mx.array``, elementwise math (``mx.exp``,
``mx.log``, ``mx.sqrt``, ``mx.square``, ``mx.power``, ``mx.abs``,
``mx.log1p``, ``mx.tanh``, ``mx.sigmoid``, ``mx.where`` over a data mask) —
and a few more on the returned samples (``mx.mean``, ``mx.std``, ``mx.all``,
``mx.allclose``) and ``mx.random.key``.  Inside a traced ``log_prob`` these
build the term program (_trace.py: fused terms, or expression terms for
general elementwise arithmetic); on concrete arrays they are ordinary NumPy
float32 operations on the host (post-processing only: sampling itself runs in
the HIP kernels).
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


def _as_log_density(x):
    """A traced value summed into a log density: itself, or a parameter
    expression (`mx.sum(log_x)`, the Jacobian of a vector reparameterisation)
    as identity terms, or an expression term when it is more general."""
    if isinstance(x, _trace.LogProbExpr):
        return x
    if isinstance(x, (_trace.Param, _trace.Affine)):
        try:
            return _trace.identity_expr(x)
        except _trace.TraceError:
            return _trace.expr_term(_trace.Expr.of(x))
    return _trace.expr_term(x)


def sum(x, axis=None, keepdims=False):  # noqa: A001 - mirrors mx.sum
    if isinstance(x, (_trace.LogProbExpr, _trace.Param, _trace.Affine, _trace.Expr)):
        return _as_log_density(x).sum(axis, keepdims)
    return np.sum(np.asarray(x), axis=axis, keepdims=keepdims)


def mean(x, axis=None, keepdims=False):
    """mx.mean: of a log density (or a parameter expression summed into one)
    its sum times 1 / n; of concrete arrays the NumPy value."""
    if isinstance(x, (_trace.LogProbExpr, _trace.Param, _trace.Affine, _trace.Expr)):
        return _as_log_density(x).mean(axis, keepdims)
    return np.mean(np.asarray(_trace._to_numpy(x)), axis=axis, keepdims=keepdims)


def _concrete(name, fn):
    def f(x, *a, **k):
        if _trace.is_symbolic(x, *a):
            raise _trace.TraceError(f"mx.{name} of a traced value: " + _trace._UNSUPPORTED)
        return fn(np.asarray(_trace._to_numpy(x)), *a, **k)

    f.__name__ = name
    return f


def _transform(name, xf, op, fn):
    """mx.exp / mx.log: of a traced parameter (or view) a transformed parameter
    operand (mc_transform_kind, the fused fast paths); of any other traced
    expression an expression node; of concrete arrays the NumPy f32 value."""
    def f(x, *a, **k):
        if isinstance(x, _trace.Param) and not x.xf and not a and not k:
            return x.transformed(xf, name)
        if _trace.is_symbolic(x, *a):
            return _trace.Expr.unary(op, x)
        return fn(np.asarray(_trace._to_numpy(x)), *a, **k)

    f.__name__ = name
    return f


def _elementwise(name, op, fn):
    """An elementwise mx function: an expression node of a traced value, the
    NumPy f32 value of a concrete one."""
    def f(x):
        if _trace.is_symbolic(x):
            return _trace.Expr.unary(op, x)
        return fn(np.asarray(_trace._to_numpy(x), np.float32))

    f.__name__ = name
    return f


def _sigmoid(x):
    return (np.float32(1) / (np.float32(1) + np.exp(-x))).astype(np.float32)


log = _transform("log", 2, _trace._lib.MC_EX_LOG, np.log)
exp = _transform("exp", 1, _trace._lib.MC_EX_EXP, np.exp)
sqrt = _elementwise("sqrt", _trace._lib.MC_EX_SQRT, np.sqrt)
square = _elementwise("square", _trace._lib.MC_EX_SQUARE, np.square)
abs = _elementwise("abs", _trace._lib.MC_EX_ABS, np.abs)  # noqa: A001
log1p = _elementwise("log1p", _trace._lib.MC_EX_LOG1P, np.log1p)
tanh = _elementwise("tanh", _trace._lib.MC_EX_TANH, np.tanh)
sigmoid = _elementwise("sigmoid", _trace._lib.MC_EX_SIGMOID, _sigmoid)
negative = _elementwise("negative", _trace._lib.MC_EX_NEG, np.negative)


def power(a, b):
    if _trace.is_symbolic(a, b):
        return _trace.Expr.binary(_trace._lib.MC_EX_POW, a, b)
    return np.power(np.asarray(_trace._to_numpy(a), np.float32),
                    np.asarray(_trace._to_numpy(b), np.float32))


def _binary(name, op, fn):
    def f(a, b):
        if _trace.is_symbolic(a, b):
            return _trace.Expr.binary(op, a, b)
        return fn(np.asarray(_trace._to_numpy(a), np.float32),
                  np.asarray(_trace._to_numpy(b), np.float32))

    f.__name__ = name
    return f


add = _binary("add", _trace._lib.MC_EX_ADD, np.add)
subtract = _binary("subtract", _trace._lib.MC_EX_SUB, np.subtract)
multiply = _binary("multiply", _trace._lib.MC_EX_MUL, np.multiply)
divide = _binary("divide", _trace._lib.MC_EX_DIV, np.divide)
std = _concrete("std", np.std)
var = _concrete("var", np.var)
median = _concrete("median", np.median)
all = _concrete("all", np.all)  # noqa: A001
any = _concrete("any", np.any)  # noqa: A001
isnan = _concrete("isnan", np.isnan)
isinf = _concrete("isinf", np.isinf)


greater = _binary("greater", _trace._lib.MC_EX_GT, np.greater)
greater_equal = _binary("greater_equal", _trace._lib.MC_EX_GE, np.greater_equal)
less = _binary("less", _trace._lib.MC_EX_LT, np.less)
less_equal = _binary("less_equal", _trace._lib.MC_EX_LE, np.less_equal)


def where(cond, a, b):
    """mx.where: over a data mask, or over a traced condition (a comparison of
    traced values; no cotangent through the condition, as mx.where's VJP)."""
    if _trace.is_symbolic(cond, a, b):
        return _trace.Expr.where(cond, a, b)
    return np.where(cond, a, b)


def allclose(a, b, rtol=1e-5, atol=1e-8, equal_nan=False):
    return bool(np.allclose(np.asarray(a), np.asarray(b), rtol=rtol, atol=atol,
                            equal_nan=equal_nan))


def eval(*args):  # noqa: A001 - mx.eval is a no-op here (results are eager)
    return None
