"""Tracing a user ``log_prob(params)`` into the engine's term program.

The reference differentiates the user's Python ``log_prob`` with ``mx.grad``
(mlx_mcmc/kernels/hmc.py:53-67, nuts.py:76-87).  Here the function is called
ONCE with symbolic parameters; ``Normal`` / ``HalfNormal`` (the distributions
on the hot path, distributions/normal.py:33-56, halfnormal.py:34-63) record a
*term* instead of computing, and ``mx.sum`` / ``+`` / ``mx.array([...])``
combine terms.  The result is a program for ``mc_program_create``: the log
density as ``lp_const + sum_t weight_t * sum_i log_prob_t(value_i; loc_i,
scale_i)``, whose forward value and reverse-mode gradient the HIP kernels
evaluate in one fused sweep per term.

Operands a term accepts (anything else raises ``TraceError``):
  constants (Python / NumPy scalars), data vectors (array-likes), a parameter
  (scalar or vector), a basic slice ``p[a:b]`` or element ``p[i]`` of a vector
  parameter, and an integer gather ``p[idx]`` (hierarchical models, e.g.
  ``Normal(theta[group], sigma).log_prob(y)``).
Per-observation Python loops (examples/01_simple_normal.py:46-48,
tests/test_nuts.py:194-196) trace to many scalar terms with identical
distribution arguments; they are folded into one vector term.

Arithmetic on parameters builds an *affine* location ``a + b * x`` (one
product and one sum, as the reference's MLX ops round them): ``b`` a
constant or scalar parameter, ``x`` a data array, a parameter vector / slice
or an injective gather, ``a`` a constant, scalar parameter, data array,
parameter vector or injective gather — linear regression ``Normal(a + b * x,
sigma)``, non-centred hierarchies ``Normal(mu + tau * z, sigma_j)``.  It is
accepted as a Normal ``loc`` only (mc_affine in include/mcmc355.h).

Reparameterised models: ``mx.exp(p)`` / ``mx.log(p)`` of a parameter (or a
slice / element / gather of one) is a *transformed* parameter operand
(mc_transform_kind), usable wherever a parameter is — ``Normal(mu,
mx.exp(log_sigma))``, ``HalfNormal(1).log_prob(mx.exp(log_tau))``,
``mu + mx.exp(log_tau) * z``, ``Normal(0, 1).log_prob(mx.log(x))``; and a
parameter expression added to a log density (``lp + log_sigma``, the
Jacobian of the transform; ``lp - mx.log(x)``; ``mx.sum(log_x)``) is an
*identity* term ``weight * sum_i value_i`` (MC_DIST_IDENTITY).

Everything else that is elementwise — two predictors ``a + b1 * x1 + b2 *
x2``, ``exp`` of an expression, products and quotients of parameters,
``mx.sqrt`` / ``mx.square`` / ``**`` / ``mx.log1p`` / ``mx.tanh`` /
``mx.sigmoid`` / ``mx.abs``, ``mx.where`` over a data mask, Normal /
HalfNormal / Exponential whose arguments are such expressions, and any such
expression summed into the log density — traces to an *expression* term
(``Expr``, MC_DIST_EXPR): a DAG of f32 elementwise ops evaluated and
differentiated per element by the chain-per-workgroup kernels (eval.h
eval_expr), as mx.grad differentiates the reference's MLX graph.  Gamma and
Beta take such expressions too (their log densities as expression nodes, with
no gradient through gammaln, as the reference's distributions/gamma.py:61-88
and beta.py:59-91).  What raises ``TraceError``, and why:

* a Python branch on a parameter value (``float(theta)``, ``if theta > 0``):
  the model is traced once, so a branch would freeze one side of it;
* ``mx.where`` over a traced condition other than one comparison of traced
  values (x > y, mx.less(x, y) ...: a comparison node, no cotangent);
* indexing a log density (``lp[i]``): per-element log densities are summed
  whole or over an axis;
* a log density times a log density (``lp * lp``), divided into a constant
  (``1 / lp``), or under a per-element weight after an axis reduction;
* reductions other than ``mx.sum`` / ``mx.mean`` of a log density,
  multi-dimensional or strided parameter indexing, and expression terms over
  32 nodes.

Indexing a parameter expression (``(a + b * x)[group]``, ``mx.exp(...)[i]``)
pushes the index to its leaves — parameters become gathers (a gather of a
gather composes), data is indexed on the host, scalars broadcast — so an
indexed affine form stays affine.  A log density under a traced or
per-element weight (``mx.sigmoid(t) * lp``, ``mx.sum(w * lp)``, ``lp /
theta``) becomes expression terms whose roots are the terms' per-element log
densities times (over) the weight, both factors differentiated as mx.grad
differentiates the reference's product.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _lib


class TraceError(TypeError):
    """The log density uses an operation the MI355X tape does not support."""


_UNSUPPORTED = (
    "the MI355X tape supports log densities built from Normal / HalfNormal / "
    "Exponential / Gamma / Beta terms and elementwise mx expressions (summed "
    "with mx.sum / mx.mean, +, -, scalar *) whose arguments are parameters, "
    "parameter slices / integer gathers, data arrays, constants or elementwise "
    "expressions of them")


_COMPARE_OPS = (_lib.MC_EX_GT, _lib.MC_EX_GE, _lib.MC_EX_LT, _lib.MC_EX_LE)


def _comparisons(cls):
    """x < y, x <= y, x > y, x >= y of traced values: a comparison expression
    node (a 1 / 0 mask, no cotangent, as mx.greater / mx.less), usable as the
    condition of mx.where; a Python branch on it (bool()) raises TraceError."""
    ops = {"__lt__": "MC_EX_LT", "__le__": "MC_EX_LE", "__gt__": "MC_EX_GT",
           "__ge__": "MC_EX_GE"}
    for name, op in ops.items():
        def f(self, other, _op=op):
            return Expr.binary(getattr(_lib, _op), self, other)
        f.__name__ = name
        setattr(cls, name, f)
    return cls


# ---------------------------------------------------------------------------
# symbolic values
# ---------------------------------------------------------------------------
@_comparisons
class Param:
    """A parameter (or a view of one) during tracing."""

    __array_priority__ = 1000  # make NumPy defer to our operators

    def __init__(self, name: str, offset: int, shape: Tuple[int, ...], view=None, xf: int = 0):
        self.name = name
        self.offset = offset          # flat offset of the base parameter
        self.base_shape = shape
        # view: None (whole param), ('elem', flat_index), ('slice', start, len),
        # ('gather', int32 index array relative to `offset`)
        self.view = view
        self.xf = xf  # mc_transform_kind: mx.exp / mx.log of the parameter (view)

    def transformed(self, xf: int, fn: str) -> "Param":
        """mx.exp / mx.log of this parameter (view): elementwise, so it commutes
        with the view."""
        if self.xf:
            raise TraceError(f"mx.{fn} of a transformed parameter: one mx.exp / mx.log of a "
                             "parameter traces; " + _UNSUPPORTED)
        return Param(self.name, self.offset, self.base_shape, self.view, xf)

    @property
    def shape(self) -> Tuple[int, ...]:
        v = self.view
        if v is None:
            return self.base_shape
        if v[0] == "elem":
            return ()
        if v[0] == "slice":
            return (v[2],)
        return tuple(v[2])

    @property
    def size(self) -> int:
        return int(np.prod(self.shape)) if self.shape else 1

    @property
    def ndim(self) -> int:
        return len(self.shape)

    def __len__(self):
        if not self.shape:
            raise TypeError("len() of a scalar parameter")
        return self.shape[0]

    def __getitem__(self, idx):
        if self.view is not None and self.view[0] == "elem":
            raise TraceError(f"indexing a scalar view of parameter '{self.name}'")
        if self.view is not None and self.view[0] == "gather":
            # a gather of a gather: the composed index (NumPy indexing of the
            # view's index array), as MLX indexes the gathered array
            sub = np.asarray(self.view[1], np.int64).reshape(self.view[2])[idx]
            if np.ndim(sub) == 0:
                return Param(self.name, self.offset, self.base_shape, ("elem", int(sub)), self.xf)
            sub = np.asarray(sub)
            return Param(self.name, self.offset, self.base_shape,
                         ("gather", sub.astype(np.int32).ravel(), sub.shape), self.xf)
        base = 0
        length = self.size
        if self.view is not None:
            base, length = self.view[1], self.view[2]
        if len(self.base_shape) > 1 and self.view is None:
            raise TraceError("indexing multi-dimensional parameters is not supported")
        if isinstance(idx, (int, np.integer)):
            i = int(idx)
            if i < 0:
                i += length
            if not 0 <= i < length:
                raise IndexError(f"index {idx} out of range for parameter '{self.name}'")
            return Param(self.name, self.offset, self.base_shape, ("elem", base + i), self.xf)
        if isinstance(idx, slice):
            start, stop, step = idx.indices(length)
            if step != 1:
                raise TraceError("strided parameter slices are not supported")
            return Param(self.name, self.offset, self.base_shape,
                         ("slice", base + start, max(0, stop - start)), self.xf)
        arr = np.asarray(idx)
        if arr.dtype.kind not in "iu":
            raise TraceError("parameters can only be gathered by an integer index array")
        arr = arr.astype(np.int64)
        arr = np.where(arr < 0, arr + length, arr)
        if arr.size and (arr.min() < 0 or arr.max() >= length):
            raise IndexError(f"gather index out of range for parameter '{self.name}'")
        return Param(self.name, self.offset, self.base_shape,
                     ("gather", (base + arr).astype(np.int32).ravel(), arr.shape), self.xf)

    def _unsupported(self, *a, **k):
        raise TraceError(f"arithmetic on traced parameter '{self.name}': " + _UNSUPPORTED)

    # affine arithmetic (a + b * x, the fast fused paths): see Affine; any
    # other elementwise arithmetic builds an expression (Expr)
    def __mul__(self, other):
        if isinstance(other, LogProbExpr):  # theta * lp: a traced weight
            return other * self
        if isinstance(other, Expr):
            return Expr.binary(_lib.MC_EX_MUL, self, other)
        return _affine_or_expr(lambda: Affine.product(self, other), _lib.MC_EX_MUL, self, other)

    def __rmul__(self, other):
        if isinstance(other, LogProbExpr):
            return other * self
        if isinstance(other, Expr):
            return Expr.binary(_lib.MC_EX_MUL, other, self)
        return _affine_or_expr(lambda: Affine.product(other, self), _lib.MC_EX_MUL, other, self)

    def __add__(self, other):
        if isinstance(other, LogProbExpr):
            return other + self
        if isinstance(other, Expr):
            return Expr.binary(_lib.MC_EX_ADD, self, other)
        return _affine_or_expr(lambda: Affine.lift(self) + other, _lib.MC_EX_ADD, self, other)

    def __radd__(self, other):
        if isinstance(other, LogProbExpr):
            return other + self
        if isinstance(other, Expr):
            return Expr.binary(_lib.MC_EX_ADD, other, self)
        return _affine_or_expr(lambda: Affine.lift(self) + other, _lib.MC_EX_ADD, other, self)

    def __sub__(self, other):
        if isinstance(other, LogProbExpr):
            return (-other) + self
        if isinstance(other, Expr):
            return Expr.binary(_lib.MC_EX_SUB, self, other)
        return _affine_or_expr(
            lambda: (Affine.lift(self) + (-1.0) * other if not isinstance(other, Affine) else
                     Affine.lift(self) + other * -1.0), _lib.MC_EX_SUB, self, other)

    def __rsub__(self, other):
        if isinstance(other, Expr):
            return Expr.binary(_lib.MC_EX_SUB, other, self)
        return _affine_or_expr(lambda: Affine.product(-1.0, self) + other, _lib.MC_EX_SUB,
                               other, self)

    def __neg__(self):
        return Affine.product(-1.0, self)

    def __truediv__(self, other):
        return Expr.binary(_lib.MC_EX_DIV, self, other)

    def __rtruediv__(self, other):
        return Expr.binary(_lib.MC_EX_DIV, other, self)

    def __pow__(self, other):
        return Expr.binary(_lib.MC_EX_POW, self, other)

    def __rpow__(self, other):
        return Expr.binary(_lib.MC_EX_POW, other, self)

    def __abs__(self):
        return Expr.unary(_lib.MC_EX_ABS, self)

    def __float__(self):
        raise TraceError(f"float() of traced parameter '{self.name}' (a Python branch on a "
                         "parameter value cannot be traced): " + _UNSUPPORTED)

    __bool__ = __int__ = __float__

    def __repr__(self):
        xf = {1: "exp ", 2: "log "}.get(self.xf, "")
        return f"Param({xf}{self.name}, view={self.view})"


def _is_slope(x) -> bool:
    """A constant or a scalar parameter (an affine slope)."""
    if isinstance(x, Param):
        return x.shape == ()
    if isinstance(x, (Affine, LogProbExpr, Expr)):
        return False
    try:
        return np.asarray(_to_numpy(x)).size == 1 and np.asarray(_to_numpy(x)).ndim == 0
    except Exception:
        return False


def _is_term_operand(x) -> bool:
    """Something to_operand accepts (a parameter or view, data, a constant)."""
    return not isinstance(x, (Affine, LogProbExpr, Expr))


@_comparisons
class Affine:
    """A traced affine location ``loc + slope * x`` (mc_affine): one product
    and one sum per element, rounded in f32 as the reference's MLX ops."""

    __array_priority__ = 1000

    def __init__(self, loc, slope, x):
        self.loc = loc      # None (0), a constant, data, or a parameter (view)
        self.slope = slope  # None (no product), a constant or a scalar parameter
        self.x = x          # None, data, or a parameter vector / view

    @staticmethod
    def lift(v) -> "Affine":
        return v if isinstance(v, Affine) else Affine(v, None, None)

    @staticmethod
    def product(a, b) -> "Affine":
        if isinstance(a, Affine) or isinstance(b, Affine):
            raise TraceError("a product of an affine expression: only loc + slope * x traces; "
                             + _UNSUPPORTED)
        if _is_slope(a) and not (_is_slope(b) and not isinstance(b, Param)):
            slope, x = a, b
        elif _is_slope(b):
            slope, x = b, a
        else:
            raise TraceError("a product of two vectors: only loc + slope * x (slope a constant "
                             "or scalar parameter) traces; " + _UNSUPPORTED)
        if isinstance(x, Param) and x.shape == () and isinstance(slope, Param):
            raise TraceError("a product of two scalar parameters: " + _UNSUPPORTED)
        if not isinstance(x, Param) and not isinstance(slope, Param):
            raise TraceError("a constant product outside a parameter expression")
        return Affine(None, slope, x)

    def __add__(self, other):
        if isinstance(other, LogProbExpr):
            return other + self
        if isinstance(other, Expr):
            return Expr.binary(_lib.MC_EX_ADD, self, other)
        return _affine_or_expr(lambda: self._add(other), _lib.MC_EX_ADD, self, other)

    def __radd__(self, other):
        if isinstance(other, LogProbExpr):
            return other + self
        if isinstance(other, Expr):
            return Expr.binary(_lib.MC_EX_ADD, other, self)
        return _affine_or_expr(lambda: self._add(other), _lib.MC_EX_ADD, other, self)

    def _add(self, other):
        o = Affine.lift(other)
        if self.x is not None and o.x is not None:
            raise TraceError("a sum of two products (a + b*x + c*z): only loc + slope * x "
                             "traces; " + _UNSUPPORTED)
        if self.loc is not None and o.loc is not None:
            if isinstance(self.loc, Param) or isinstance(o.loc, Param):
                # a + z with both symbolic: z as x with slope 1
                if self.x is None and o.x is None:
                    a, b = self.loc, o.loc
                    if _is_slope(b) and not _is_slope(a):  # the vector is x (slope 1)
                        a, b = b, a
                    if _is_slope(b):
                        if isinstance(a, Param) and isinstance(b, Param):
                            raise TraceError("a sum of two scalar parameters as a loc: "
                                             + _UNSUPPORTED)
                        raise TraceError("a scalar parameter plus a constant is not traced as "
                                         "a loc: " + _UNSUPPORTED)
                    return Affine(a, 1.0, b)  # (a + 1 * b rounds as a + b)
                raise TraceError("a sum of two parameter terms besides the product: "
                                 + _UNSUPPORTED)
            loc = np.float32(np.asarray(self.loc, np.float32) + np.asarray(o.loc, np.float32))
        else:
            loc = self.loc if self.loc is not None else o.loc
        prod = self if self.x is not None else o
        return Affine(loc, prod.slope, prod.x)

    def __sub__(self, other):
        if isinstance(other, LogProbExpr):
            return (-other) + self
        if isinstance(other, (Affine, Expr)):
            return Expr.binary(_lib.MC_EX_SUB, self, other)
        if isinstance(other, Param):
            return _affine_or_expr(lambda: self._add(Affine.product(-1.0, other)),
                                   _lib.MC_EX_SUB, self, other)
        return _affine_or_expr(lambda: self._add(-np.asarray(_to_numpy(other), np.float32)),
                               _lib.MC_EX_SUB, self, other)

    def __rsub__(self, other):
        return Expr.binary(_lib.MC_EX_SUB, other, self)

    def __mul__(self, other):
        if isinstance(other, LogProbExpr):
            return other * self
        return Expr.binary(_lib.MC_EX_MUL, self, other)

    def __rmul__(self, other):
        if isinstance(other, LogProbExpr):
            return other * self
        return Expr.binary(_lib.MC_EX_MUL, other, self)

    def __truediv__(self, other):
        return Expr.binary(_lib.MC_EX_DIV, self, other)

    def __rtruediv__(self, other):
        return Expr.binary(_lib.MC_EX_DIV, other, self)

    def __pow__(self, other):
        return Expr.binary(_lib.MC_EX_POW, self, other)

    def __rpow__(self, other):
        return Expr.binary(_lib.MC_EX_POW, other, self)

    def __neg__(self):
        return Expr.unary(_lib.MC_EX_NEG, self)

    def __abs__(self):
        return Expr.unary(_lib.MC_EX_ABS, self)

    def __getitem__(self, item):
        """(loc + slope * x)[i] = loc[i] + slope * x[i]: the index pushed to
        the vector operands (an elementwise expression commutes with a
        gather), so the result is the same affine form, rounded per element as
        the reference's indexed MLX array.  A gather that repeats parameters
        anywhere but in the loc over a data x (the fused affine terms' rule,
        api.hip) makes it an expression instead."""
        loc, x = _index_operand(self.loc, item), _index_operand(self.x, item)
        x_data = x is None or not isinstance(x, Param)
        if _repeats(x) or (_repeats(loc) and not x_data):
            e = Expr.of(self)
            return _index_expr(e, item, np.empty(e.shape, np.int8)[item].shape)
        return Affine(loc, self.slope, x)

    def __float__(self):
        raise TraceError("float() of a traced parameter expression: " + _UNSUPPORTED)

    __bool__ = __int__ = __float__

    def operands(self):
        """(loc, slope, x) operands for mc_term / mc_affine."""
        loc = to_operand(self.loc if self.loc is not None else 0.0)
        if self.x is None:
            return loc, None, None
        return loc, to_operand(self.slope), to_operand(self.x)

    def __repr__(self):
        return f"Affine({self.loc!r} + {self.slope!r} * {self.x!r})"


def _affine_or_expr(build, op, a, b):
    """The affine form when it exists (the fused fast paths), else an Expr."""
    try:
        return build()
    except TraceError:
        return Expr.binary(op, a, b)


def _bshape(name: str, shapes) -> Tuple[int, ...]:
    """Elementwise broadcast: scalars and one common shape."""
    vec = [tuple(s) for s in shapes if tuple(s) != ()]
    for s in vec[1:]:
        if s != vec[0]:
            raise TraceError(f"{name}: cannot broadcast shapes {vec} (operands must be scalars "
                             "or share one shape)")
    return vec[0] if vec else ()


@_comparisons
class Expr:
    """A traced elementwise expression (MC_DIST_EXPR nodes, include/mcmc355.h
    mc_expr_node): op an MC_EX_* code, args its argument Exprs; a leaf holds
    a parameter (view, untransformed), a data array or a constant."""

    __array_priority__ = 1000

    def __init__(self, op: int, args=(), leaf=None, shape: Tuple[int, ...] = ()):
        self.op = op
        self.args = tuple(args)
        self.leaf = leaf
        self.shape = tuple(shape)

    # -- construction --------------------------------------------------------
    @staticmethod
    def of(x) -> "Expr":
        if isinstance(x, Expr):
            return x
        if isinstance(x, LogProbExpr):
            raise TraceError("a log density inside a parameter expression or as a distribution "
                             "argument (only + / - / scalar * / mx.sum / mx.mean combine log "
                             "densities, and mx.sum / mx.mean of a parameter expression is read "
                             "as a log density): " + _UNSUPPORTED)
        if isinstance(x, Param):
            if x.xf:
                raw = Param(x.name, x.offset, x.base_shape, x.view, 0)
                op = _lib.MC_EX_EXP if x.xf == _lib.MC_XF_EXP else _lib.MC_EX_LOG
                return Expr(op, [Expr.of(raw)], shape=raw.shape)
            return Expr(_lib.MC_EX_LEAF, leaf=x, shape=x.shape)
        if isinstance(x, Affine):
            if x.x is None:
                return Expr.of(x.loc if x.loc is not None else 0.0)
            prod = Expr.binary(_lib.MC_EX_MUL, x.slope, x.x)
            return prod if x.loc is None else Expr.binary(_lib.MC_EX_ADD, x.loc, prod)
        arr = np.asarray(_to_numpy(x))
        if arr.dtype == object:
            raise TraceError("unsupported value in a parameter expression: " + _UNSUPPORTED)
        arr = arr.astype(np.float32)
        if arr.ndim == 0:
            return Expr(_lib.MC_EX_LEAF, leaf=float(arr), shape=())
        return Expr(_lib.MC_EX_LEAF, leaf=np.ascontiguousarray(arr), shape=arr.shape)

    @staticmethod
    def unary(op: int, a) -> "Expr":
        ea = Expr.of(a)
        return Expr(op, [ea], shape=ea.shape)

    @staticmethod
    def binary(op: int, a, b) -> "Expr":
        ea, eb = Expr.of(a), Expr.of(b)
        return Expr(op, [ea, eb], shape=_bshape("expression", [ea.shape, eb.shape]))

    @staticmethod
    def where(mask, a, b) -> "Expr":
        if is_symbolic(mask):
            # a traced condition: a comparison of traced values (no cotangent
            # through it, as mx.where's VJP)
            if not (isinstance(mask, Expr) and mask.op in _COMPARE_OPS):
                raise TraceError("mx.where over a traced condition other than one comparison "
                                 "(x > y, x < y, x >= y, x <= y of traced values): "
                                 + _UNSUPPORTED)
            em = mask
        else:
            m = np.asarray(_to_numpy(mask))
            if m.dtype == object:
                raise TraceError("mx.where over an unsupported condition: " + _UNSUPPORTED)
            em = Expr.of(m.astype(np.float32))
        ea, eb = Expr.of(a), Expr.of(b)
        e = Expr(_lib.MC_EX_WHERE, [em, ea, eb],
                 shape=_bshape("mx.where", [em.shape, ea.shape, eb.shape]))
        return e

    # -- arithmetic ------------------------------------------------------------
    def __add__(self, other):
        if isinstance(other, LogProbExpr):
            return other + self
        return Expr.binary(_lib.MC_EX_ADD, self, other)

    def __radd__(self, other):
        if isinstance(other, LogProbExpr):
            return other + self
        return Expr.binary(_lib.MC_EX_ADD, other, self)

    def __sub__(self, other):
        if isinstance(other, LogProbExpr):
            return (-other) + self
        return Expr.binary(_lib.MC_EX_SUB, self, other)

    def __rsub__(self, other):
        return Expr.binary(_lib.MC_EX_SUB, other, self)

    def __mul__(self, other):
        if isinstance(other, LogProbExpr):
            return other * self
        return Expr.binary(_lib.MC_EX_MUL, self, other)

    def __rmul__(self, other):
        if isinstance(other, LogProbExpr):
            return other * self
        return Expr.binary(_lib.MC_EX_MUL, other, self)

    def __truediv__(self, other):
        return Expr.binary(_lib.MC_EX_DIV, self, other)

    def __rtruediv__(self, other):
        return Expr.binary(_lib.MC_EX_DIV, other, self)

    def __pow__(self, other):
        return Expr.binary(_lib.MC_EX_POW, self, other)

    def __rpow__(self, other):
        return Expr.binary(_lib.MC_EX_POW, other, self)

    def __neg__(self):
        return Expr.unary(_lib.MC_EX_NEG, self)

    def __abs__(self):
        return Expr.unary(_lib.MC_EX_ABS, self)

    def __getitem__(self, item):
        """expr[i]: the index pushed down to the leaves (every node is
        elementwise, so indexing commutes with it): parameter leaves become
        gathers / element views, data leaves are indexed on the host, scalar
        operands broadcast unchanged.  The same per-element arithmetic as the
        reference's indexed MLX array."""
        if self.shape == ():
            raise TraceError("indexing a scalar traced expression")
        shape = np.empty(self.shape, np.int8)[item].shape  # (IndexError as NumPy's)
        return _index_expr(self, item, shape)

    def __float__(self):
        raise TraceError("float() of a traced expression (a Python branch on a parameter value "
                         "cannot be traced): " + _UNSUPPORTED)

    __bool__ = __int__ = __float__

    @property
    def size(self) -> int:
        return int(np.prod(self.shape)) if self.shape else 1

    def __repr__(self):
        if self.op == _lib.MC_EX_LEAF:
            return f"Expr(leaf {self.leaf!r})"
        return f"Expr(op {self.op}, {len(self.args)} args, shape={self.shape})"


def _index_operand(v, item):
    """An affine operand indexed: vectors (a parameter or data) take the index,
    scalars broadcast unchanged."""
    if v is None:
        return None
    if isinstance(v, Param):
        return v if v.shape == () else v[item]
    arr = np.asarray(_to_numpy(v))
    if arr.ndim == 0:
        return v
    return np.ascontiguousarray(np.asarray(arr, np.float32)[item])


def _repeats(v) -> bool:
    """A parameter gather whose index repeats an element (non-injective)."""
    if not (isinstance(v, Param) and v.view is not None and v.view[0] == "gather"):
        return False
    idx = np.asarray(v.view[1])
    return np.unique(idx).size != idx.size


def _index_expr(e: "Expr", item, shape) -> "Expr":
    """e[item] with the index pushed to e's leaves (Expr.__getitem__)."""
    if e.shape == ():
        return e
    if e.op == _lib.MC_EX_LEAF:
        if isinstance(e.leaf, Param):
            return Expr.of(e.leaf[item])
        if isinstance(e.leaf, np.ndarray):
            return Expr.of(e.leaf[item])
        return e
    args = [None if a is None else _index_expr(a, item, shape) for a in e.args]
    return Expr(e.op, args, shape=shape)


def expr_term(root: Expr) -> "LogProbExpr":
    """An expression summed into a log density: weight * sum_i root_i."""
    n = root.size
    return LogProbExpr([Term(_lib.MC_DIST_EXPR, NONE_OPERAND, NONE_OPERAND, NONE_OPERAND, n,
                             1.0, None, root)], 0.0, root.shape)


_EXPR_DIST = {"Normal": _lib.MC_EX_NORMAL_LP, "HalfNormal": _lib.MC_EX_HALFNORMAL_LP,
              "Exponential": _lib.MC_EX_EXPONENTIAL_LP, "Gamma": _lib.MC_EX_GAMMA_LP,
              "Beta": _lib.MC_EX_BETA_LP}


def dist_expr(dist_name: str, value, loc, scale) -> "LogProbExpr":
    """Distribution.log_prob over expression arguments (MC_EX_*_LP node;
    Gamma / Beta: loc and scale are the shapes alpha, beta)."""
    op = _EXPR_DIST.get(dist_name)
    if op is None:
        raise TraceError(f"{dist_name} with parameter-expression arguments (Normal, HalfNormal, "
                         "Exponential, Gamma and Beta take them): " + _UNSUPPORTED)
    ev, es = Expr.of(value), Expr.of(scale)
    if op in (_lib.MC_EX_NORMAL_LP, _lib.MC_EX_GAMMA_LP, _lib.MC_EX_BETA_LP):
        el = Expr.of(loc)
        root = Expr(op, [ev, el, es], shape=_bshape(dist_name, [ev.shape, el.shape, es.shape]))
    else:
        root = Expr(op, [ev, None, es], shape=_bshape(dist_name, [ev.shape, es.shape]))
    return expr_term(root)


@dataclass
class Operand:
    kind: int
    param_offset: int = 0
    value: float = 0.0
    data: Optional[np.ndarray] = None    # float32, DATA
    index: Optional[np.ndarray] = None   # int32,   GATHER
    shape: Tuple[int, ...] = ()
    transform: int = 0                   # mc_transform_kind (parameter operands)

    def key(self):
        if self.kind == _lib.MC_OP_CONST:
            return ("c", float(np.float32(self.value)))
        if self.kind == _lib.MC_OP_PSCALAR:
            return ("p", self.param_offset, self.transform)
        if self.kind == _lib.MC_OP_PVEC:
            return ("v", self.param_offset, self.shape, self.transform)
        if self.kind == _lib.MC_OP_DATA:
            return ("d", id(self.data))
        if self.kind == _lib.MC_OP_GATHER:
            return ("g", self.param_offset, id(self.index), self.transform)
        return ("n",)


NONE_OPERAND = Operand(_lib.MC_OP_NONE)


def to_operand(x) -> Operand:
    """Classify a distribution argument."""
    if isinstance(x, Param):
        v = x.view
        xf = x.xf
        if v is None:
            if x.base_shape == ():
                return Operand(_lib.MC_OP_PSCALAR, param_offset=x.offset, transform=xf)
            return Operand(_lib.MC_OP_PVEC, param_offset=x.offset, shape=x.base_shape,
                           transform=xf)
        if v[0] == "elem":
            return Operand(_lib.MC_OP_PSCALAR, param_offset=x.offset + v[1], transform=xf)
        if v[0] == "slice":
            return Operand(_lib.MC_OP_PVEC, param_offset=x.offset + v[1], shape=(v[2],),
                           transform=xf)
        return Operand(_lib.MC_OP_GATHER, param_offset=x.offset, index=v[1], shape=tuple(v[2]),
                       transform=xf)
    if isinstance(x, LogProbExpr):
        raise TraceError("a log density cannot be a distribution argument: " + _UNSUPPORTED)
    if isinstance(x, (Affine, Expr)):
        raise TraceError("a parameter expression is not a fused-term operand: " + _UNSUPPORTED)
    try:
        import torch

        if isinstance(x, torch.Tensor):
            x = x.detach().cpu().numpy()
    except ImportError:  # pragma: no cover
        pass
    arr = np.asarray(x)
    if arr.dtype == object:
        raise TraceError("unsupported distribution argument: " + _UNSUPPORTED)
    arr = arr.astype(np.float32)
    if arr.ndim == 0:
        return Operand(_lib.MC_OP_CONST, value=float(arr))
    return Operand(_lib.MC_OP_DATA, data=np.ascontiguousarray(arr).ravel(), shape=arr.shape)


def is_symbolic(*xs) -> bool:
    return any(isinstance(x, (Param, LogProbExpr, Affine, Expr)) for x in xs)


@dataclass
class Term:
    dist: int
    value: Operand
    loc: Operand
    scale: Operand
    n: int
    weight: float = 1.0
    aff: Optional[Tuple[Operand, Operand]] = None  # affine loc: (slope, x)
    expr: Optional["Expr"] = None                   # MC_DIST_EXPR: the root node
    # the traced arguments the term was made from — (dist name, value, loc,
    # scale) or ("identity", value) — so a traced or per-element weight can
    # rebuild it as an expression (LogProbExpr._weighted)
    src: Optional[tuple] = None


def broadcast_n(dist_name: str, ops: List[Operand]) -> Tuple[int, Tuple[int, ...]]:
    shapes = [o.shape for o in ops if o.kind not in (_lib.MC_OP_NONE,) and o.shape != ()]
    if not shapes:
        return 1, ()
    s0 = shapes[0]
    for s in shapes[1:]:
        if s != s0:
            raise TraceError(f"{dist_name}: cannot broadcast operand shapes {shapes} "
                             "(operands must be scalars or share one shape)")
    return int(np.prod(s0)), s0


class LogProbExpr:
    """A bag of weighted terms plus a constant; shape () once summed."""

    __array_priority__ = 1000

    def __init__(self, terms: List[Term], const: float, shape: Tuple[int, ...]):
        self.terms = terms
        self.const = const
        self.shape = shape

    # -- arithmetic ----------------------------------------------------------
    def _combine(self, other, sign: float):
        if isinstance(other, LogProbExpr):
            if self.shape != other.shape:
                if self.shape == () or other.shape == ():
                    raise TraceError("adding a scalar log density to an unsummed vector one "
                                     "(sum it with mx.sum first)")
                raise TraceError(f"shape mismatch {self.shape} vs {other.shape}")
            terms = list(self.terms) + [_scaled(t, sign) for t in other.terms]
            return LogProbExpr(terms, self.const + sign * other.const, self.shape)
        if isinstance(other, (Param, Affine)):
            try:
                ident = identity_expr(other)
            except TraceError:
                ident = expr_term(Expr.of(other))
            return self._combine(ident, sign)
        if isinstance(other, Expr):
            return self._combine(expr_term(other), sign)
        c = _scalar_const(other)
        if self.shape != ():
            raise TraceError("adding a constant to an unsummed vector log density")
        return LogProbExpr(list(self.terms), self.const + sign * c, ())

    def __add__(self, other):
        return self._combine(other, 1.0)

    def __radd__(self, other):
        return self._combine(other, 1.0)

    def __sub__(self, other):
        return self._combine(other, -1.0)

    def __rsub__(self, other):
        return (-self)._combine(other, 1.0)

    def __neg__(self):
        return self * -1.0

    def __mul__(self, other):
        if isinstance(other, (Param, Affine, Expr)) or _is_vector_const(other):
            return self._weighted(other, _lib.MC_EX_MUL)
        c = _scalar_const(other)
        return LogProbExpr([_scaled(t, c) for t in self.terms], self.const * c, self.shape)

    __rmul__ = __mul__

    def __truediv__(self, other):
        if isinstance(other, (Param, Affine, Expr)) or _is_vector_const(other):
            return self._weighted(other, _lib.MC_EX_DIV)
        c = _scalar_const(other)
        return self * float(np.float32(1.0) / np.float32(c))

    def __rtruediv__(self, other):
        raise TraceError("dividing by a log density: " + _UNSUPPORTED)

    def _weighted(self, w, op: int) -> "LogProbExpr":
        """lp * w or lp / w with w a traced value (a parameter, an affine or
        elementwise expression) or a per-element data array: every term
        becomes an expression term whose root is the term's per-element log
        density times (or over) w — sum_i lp_i * w_i, as the reference's MLX
        graph computes it and mx.grad differentiates it (both factors get a
        cotangent).  w is a scalar or has the log density's shape."""
        W = Expr.of(w)
        if W.shape not in ((), self.shape):
            raise TraceError(f"a log density of shape {self.shape} weighted by shape {W.shape} "
                             "(a weight is a scalar or has the log density's shape)")
        terms = []
        for t in self.terms:
            root = _term_root(t)
            if W.shape != () and root.shape != self.shape:
                raise TraceError("a per-element weight on a log density summed over some axes "
                                 "(weight the unreduced log density): " + _UNSUPPORTED)
            node = Expr(op, [root, W], shape=_bshape("weighted log density", [root.shape, W.shape]))
            terms.append(Term(_lib.MC_DIST_EXPR, NONE_OPERAND, NONE_OPERAND, NONE_OPERAND,
                              node.size, t.weight, None, node))
        if self.const != 0.0:
            terms += expr_term(Expr.binary(op, float(self.const), W)).terms
        return LogProbExpr(terms, 0.0, self.shape)

    def _reduced(self, axis, keepdims):
        """The shape after summing `axis` (None, an int or a tuple; negative
        axes count from the end), and the number of elements summed into each
        entry."""
        nd = len(self.shape)
        if axis is None:
            axes = tuple(range(nd))
        else:
            axes = tuple(axis) if isinstance(axis, (tuple, list)) else (axis,)
            norm = []
            for a in axes:
                a = int(a)
                if not -nd <= a < nd:
                    raise TraceError(f"axis {a} out of range for a log density of shape "
                                     f"{self.shape}")
                norm.append(a % nd)
            if len(set(norm)) != len(norm):
                raise TraceError(f"repeated axis in {axes}")
            axes = tuple(norm)
        shape = tuple((1 if keepdims else None) if i in axes else d
                      for i, d in enumerate(self.shape))
        count = int(np.prod([self.shape[i] for i in axes])) if axes else 1
        return tuple(d for d in shape if d is not None), count

    def sum(self, axis=None, keepdims=False):
        """mx.sum of a log density: over every axis the scalar the sampler
        needs; over some axes a smaller log density whose later use must stay
        linear (sums, + / -, scalar weights) — the terms are unchanged, only
        the shape they are summed into (the total is the same)."""
        shape, _ = self._reduced(axis, keepdims)
        return LogProbExpr(list(self.terms), self.const, shape)

    def mean(self, axis=None, keepdims=False):
        """mx.mean of a log density: its sum over `axis` times the f32
        reciprocal of the element count (MLX's mean, mx.sum(x) * (1 / n))."""
        shape, count = self._reduced(axis, keepdims)
        r = float(np.float32(1.0) / np.float32(count))
        return LogProbExpr(list(self.terms), self.const, shape) * r

    def __getitem__(self, item):
        raise TraceError("indexing a log density (lp[i]: per-element log densities are summed "
                         "whole, or over an axis with mx.sum(lp, axis=k)): " + _UNSUPPORTED)

    def __float__(self):
        raise TraceError("float() of a traced log density: " + _UNSUPPORTED)

    __bool__ = __float__

    def __repr__(self):
        return f"LogProbExpr({len(self.terms)} terms, shape={self.shape})"


def identity_expr(x) -> LogProbExpr:
    """A parameter expression added to a log density (``lp + log_sigma``,
    ``lp - mx.log(x)``): identity terms ``weight * value`` (MC_DIST_IDENTITY),
    unsummed — ``mx.sum`` reduces it like any log density.  Accepted: a
    parameter or view, transformed or not, times a constant, plus a constant."""
    const = 0.0
    weight = 1.0
    if isinstance(x, Affine):
        if x.x is None:
            raise TraceError("adding a parameter loc expression to a log density: "
                             + _UNSUPPORTED)
        if isinstance(x.slope, Param):
            raise TraceError("adding a product of parameters to a log density: " + _UNSUPPORTED)
        if x.loc is not None:
            loc = np.asarray(_to_numpy(x.loc))
            if isinstance(x.loc, Param) or loc.dtype == object or loc.size != 1:
                raise TraceError("adding a sum of a parameter and a vector to a log density: "
                                 + _UNSUPPORTED)
            const = float(loc.reshape(()))
        weight = float(np.asarray(_to_numpy(x.slope)).reshape(()))
        x = x.x
    if not isinstance(x, Param):
        raise TraceError("adding this expression to a log density: " + _UNSUPPORTED)
    op = to_operand(x)
    n, shape = broadcast_n("identity", [op])
    if op.kind == _lib.MC_OP_GATHER and op.shape == ():
        op.shape = (1,)
    if const and shape != ():
        raise TraceError("adding a parameter vector plus a constant to a log density: "
                         + _UNSUPPORTED)
    term = Term(_lib.MC_DIST_IDENTITY, op, NONE_OPERAND, NONE_OPERAND, n, weight,
                src=("identity", x))
    return LogProbExpr([term], const, shape)


def _scaled(t: Term, c: float) -> Term:
    return Term(t.dist, t.value, t.loc, t.scale, t.n, t.weight * c, t.aff, t.expr, t.src)


def _term_root(t: Term) -> "Expr":
    """A term's per-element log density as an expression (its weight apart)."""
    if t.dist == _lib.MC_DIST_EXPR:
        return t.expr
    if t.src is None:
        raise TraceError("this log density cannot take a traced or per-element weight: "
                         + _UNSUPPORTED)
    if t.src[0] == "identity":
        return Expr.of(t.src[1])
    name, value, loc, scale = t.src
    if name not in _EXPR_DIST:
        raise TraceError(f"{name} under a traced or per-element weight: " + _UNSUPPORTED)
    return dist_expr(name, value, loc, scale).terms[0].expr


def _is_vector_const(x) -> bool:
    """A non-scalar numeric constant (data), i.e. a per-element weight."""
    if is_symbolic(x):
        return False
    try:
        arr = np.asarray(_to_numpy(x))
    except Exception:
        return False
    return arr.dtype != object and arr.size != 1


def _scalar_const(x) -> float:
    if isinstance(x, (Param, LogProbExpr, Affine, Expr)):
        raise TraceError("a log density times a traced value (lp * theta, lp * lp: log "
                         "densities combine linearly, with constant weights): " + _UNSUPPORTED)
    arr = np.asarray(x)
    if arr.dtype == object or arr.size != 1:
        raise TraceError("a log density times a non-scalar constant (per-element weights: "
                         "only scalar constants combine with a log density)")
    return float(arr.reshape(()))


def make_term(dist: int, dist_name: str, value, loc, scale) -> LogProbExpr:
    if any(isinstance(x, Expr) for x in (value, loc, scale)):
        return dist_expr(dist_name, value, loc, scale)
    try:
        return _make_fused_term(dist, dist_name, value, loc, scale)
    except TraceError:
        # arguments the fused terms do not take (an affine value or scale, a
        # transformed parameter times a parameter ...): an expression term
        if dist_name not in _EXPR_DIST or not any(
                isinstance(x, (Param, Affine)) for x in (value, loc, scale)):
            raise
        return dist_expr(dist_name, value, loc, scale)


def _make_fused_term(dist: int, dist_name: str, value, loc, scale) -> LogProbExpr:
    aff = None
    if isinstance(loc, Param) and dist_name == "Normal":
        loc_op = to_operand(loc)
    elif isinstance(loc, Affine):
        if dist_name != "Normal":
            raise TraceError(f"{dist_name}: a parameter expression as a shape operand: "
                             + _UNSUPPORTED)
        loc_op, slope_op, x_op = loc.operands()
        if x_op is not None:
            if x_op.kind == _lib.MC_OP_PSCALAR:
                raise TraceError("a constant times a scalar parameter as a Normal loc: "
                                 + _UNSUPPORTED)
            aff = (slope_op, x_op)
    else:
        loc_op = NONE_OPERAND if loc is None else to_operand(loc)
    ops = [to_operand(value), loc_op, to_operand(scale)]
    n, shape = broadcast_n(dist_name, ops + ([aff[1]] if aff else []))
    for o in ops + (list(aff) if aff else []):
        if o.kind in (_lib.MC_OP_DATA, _lib.MC_OP_GATHER) and o.shape == ():
            o.shape = (1,)
    return LogProbExpr([Term(dist, ops[0], ops[1], ops[2], n, 1.0, aff,
                             src=(dist_name, value, loc, scale))], 0.0, shape)


def stack(items) -> LogProbExpr:
    """mx.array([lp_1, ..., lp_k]) over traced scalar log densities."""
    terms: List[Term] = []
    const = 0.0
    for it in items:
        if isinstance(it, LogProbExpr):
            if it.shape != ():
                raise TraceError("mx.array of vector log densities is not supported")
            terms += it.terms
            const += it.const
        else:
            const += _scalar_const(it)
    return LogProbExpr(terms, const, (len(items),))


# ---------------------------------------------------------------------------
# folding + program building
# ---------------------------------------------------------------------------
def fold_terms(terms: List[Term]) -> List[Term]:
    """Merge terms that differ only in a constant/data `value`.

    ``for y in data: lp += Normal(mu, sigma).log_prob(y)`` yields one scalar
    term per observation; folding gives the single vector term the reference
    would have written as ``mx.sum(Normal(mu, sigma).log_prob(data))``.
    """
    out: List[Term] = []
    groups: Dict[tuple, int] = {}
    for t in terms:
        foldable = (t.aff is None and t.value.kind in (_lib.MC_OP_CONST, _lib.MC_OP_DATA)
                    and t.loc.kind in (_lib.MC_OP_CONST, _lib.MC_OP_PSCALAR, _lib.MC_OP_NONE)
                    and t.scale.kind in (_lib.MC_OP_CONST, _lib.MC_OP_PSCALAR))
        if not foldable:
            out.append(t)
            continue
        key = (t.dist, float(np.float32(t.weight)), t.loc.key(), t.scale.key())
        vals = (np.array([t.value.value], np.float32) if t.value.kind == _lib.MC_OP_CONST
                else t.value.data)
        if key in groups:
            g = out[groups[key]]
            g.value.data = np.concatenate([g.value.data, vals])
            g.value.shape = (g.value.data.size,)
            g.n = g.value.data.size
        else:
            groups[key] = len(out)
            out.append(Term(t.dist, Operand(_lib.MC_OP_DATA, data=vals.copy(),
                                            shape=(vals.size,)),
                            t.loc, t.scale, int(vals.size), t.weight))
    return out


@dataclass
class ParamLayout:
    names: List[str]
    shapes: List[Tuple[int, ...]]
    offsets: List[int]
    size: int

    def flatten(self, params: dict) -> np.ndarray:
        out = np.empty(self.size, np.float32)
        for name, shp, off in zip(self.names, self.shapes, self.offsets):
            v = np.asarray(_to_numpy(params[name]), np.float32)
            if v.shape != shp:
                raise ValueError(f"parameter '{name}' has shape {v.shape}, expected {shp}")
            n = int(np.prod(shp)) if shp else 1
            out[off:off + n] = v.ravel()
        return out

    def unflatten(self, flat: np.ndarray) -> Dict[str, np.ndarray]:
        """flat: [..., D] -> {name: [..., *shape]}"""
        lead = flat.shape[:-1]
        out = {}
        for name, shp, off in zip(self.names, self.shapes, self.offsets):
            n = int(np.prod(shp)) if shp else 1
            out[name] = flat[..., off:off + n].reshape(lead + shp)
        return out


def _to_numpy(x):
    try:
        import torch

        if isinstance(x, torch.Tensor):
            return x.detach().cpu().numpy()
    except ImportError:  # pragma: no cover
        pass
    return x


def layout_of(initial_params: dict) -> ParamLayout:
    names, shapes, offsets = [], [], []
    off = 0
    for name, v in initial_params.items():
        arr = np.asarray(_to_numpy(v), np.float32)
        names.append(name)
        shapes.append(tuple(arr.shape))
        offsets.append(off)
        off += int(arr.size)
    if off == 0:
        raise ValueError("initial_params is empty")
    return ParamLayout(names, shapes, offsets, off)


@dataclass
class TracedModel:
    layout: ParamLayout
    terms: List[Term]
    lp_const: float
    # pools handed to mc_program_create
    data: np.ndarray = field(default_factory=lambda: np.zeros(0, np.float32))
    index: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    c_terms: object = None
    c_affines: object = None
    n_affines: int = 0
    c_exprs: object = None
    c_nodes: object = None
    n_exprs: int = 0
    n_nodes: int = 0


def trace(log_prob_fn, initial_params: dict) -> TracedModel:
    layout = layout_of(initial_params)
    sym = {name: Param(name, off, shp)
           for name, shp, off in zip(layout.names, layout.shapes, layout.offsets)}
    out = log_prob_fn(sym)
    if isinstance(out, (Param, Affine, Expr)) and tuple(out.shape) == ():
        # a scalar parameter expression returned as the log density itself
        out = expr_term(Expr.of(out))
    if not isinstance(out, LogProbExpr):
        raise TraceError("log_prob did not build its value from Normal / HalfNormal terms: "
                         + _UNSUPPORTED)
    if out.shape != ():
        raise TraceError(f"log_prob must return a scalar (got shape {out.shape}); "
                         "sum the likelihood with mx.sum as the reference does")
    terms = fold_terms(out.terms)
    model = TracedModel(layout, terms, float(np.float32(out.const)))
    _build_pools(model)
    return model


def _build_pools(model: TracedModel) -> None:
    data_parts: List[np.ndarray] = []
    index_parts: List[np.ndarray] = []
    nd = 0
    ni = 0
    arr = (_lib.McTerm * max(1, len(model.terms)))()
    affs = [t for t in model.terms if t.aff is not None]
    aarr = (_lib.McAffine * max(1, len(affs)))()
    na = 0
    exprs: List[Tuple[int, int]] = []
    nodes: List[tuple] = []   # (op, a, b, c, Operand or None)
    for k, t in enumerate(model.terms):
        ct = arr[k]
        ct.dist = t.dist
        ct.n = t.n
        ct.weight = t.weight
        if t.dist == _lib.MC_DIST_EXPR:
            first = len(nodes)
            nodes.extend(_linearize(t.expr, t.n))
            exprs.append((first, len(nodes) - first))
            ct.affine = len(exprs)
            continue
        slots = [(ct, "value", t.value), (ct, "loc", t.loc), (ct, "scale", t.scale)]
        if t.aff is not None:
            ct.affine = na + 1
            slots += [(aarr[na], "slope", t.aff[0]), (aarr[na], "x", t.aff[1])]
            na += 1
        for owner, slot, o in slots:
            co = getattr(owner, slot)
            co.kind = o.kind
            co.param_offset = o.param_offset
            co.value = o.value
            co.transform = o.transform
            if o.kind == _lib.MC_OP_DATA:
                co.pool_offset = nd
                data_parts.append(o.data.astype(np.float32))
                nd += o.data.size
            elif o.kind == _lib.MC_OP_GATHER:
                co.pool_offset = ni
                index_parts.append(o.index.astype(np.int32))
                ni += o.index.size
    carr = (_lib.McExprNode * max(1, len(nodes)))()
    index_ids: Dict[bytes, int] = {}   # one pool copy per gather index
    for k, (op, a, b, c, o) in enumerate(nodes):
        cn = carr[k]
        cn.op, cn.a, cn.b, cn.c = op, a, b, c
        if o is None:
            continue
        co = cn.leaf
        co.kind = o.kind
        co.param_offset = o.param_offset
        co.value = o.value
        co.transform = 0
        if o.kind == _lib.MC_OP_DATA:
            co.pool_offset = nd
            data_parts.append(o.data.astype(np.float32))
            nd += o.data.size
        elif o.kind == _lib.MC_OP_GATHER:
            ik = o.index.tobytes()
            if ik not in index_ids:
                index_ids[ik] = ni
                index_parts.append(o.index.astype(np.int32))
                ni += o.index.size
            co.pool_offset = index_ids[ik]
    xarr = (_lib.McExpr * max(1, len(exprs)))()
    for k, (first, count) in enumerate(exprs):
        xarr[k].first, xarr[k].count = first, count
    model.c_exprs, model.c_nodes = xarr, carr
    model.n_exprs, model.n_nodes = len(exprs), len(nodes)
    model.data = (np.concatenate(data_parts) if data_parts else np.zeros(0, np.float32))
    model.index = (np.concatenate(index_parts) if index_parts else np.zeros(0, np.int32))
    model.c_terms = arr
    model.c_affines = aarr
    model.n_affines = na


def _linearize(root: Expr, n: int) -> List[tuple]:
    """Post-order node list of an expression term (arguments before their
    users, the root last); identical leaves share one node."""
    out: List[tuple] = []
    memo: Dict[int, int] = {}
    leaves: Dict[tuple, int] = {}

    def leaf_operand(e: Expr) -> Operand:
        x = e.leaf
        if isinstance(x, Param):
            op = to_operand(x)
            if op.kind == _lib.MC_OP_GATHER and op.shape == ():
                op.shape = (1,)
            return op
        if isinstance(x, np.ndarray):
            if x.size == 1 and n > 1 and x.shape == ():
                return Operand(_lib.MC_OP_CONST, value=float(x))
            return Operand(_lib.MC_OP_DATA, data=x.ravel(), shape=x.shape)
        return Operand(_lib.MC_OP_CONST, value=float(x))

    def visit(e: Expr) -> int:
        if id(e) in memo:
            return memo[id(e)]
        if e.op == _lib.MC_EX_LEAF:
            o = leaf_operand(e)
            key = (("g", o.param_offset, o.index.tobytes()) if o.kind == _lib.MC_OP_GATHER
                   else o.key())
            if key in leaves:
                memo[id(e)] = leaves[key]
                return leaves[key]
            out.append((e.op, -1, -1, -1, o))
            leaves[key] = memo[id(e)] = len(out) - 1
            return len(out) - 1
        ids = [visit(a) if a is not None else -1 for a in e.args]
        ids += [-1] * (3 - len(ids))
        out.append((e.op, ids[0], ids[1], ids[2], None))
        memo[id(e)] = len(out) - 1
        return len(out) - 1

    visit(root)
    if len(out) > _lib.MC_EXPR_MAX_NODES:
        raise TraceError(f"an expression term of {len(out)} nodes (at most "
                         f"{_lib.MC_EXPR_MAX_NODES}): split the log density into several sums")
    return out


class Program:
    """An mc_program handle owning its device copy of the model."""

    def __init__(self, model: TracedModel):
        lib = _lib.load()
        self.model = model
        self.layout = model.layout
        self.D = model.layout.size
        h = ctypes.c_void_p()
        data = np.ascontiguousarray(model.data, np.float32)
        index = np.ascontiguousarray(model.index, np.int32)
        _lib.check(lib.mc_program_create_expr(
            model.c_terms, len(model.terms), model.c_affines, model.n_affines, model.c_exprs,
            model.n_exprs, model.c_nodes, model.n_nodes, self.D,
            model.lp_const, data.ctypes.data_as(ctypes.c_void_p), data.size,
            index.ctypes.data_as(ctypes.c_void_p), index.size, ctypes.byref(h)))
        self.handle = h
        self.waves_per_chain = lib.mc_program_waves_per_chain(h)
        self.num_slices = lib.mc_program_num_slices(h)

    def set_slices(self, num_slices: int) -> None:
        """HMC work split (include/mcmc355.h mc_program_set_slices): 0 automatic,
        1 one chain per workgroup, >= 2 that many data slices per chain."""
        lib = _lib.load()
        _lib.check(lib.mc_program_set_slices(self.handle, int(num_slices)))
        self.num_slices = lib.mc_program_num_slices(self.handle)

    SLICE_KERNELS = {"auto": 0, "interpreter": 1, "lanes": 2}

    def set_slice_kernel(self, kernel: str) -> None:
        """Kernel of a sliced HMC program (mc_program_set_slice_kernel):
        "auto" (lane-resident when the layout qualifies), "interpreter"
        (k_hmc_sl, csrc/sliced.h) or "lanes" (k_hmc_lr, csrc/lanes.h; raises
        EngineError when the layout does not qualify).  On an unsliced program
        "lanes" plans one slice (no exchange) and "auto" / "interpreter" keep
        the chain-per-workgroup kernel (k_hmc)."""
        _lib.check(_lib.load().mc_program_set_slice_kernel(self.handle,
                                                           self.SLICE_KERNELS[kernel]))

    @property
    def slice_kernel(self) -> str:
        """"unsliced", "interpreter" or "lanes": what an HMC launch will run."""
        k = _lib.load().mc_program_slice_kernel(self.handle)
        return {0: "unsliced", 1: "interpreter", 2: "lanes"}[k]

    def nuts_kernel(self, max_tree_depth: int = 10) -> str:
        """"lanes" (k_nuts_lr), "sliced" (k_nuts_sl: a sliced fast-form
        program, csrc/nuts_sliced.h) or "tape" (k_nuts): what mc_nuts_run will
        run."""
        k = _lib.load().mc_program_nuts_lanes(self.handle, int(max_tree_depth))
        return {1: "lanes", 2: "lanes", 3: "sliced"}.get(k, "tape")

    def nuts_register_only(self, max_tree_depth: int = 10) -> bool:
        """True when mc_nuts_run runs k_nuts_lr's register-only variant."""
        return _lib.load().mc_program_nuts_lanes(self.handle, int(max_tree_depth)) == 2

    @property
    def kernel_note(self) -> str:
        """Why HMC launches miss the lane-resident kernel ("" when they run it)."""
        return (_lib.load().mc_program_kernel_note(self.handle) or b"").decode()

    @property
    def program_elements(self) -> int:
        """Element count over the traced terms (the slice planner's size measure)."""
        return int(sum(t.n for t in self.model.terms))

    @property
    def lanes_fast(self) -> bool:
        """True when a lane-resident launch runs the fast-form kernel k_hmc_lf."""
        return _lib.load().mc_program_lanes_fast(self.handle) == 1

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                _lib.load().mc_program_destroy(h)
            except Exception:  # pragma: no cover - interpreter shutdown
                pass
            self.handle = None


def _has_data_leaf(e: "Expr") -> bool:
    if e.op == _lib.MC_EX_LEAF:
        return isinstance(e.leaf, np.ndarray)
    return any(a is not None and _has_data_leaf(a) for a in e.args)


def _own_prior_like(t: Term) -> bool:
    """A scalar term the sliced kernels evaluate as a shared parameter's own
    prior (api.hip plan_lanes LrSterm::own): Normal / HalfNormal of an
    untransformed scalar parameter with constant loc and scale."""
    return (t.dist in (_lib.MC_DIST_NORMAL, _lib.MC_DIST_HALFNORMAL) and t.aff is None
            and t.value.kind == _lib.MC_OP_PSCALAR and t.value.transform == 0
            and t.loc.kind in (_lib.MC_OP_CONST, _lib.MC_OP_NONE)
            and t.scale.kind == _lib.MC_OP_CONST)


def affine_as_expressions(model: TracedModel, scalars: bool = False) -> Optional[TracedModel]:
    """The same model with every fused affine-loc term (``Normal(a + b * x,
    s)``, mc_affine) rebuilt as an expression term of the same per-element
    arithmetic (its MC_EX_NORMAL_LP node over ADD(a, MUL(b, x))), the other
    terms unchanged; None when nothing changes.  The sliced NUTS / MH kernels
    take expression terms (LS_EXPR, csrc/nuts_sliced.h, mh_sliced.h) but not
    affine ones, so this form moves NUTS and MH on a large regression off the
    tape.  scalars: also every scalar term those kernels cannot take as a
    shared parameter's own prior (``Exponential(1).log_prob(sigma)``, a
    second prior on one parameter, a prior with a parameter argument) — the
    kernels evaluate scalar terms only as own priors."""
    owned = set()
    convert = []
    for t in model.terms:
        c = t.aff is not None
        if scalars and not c and t.n == 1 and t.dist not in (_lib.MC_DIST_EXPR,
                                                             _lib.MC_DIST_IDENTITY):
            own = _own_prior_like(t) and t.value.param_offset not in owned
            if own:
                owned.add(t.value.param_offset)
            c = not own and t.src is not None and t.src[0] in _EXPR_DIST
        convert.append(c)
    if not any(convert):
        return None
    terms = []
    for t, c in zip(model.terms, convert):
        if not c:
            terms.append(t)
            continue
        root = _term_root(t)
        if not _has_data_leaf(root):
            # the lane planner tiles an expression term by its data arrays
            # (host.h expr_lanes_ok): a scalar prior gets a one-element mask,
            # where(1, lp, lp) — the same value and the same cotangent
            mask = Expr.of(np.ones(max(root.size, 1), np.float32).reshape(root.shape or (1,)))
            root = Expr(_lib.MC_EX_WHERE, [mask, root, root], shape=mask.shape)
        terms.append(Term(_lib.MC_DIST_EXPR, NONE_OPERAND, NONE_OPERAND, NONE_OPERAND,
                          root.size, t.weight, None, root))
    out = TracedModel(model.layout, terms, model.lp_const)
    _build_pools(out)
    return out


def nuts_program(prog: "Program", max_tree_depth: int = 10) -> "Program":
    """The program NUTS runs: `prog`, or — when its affine-loc terms (and,
    failing that, its scalar terms other than own priors) keep NUTS on the
    chain-per-workgroup tape and the same model with those terms as
    expression terms plans onto the sliced kernel — that program.  (HMC keeps
    `prog`: the lane kernel k_hmc_lr runs affine and generic scalar terms.)"""
    if prog.nuts_kernel(max_tree_depth) != "tape":
        return prog
    for scalars in (False, True):
        try:
            alt = affine_as_expressions(prog.model, scalars)
        except TraceError:
            continue
        if alt is None:
            continue
        p2 = Program(alt)
        # (the sliced kernel runs expression terms compiled: with the JIT off
        # they would run interpreted on the tape, slower than the fused terms)
        if p2.nuts_kernel(max_tree_depth) == "sliced" and _lib.load().mc_program_expr_jit(
                p2.handle) == 1:
            return p2
    return prog


def mh_program(prog: "Program") -> "Program":
    """The program random-walk MH runs: `prog`, or its affine-loc (and then
    non-own scalar) terms as expression terms (affine_as_expressions) when
    that moves MH from the tape (k_mh) onto the sliced kernel k_mh_sl
    (value-only LS_EXPR pass)."""
    lib = _lib.load()
    if lib.mc_program_mh_sliced(prog.handle) == 1:
        return prog
    for scalars in (False, True):
        try:
            alt = affine_as_expressions(prog.model, scalars)
        except TraceError:
            continue
        if alt is None:
            continue
        p2 = Program(alt)
        if lib.mc_program_mh_sliced(p2.handle) == 1 and lib.mc_program_expr_jit(p2.handle) == 1:
            return p2
    return prog


def compile_model(log_prob_fn, initial_params: dict, slices: int = 0,
                  slice_kernel: str = "auto") -> Program:
    _lib.require_device()
    prog = Program(trace(log_prob_fn, initial_params))
    if slices:
        prog.set_slices(slices)
    if slice_kernel != "auto":
        prog.set_slice_kernel(slice_kernel)
    return prog
