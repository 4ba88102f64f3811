"""Host logic without a GPU: tracing user models into the term program."""
import re

import numpy as np
import pytest

import mlx_mcmc_amd as m
import mlx_mcmc_amd.core as mx
import workloads as W
from mlx_mcmc_amd import _lib, _trace


def kinds(t):
    return (t.dist, t.value.kind, t.loc.kind, t.scale.kind, t.n)


def test_config1_model_traces_to_three_terms():
    lp, init = W.simple_normal(W.ns_product())
    tm = _trace.trace(lp, init)
    assert tm.layout.names == ["mu", "sigma"] and tm.layout.size == 2
    got = [kinds(t) for t in tm.terms]
    assert got == [
        (_lib.MC_DIST_NORMAL, _lib.MC_OP_PSCALAR, _lib.MC_OP_CONST, _lib.MC_OP_CONST, 1),
        (_lib.MC_DIST_HALFNORMAL, _lib.MC_OP_PSCALAR, _lib.MC_OP_NONE, _lib.MC_OP_CONST, 1),
        (_lib.MC_DIST_NORMAL, _lib.MC_OP_DATA, _lib.MC_OP_PSCALAR, _lib.MC_OP_PSCALAR, 100),
    ]
    np.testing.assert_array_equal(tm.data, W.simple_normal_data().astype(np.float32))


def test_per_observation_loop_is_folded():
    """examples/01_simple_normal.py:46-48 and tests/test_nuts.py:194-196 style."""
    y = W.simple_normal_data()

    def loop_model(p):
        lp = m.Normal(0, 10).log_prob(p["mu"]) + m.HalfNormal(5).log_prob(p["sigma"])
        ll = mx.array(0.0)
        for yi in y:
            ll = ll + m.Normal(p["mu"], p["sigma"]).log_prob(mx.array(yi))
        return lp + ll

    def stacked_model(p):
        lp = m.Normal(0, 10).log_prob(p["mu"]) + m.HalfNormal(5).log_prob(p["sigma"])
        return lp + mx.sum(mx.array([m.Normal(p["mu"], p["sigma"]).log_prob(mx.array(v))
                                     for v in y]))

    for fn in (loop_model, stacked_model):
        tm = _trace.trace(fn, {"mu": 0.0, "sigma": 1.0})
        assert len(tm.terms) == 3
        assert tm.terms[2].n == 100
        np.testing.assert_array_equal(tm.terms[2].value.data, y.astype(np.float32))


def test_hierarchical_gather_operands():
    G, N = W.SHAPES["small"]
    lp, init = W.hierarchical(W.ns_product(), G, N)
    tm = _trace.trace(lp, init)
    assert tm.layout.size == G + 3
    lik = tm.terms[-1]
    assert kinds(lik) == (_lib.MC_DIST_NORMAL, _lib.MC_OP_DATA, _lib.MC_OP_GATHER,
                          _lib.MC_OP_PSCALAR, N)
    _, group = W.hierarchical_data(G, N)
    np.testing.assert_array_equal(lik.loc.index, group)
    assert lik.loc.param_offset == tm.layout.offsets[tm.layout.names.index("theta")]
    prior = tm.terms[-2]
    assert kinds(prior) == (_lib.MC_DIST_NORMAL, _lib.MC_OP_PVEC, _lib.MC_OP_PSCALAR,
                            _lib.MC_OP_PSCALAR, G)


def test_slices_elements_and_weights():
    def model(p):
        x = p["x"]
        lp = m.Normal(x[0], 1.0).log_prob(x[1:4])           # element + slice
        lp = mx.sum(lp) - 0.5 * mx.sum(m.Normal(0, 2).log_prob(x))
        return lp + 3.0
    tm = _trace.trace(model, {"x": np.zeros(5, np.float32)})
    a, b = tm.terms
    assert (a.loc.kind, a.loc.param_offset) == (_lib.MC_OP_PSCALAR, 0)
    assert (a.value.kind, a.value.param_offset, a.n) == (_lib.MC_OP_PVEC, 1, 3)
    assert b.weight == -0.5 and tm.lp_const == 3.0


def test_affine_loc_traces():
    """Linear predictors trace to one Normal term with an affine loc
    (include/mcmc355.h mc_affine): regression a + b * x over data, and the
    non-centred mu + tau * z over a parameter vector."""
    lp, init = W.linear_regression(W.ns_product(), 50)
    tm = _trace.trace(lp, init)
    lik = [t for t in tm.terms if t.aff is not None]
    assert len(lik) == 1 and tm.n_affines == 1
    t = lik[0]
    assert (t.loc.kind, t.loc.param_offset) == (_lib.MC_OP_PSCALAR, 0)        # a
    assert (t.aff[0].kind, t.aff[0].param_offset) == (_lib.MC_OP_PSCALAR, 1)  # b
    assert t.aff[1].kind == _lib.MC_OP_DATA and t.n == 50
    np.testing.assert_array_equal(t.aff[1].data, W.regression_data(50)[0])
    assert tm.c_terms[[k for k, u in enumerate(tm.terms) if u.aff][0]].affine == 1
    lp, init = W.eight_schools_nc(W.ns_product())
    tm = _trace.trace(lp, init)
    (t,) = [t for t in tm.terms if t.aff is not None]
    assert t.loc.kind == _lib.MC_OP_PSCALAR and t.aff[0].kind == _lib.MC_OP_PSCALAR
    assert (t.aff[1].kind, t.aff[1].param_offset, t.n) == (_lib.MC_OP_PVEC, 2, 8)
    assert t.scale.kind == _lib.MC_OP_DATA and t.value.kind == _lib.MC_OP_DATA


def test_affine_varying_intercept_traces():
    """alpha[group] + beta * x: an affine loc whose own operand is a
    non-injective gather (the segmented tape path)."""
    lp, init = W.varying_intercept(W.ns_product())
    tm = _trace.trace(lp, init)
    (t,) = [t for t in tm.terms if t.aff is not None]
    assert t.loc.kind == _lib.MC_OP_GATHER and t.n == 2000
    assert t.aff[0].kind == _lib.MC_OP_PSCALAR and t.aff[1].kind == _lib.MC_OP_DATA


@pytest.mark.parametrize("expr, want", [
    (lambda p: p["a"] + p["b"] * X3, ("p", "p", "d")),
    (lambda p: X3 * p["b"] + p["a"], ("p", "p", "d")),
    (lambda p: p["a"] - X3, ("p", "c", "d")),           # slope -1
    (lambda p: 2.0 * p["v"], ("c", "c", "v")),            # loc 0
    (lambda p: p["v"] + p["a"], ("p", "c", "v")),         # slope 1
    (lambda p: p["b"] * p["v"] + 1.0, ("c", "p", "v")),
])
def test_affine_forms(expr, want):
    def lp(p):
        return mx.sum(m.Normal(expr(p), 1.0).log_prob(np.zeros(3, np.float32)))

    tm = _trace.trace(lp, {"a": 1.0, "b": 2.0, "v": np.zeros(3, np.float32)})
    (t,) = tm.terms
    code = {_lib.MC_OP_PSCALAR: "p", _lib.MC_OP_CONST: "c", _lib.MC_OP_DATA: "d",
            _lib.MC_OP_PVEC: "v"}
    got = (code[t.loc.kind],) + ((code[t.aff[0].kind], code[t.aff[1].kind]) if t.aff else ())
    assert got == want


X3 = np.arange(3, dtype=np.float32)


# Constructs that still raise: each error names its construct
@pytest.mark.parametrize("bad,names", [
    (lambda p: m.Normal(0, 1).log_prob(p["x"]) if p["x"] > 0 else 0,     # Python branch
     "a Python branch on a parameter value"),
    (lambda p: m.Normal(0, 1).log_prob(p["v"]), "must return a scalar"),  # unsummed vector
    (lambda p: m.Normal(0, 1).log_prob(p["x"]) + p["v"],                   # unsummed identity
     "adding a scalar log density to an unsummed vector one"),
    (lambda p: m.Normal(0, 1).log_prob(mx.tanh(p["x"])[0]),                 # indexing a scalar
     "indexing a scalar"),
    (lambda p: mx.sum(mx.where((p["v"] > 0) * 1.0, p["v"], 0.0)),           # arithmetic mask
     "mx.where over a traced condition other than one comparison"),
    (lambda p: m.Normal(0, 1).log_prob(p["x"]) * m.Normal(0, 1).log_prob(p["x"]),  # lp * lp
     "a log density times a traced value"),
    (lambda p: mx.sum(m.Normal(0, 1).log_prob(p["v"]) * np.ones(4, np.float32)),  # bad weight
     "weighted by shape (4,)"),
    (lambda p: mx.sum(mx.sum(m.Normal(p["x"], 1.0).log_prob(np.ones((2, 3), np.float32)),
                             axis=1) * np.ones(2, np.float32)),          # weight after an axis sum
     "a per-element weight on a log density summed over some axes"),
    (lambda p: 1.0 / m.Normal(0, 1).log_prob(p["x"]), "dividing by a log density"),
    (lambda p: mx.sum(m.Normal(p["v"] * X3, 1.0).log_prob(np.zeros(4, np.float32))),
     "cannot broadcast shapes"),
    (lambda p: mx.sum(_deep(p["v"], 40)), "nodes (at most 32)"),           # too deep
    (lambda p: mx.exp(mx.sum(m.Normal(0, 1).log_prob(p["v"]))),            # logsumexp-like
     "a log density inside a parameter expression"),
    (lambda p: mx.sum(m.Normal(0, 1).log_prob(p["v"])[1:]), "indexing a log density"),
    (lambda p: mx.sum(m.Normal(0, 1).log_prob(p["v"]), axis=2), "axis 2 out of range"),
    (lambda p: m.Normal(mx.mean(p["v"]), 1.0).log_prob(p["x"]),            # a reduction as a value
     "as a distribution argument"),
    (lambda p: float(m.Normal(0, 1).log_prob(p["x"])), "float() of a traced log density"),
    (lambda p: mx.std(p["v"]), "mx.std of a traced value"),
])
def test_unsupported_models_raise(bad, names):
    with pytest.raises(_trace.TraceError, match=re.escape(names)):
        _trace.trace(bad, {"x": 1.0, "v": np.zeros(3, np.float32)})


def _deep(x, k):
    for i in range(k):
        x = mx.tanh(x * (1.0 + i))
    return x


# Expressions the fused terms do not cover trace to expression terms
# (MC_DIST_EXPR, eval.h eval_expr) — each of these raised TraceError before
@pytest.mark.parametrize("good", [
    lambda p: m.Normal(0, 1).log_prob(p["x"] * 2.0),          # an expression as a value
    lambda p: mx.sum(m.Normal(p["x"] + p["x"] * X3 + p["x"] * X3, 1.0).log_prob(X3)),  # 2 products
    lambda p: mx.sum(m.Normal(p["x"] * p["x"], 1.0).log_prob(X3)),  # product of parameters
    lambda p: mx.sum(m.Normal(0.0, p["x"] * 2.0).log_prob(X3)),  # an expression as a scale
    lambda p: mx.sum(m.Normal((p["x"] + p["x"] * X3) * 2.0, 1.0).log_prob(X3)),  # scaled affine
    lambda p: mx.log(p["x"]),                                   # a scalar expression as lp
    lambda p: m.Normal(0, 1).log_prob(mx.exp(mx.exp(p["x"]))),  # a transform of a transform
    lambda p: m.Normal(0, 1).log_prob(mx.exp(p["x"] * 2.0)),    # exp of an expression
    lambda p: m.Normal(0, 1).log_prob(p["x"]) + p["x"] * p["x"],  # a product added to lp
    lambda p: mx.sum(m.Normal(2.0 * p["x"], 1.0).log_prob(X3)),  # const * scalar as a loc
    lambda p: mx.sum(m.Normal(p["x"] + 1.0, 1.0).log_prob(X3)),  # scalar + constant as a loc
    lambda p: mx.sum(m.Normal(p["x"] + p["y"], 1.0).log_prob(X3)),  # sum of scalars as a loc
    lambda p: mx.sum(-0.5 * mx.square(p["v"] - X3) / p["x"]),   # a hand-written density
    lambda p: mx.sum(mx.where(X3 > 1, mx.sqrt(mx.abs(p["v"])), mx.tanh(p["v"]))),
    lambda p: mx.sum(mx.log1p(mx.sigmoid(p["v"]) ** 2.0)),
    lambda p: m.HalfNormal(mx.exp(p["x"]) + 1.0).log_prob(p["y"] * p["y"]),
    lambda p: m.Exponential(p["x"] * p["y"]).log_prob(mx.exp(p["y"])),
    lambda p: m.Gamma(p["x"] * 2.0, 1.0).log_prob(p["y"]),      # Gamma over expressions
    lambda p: mx.sum(m.Gamma(mx.exp(p["x"]), p["y"] * X3 + 1.0).log_prob(X3 + 1.0)),
    lambda p: mx.sum(m.Beta(p["y"] * 4.0, (1.0 - p["y"]) * 4.0).log_prob(X3 * 0.2 + 0.1)),
    lambda p: m.Beta(2.0, 3.0).log_prob(mx.sigmoid(p["x"])),     # Beta of an expression
    lambda p: mx.mean(-0.5 * mx.square(p["v"] - X3)),             # mx.mean of an expression
    lambda p: mx.sum(mx.where(p["v"] > 0, p["v"], 0.0)),          # a traced condition
    lambda p: mx.sum(mx.where(mx.abs(p["v"] - X3) < p["x"], mx.square(p["v"]), p["v"])),
    lambda p: mx.sum(mx.where(mx.less_equal(X3, p["v"]), 1.0, -mx.square(p["v"]))),
    # indexing pushed to the leaves: an expression, an affine form, a gather
    # of a gather
    lambda p: mx.sum(m.Normal(0, 1).log_prob((p["v"] * 2.0)[np.array([0, 2, 2])])),
    lambda p: mx.sum(m.Normal(mx.exp(p["x"] * X3)[1:], 1.0).log_prob(X3[:2])),
    lambda p: mx.sum(m.Normal(0, 1).log_prob(mx.tanh(p["v"][np.array([2, 1, 0])])[np.array([0, 0])])),
    # log densities under traced or per-element weights
    lambda p: m.Normal(0, 1).log_prob(p["x"]) * p["x"],
    lambda p: mx.sigmoid(p["y"]) * mx.sum(m.Normal(p["x"], 1.0).log_prob(X3)),
    lambda p: mx.sum(m.Normal(0, 1).log_prob(p["v"]) * X3),
    lambda p: mx.sum(X3 * m.HalfNormal(mx.exp(p["x"])).log_prob(X3 + 1.0)),
    lambda p: (m.Normal(0, 1).log_prob(p["x"]) + 2.0) / (1.0 + p["y"] * p["y"]),
])
def test_general_expressions_trace(good):
    tm = _trace.trace(good, {"x": 1.0, "y": 0.5, "v": np.zeros(3, np.float32)})
    exprs = [t for t in tm.terms if t.dist == _lib.MC_DIST_EXPR]
    assert exprs and tm.n_exprs == len(exprs) and tm.n_nodes >= 2
    for k in range(tm.n_exprs):
        first, count = tm.c_exprs[k].first, tm.c_exprs[k].count
        for i in range(first, first + count):
            nd = tm.c_nodes[i]
            for a in (nd.a, nd.b, nd.c):   # arguments precede their users
                assert a < i - first
            if nd.op == _lib.MC_EX_LEAF:
                assert nd.leaf.transform == 0 and (nd.a, nd.b, nd.c) == (-1, -1, -1)


def test_expression_models_trace_to_expected_terms():
    """The expression workloads keep their fused parts fused (priors, the
    log-Jacobian identity term) and put only the rest in expression terms;
    the varying-slopes likelihood gathers alpha and beta through one index."""
    lp, init = W.two_predictor_regression(W.ns_product())
    tm = _trace.trace(lp, init)
    assert [t.dist for t in tm.terms].count(_lib.MC_DIST_EXPR) == 1
    assert _lib.MC_DIST_IDENTITY in [t.dist for t in tm.terms]
    ops = [tm.c_nodes[i].op for i in range(tm.n_nodes)]
    assert ops[-1] == _lib.MC_EX_NORMAL_LP and _lib.MC_EX_EXP in ops
    lp, init = W.varying_slopes(W.ns_product())
    tm = _trace.trace(lp, init)
    gathers = [tm.c_nodes[i].leaf for i in range(tm.n_nodes)
               if tm.c_nodes[i].op == _lib.MC_EX_LEAF and tm.c_nodes[i].leaf.kind == _lib.MC_OP_GATHER]
    assert len(gathers) == 2 and gathers[0].pool_offset == gathers[1].pool_offset
    for f in (W.logistic_regression, W.cauchy_location):
        tm = _trace.trace(*f(W.ns_product()))
        assert any(t.dist == _lib.MC_DIST_EXPR for t in tm.terms)


def test_indexing_pushes_to_the_leaves():
    """(alpha + beta * z)[group] stays the fused affine form (loc a gather of
    alpha, x the host-indexed z); an elementwise expression indexed by the
    group gathers its parameter leaves; the gather of a gather composes."""
    z = np.arange(4, dtype=np.float32)
    grp = np.array([0, 3, 3, 1, 2, 0])
    y = np.linspace(-1, 1, 6).astype(np.float32)

    def lp(p):
        mu = (p["a"] + p["b"] * z)[grp]
        sc = mx.exp(p["b"] * z + 0.5)[grp]
        return mx.sum(m.Normal(mu, 1.0).log_prob(y)) + mx.sum(m.Normal(0, sc).log_prob(y))

    tm = _trace.trace(lp, {"a": np.zeros(4, np.float32), "b": 0.5})
    aff = [t for t in tm.terms if t.aff is not None]
    assert len(aff) == 1 and aff[0].loc.kind == _lib.MC_OP_GATHER
    assert list(aff[0].loc.index) == list(grp)
    assert aff[0].aff[1].kind == _lib.MC_OP_DATA and np.array_equal(aff[0].aff[1].data, z[grp])
    ex = [t for t in tm.terms if t.dist == _lib.MC_DIST_EXPR]
    assert len(ex) == 1 and ex[0].n == 6
    v = _trace.Param("v", 0, (5,))
    g = v[np.array([4, 3, 2])][np.array([2, 2, 0])]
    assert g.view[0] == "gather" and list(g.view[1]) == [2, 2, 4]
    assert v[np.array([4, 3])][1].view == ("elem", 3)


def test_traced_weights_make_expression_terms():
    """lp * w with w traced or per-element data: every term of lp becomes an
    expression term whose root is its log density times w (the fused
    Normal's arguments rebuilt as an MC_EX_NORMAL_LP node); a constant part
    of lp becomes a term of its own."""
    X = np.arange(3, dtype=np.float32)

    def lp(p):
        base = m.Normal(p["x"], 1.0).log_prob(X)                 # fused, vector
        return mx.sum(base * X) + (m.HalfNormal(2).log_prob(p["y"]) + 1.5) * p["x"]

    tm = _trace.trace(lp, {"x": 1.0, "y": 0.5})
    assert [t.dist for t in tm.terms] == [_lib.MC_DIST_EXPR] * 3
    assert [t.n for t in tm.terms] == [3, 1, 1]
    ops = [tm.c_nodes[i].op for i in range(tm.n_nodes)]
    assert _lib.MC_EX_NORMAL_LP in ops and _lib.MC_EX_HALFNORMAL_LP in ops
    assert ops.count(_lib.MC_EX_MUL) == 3


def test_affine_terms_as_expressions():
    """_trace.affine_as_expressions (the NUTS program of a regression): the
    fused affine-loc term becomes one expression term, NORMAL_LP over
    ADD(a, MUL(b, x)), the priors stay fused; a model without affine terms
    gives None."""
    lp, init = W.linear_regression(W.ns_product(), 50)
    tm = _trace.trace(lp, init)
    assert tm.n_affines == 1
    alt = _trace.affine_as_expressions(tm)
    assert alt.n_affines == 0 and alt.n_exprs == 1
    assert [t.dist for t in alt.terms].count(_lib.MC_DIST_EXPR) == 1
    assert len(alt.terms) == len(tm.terms) and alt.lp_const == tm.lp_const
    ops = [alt.c_nodes[i].op for i in range(alt.n_nodes)]
    assert ops[-1] == _lib.MC_EX_NORMAL_LP and _lib.MC_EX_ADD in ops and _lib.MC_EX_MUL in ops
    lp2, init2 = W.two_predictor_regression(W.ns_product())
    assert _trace.affine_as_expressions(_trace.trace(lp2, init2)) is None


def test_layout_roundtrip():
    init = {"a": 1.0, "b": np.arange(6, dtype=np.float32).reshape(2, 3), "c": 2.0}
    lay = _trace.layout_of(init)
    flat = lay.flatten(init)
    np.testing.assert_array_equal(flat, [1, 0, 1, 2, 3, 4, 5, 2])
    back = lay.unflatten(np.stack([flat, flat + 1]))
    assert back["b"].shape == (2, 2, 3) and back["a"].shape == (2,)


def test_random_keys_are_deterministic():
    k = m.random.key(42)
    assert m.random.split(k, 3) == m.random.split(m.random.key(42), 3)
    assert len(set(x.seed for x in m.random.split(k, 8))) == 8


def test_mcmc_method_errors():
    mc = m.MCMC(lambda p: m.Normal(0, 1).log_prob(p["x"]))
    with pytest.raises(ValueError):
        mc.run({"x": 0.0}, method="gibbs")
    import torch

    if not torch.cuda.is_available():
        # no CPU fallback: the GPU sampler fails loudly without a device
        from mlx_mcmc_amd import _lib

        with pytest.raises(_lib.EngineUnavailable):
            mc.run({"x": 0.0}, method="metropolis", verbose=False)
    with pytest.raises(ValueError):
        mc.summary()


def test_nuts_kernel_choice_is_checked():
    """nuts(nuts_kernel=...) accepts only 'auto' and 'tape' (ADVICE r5): a
    typo raises before anything is traced or launched."""
    lp = lambda p: m.Normal(0, 1).log_prob(p["x"])  # noqa: E731
    for bad in ("lanes", "sliced", "Auto", ""):
        with pytest.raises(ValueError, match="nuts_kernel"):
            m.nuts(lp, {"x": 0.0}, num_samples=1, num_warmup=0, nuts_kernel=bad)


def test_transformed_operands_and_identity_terms():
    """Reparameterised models (include/mcmc355.h mc_transform_kind,
    MC_DIST_IDENTITY): mx.exp / mx.log of a parameter is a transformed
    operand wherever a parameter may stand; a parameter expression added to
    the log density is an identity term with its constant weight."""
    XF = {_lib.MC_XF_NONE: "", _lib.MC_XF_EXP: "exp", _lib.MC_XF_LOG: "log"}

    def desc(o):
        return (o.kind, XF[o.transform])

    lp, init = W.hierarchical_reparam(W.ns_product(), *W.SHAPES["small"])
    tm = _trace.trace(lp, init)
    P, N, PV, G_, D = (_lib.MC_OP_PSCALAR, _lib.MC_OP_NONE, _lib.MC_OP_PVEC, _lib.MC_OP_GATHER,
                       _lib.MC_OP_DATA)
    C = _lib.MC_OP_CONST
    got = [(t.dist, desc(t.value), desc(t.loc), desc(t.scale), t.weight) for t in tm.terms]
    assert got == [
        (_lib.MC_DIST_NORMAL, (P, ""), (C, ""), (C, ""), 1.0),
        (_lib.MC_DIST_HALFNORMAL, (P, "exp"), (N, ""), (C, ""), 1.0),     # HalfNormal(5)(e^lt)
        (_lib.MC_DIST_IDENTITY, (P, ""), (N, ""), (N, ""), 1.0),          # + log_tau
        (_lib.MC_DIST_HALFNORMAL, (P, "exp"), (N, ""), (C, ""), 1.0),
        (_lib.MC_DIST_IDENTITY, (P, ""), (N, ""), (N, ""), 1.0),
        (_lib.MC_DIST_NORMAL, (PV, ""), (P, ""), (P, "exp"), 1.0),        # theta ~ N(mu, e^lt)
        (_lib.MC_DIST_NORMAL, (D, ""), (G_, ""), (P, "exp"), 1.0),        # y ~ N(theta[g], e^ls)
    ]
    assert [tm.c_terms[k].scale.transform for k in range(len(tm.terms))][-1] == _lib.MC_XF_EXP
    # the affine slope exp(log_tau) of the non-centred model
    lp, init = W.eight_schools_nc_log(W.ns_product())
    tm = _trace.trace(lp, init)
    (t,) = [t for t in tm.terms if t.aff is not None]
    assert desc(t.aff[0]) == (P, "exp") and desc(t.aff[1]) == (PV, "")
    assert tm.c_affines[0].slope.transform == _lib.MC_XF_EXP
    # a log-transformed vector value and `- mx.sum(mx.log(x))`
    lp, init = W.lognormal(W.ns_product())
    tm = _trace.trace(lp, init)
    a, b = tm.terms
    assert desc(a.value) == (PV, "log") and a.n == 20
    assert (b.dist, desc(b.value), b.weight, b.n) == (_lib.MC_DIST_IDENTITY, (PV, "log"), -1.0, 20)
    # forms of an identity: sign, constant weight and offset, views
    def forms(p):
        lp0 = m.Normal(0, 1).log_prob(p["x"])
        return (lp0 - p["x"], -p["x"] + lp0, lp0 + 0.5 * p["x"], lp0 + (2.0 * p["x"] + 1.0),
                lp0 + mx.sum(mx.log(p["v"][1:3])), lp0 - mx.sum(p["v"][np.array([0, 0, 2])]))
    outs = forms({"x": _trace.Param("x", 0, ()), "v": _trace.Param("v", 1, (3,))})
    ids = [[t for t in o.terms if t.dist == _lib.MC_DIST_IDENTITY][0] for o in outs]
    assert [t.weight for t in ids] == [-1.0, -1.0, 0.5, 2.0, 1.0, -1.0]
    assert outs[3].const == 1.0
    assert desc(ids[4].value) == (PV, "log") and ids[4].value.param_offset == 2 and ids[4].n == 2
    assert desc(ids[5].value) == (G_, "") and ids[5].n == 3
    # a transform commutes with a view: exp(v)[1] and exp(v[1]) are one operand
    o1 = _trace.to_operand(mx.exp(_trace.Param("v", 1, (3,)))[1])
    o2 = _trace.to_operand(mx.exp(_trace.Param("v", 1, (3,))[1]))
    assert o1.key() == o2.key() == ("p", 2, _lib.MC_XF_EXP)
    # transformed and plain operands never fold together
    y = W.simple_normal_data()

    def two_scales(p):
        lp = 0.0
        for v in y[:3]:
            lp = lp + m.Normal(p["mu"], p["s"]).log_prob(mx.array(v))
        for v in y[3:6]:
            lp = lp + m.Normal(p["mu"], mx.exp(p["s"])).log_prob(mx.array(v))
        return lp
    tm = _trace.trace(two_scales, {"mu": 0.0, "s": 0.0})
    assert [(t.n, t.scale.transform) for t in tm.terms] == [(3, 0), (3, _lib.MC_XF_EXP)]


def test_axis_sums_and_means():
    """mx.sum(lp, axis=k) keeps the terms and reduces the shape; mx.mean is
    the sum times f32(1 / n); a row-summed log density summed again (or G
    times its mean) is the whole; the traced model W.axis_reductions (run on
    the GPU against autograd in tests/test_gpu_expr.py) carries those
    weights."""
    Y = np.ones((4, 5), np.float32)

    def f(axis_ops):
        def lp(p):
            per = m.Normal(p["x"], 1.0).log_prob(Y)
            return axis_ops(per)
        return _trace.trace(lp, {"x": 1.0})

    tm = f(lambda per: mx.sum(mx.sum(per, axis=1)))
    assert [t.weight for t in tm.terms] == [1.0] and tm.terms[0].n == 20
    tm = f(lambda per: mx.sum(mx.sum(per, axis=-1, keepdims=True)))
    assert [t.weight for t in tm.terms] == [1.0]
    tm = f(lambda per: mx.mean(per))
    assert tm.terms[0].weight == pytest.approx(float(np.float32(1) / np.float32(20)))
    tm = f(lambda per: mx.sum(mx.mean(per, axis=0)))
    assert tm.terms[0].weight == pytest.approx(0.25)
    tm = f(lambda per: mx.mean(per, axis=(0, 1)))
    assert tm.terms[0].weight == pytest.approx(0.05)
    tm = _trace.trace(*W.axis_reductions(W.ns_product()))
    assert sorted(round(t.weight, 6) for t in tm.terms if t.n == 400) == [0.00125, 1.0]
    with pytest.raises(_trace.TraceError, match="must return a scalar"):
        f(lambda per: mx.sum(per, axis=1))
