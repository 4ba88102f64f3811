"""Expression terms (include/mcmc355.h MC_DIST_EXPR / mc_expr_node;
_trace.Expr; eval.h eval_expr): the reference differentiates any MLX
expression of the parameters with mx.grad (hmc.py:53-67, nuts.py:76-87).
Models beyond the fused terms — two predictors with a log-scale noise, a
Bernoulli likelihood through mx.sigmoid / mx.log1p, varying slopes (two
gathers through one non-injective index: the segmented expression path), a
hand-written Cauchy likelihood using every other op (sqrt, square, log1p,
tanh, abs, power, where), Gamma and Beta likelihoods with expression shapes —
run on the GPU tape and are checked against the CPU
oracle, whose gradients are torch autograd over the same user model.

Bars: tape log p within 2e-6 * 50 of max(1, |lp|) (f32 summation order and
ocml vs torch transcendental rounding), gradients rtol 1e-4; HMC decisions /
H / ratios equal to the oracle's until a proven near-tie (tests/_near_tie.py);
NUTS trees identical for >= 10 iterations; MH decisions identical over 150
iterations; the two-predictor posterior means within 4 MCSE of least squares
(flat-ish priors)."""
import numpy as np
import pytest

import workloads as W
from _near_tie import compare_trace, log_u
from oracle import samplers as S

pytestmark = pytest.mark.gpu


def tiny_scalar(ns):
    """Only broadcast parameters in small expression terms (the wave-task path)."""
    def log_prob(params):
        a, b = params["a"], params["b"]
        lp = ns.Normal(0, 1).log_prob(a * b) + ns.Normal(a / (1.0 + b * b), 2.0).log_prob(0.3)
        return lp + ns.Normal(0, 3).log_prob(a) + ns.Normal(0, 3).log_prob(b) - 0.1 * ns.square(a - b)

    return log_prob, {"a": np.float32(0.5), "b": np.float32(-0.4)}


MODELS = {"two_predictor": W.two_predictor_regression,
          "logistic": W.logistic_regression,
          "varying_slopes": W.varying_slopes,
          "cauchy": W.cauchy_location,
          "gamma_beta": W.gamma_beta_regression,
          "axis_reductions": W.axis_reductions,
          "huber": W.huber_regression,
          "weighted_indexed": W.weighted_indexed,
          "tempered": W.tempered,
          "tiny_scalar": tiny_scalar}
POSITIVE = ("sigma", "v")


def _points(prog, init, k=6, spread=0.3, seed=7):
    rng = np.random.default_rng(seed)
    base = prog.layout.flatten(init)
    pts = np.stack([base + rng.normal(0, spread, base.size).astype(np.float32) for _ in range(k)])
    for nm in POSITIVE:
        if nm in prog.layout.names:
            j = prog.layout.offsets[prog.layout.names.index(nm)]
            pts[:, j] = np.abs(pts[:, j]) + 0.2
    return pts


@pytest.mark.parametrize("model", list(MODELS))
def test_expr_tape_matches_autograd(gpu, model):
    from mlx_mcmc_amd import _engine, _lib, _trace

    lp_fn, init = MODELS[model](W.ns_product())
    prog = _trace.compile_model(lp_fn, init)
    assert any(t.dist == _lib.MC_DIST_EXPR for t in prog.model.terms)
    assert prog.slice_kernel == "unsliced"   # the chain-per-workgroup tape
    olp, oinit = MODELS[model](W.ns_oracle())
    M = S.EagerModel(olp, oinit)
    pts = _points(prog, init)
    lp, g = _engine.logp_grad(prog, pts)
    lp, g = lp.cpu().numpy(), g.cpu().numpy()
    for i, q in enumerate(pts):
        rl, rg = M.logp_grad(q)
        assert abs(lp[i] - rl) <= 2e-6 * max(1.0, abs(rl)) * 50, (i, lp[i], rl)
        np.testing.assert_allclose(g[i], rg, rtol=1e-4, atol=1e-3 * max(1.0, np.abs(rg).max()))
    # bit-reproducible: the same points evaluate to the same bits
    lp2, g2 = _engine.logp_grad(prog, pts)
    assert np.array_equal(lp, lp2.cpu().numpy()) and np.array_equal(g, g2.cpu().numpy())


def test_expr_nan_and_support(gpu):
    """log of a negative parameter gives NaN log p (Q14), HalfNormal of a
    negative expression -inf with zero gradient through mx.where (halfnormal.py:63)."""
    import mlx_mcmc_amd as m
    import mlx_mcmc_amd.core as mx
    from mlx_mcmc_amd import _engine, _trace

    prog = _trace.compile_model(
        lambda p: m.Normal(0, 1).log_prob(mx.log(p["x"] * 2.0)) + m.HalfNormal(1.0).log_prob(
            p["y"] - 1.0), {"x": 1.0, "y": 2.0})
    lp, g = _engine.logp_grad(prog, np.array([[-1.0, 2.0], [1.0, 0.5]], np.float32))
    lp, g = lp.cpu().numpy(), g.cpu().numpy()
    assert np.isnan(lp[0])
    assert lp[1] == -np.inf and g[1, 1] == 0.0


@pytest.mark.parametrize("model,start,eps,seed", [
    ("two_predictor", {"a": 0.5, "b1": 1.2, "b2": -0.8, "log_sigma": -0.5}, 0.004, 0),
    ("logistic", {"a": -0.3, "b": 1.1}, 0.05, 1),
    ("cauchy", {"mu": 2.0, "v": 0.5, "w": 0.1}, 0.02, 2),
    # (the shapes' gradients omit digamma, as the reference's host gammaln
    # does: the trajectories follow a biased force, so only small steps accept)
    ("gamma_beta", {"b0": 0.3, "b1": 0.2, "c0": 0.0, "c1": 0.5, "log_a": 1.0, "log_phi": 2.0},
     1e-4, 4),
    ("axis_reductions", {"a": 0.4, "b": 1.4, "log_sigma": -0.4}, 0.01, 5),
    # mx.where over a traced condition (|residual| < c: comparison nodes)
    ("huber", {"a": 0.4, "b": 1.3}, 0.01, 6),
    # per-observation weights, indexed affine / elementwise expressions
    ("weighted_indexed", {"alpha": np.zeros(8), "beta": 0.5, "log_sigma": -0.3, "c": 0.0},
     0.02, 7),
    # a likelihood under a traced weight (mx.sigmoid(t) * lp), a log density
    # divided by a parameter expression
    ("tempered", {"mu": 1.0, "t": 0.5, "log_s": 0.0}, 0.05, 8),
])
def test_expr_hmc_trace_matches_oracle(gpu, model, start, eps, seed):
    import mlx_mcmc_amd as m

    lp, _ = MODELS[model](W.ns_product())
    olp, _ = MODELS[model](W.ns_oracle())
    start = {k: np.asarray(v, np.float32) if np.ndim(v) else np.float32(v) for k, v in start.items()}
    kw = dict(num_samples=40, num_warmup=40, step_size=eps, num_leapfrog_steps=10)
    s, rate, info = m.hmc(lp, start, key=m.random.key(seed), progress=False, return_info=True,
                          return_trace=True, **kw)
    assert info.extra["kernel"] == "unsliced"
    ref = S.hmc(olp, start, seed=seed, **kw)
    # the warmup iterations: once the warmup rule (Q4) has grown eps into the
    # unstable regime, a strongly rejected trajectory amplifies the 1-ulp
    # differences of ocml's and torch's sigmoid / log1p / sqrt past the
    # 8-ulp tie bound (both still reject it)
    n = 40
    tr = info.trace
    gpu_c = {"accepted": tr["accepted"][0][:n], "ratio": tr["accept_stat"][0][:n],
             "step_size": tr["step_size"][0][:n], "energy": tr["energy"][0][:n]}
    ref_c = {k: np.asarray(ref.trace[k])[:n] for k in ("accepted", "ratio", "step_size", "energy")}
    ref_c["log_u"] = log_u(seed, 0, n)
    same = compare_trace(gpu_c, ref_c, f"{model} seed {seed}", verbose=True)
    acc = np.asarray(ref.trace["accepted"][:same])
    assert same >= 30 and acc.any()
    ns = max(0, min(same, 40) - 10)
    name = list(start)[0]
    # positions: the same draws and decisions, 1-ulp transcendental
    # differences carried through the leapfrog steps
    first = np.asarray(s[name]).reshape(np.asarray(s[name]).shape[0], -1)[:, 0]
    np.testing.assert_allclose(first[:ns], ref.samples[:ns, 0], rtol=1e-3, atol=2e-3)


def test_expr_varying_slopes_hmc_trace(gpu):
    """alpha[g] + beta[g] * x over an unsorted group index: the segmented
    expression path against the oracle's HMC trace."""
    import mlx_mcmc_amd as m

    lp, init = W.varying_slopes(W.ns_product())
    olp, _ = W.varying_slopes(W.ns_oracle())
    x, y, g = W.varying_slopes_data()
    start = dict(init)
    ab = np.array([np.polyfit(x[g == k], y[g == k], 1) for k in range(16)], np.float32)
    start["alpha"], start["beta"] = ab[:, 1].copy(), ab[:, 0].copy()
    # (from eps 0.01 the warmup rule reaches the unstable regime at iteration
    # 24, where both trajectories blow up: ratios -15 then -4.9e6)
    kw = dict(num_samples=30, num_warmup=30, step_size=0.005, num_leapfrog_steps=10)
    s, rate, info = m.hmc(lp, start, key=m.random.key(3), progress=False, return_info=True,
                          return_trace=True, **kw)
    ref = S.hmc(olp, start, seed=3, **kw)
    n = 30
    tr = info.trace
    gpu_c = {"accepted": tr["accepted"][0][:n], "ratio": tr["accept_stat"][0][:n],
             "step_size": tr["step_size"][0][:n], "energy": tr["energy"][0][:n]}
    ref_c = {k: np.asarray(ref.trace[k])[:n] for k in ("accepted", "ratio", "step_size", "energy")}
    ref_c["log_u"] = log_u(3, 0, n)
    same = compare_trace(gpu_c, ref_c, "varying slopes", verbose=True)
    acc = np.asarray(ref.trace["accepted"][:same])
    assert same >= 25 and acc.any()


def test_expr_nuts_trace_matches_oracle(gpu):
    import mlx_mcmc_amd as m

    plp, pinit = W.logistic_regression(W.ns_product())
    olp, oinit = W.logistic_regression(W.ns_oracle())
    n_w, n_s = 30, 10
    _, _, info = m.nuts(plp, pinit, num_samples=n_s, num_warmup=n_w, key=m.random.key(2),
                        progress=False, return_info=True, return_trace=True)
    assert info.extra["kernel"] == "tape"
    ref = S.nuts(olp, oinit, num_samples=n_s, num_warmup=n_w, seed=2)
    same = 0
    for i in range(n_w + n_s):
        if (info.trace["tree_depth"][0][i] != ref.trace["depth"][i]
                or info.trace["n_leapfrog"][0][i] != ref.trace["leaves"][i]):
            break
        same += 1
    assert same >= 10, f"trees diverged at iteration {same}"
    assert max(ref.trace["depth"][:same]) >= 2


def test_expr_mh_trace_matches_oracle(gpu):
    """The value-only tape (eval_lp_grad<WPC, true>) on an expression model."""
    import mlx_mcmc_amd as m

    lp, _ = W.cauchy_location(W.ns_product())
    olp, _ = W.cauchy_location(W.ns_oracle())
    start = {"mu": 2.0, "v": 0.5, "w": 0.1}
    n = 150
    s, rate, info = m.metropolis_hastings(lp, start, num_samples=n, proposal_scale=0.1,
                                          random_seed=5, return_info=True, return_trace=True)
    ref = S.metropolis_hastings(olp, start, num_samples=n, proposal_scale=0.1, random_seed=5)
    acc = info.trace["accepted"][0].astype(bool)
    assert list(acc) == ref.trace["accepted"] and 0 < acc.mean() < 1
    np.testing.assert_allclose(s["mu"], ref.samples[:, 0], rtol=1e-5, atol=1e-6)


def test_expr_two_predictor_posterior(gpu):
    import mlx_mcmc_amd as m

    lp, _ = W.two_predictor_regression(W.ns_product())
    x1, x2, y = W.two_predictor_data()
    X = np.stack([np.ones_like(x1), x1, x2], 1).astype(np.float64)
    beta = np.linalg.lstsq(X, y.astype(np.float64), rcond=None)[0]
    resid = y - X @ beta
    start = {"a": np.float32(beta[0]), "b1": np.float32(beta[1]), "b2": np.float32(beta[2]),
             "log_sigma": np.float32(np.log(resid.std()))}
    # HMC: with |H0| ~ 950 the reference's f32 slice (Q7) underflows to
    # log u = -inf and its NUTS stops testing the slice; the oracle and the
    # GPU reproduce that, so the posterior check runs HMC
    s, rate, info = m.hmc(lp, start, num_samples=500, num_warmup=300, step_size=0.01,
                          num_leapfrog_steps=10, key=m.random.key(1), num_chains=32,
                          progress=False, return_info=True)
    live = info.accept_rate > 0.05
    assert live.sum() >= 16
    for k, name in enumerate(("a", "b1", "b2")):
        d = s[name][live]                # [C, S]
        mcse = d.mean(1).std() / np.sqrt(d.shape[0])
        assert abs(d.mean() - beta[k]) < 4 * mcse + 2e-3, (name, d.mean(), beta[k], mcse)
    sd = np.exp(s["log_sigma"][live]).mean()
    assert abs(sd - resid.std()) < 0.02


@pytest.mark.parametrize("G", [1, 4])
def test_expr_segmented_few_groups_large_n(gpu, G):
    """alpha[g] + beta[g] * x with 1 or 4 groups over 200 K elements: the
    segmented expression path splits each group's run into virtual segments
    (partials per gathered leaf, added per group in order after a barrier)
    instead of walking it in one lane.  Log p and gradients against torch
    autograd (f32 summation over 200 K elements: lp within 1e-5 relative,
    gradients rtol 2e-4), and bit-reproducible."""
    from mlx_mcmc_amd import _engine, _trace

    n = 200_000
    lp_fn, init = W.varying_slopes(W.ns_product(), G=G, N=n)
    prog = _trace.compile_model(lp_fn, init)
    olp, oinit = W.varying_slopes(W.ns_oracle(), G=G, N=n)
    M = S.EagerModel(olp, oinit)
    pts = _points(prog, init, k=3, spread=0.2)
    lp, g = _engine.logp_grad(prog, pts)
    lp, g = lp.cpu().numpy(), g.cpu().numpy()
    for i, q in enumerate(pts):
        rl, rg = M.logp_grad(q)
        assert abs(lp[i] - rl) <= 1e-5 * max(1.0, abs(rl)), (i, lp[i], rl)
        np.testing.assert_allclose(g[i], rg, rtol=2e-4, atol=2e-5 * max(1.0, np.abs(rg).max()))
    lp2, g2 = _engine.logp_grad(prog, pts)
    assert np.array_equal(lp, lp2.cpu().numpy()) and np.array_equal(g, g2.cpu().numpy())
