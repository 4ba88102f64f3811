"""Synthetic workloads of BASELINE.json's configs, as model factories.

Each factory takes a namespace ``ns`` with ``Normal``, ``HalfNormal`` and ``sum``
— the product (``ns_product()``: mlx_mcmc_amd) or the CPU oracle
(``ns_oracle()``: oracle.ns) — and returns ``(log_prob_fn, initial_params)``,
so the same model definition is traced for the GPU and differentiated by
autograd on the CPU.  Data are fixed synthetic draws (no datasets).
"""
from __future__ import annotations

from types import SimpleNamespace

import numpy as np


def ns_product():
    import mlx_mcmc_amd as m
    import mlx_mcmc_amd.core as mx

    return SimpleNamespace(Normal=m.Normal, HalfNormal=m.HalfNormal, Exponential=m.Exponential,
                           Gamma=m.Gamma, Beta=m.Beta, sum=mx.sum, mean=mx.mean, array=mx.array,
                           exp=mx.exp, log=mx.log, sqrt=mx.sqrt, square=mx.square,
                           power=mx.power, abs=mx.abs, log1p=mx.log1p, tanh=mx.tanh,
                           sigmoid=mx.sigmoid, where=mx.where, pi=mx.pi, name="product")


def ns_oracle():
    from oracle import ns

    return SimpleNamespace(Normal=ns.Normal, HalfNormal=ns.HalfNormal, Exponential=ns.Exponential,
                           Gamma=ns.Gamma, Beta=ns.Beta, sum=ns.sum, mean=ns.mean, array=ns.array,
                           exp=ns.exp, log=ns.log, sqrt=ns.sqrt, square=ns.square,
                           power=ns.power, abs=ns.abs, log1p=ns.log1p, tanh=ns.tanh,
                           sigmoid=ns.sigmoid, where=ns.where, pi=ns.pi, name="oracle")


# ---- config 1: examples/01_simple_normal.py:26-50 (vectorised as in
#      examples/02_hmc_comparison.py:40-52) ------------------------------------
def simple_normal_data(n=100):
    np.random.seed(42)
    return np.random.normal(5.0, 2.0, n)


def simple_normal(ns, n=100):
    data = simple_normal_data(n)

    def log_prob(params):
        mu = params["mu"]
        sigma = params["sigma"]
        lp = ns.Normal(0, 10).log_prob(mu) + ns.HalfNormal(5).log_prob(sigma)
        return lp + ns.sum(ns.Normal(mu, sigma).log_prob(ns.array(data)))

    return log_prob, {"mu": 0.0, "sigma": 1.0}


# ---- config 2: isotropic D-dim standard normal --------------------------------
def iso_normal(ns, D=100):
    def log_prob(params):
        return ns.sum(ns.Normal(0, 1).log_prob(params["x"]))

    return log_prob, {"x": np.zeros(D, np.float32)}


# ---- configs 3/4: hierarchical Normal (README "Large" row) ---------------------
SHAPES = {"small": (7, 1_000), "medium": (97, 10_000), "large": (997, 100_000)}


def hierarchical_data(G, N, seed=0):
    rng = np.random.default_rng(seed)
    group = (np.arange(N, dtype=np.int64) * G) // N
    theta_true = rng.normal(1.0, 2.0, G)
    y = rng.normal(theta_true[group], 1.0).astype(np.float32)
    return y, group.astype(np.int32)


def hierarchical(ns, G=997, N=100_000, seed=0):
    y, group = hierarchical_data(G, N, seed)

    def log_prob(params):
        mu, tau, sigma, theta = params["mu"], params["tau"], params["sigma"], params["theta"]
        lp = ns.Normal(0, 10).log_prob(mu)
        lp = lp + ns.HalfNormal(5).log_prob(tau)
        lp = lp + ns.HalfNormal(5).log_prob(sigma)
        lp = lp + ns.sum(ns.Normal(mu, tau).log_prob(theta))
        lp = lp + ns.sum(ns.Normal(theta[group], sigma).log_prob(y))
        return lp

    sums = np.bincount(group, weights=y, minlength=G)
    counts = np.bincount(group, minlength=G)
    gm = (sums / np.maximum(counts, 1)).astype(np.float32)
    init = {"mu": np.float32(gm.mean()), "tau": np.float32(gm.std()),
            "sigma": np.float32(1.0), "theta": gm}
    return log_prob, init


def hierarchical_reparam(ns, G=997, N=100_000, seed=0):
    """The hierarchical model with unconstrained scales: tau = exp(log_tau),
    sigma = exp(log_sigma), the same HalfNormal priors on tau and sigma plus
    the log-Jacobians (`lp + log_tau`), so (mu, exp(log_tau), exp(log_sigma),
    theta) has exactly `hierarchical`'s posterior (oracle/exact.py
    log_tau_sigma moments).  Transformed scale operands and identity terms
    (include/mcmc355.h mc_transform_kind, MC_DIST_IDENTITY)."""
    y, group = hierarchical_data(G, N, seed)

    def log_prob(params):
        mu, log_tau, log_sigma = params["mu"], params["log_tau"], params["log_sigma"]
        theta = params["theta"]
        tau, sigma = ns.exp(log_tau), ns.exp(log_sigma)
        lp = ns.Normal(0, 10).log_prob(mu)
        lp = lp + ns.HalfNormal(5).log_prob(tau) + log_tau
        lp = lp + ns.HalfNormal(5).log_prob(sigma) + log_sigma
        lp = lp + ns.sum(ns.Normal(mu, tau).log_prob(theta))
        lp = lp + ns.sum(ns.Normal(theta[group], sigma).log_prob(y))
        return lp

    _, init = hierarchical(ns, G, N, seed)
    return log_prob, {"mu": init["mu"], "log_tau": np.float32(np.log(init["tau"])),
                      "log_sigma": np.float32(0.0), "theta": init["theta"]}


def hierarchical_flops_per_step(G, N):
    """SURVEY §8d canonical algorithmic FP32 flops per chain-leapfrog-step."""
    return 5 * N + 13 * (G + 3)


# ---- config 5: ill-conditioned diagonal Gaussian (kappa = 1000) ----------------
def illcond_scales(D=100):
    return (10.0 ** (-1.5 * np.arange(D) / (D - 1))).astype(np.float32)


def illcond_normal(ns, D=100):
    scales = illcond_scales(D)

    def log_prob(params):
        return ns.sum(ns.Normal(0, scales).log_prob(params["x"]))

    return log_prob, {"x": np.zeros(D, np.float32)}


# ---- SURVEY 8f-1 models: examples/03_ab_testing.py:26-59 and
#      examples/04_event_rates.py:26-55 (same data generation and log_prob) ------
def ab_testing_data():
    np.random.seed(42)
    n = 1000
    ca = int(np.random.binomial(n, 0.12))
    cb = int(np.random.binomial(n, 0.15))
    return n, ca, cb


def ab_testing(ns):
    """Beta(1, 1) priors and Beta(k + 1, n - k + 1) 'likelihoods' on p_A, p_B:
    the posterior of p_X is Beta(k_X + 1, n - k_X + 1)."""
    n, ca, cb = ab_testing_data()

    def log_prob(params):
        p_a, p_b = params["p_A"], params["p_B"]
        return (ns.Beta(1, 1).log_prob(p_a) + ns.Beta(1, 1).log_prob(p_b)
                + ns.Beta(ca + 1, n - ca + 1).log_prob(p_a)
                + ns.Beta(cb + 1, n - cb + 1).log_prob(p_b))

    return log_prob, {"p_A": 0.1, "p_B": 0.1}


def event_rates_data():
    np.random.seed(42)
    return np.random.exponential(scale=1 / 3.0, size=50)


def event_rates(ns):
    """Gamma(2, 1) prior, Exponential likelihood written as the reference's loop:
    the posterior of the rate is Gamma(2 + n, 1 + sum t)."""
    t = event_rates_data()

    def log_prob(params):
        rate = params["rate"]
        lp = ns.Gamma(alpha=2, beta=1).log_prob(rate)
        ll = ns.array(0.0)
        for ti in t:
            ll = ll + ns.Exponential(rate).log_prob(ns.array(ti))
        return lp + ll

    return log_prob, {"rate": 2.0}


# ---- per-element data scales (known measurement error): eight schools ---------
EIGHT_SCHOOLS_Y = np.array([28.0, 8.0, -3.0, 7.0, -1.0, 1.0, 18.0, 12.0], np.float32)
EIGHT_SCHOOLS_SIGMA = np.array([15.0, 10.0, 16.0, 11.0, 9.0, 11.0, 10.0, 18.0], np.float32)


def eight_schools(ns):
    """Centred eight schools: y_j ~ N(theta_j, sigma_j) with known sigma_j,
    theta ~ N(mu, tau): a likelihood whose scale is a per-element data vector."""
    y, sig = EIGHT_SCHOOLS_Y, EIGHT_SCHOOLS_SIGMA

    def log_prob(params):
        mu, tau, theta = params["mu"], params["tau"], params["theta"]
        lp = ns.Normal(0, 5).log_prob(mu) + ns.HalfNormal(5).log_prob(tau)
        lp = lp + ns.sum(ns.Normal(mu, tau).log_prob(theta))
        return lp + ns.sum(ns.Normal(theta, sig).log_prob(ns.array(y)))

    return log_prob, {"mu": np.float32(4.0), "tau": np.float32(3.0),
                      "theta": np.full(8, 4.0, np.float32)}


def eight_schools_nc(ns):
    """Non-centred eight schools: theta_j = mu + tau * z_j (an affine loc),
    y_j ~ N(theta_j, sigma_j), z ~ N(0, 1)."""
    y, sig = EIGHT_SCHOOLS_Y, EIGHT_SCHOOLS_SIGMA

    def log_prob(params):
        mu, tau, z = params["mu"], params["tau"], params["z"]
        lp = ns.Normal(0, 5).log_prob(mu) + ns.HalfNormal(5).log_prob(tau)
        lp = lp + ns.sum(ns.Normal(0, 1).log_prob(z))
        return lp + ns.sum(ns.Normal(mu + tau * z, sig).log_prob(ns.array(y)))

    return log_prob, {"mu": np.float32(4.0), "tau": np.float32(3.0),
                      "z": np.zeros(8, np.float32)}


def eight_schools_nc_log(ns):
    """Non-centred eight schools with tau = exp(log_tau): the affine loc's
    slope is a transformed parameter (mu + exp(log_tau) * z), plus the
    log-Jacobian identity term."""
    y, sig = EIGHT_SCHOOLS_Y, EIGHT_SCHOOLS_SIGMA

    def log_prob(params):
        mu, log_tau, z = params["mu"], params["log_tau"], params["z"]
        tau = ns.exp(log_tau)
        lp = ns.Normal(0, 5).log_prob(mu) + ns.HalfNormal(5).log_prob(tau) + log_tau
        lp = lp + ns.sum(ns.Normal(0, 1).log_prob(z))
        return lp + ns.sum(ns.Normal(mu + tau * z, sig).log_prob(ns.array(y)))

    return log_prob, {"mu": np.float32(4.0), "log_tau": np.float32(1.0),
                      "z": np.zeros(8, np.float32)}


# ---- a positive vector through mx.log: log-normal components -----------------------
def lognormal_params(D=20):
    m = np.linspace(-1.0, 1.0, D).astype(np.float32)
    s = np.linspace(0.2, 0.4, D).astype(np.float32)
    return m, s


def lognormal(ns, D=20):
    """x_i > 0 with log x_i ~ N(m_i, s_i), written as the change of variables
    Normal(m, s).log_prob(log x) - sum(log x): a log-transformed parameter
    vector as a value operand and a vector identity term.  Known answer:
    E x_i = exp(m_i + s_i^2 / 2), Var x_i = (exp(s_i^2) - 1) exp(2 m_i + s_i^2)."""
    m, s = lognormal_params(D)

    def log_prob(params):
        x = params["x"]
        lp = ns.sum(ns.Normal(ns.array(m), ns.array(s)).log_prob(ns.log(x)))
        return lp - ns.sum(ns.log(x))

    return log_prob, {"x": np.exp(m).astype(np.float32)}


def lognormal_moments(D=20):
    m, s = (v.astype(np.float64) for v in lognormal_params(D))
    return {"mean": np.exp(m + s * s / 2), "var": np.expm1(s * s) * np.exp(2 * m + s * s)}


# ---- linear regression: an affine loc a + b * x over data ------------------------
def regression_data(n=1000, seed=3):
    rng = np.random.default_rng(seed)
    x = rng.normal(0.0, 1.0, n).astype(np.float32)
    y = (1.5 + 2.0 * x + rng.normal(0.0, 0.5, n)).astype(np.float32)
    return x, y


def linear_regression(ns, n=1000):
    x, y = regression_data(n)

    def log_prob(params):
        a, b, sigma = params["a"], params["b"], params["sigma"]
        lp = ns.Normal(0, 10).log_prob(a) + ns.Normal(0, 10).log_prob(b)
        lp = lp + ns.HalfNormal(5).log_prob(sigma)
        return lp + ns.sum(ns.Normal(a + b * ns.array(x), sigma).log_prob(ns.array(y)))

    return log_prob, {"a": np.float32(0.0), "b": np.float32(0.0), "sigma": np.float32(1.0)}


def linear_regression_exp(ns, n=1000):
    """The linear regression with an Exponential(1) prior on the noise scale
    (a scalar term the sliced kernels cannot take as an own prior)."""
    x, y = regression_data(n)

    def log_prob(params):
        a, b, sigma = params["a"], params["b"], params["sigma"]
        lp = ns.Normal(0, 10).log_prob(a) + ns.Normal(0, 10).log_prob(b)
        lp = lp + ns.Exponential(1.0).log_prob(sigma)
        return lp + ns.sum(ns.Normal(a + b * ns.array(x), sigma).log_prob(ns.array(y)))

    return log_prob, {"a": np.float32(0.0), "b": np.float32(0.0), "sigma": np.float32(1.0)}


def varying_intercept_data(G=20, N=2000, seed=4):
    rng = np.random.default_rng(seed)
    group = np.sort(rng.integers(0, G, N)).astype(np.int32)
    alpha = rng.normal(1.0, 1.5, G)
    x = rng.normal(0.0, 1.0, N).astype(np.float32)
    y = (alpha[group] + 0.7 * x + rng.normal(0.0, 0.8, N)).astype(np.float32)
    return x, y, group


def varying_intercept(ns, G=20, N=2000):
    """Varying-intercept regression: y_i ~ N(alpha[g_i] + beta * x_i, sigma)
    (an affine loc through a non-injective gather), alpha ~ N(mu, tau)."""
    x, y, group = varying_intercept_data(G, N)

    def log_prob(params):
        mu, tau, beta, sigma = params["mu"], params["tau"], params["beta"], params["sigma"]
        alpha = params["alpha"]
        lp = ns.Normal(0, 10).log_prob(mu) + ns.HalfNormal(5).log_prob(tau)
        lp = lp + ns.Normal(0, 10).log_prob(beta) + ns.HalfNormal(5).log_prob(sigma)
        lp = lp + ns.sum(ns.Normal(mu, tau).log_prob(alpha))
        return lp + ns.sum(ns.Normal(alpha[group] + beta * ns.array(x), sigma)
                           .log_prob(ns.array(y)))

    return log_prob, {"mu": np.float32(1.0), "tau": np.float32(1.5), "beta": np.float32(0.7),
                      "sigma": np.float32(0.8), "alpha": np.ones(G, np.float32)}


# ---- general elementwise expressions (expression terms, MC_DIST_EXPR) ------------
def two_predictor_data(n=1000, seed=5):
    rng = np.random.default_rng(seed)
    x1 = rng.normal(0.0, 1.0, n).astype(np.float32)
    x2 = rng.normal(0.0, 1.0, n).astype(np.float32)
    y = (0.5 + 1.2 * x1 - 0.8 * x2 + rng.normal(0.0, 0.6, n)).astype(np.float32)
    return x1, x2, y


def two_predictor_regression(ns, n=1000):
    """y ~ N(a + b1 x1 + b2 x2, exp(log_sigma)): two products in the loc and
    a log-scale noise with its Jacobian (an expression term)."""
    x1, x2, y = two_predictor_data(n)

    def log_prob(params):
        a, b1, b2, log_sigma = params["a"], params["b1"], params["b2"], params["log_sigma"]
        sigma = ns.exp(log_sigma)
        lp = ns.Normal(0, 10).log_prob(a) + ns.Normal(0, 10).log_prob(b1)
        lp = lp + ns.Normal(0, 10).log_prob(b2) + ns.HalfNormal(5).log_prob(sigma) + log_sigma
        mean = a + b1 * ns.array(x1) + b2 * ns.array(x2)
        return lp + ns.sum(ns.Normal(mean, sigma).log_prob(ns.array(y)))

    return log_prob, {"a": np.float32(0.0), "b1": np.float32(0.0), "b2": np.float32(0.0),
                      "log_sigma": np.float32(0.0)}


def huber_data(n=1000, seed=8):
    rng = np.random.default_rng(seed)
    x = rng.normal(0.0, 1.0, n).astype(np.float32)
    noise = np.where(rng.random(n) < 0.1, rng.normal(0.0, 6.0, n), rng.normal(0.0, 0.5, n))
    y = (0.4 + 1.3 * x + noise).astype(np.float32)
    return x, y


def huber_regression(ns, n=1000, c=1.0):
    """A robust regression: the Huber loss of the residuals as the negative
    log density, its two branches chosen by mx.where over a traced condition
    (|r| < c, a comparison of a parameter expression)."""
    x, y = huber_data(n)

    def log_prob(params):
        a, b = params["a"], params["b"]
        lp = ns.Normal(0, 10).log_prob(a) + ns.Normal(0, 10).log_prob(b)
        r = ns.array(y) - (a + b * ns.array(x))
        ar = ns.abs(r)
        loss = ns.where(ar < c, 0.5 * (r * r), c * ar - 0.5 * c * c)
        return lp - ns.sum(loss)

    return log_prob, {"a": np.float32(0.4), "b": np.float32(1.3)}


def weighted_indexed_data(G=8, n=400, seed=9):
    rng = np.random.default_rng(seed)
    group = rng.integers(0, G, n).astype(np.int64)           # unsorted, repeats
    z = rng.normal(0.0, 1.0, G).astype(np.float32)            # a group-level covariate
    w = rng.uniform(0.5, 1.5, n).astype(np.float32)           # per-observation weights
    alpha = rng.normal(0.5, 1.0, G)
    y = (alpha[group] + 0.8 * z[group] + rng.normal(0.0, 0.6, n)).astype(np.float32)
    return group, z, w, y


def weighted_indexed(ns, G=8, n=400):
    """Per-observation weights on a log density (mx.sum(w * lp)), an indexed
    affine expression ((alpha + beta * z)[group]) and an indexed elementwise
    expression (mx.exp(...)[group] as a per-group scale)."""
    group, z, w, y = weighted_indexed_data(G, n)

    def log_prob(params):
        al, b, ls, c = params["alpha"], params["beta"], params["log_sigma"], params["c"]
        lp = ns.sum(ns.Normal(0, 2).log_prob(al)) + ns.Normal(0, 2).log_prob(b)
        lp = lp + ns.Normal(0, 1).log_prob(ls) + ns.Normal(0, 1).log_prob(c)
        mu = (al + b * ns.array(z))[group]
        scale = ns.exp(ls + c * ns.array(z))[group]
        return lp + ns.sum(ns.array(w) * ns.Normal(mu, scale).log_prob(ns.array(y)))

    return log_prob, {"alpha": np.zeros(G, np.float32), "beta": np.float32(0.5),
                      "log_sigma": np.float32(-0.3), "c": np.float32(0.0)}


def tempered_data(n=300, seed=10):
    rng = np.random.default_rng(seed)
    return rng.normal(1.5, 0.8, n).astype(np.float32)


def tempered(ns, n=300):
    """A likelihood weighted by a parameter (mx.sigmoid(t) * lp, a power
    posterior whose temperature is sampled) and a log density divided by a
    parameter expression: log densities under traced weights."""
    y = tempered_data(n)

    def log_prob(params):
        mu, t, ls = params["mu"], params["t"], params["log_s"]
        lp = ns.Normal(0, 5).log_prob(mu) + ns.Normal(0, 1).log_prob(t)
        lp = lp + ns.Normal(0, 1).log_prob(ls) / (1.0 + ns.square(t))
        lik = ns.sum(ns.Normal(mu, ns.exp(ls)).log_prob(ns.array(y)))
        return lp + ns.sigmoid(t) * lik

    return log_prob, {"mu": np.float32(1.0), "t": np.float32(0.5), "log_s": np.float32(0.0)}


def logistic_data(n=500, seed=6):
    rng = np.random.default_rng(seed)
    x = rng.normal(0.0, 1.0, n).astype(np.float32)
    p = 1.0 / (1.0 + np.exp(-(-0.3 + 1.1 * x)))
    y = (rng.random(n) < p).astype(np.float32)
    return x, y


def logistic_regression(ns, n=500):
    """Bernoulli likelihood written out with mx.sigmoid / mx.log / mx.log1p."""
    x, y = logistic_data(n)

    def log_prob(params):
        a, b = params["a"], params["b"]
        lp = ns.Normal(0, 5).log_prob(a) + ns.Normal(0, 5).log_prob(b)
        p = ns.sigmoid(a + b * ns.array(x))
        ll = ns.array(y) * ns.log(p) + (1.0 - ns.array(y)) * ns.log1p(-p)
        return lp + ns.sum(ll)

    return log_prob, {"a": np.float32(0.0), "b": np.float32(0.0)}


def varying_slopes_data(G=16, N=1600, seed=7):
    rng = np.random.default_rng(seed)
    group = rng.integers(0, G, N).astype(np.int32)          # unsorted: the tape sorts it
    alpha = rng.normal(1.0, 1.0, G)
    beta = rng.normal(-0.5, 0.7, G)
    x = rng.normal(0.0, 1.0, N).astype(np.float32)
    y = (alpha[group] + beta[group] * x + rng.normal(0.0, 0.5, N)).astype(np.float32)
    return x, y, group


def varying_slopes(ns, G=16, N=1600):
    """y_i ~ N(alpha[g_i] + beta[g_i] x_i, sigma): two gathers through one
    non-injective index in a product and a sum (the segmented expression
    path), alpha ~ N(mu_a, 2), beta ~ N(mu_b, 2)."""
    x, y, group = varying_slopes_data(G, N)

    def log_prob(params):
        mu_a, mu_b, sigma = params["mu_a"], params["mu_b"], params["sigma"]
        alpha, beta = params["alpha"], params["beta"]
        lp = ns.Normal(0, 5).log_prob(mu_a) + ns.Normal(0, 5).log_prob(mu_b)
        lp = lp + ns.HalfNormal(2).log_prob(sigma)
        lp = lp + ns.sum(ns.Normal(mu_a, 2.0).log_prob(alpha))
        lp = lp + ns.sum(ns.Normal(mu_b, 2.0).log_prob(beta))
        mean = alpha[group] + beta[group] * ns.array(x)
        return lp + ns.sum(ns.Normal(mean, sigma).log_prob(ns.array(y)))

    return log_prob, {"mu_a": np.float32(1.0), "mu_b": np.float32(-0.5),
                      "sigma": np.float32(0.5), "alpha": np.ones(G, np.float32),
                      "beta": np.zeros(G, np.float32)}


def gamma_beta_data(n=300, seed=9):
    rng = np.random.default_rng(seed)
    x = rng.normal(0.0, 1.0, n).astype(np.float32)
    mu = np.exp(0.4 + 0.3 * x)
    y = rng.gamma(3.0, mu / 3.0).astype(np.float32)             # shape 3, mean mu
    p = 1.0 / (1.0 + np.exp(-(-0.2 + 0.8 * x)))
    z = np.clip(rng.beta(8.0 * p, 8.0 * (1.0 - p)), 1e-4, 1 - 1e-4).astype(np.float32)
    return x, y, z


def gamma_beta_regression(ns, n=300):
    """Gamma and Beta likelihoods with parameter-expression arguments
    (gamma.py:48-88, beta.py:45-91): a Gamma GLM y ~ Gamma(a, a / mu),
    mu = exp(b0 + b1 x), and a Beta regression z ~ Beta(phi p, phi (1 - p)),
    p = sigmoid(c0 + c1 x) — the shapes are expressions, so their gammaln
    normalisers are evaluated per element at the current values, and (as in
    the reference, whose gammaln is a host scipy constant) the shape
    gradients carry no digamma term."""
    x, y, z = gamma_beta_data(n)

    def log_prob(params):
        b0, b1, c0, c1 = params["b0"], params["b1"], params["c0"], params["c1"]
        la, lphi = params["log_a"], params["log_phi"]
        lp = ns.Normal(0, 2).log_prob(b0) + ns.Normal(0, 2).log_prob(b1)
        lp = lp + ns.Normal(0, 2).log_prob(c0) + ns.Normal(0, 2).log_prob(c1)
        lp = lp + ns.Normal(1, 1).log_prob(la) + ns.Normal(2, 1).log_prob(lphi)
        a = ns.exp(la)
        mu = ns.exp(b0 + b1 * ns.array(x))
        lp = lp + ns.sum(ns.Gamma(a, a / mu).log_prob(ns.array(y)))
        phi = ns.exp(lphi)
        p = ns.sigmoid(c0 + c1 * ns.array(x))
        return lp + ns.sum(ns.Beta(phi * p, phi * (1.0 - p)).log_prob(ns.array(z)))

    return log_prob, {"b0": np.float32(0.3), "b1": np.float32(0.2), "c0": np.float32(0.0),
                      "c1": np.float32(0.5), "log_a": np.float32(1.0),
                      "log_phi": np.float32(2.0)}


def axis_reduction_data(G=8, K=50, seed=10):
    rng = np.random.default_rng(seed)
    x = rng.normal(0.0, 1.0, (G, K)).astype(np.float32)
    y = (0.5 + 1.5 * x + rng.normal(0.0, 0.6, (G, K))).astype(np.float32)
    return x, y


def axis_reductions(ns, G=8, K=50):
    """Log densities reduced over axes and averaged (mx.sum(lp, axis=1),
    mx.mean): a 2-D regression likelihood written out (an expression term)
    summed per row, then G times the mean of the rows (the total), and a
    fused 2-D term averaged over both axes with a weight."""
    x, y = axis_reduction_data(G, K)

    def log_prob(params):
        a, b, ls = params["a"], params["b"], params["log_sigma"]
        lp = ns.Normal(0, 5).log_prob(a) + ns.Normal(0, 5).log_prob(b)
        lp = lp + ns.Normal(0, 1).log_prob(ls)
        z = (ns.array(y) - (a + b * ns.array(x))) / ns.exp(ls)
        per = -0.5 * ns.square(z) - ls - 0.9189385                              # (G, K)
        rows = ns.sum(per, axis=1)                                               # (G,)
        lp = lp + float(G) * ns.mean(rows)
        return lp + 0.5 * ns.mean(ns.Normal(a, 2.0).log_prob(ns.array(y)), axis=(0, 1))

    return log_prob, {"a": np.float32(0.4), "b": np.float32(1.4), "log_sigma": np.float32(-0.4)}


def cauchy_location(ns, n=200, seed=8):
    """A Cauchy location-scale likelihood written by hand (the reference has no
    Cauchy): -log(pi s) - log1p(((y - mu) / s)^2), s = sqrt(v); plus the other
    elementwise ops (tanh, abs, power, where over a data mask) in a weak
    extra term, so every expression op is differentiated somewhere."""
    rng = np.random.default_rng(seed)
    y = (2.0 + rng.standard_cauchy(n) * 0.7).astype(np.float32)
    mask = (np.arange(n) % 3 == 0).astype(np.float32)

    def log_prob(params):
        mu, v, w = params["mu"], params["v"], params["w"]
        s = ns.sqrt(v)
        lp = ns.Normal(0, 10).log_prob(mu) + ns.Exponential(1.0).log_prob(v)
        lp = lp + ns.Normal(0, 1).log_prob(w)
        z = (ns.array(y) - mu) / s
        lp = lp + ns.sum(-ns.log(ns.pi * s) - ns.log1p(ns.square(z)))
        extra = ns.where(ns.array(mask), ns.tanh(w * z), -0.1 * ns.power(ns.abs(w) + 1.0, 1.5))
        return lp + 0.01 * ns.sum(extra)

    return log_prob, {"mu": np.float32(2.0), "v": np.float32(0.5), "w": np.float32(0.1)}
