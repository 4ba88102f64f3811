"""Exponential, Gamma and Beta on the GPU tape.

Parity bars: elementwise log_prob within 2e-6 relative (+ absolute slack for
the float32 log B / gammaln normalisers) of the oracle restatement
(oracle/ns.py, pinned to scipy by tests/test_oracle_pins.py), identical
support (-inf) decisions; tape log p and gradient vs oracle autograd (rtol
1e-4) on the reference's example 03/04 models and on vector-shape variants;
HMC / NUTS posteriors of those models against their analytic conjugate
posteriors; the sliced kernel against the chain-per-workgroup kernel; and the
reference's sampling statistics (tests/test_new_distributions.py).
"""
import numpy as np
import pytest

import workloads as W

pytestmark = pytest.mark.gpu


def _m():
    import mlx_mcmc_amd as m

    return m


def _oracle():
    from oracle import ns

    return ns


@pytest.mark.parametrize("name", ["Exponential", "Gamma", "Beta"])
def test_elementwise_log_prob_matches_oracle(gpu, name):
    m, ns = _m(), _oracle()
    rng = np.random.default_rng(7)
    n = 4096
    if name == "Beta":
        x = rng.uniform(-0.2, 1.2, n).astype(np.float32)
        x[:4] = [0.0, 1.0, -0.1, 1.5]
    else:
        x = rng.uniform(-1.0, 6.0, n).astype(np.float32)
        x[:2] = [0.0, -1.0]
    a = rng.uniform(0.5, 8.0, n).astype(np.float32)
    b = rng.uniform(0.3, 5.0, n).astype(np.float32)
    if name == "Exponential":
        got, ref = m.Exponential(b).log_prob(x), ns.Exponential(b).log_prob(x).numpy()
    elif name == "Gamma":
        got, ref = m.Gamma(a, b).log_prob(x), ns.Gamma(a, b).log_prob(x).numpy()
    else:
        got, ref = m.Beta(a, b).log_prob(x), ns.Beta(a, b).log_prob(x).numpy()
    np.testing.assert_array_equal(np.isfinite(got), np.isfinite(ref))
    f = np.isfinite(ref)
    np.testing.assert_allclose(got[f], ref[f], rtol=2e-6, atol=2e-5)
    # the reference's scalar known answers through the product API
    if name == "Exponential":
        assert np.isclose(float(m.Exponential(2.0).log_prob(0.0)), np.log(2.0))


def _tape_vs_oracle(lp_p, lp_o, init, points):
    import torch

    from mlx_mcmc_amd import _engine, _trace
    from oracle import samplers as S

    prog = _trace.compile_model(lp_p, init)
    M = S.EagerModel(lp_o, init)
    q = np.array(points, np.float32)
    glp, gg = _engine.logp_grad(prog, q)
    glp, gg = glp.cpu().numpy(), gg.cpu().numpy()
    for i in range(len(q)):
        l, g = M.logp_grad(q[i])
        assert abs(glp[i] - l) <= 2e-6 * (abs(l) + 1) + 1e-3
        np.testing.assert_allclose(gg[i], g, rtol=1e-4, atol=1e-4 * np.abs(g).max() + 1e-5)
    return prog


def test_tape_example03_ab_testing(gpu):
    lp_p, init = W.ab_testing(W.ns_product())
    lp_o, _ = W.ab_testing(W.ns_oracle())
    _tape_vs_oracle(lp_p, lp_o, init, [[0.1, 0.1], [0.12, 0.16], [0.3, 0.05]])


def test_tape_example04_event_rates(gpu):
    lp_p, init = W.event_rates(W.ns_product())
    lp_o, _ = W.event_rates(W.ns_oracle())
    prog = _tape_vs_oracle(lp_p, lp_o, init, [[2.0], [3.1], [0.4]])
    # the reference's per-observation loop folds into one vector term
    assert len(prog.model.terms) == 2


def test_tape_vector_shapes_and_params(gpu):
    """Per-element shapes, shape parameters (gammaln evaluated, no gradient),
    and a gathered per-group rate."""
    rng = np.random.default_rng(3)
    G, n = 12, 600
    g = np.sort(rng.integers(0, G, n)).astype(np.int32)
    t = rng.exponential(0.5, n).astype(np.float32)
    a_vec = rng.uniform(1.5, 4.0, G).astype(np.float32)

    def model(ns):
        def lp(p):
            return (ns.sum(ns.Gamma(ns.array(a_vec), p["b"]).log_prob(p["rate"]))
                    + ns.sum(ns.Exponential(p["rate"][g]).log_prob(ns.array(t)))
                    + ns.Gamma(p["a"], 1.0).log_prob(p["b"])
                    + ns.sum(ns.Beta(p["a"], p["b"]).log_prob(p["u"])))
        return lp

    init = {"rate": np.full(G, 2.0, np.float32), "b": np.float32(1.3),
            "a": np.float32(2.2), "u": np.full(5, 0.4, np.float32)}
    pts = []
    for s in range(3):
        r = np.random.default_rng(s)
        pts.append(np.concatenate([r.uniform(0.5, 3, G), [r.uniform(0.5, 2)],
                                   [r.uniform(1, 3)], r.uniform(0.1, 0.9, 5)]).astype(np.float32))
    _tape_vs_oracle(model(W.ns_product()), model(W.ns_oracle()), init, pts)


def test_hmc_example03_posterior(gpu):
    """Posterior of p_X is Beta(k_X + 1, n - k_X + 1)."""
    m = _m()
    n, ca, cb = W.ab_testing_data()
    lp, init = W.ab_testing(W.ns_product())
    s, rate = m.hmc(lp, init, num_samples=2000, num_warmup=1000, step_size=0.01,
                    num_leapfrog_steps=10, key=m.random.key(0), num_chains=8, progress=False)
    for name, k in (("p_A", ca), ("p_B", cb)):
        a, b = k + 1, n - k + 1
        mean = a / (a + b)
        sd = np.sqrt(a * b / ((a + b) ** 2 * (a + b + 1)))
        x = s[name]
        assert abs(float(x.mean()) - mean) < 0.2 * sd
        assert abs(float(x.std()) / sd - 1) < 0.1
    assert np.all(rate > 0.5)


def test_nuts_example04_posterior(gpu):
    """Posterior of the rate is Gamma(2 + n, 1 + sum t) (fixed step size)."""
    m = _m()
    t = W.event_rates_data()
    lp, init = W.event_rates(W.ns_product())
    s, _ = m.nuts(lp, init, num_samples=1000, num_warmup=200, step_size=0.2,
                  adapt_step_size=False, key=m.random.key(1), num_chains=8, progress=False)
    a, b = 2 + len(t), 1 + t.sum()
    x = s["rate"]
    assert abs(float(x.mean()) - a / b) < 0.1 * np.sqrt(a) / b
    assert abs(float(x.std()) / (np.sqrt(a) / b) - 1) < 0.1


def test_nuts_adaptation_freeze_matches_oracle(gpu):
    """With adaptation on, the reference's dual averaging runs away on this
    model: a proposal with rate < 0 makes log(rate) NaN, the NaN acceptance
    statistic counts as 1 (nuts.py:173), and the step size grows
    until every trajectory leaves the support, freezing the chain.  The GPU
    kernel must freeze at the same point as the oracle."""
    m = _m()
    from oracle import samplers as S

    lp, init = W.event_rates(W.ns_product())
    lp_o, _ = W.event_rates(W.ns_oracle())
    s, _ = m.nuts(lp, init, num_samples=200, num_warmup=200, step_size=0.1,
                  key=m.random.key(1), num_chains=1, progress=False)
    ref = S.nuts(lp_o, init, num_samples=200, num_warmup=200, step_size=0.1, seed=1)
    x = np.asarray(s["rate"]).ravel()
    assert len(np.unique(x)) == 1 and len(np.unique(ref.samples[:, 0])) == 1
    np.testing.assert_allclose(x[-1], ref.samples[-1, 0], rtol=1e-4)


def test_sliced_exponential_gamma_model(gpu):
    """A 20 000-observation Exponential likelihood (rate per group, Gamma
    prior on the rates and their scale): sliced vs chain-per-workgroup."""
    m = _m()
    rng = np.random.default_rng(11)
    G, n = 40, 20000
    g = np.sort(rng.integers(0, G, n)).astype(np.int32)
    t = rng.exponential(1 / rng.uniform(1, 4, G)[g]).astype(np.float32)

    def lp(p):
        ns = W.ns_product()
        return (ns.Gamma(2.0, 1.0).log_prob(p["b"])
                + ns.sum(ns.Gamma(2.0, p["b"]).log_prob(p["rate"]))
                + ns.sum(ns.Exponential(p["rate"][g]).log_prob(ns.array(t))))

    init = {"rate": np.full(G, 2.0, np.float32), "b": np.float32(1.0)}
    kw = dict(num_samples=10, num_warmup=10, step_size=0.01, num_leapfrog_steps=8,
              key=m.random.key(4), num_chains=8, progress=False, return_info=True,
              return_trace=True)
    a, _, ia = m.hmc(lp, init, num_slices=1, **kw)
    b, _, ib = m.hmc(lp, init, num_slices=4, **kw)
    np.testing.assert_array_equal(ia.trace["accepted"], ib.trace["accepted"])
    for k in a:
        np.testing.assert_allclose(b[k], a[k], rtol=1e-3, atol=1e-4)


def test_sampling_statistics(gpu):
    """tests/test_new_distributions.py:46-60,101-118,156-172."""
    m = _m()
    x = m.Beta(5, 2).sample(m.random.key(42), (10000,))
    assert np.all((x > 0) & (x < 1))
    assert np.isclose(x.mean(), 5 / 7, atol=0.05) and np.isclose(x.var(), 10 / (49 * 8), atol=0.01)
    x = m.Gamma(4, 2).sample(m.random.key(42), (10000,))
    assert np.all(x > 0)
    assert np.isclose(x.mean(), 2.0, rtol=0.1) and np.isclose(x.var(), 1.0, rtol=0.15)
    x = m.Exponential(2.0).sample(m.random.key(42), (10000,))
    assert np.all(x >= 0)
    assert np.isclose(x.mean(), 0.5, rtol=0.1) and np.isclose(x.var(), 0.25, rtol=0.15)
    assert np.isclose(float(m.Gamma(6, 3).mean()), 2.0)
    assert np.isclose(float(m.Beta(3, 7).mean()), 0.3)
    assert np.isclose(float(m.Exponential(3.0).mean()), 1 / 3)
