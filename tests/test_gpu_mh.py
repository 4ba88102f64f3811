"""Metropolis-Hastings: k_mh against the CPU oracle's restatement
of mlx_mcmc/kernels/metropolis.py:6-101, and the reference's MCMC.run
metropolis branch (mcmc.py:135-189) through the product API.

The reference has no MH test of its own; its examples (01, 03, 04) run MH
through MCMC.run, and their analytic posteriors are the statistical targets.
Parity bar: same draws (Philox), so accept decisions and samples equal the
oracle's while the two f32 log densities agree; the tape's f32 summation order
differs from autograd's by ~1 ulp of |log p|, so decisions are asserted
identical over the first 150 iterations (a flip needs log U within that ulp of
the ratio) and the samples to rtol 1e-5 while the decisions agree.
"""
import numpy as np
import pytest

import mlx_mcmc_amd as m
import mlx_mcmc_amd.core as mx
import workloads as W
from oracle import samplers as S

pytestmark = pytest.mark.gpu


def test_mh_trace_parity_simple_normal(gpu):
    lp, init = W.simple_normal(W.ns_product())
    olp, oinit = W.simple_normal(W.ns_oracle())
    n = 150
    s, rate, info = m.metropolis_hastings(lp, init, num_samples=n, proposal_scale=0.3,
                                          random_seed=11, return_info=True, return_trace=True)
    ref = S.metropolis_hastings(olp, oinit, num_samples=n, proposal_scale=0.3, random_seed=11)
    acc = info.trace["accepted"][0].astype(bool)
    assert list(acc) == ref.trace["accepted"]
    np.testing.assert_allclose(s["mu"], ref.samples[:, 0], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(s["sigma"], ref.samples[:, 1], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(info.trace["accept_stat"][0], ref.trace["ratio"], rtol=1e-4,
                               atol=2e-4)
    assert rate == pytest.approx(ref.accept_rate, abs=1e-12)
    assert s["mu"].shape == (n,) and s["sigma"].dtype == np.float32


def test_mh_trace_parity_hierarchical_medium(gpu):
    """A gathered, segmented tape (D = 100, N = 10k) in value-only mode."""
    G, N = W.SHAPES["medium"]
    lp, init = W.hierarchical(W.ns_product(), G, N)
    olp, oinit = W.hierarchical(W.ns_oracle(), G, N)
    n = 60
    s, rate, info = m.metropolis_hastings(lp, init, num_samples=n, proposal_scale=0.01,
                                          random_seed=3, return_info=True, return_trace=True)
    ref = S.metropolis_hastings(olp, oinit, num_samples=n, proposal_scale=0.01, random_seed=3)
    assert list(info.trace["accepted"][0].astype(bool)) == ref.trace["accepted"]
    assert 0 < sum(ref.trace["accepted"]) < n
    np.testing.assert_allclose(s["theta"], ref.samples[:, 3:], rtol=1e-5, atol=1e-5)
    # the tape's log density at every stored point (value-only evaluation)
    np.testing.assert_allclose(info.trace["energy"][0], ref.trace["logp"], rtol=2e-6)


def test_mh_posterior_and_chains(gpu):
    """Normal(0, 1) target: 64 chains; moments; chain_offset / launch-split invariance."""
    def lp(p):
        return mx.sum(m.Normal(0, 1).log_prob(p["x"]))

    init = {"x": np.zeros(4, np.float32)}
    s, rate = m.metropolis_hastings(lp, init, num_samples=4000, proposal_scale=1.5,
                                    random_seed=5, num_chains=64)
    x = s["x"][:, 500:]
    assert x.shape == (64, 3500, 4)
    assert abs(float(x.mean())) < 0.03 and abs(float(x.std()) - 1) < 0.03
    assert np.all((rate > 0.15) & (rate < 0.3))  # 4-D random walk at scale 1.5: ~0.21
    # chains 16..31 alone, as a shard with chain_offset 16
    s2, r2 = m.metropolis_hastings(lp, init, num_samples=4000, proposal_scale=1.5,
                                   random_seed=5, num_chains=16, chain_offset=16)
    assert np.array_equal(s2["x"], s["x"][16:32]) and np.array_equal(r2, rate[16:32])
    # progress printing splits the run into 500-iteration launches: same draws
    s3, r3 = m.metropolis_hastings(lp, init, num_samples=4000, proposal_scale=1.5,
                                   random_seed=5, num_chains=16, chain_offset=16, verbose=True)
    assert np.array_equal(s3["x"], s2["x"]) and np.array_equal(r3, r2)


def test_mh_support_and_errors(gpu):
    # hard support (halfnormal.py:63): proposals below 0 give -inf and are rejected
    s, rate = m.metropolis_hastings(lambda p: m.HalfNormal(1.0).log_prob(p["s"]), {"s": 0.05},
                                    num_samples=2000, proposal_scale=0.5, random_seed=1)
    assert np.all(s["s"] > 0) and 0.1 < rate < 0.9
    assert abs(float(np.mean(s["s"][200:])) - np.sqrt(2 / np.pi)) < 0.12
    with pytest.raises(ZeroDivisionError):  # metropolis.py:99
        m.metropolis_hastings(lambda p: m.Normal(0, 1).log_prob(p["x"]), {"x": 0.0},
                              num_samples=0)


def test_mcmc_run_metropolis(gpu, capsys):
    """examples/01_simple_normal.py:52-73 through MCMC.run (the reference default method)."""
    lp, init = W.simple_normal(W.ns_product())
    mc = m.MCMC(lp)
    out = mc.run(init, num_samples=5000, num_warmup=1000, proposal_scale=0.3, random_seed=42)
    text = capsys.readouterr().out
    assert "MLX-MCMC: METROPOLIS Sampling" in text and "Warmup phase: 1000 samples" in text
    assert "Running 5000 Metropolis-Hastings iterations..." in text
    assert "Iteration 5000/5000 (accept rate:" in text
    assert set(out) == {"mu", "sigma"} and out["mu"].shape == (5000,)
    data = W.simple_normal_data()
    assert abs(out["mu"].mean() - data.mean()) < 0.15
    assert abs(out["sigma"].mean() - data.std()) < 0.15
    assert 0.1 < mc.acceptance_rate < 0.9
    summ = mc.summary()
    assert abs(summ["mu"]["mean"] - float(out["mu"].mean())) < 1e-4
    # warmup then sampling with random_seed + 1 from the last warmup draw (mcmc.py:162,175)
    w, _ = m.metropolis_hastings(lp, init, num_samples=1000, proposal_scale=0.3, random_seed=42)
    s, _ = m.metropolis_hastings(lp, {k: v[-1] for k, v in w.items()}, num_samples=5000,
                                 proposal_scale=0.3, random_seed=43)
    assert np.array_equal(s["mu"], out["mu"])
    with pytest.raises(ValueError):
        mc.run(init, method="gibbs", verbose=False)
