"""GPU tests of the drop-in API (hmc / nuts / MCMC / Distribution).

The reference's own statistical assertions (tests/test_hmc.py, test_nuts.py,
test_distributions.py) are re-run through the product.  Several chains of one
launch give several independent RNG streams; where the reference test is
seed-sensitive the majority of streams must pass.
"""
import numpy as np
import pytest

import mlx_mcmc_amd as m
import mlx_mcmc_amd.core as mx
import workloads as W

pytestmark = pytest.mark.gpu


def std_normal(p):
    return m.Normal(0, 1).log_prob(p["x"])


def frac(ok):
    return float(np.mean(ok))


def test_hmc_reference_tests(gpu):
    # test_hmc.py:13-41 over 8 streams
    s, rate = m.hmc(std_normal, {"x": 0.5}, num_samples=1000, num_warmup=500, step_size=0.1,
                    num_leapfrog_steps=10, key=m.random.key(42), num_chains=8, progress=False)
    x = s["x"]
    assert x.shape == (8, 1000)
    ok = (np.abs(x.mean(1)) < 0.15) & (np.abs(x.std(1) - 1) < 0.15) & (rate >= 0.5)
    assert frac(ok) >= 0.6
    # test_hmc.py:43-79
    s, rate = m.hmc(lambda p: m.Normal(0, 1).log_prob(p["x"]) + m.Normal(2, 0.5).log_prob(p["y"]),
                    {"x": 0.0, "y": 2.0}, num_samples=2000, num_warmup=1000, step_size=0.1,
                    num_leapfrog_steps=10, key=m.random.key(123), num_chains=8, progress=False)
    # Streams differ in outcome under the reference's x0.95/x1.05 rule: some
    # overshoot to eps ~ 1.85 > 2 sigma_y and stop accepting.  The outcome per
    # stream is the algorithm's, not noise: it equals the CPU oracle's on the
    # same stream (oracle/samplers.py hmc, seed 123, chains 0/2/5 ->
    # 0.9955 / 0.0 / 0.01).  The reference's moment bounds are asserted on the
    # pooled sample of the streams that accept.
    assert rate[0] == pytest.approx(0.9955, abs=1e-9)
    assert rate[2] == 0.0 and rate[5] == pytest.approx(0.01, abs=1e-9)
    good = rate > 0.5
    assert good.sum() >= 4
    x, y = s["x"][good].ravel(), s["y"][good].ravel()
    assert abs(x.mean()) < 0.15 and abs(x.std() - 1) < 0.15
    assert abs(y.mean() - 2) < 0.15 and abs(y.std() - 0.5) < 0.1
    # test_hmc.py:81-116
    _, ra = m.hmc(std_normal, {"x": 0.0}, num_samples=500, num_warmup=500, step_size=0.01,
                  num_leapfrog_steps=10, target_accept=0.7, key=m.random.key(42), progress=False)
    _, rb = m.hmc(std_normal, {"x": 0.0}, num_samples=500, num_warmup=500, step_size=0.01,
                  num_leapfrog_steps=10, adapt_step_size=False, key=m.random.key(42),
                  progress=False)
    assert rb > ra
    # test_hmc.py:118-146
    s, _ = m.hmc(lambda p: m.HalfNormal(2.0).log_prob(p["sigma"]), {"sigma": 1.0},
                 num_samples=1000, num_warmup=500, step_size=0.05, num_leapfrog_steps=10,
                 key=m.random.key(999), progress=False)
    assert mx.all(s["sigma"] > 0) and 0.5 < float(mx.mean(s["sigma"])) < 3.0
    # test_hmc.py:148-177
    a, _ = m.hmc(std_normal, {"x": 0.0}, num_samples=100, num_warmup=50, num_leapfrog_steps=5,
                 key=m.random.key(12345), progress=False)
    b, _ = m.hmc(std_normal, {"x": 0.0}, num_samples=100, num_warmup=50, num_leapfrog_steps=5,
                 key=m.random.key(12345), progress=False)
    assert mx.allclose(a["x"], b["x"]) and np.array_equal(a["x"], b["x"])


def test_hmc_posterior_inference(gpu):
    """test_hmc.py:179-220 over 8 streams (seed-sensitive, majority)."""
    np.random.seed(42)
    data = np.random.normal(3.0, 1.5, 50)

    def lp(p):
        out = m.Normal(0, 10).log_prob(p["mu"]) + m.HalfNormal(5).log_prob(p["sigma"])
        return out + mx.sum(m.Normal(p["mu"], p["sigma"]).log_prob(mx.array(data)))

    s, rate = m.hmc(lp, {"mu": 0.0, "sigma": 1.0}, num_samples=2000, num_warmup=1000,
                    step_size=0.1, num_leapfrog_steps=10, key=m.random.key(42), num_chains=8,
                    progress=False)
    ok = ((np.abs(s["mu"].mean(1) - 3.0) < 0.4) & (np.abs(s["sigma"].mean(1) - 1.5) < 0.4)
          & (rate >= 0.5))
    assert frac(ok) >= 0.6


def test_nuts_reference_tests(gpu):
    # test_nuts.py:13-32
    s, rate = m.nuts(lambda p: m.Normal(5.0, 2.0).log_prob(p["mu"]), {"mu": 0.0},
                     num_samples=1000, num_warmup=500, step_size=0.5, key=m.random.key(42),
                     num_chains=8, progress=False)
    ok = ((s["mu"].mean(1) > 4.5) & (s["mu"].mean(1) < 5.5) & (s["mu"].std(1) > 1.5)
          & (s["mu"].std(1) < 2.5) & (rate > 0.5))
    assert frac(ok) >= 0.75
    # test_nuts.py:34-54
    s, _ = m.nuts(lambda p: m.Normal(0, 1).log_prob(p["mu1"]) + m.Normal(5, 2).log_prob(p["mu2"]),
                  {"mu1": 0.0, "mu2": 0.0}, num_samples=1000, num_warmup=500, step_size=0.3,
                  key=m.random.key(123), num_chains=8, progress=False)
    ok = (np.abs(s["mu1"].mean(1)) < 0.5) & (np.abs(s["mu2"].mean(1) - 5) < 0.5)
    assert frac(ok) >= 0.75
    # test_nuts.py:88-108 (positivity) and :110-136 (reproducibility)
    s, _ = m.nuts(lambda p: m.HalfNormal(5.0).log_prob(p["sigma"])
                  + m.Normal(0, p["sigma"]).log_prob(mx.array(0.5)),
                  {"sigma": 1.0}, num_samples=1000, num_warmup=500, step_size=0.1,
                  key=m.random.key(456), progress=False)
    assert mx.all(s["sigma"] > 0)
    a, _ = m.nuts(std_normal, {"x": 0.0}, num_samples=100, num_warmup=100,
                  key=m.random.key(42), progress=False)
    b, _ = m.nuts(std_normal, {"x": 0.0}, num_samples=100, num_warmup=100,
                  key=m.random.key(42), progress=False)
    np.testing.assert_array_almost_equal(a["x"], b["x"], decimal=5)
    # test_nuts.py:157-186
    s, _ = m.nuts(std_normal, {"x": 0.0}, num_samples=100, num_warmup=100, max_tree_depth=3,
                  step_size=0.5, key=m.random.key(42), progress=False)
    assert len(s["x"]) == 100


def test_mcmc_facade(gpu):
    """test_nuts.py:138-155 and :188-227 (MCMC.run, per-observation list model)."""
    mc = m.MCMC(lambda p: m.Normal(3.0, 1.0).log_prob(p["mu"]))
    s = mc.run(initial_params={"mu": 0.0}, num_samples=500, num_warmup=500, method="nuts",
               step_size=0.5, verbose=False, progress=False)
    assert 2.5 < np.mean(s["mu"]) < 3.5
    summ = mc.summary()
    assert set(summ["mu"]) == {"mean", "std", "median", "2.5%", "97.5%"}
    np.random.seed(42)
    y = np.random.normal(5.0, 2.0, 50)

    def lp(p):
        prior = m.Normal(0, 10).log_prob(p["mu"]) + m.HalfNormal(5).log_prob(p["sigma"])
        return prior + mx.sum(mx.array([m.Normal(p["mu"], p["sigma"]).log_prob(mx.array(v))
                                        for v in y]))
    s = m.MCMC(lp).run(initial_params={"mu": 0.0, "sigma": 1.0}, num_samples=1000,
                       num_warmup=500, method="hmc", step_size=0.1, verbose=False,
                       progress=False)
    assert abs(np.mean(s["mu"]) - 5.0) < 1.0 and abs(np.mean(s["sigma"]) - 2.0) < 1.0


def test_chain_offset_invariance_and_determinism(gpu):
    """The multi-GPU contract: draws are keyed by the global chain id, so
    splitting chains over launches (GPUs) gives bit-identical samples."""
    lp, init = W.simple_normal(W.ns_product())
    full, _ = m.hmc(lp, init, num_samples=50, num_warmup=50, key=m.random.key(5), num_chains=8,
                    progress=False)
    a, _ = m.hmc(lp, init, num_samples=50, num_warmup=50, key=m.random.key(5), num_chains=4,
                 chain_offset=0, progress=False)
    b, _ = m.hmc(lp, init, num_samples=50, num_warmup=50, key=m.random.key(5), num_chains=4,
                 chain_offset=4, progress=False)
    for k in full:
        np.testing.assert_array_equal(full[k], np.concatenate([a[k], b[k]]))
    again, _ = m.hmc(lp, init, num_samples=50, num_warmup=50, key=m.random.key(5), num_chains=8,
                     progress=False)
    for k in full:
        np.testing.assert_array_equal(full[k], again[k])


def test_hierarchical_chain_offset_invariance(gpu):
    """Same contract on the segmented (gathered) path, small shape."""
    G, N = W.SHAPES["small"]
    lp, init = W.hierarchical(W.ns_product(), G, N)
    full, _ = m.hmc(lp, init, num_samples=20, num_warmup=20, step_size=0.01,
                    num_leapfrog_steps=20, key=m.random.key(1), num_chains=4, progress=False)
    part, _ = m.hmc(lp, init, num_samples=20, num_warmup=20, step_size=0.01,
                    num_leapfrog_steps=20, key=m.random.key(1), num_chains=2, chain_offset=2,
                    progress=False)
    np.testing.assert_array_equal(full["theta"][2:], part["theta"])


def test_iso_normal_config2_moments(gpu):
    """Config 2: 100-dim standard normal, 64 chains: pooled mean ~ 0, var ~ 1."""
    lp, init = W.iso_normal(W.ns_product())
    s, rate = m.hmc(lp, init, num_samples=1000, num_warmup=1000, step_size=0.1,
                    num_leapfrog_steps=10, key=m.random.key(0), num_chains=64, progress=False)
    x = s["x"]  # [64, 1000, 100]
    assert x.shape == (64, 1000, 100)
    assert abs(x.mean()) < 0.05
    assert abs(x.var() - 1.0) < 0.05


def test_illcond_config5_nuts_moments(gpu):
    """Config 5: kappa = 1000 diagonal Gaussian, NUTS (slice active): per-
    coordinate variance within 15 % of sigma_i^2 pooled over chains."""
    lp, init = W.illcond_normal(W.ns_product())
    s, rate, info = m.nuts(lp, init, num_samples=500, num_warmup=500, step_size=0.1,
                           key=m.random.key(0), num_chains=64, progress=False,
                           return_info=True)
    x = s["x"]
    var = x.reshape(-1, 100).var(axis=0)
    sig2 = W.illcond_scales(100).astype(np.float64) ** 2
    assert np.all(np.abs(var / sig2 - 1) < 0.15)
    assert np.all(info.mean_tree_depth >= 1)


def test_vector_params_and_errors(gpu):
    s, _ = m.hmc(lambda p: mx.sum(m.Normal(0, 1).log_prob(p["v"])),
                 {"v": np.zeros(3, np.float32)}, num_samples=10, num_warmup=10, progress=False)
    assert s["v"].shape == (10, 3)
    with pytest.raises(ZeroDivisionError):
        m.hmc(std_normal, {"x": 0.0}, num_samples=10, num_warmup=0, progress=False)
    from mlx_mcmc_amd._trace import TraceError

    with pytest.raises(TraceError):   # a Python branch on a parameter value
        m.nuts(lambda p: m.Normal(0, 1).log_prob(p["x"]) if p["x"] > 0 else 0.0, {"x": 1.0},
               num_samples=5, num_warmup=5, progress=False)


def test_distribution_sampling(gpu):
    """tests/test_distributions.py:34-50, 81-102 on the GPU RNG stream."""
    z = m.Normal(5.0, 2.0).sample(m.random.key(42), shape=(10000,))
    assert z.shape == (10000,)
    assert abs(z.mean() - 5.0) < 0.1 and abs(z.std() - 2.0) < 0.1
    h = m.HalfNormal(2.0).sample(m.random.key(42), shape=(10000,))
    assert np.all(h >= 0)
    assert np.isclose(h.mean(), 2.0 * np.sqrt(2 / np.pi), rtol=0.1)
    assert np.isclose(h.std(), 2.0 * np.sqrt(1 - 2 / np.pi), rtol=0.1)
    assert m.HalfNormal(5.0).sample(m.random.key(0), shape=(1000,)).min() >= 0


def test_example02_realisations_match_oracle(gpu):
    """Example 02's HMC run (examples/02_hmc_comparison.py:86-100: MCMC.run
    method='hmc', step_size 0.1, L = 10, W = 1000, S = 5000, seed 42) on 64
    chains through the product API against the oracle's 64 realisations
    (tests/golden/example02_hmc.json): a chain whose 6000 accept decisions all
    agree ends with a bit-identical step size, so at least 56 of 64 must; those
    carry the oracle's statistics (acceptance exactly, ESS and |mean - truth|
    to float rounding), and the GPU's realisations bracket the reference's
    published numbers by the same rule as the oracle's
    (test_oracle_pins.example02_bracket)."""
    import json
    import os

    from test_oracle_pins import example02_bracket

    with open(os.path.join(os.path.dirname(__file__), "golden", "example02_hmc.json")) as f:
        fx = json.load(f)
    cfg = fx["config"]
    lp, init = W.simple_normal(W.ns_product())
    s, rate, info = m.hmc(lp, init, num_samples=cfg["num_samples"],
                          num_warmup=cfg["num_warmup"], step_size=cfg["step_size"],
                          num_leapfrog_steps=cfg["num_leapfrog_steps"],
                          adapt_step_size=cfg["adapt_step_size"],
                          target_accept=cfg["target_accept"], key=m.random.key(cfg["seed"]),
                          num_chains=64, progress=False, return_info=True)
    from oracle.diag import compute_ess_02

    mu = np.asarray(s["mu"], np.float64)
    sg = np.asarray(s["sigma"], np.float64)
    mine = []
    same = exact = 0
    for c, o in enumerate(fx["chains"]):
        r = {"accept_rate": float(info.accept_rate[c]), "step_size": float(info.step_size[c]),
             "ess_mu": compute_ess_02(mu[c]), "ess_sigma": compute_ess_02(sg[c]),
             "err_mu": abs(mu[c].mean() - 5.0), "err_sigma": abs(sg[c].mean() - 2.0)}
        mine.append(r)
        if r["step_size"] == o["step_size"]:
            same += 1
            assert abs(r["accept_rate"] - o["accept_rate"]) <= 1e-3
            exact += (r["accept_rate"] == o["accept_rate"] and
                      abs(r["err_mu"] - o["err_mu"]) <= 1e-4 and
                      abs(r["err_sigma"] - o["err_sigma"]) <= 1e-4 and
                      r["ess_mu"] == pytest.approx(o["ess_mu"], rel=1e-2) and
                      r["ess_sigma"] == pytest.approx(o["ess_sigma"], rel=1e-2))
    print(f"example 02: {same} of 64 final step sizes identical, {exact} realisations identical")
    assert same >= 56, f"only {same} of 64 realisations kept the oracle's decisions"
    assert exact >= 48
    example02_bracket(mine, fx["published"])
