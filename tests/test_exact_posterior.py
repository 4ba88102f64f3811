"""The float64 known answers (oracle/exact.py, tests/golden/posterior_exact.json)
pinned before any GPU test trusts them (CPU only):

  * the closed-form conditioning agrees with dense Gaussian conditioning of
    the joint (mu, theta) given (tau, sigma) (precision matrix inverted);
  * the marginal of (tau, sigma) agrees with the joint log density of the
    model (workloads.hierarchical through the oracle's distributions,
    restating normal.py:28-31 / halfnormal.py:55-63) integrated over
    (mu, theta) by Laplace's method, which is exact for a Gaussian;
  * the committed fixture is what the code computes;
  * the oracle's HMC (restating hmc.py:7-206) agrees with it on the small
    and large shapes within its own Monte-Carlo error
    (tests/golden/posterior_small.json, posterior_large.json): the
    z-scores |mean_oracle - mean_exact| / MCSE are standard-normal-like.
"""
import json
import os

import numpy as np
import pytest

import workloads as W
from oracle import exact as E

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _fixture():
    with open(os.path.join(GOLD, "posterior_exact.json")) as f:
        return json.load(f)


def test_conditional_moments_match_dense_gaussian():
    G, N = W.SHAPES["small"]
    y, g = W.hierarchical_data(G, N)
    n, ybar, ss = E.group_stats(y, g, G)
    M = E._Marginal(n, ybar, ss)
    for tau, sigma in [(1.3, 0.97), (0.4, 1.2)]:
        # precision of (mu, theta) given (tau, sigma, y)
        Q = np.zeros((G + 1, G + 1))
        h = np.zeros(G + 1)
        Q[0, 0] = 1 / E.PRIOR_MU_SD ** 2 + G / tau ** 2
        Q[0, 1:] = Q[1:, 0] = -1 / tau ** 2
        Q[1:, 1:] = np.diag(1 / tau ** 2 + n / sigma ** 2)
        h[1:] = n * ybar / sigma ** 2
        cov = np.linalg.inv(Q)
        mean = cov @ h
        m, vm, et, vt = M.conditional(tau, sigma)
        np.testing.assert_allclose(m, mean[0], rtol=1e-12)
        np.testing.assert_allclose(vm, cov[0, 0], rtol=1e-12)
        np.testing.assert_allclose(et, mean[1:], rtol=1e-12)
        np.testing.assert_allclose(vt, np.diag(cov)[1:], rtol=1e-12)


def test_marginal_matches_joint_density():
    """log p(tau, sigma | y) differences equal those of the joint density
    integrated over (mu, theta) — Gaussian in (mu, theta), so Laplace at the
    conditional mode is exact: log p(tau, sigma, m*) + 0.5 log det(2 pi Q^-1)."""
    import torch

    G, N = W.SHAPES["small"]
    y, g = W.hierarchical_data(G, N)
    M = E._Marginal(*E.group_stats(y, g, G))
    lp_fn, _ = W.hierarchical(W.ns_oracle(), G, N)

    def joint(tau, sigma):
        m, _, et, _ = M.conditional(tau, sigma)
        n = M.n
        Q = np.zeros((G + 1, G + 1))
        Q[0, 0] = 1 / E.PRIOR_MU_SD ** 2 + G / tau ** 2
        Q[0, 1:] = Q[1:, 0] = -1 / tau ** 2
        Q[1:, 1:] = np.diag(1 / tau ** 2 + n / sigma ** 2)
        params = {"mu": torch.tensor(m, dtype=torch.float64),
                  "tau": torch.tensor(tau, dtype=torch.float64),
                  "sigma": torch.tensor(sigma, dtype=torch.float64),
                  "theta": torch.tensor(et, dtype=torch.float64)}
        with torch.no_grad():
            lp = float(lp_fn(params))
        return lp - 0.5 * np.linalg.slogdet(Q)[1]

    pts = [(1.3, 0.97), (0.9, 1.02), (2.1, 0.95)]
    a = M.logp(np.array([p[0] for p in pts]), np.array([p[1] for p in pts]))
    b = np.array([joint(*p) for p in pts])
    np.testing.assert_allclose(a - a[0], b - b[0], atol=1e-6)


def test_fixture_is_reproduced():
    fx = _fixture()["shapes"]
    for shape in ("small", "medium"):
        G, N = W.SHAPES[shape]
        y, g = W.hierarchical_data(G, N)
        r = E.hierarchical_moments(y, g, G, n_grid=81)
        np.testing.assert_allclose(r["mean"], fx[shape]["mean"], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(r["var"], fx[shape]["var"], rtol=1e-9)
        np.testing.assert_allclose(r["log_tau_sigma_mean"], fx[shape]["log_tau_sigma_mean"],
                                   rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(r["log_tau_sigma_var"], fx[shape]["log_tau_sigma_var"],
                                   rtol=1e-9)
        assert fx[shape]["quadrature_rel_error_mean"] < 1e-9
        assert fx[shape]["quadrature_rel_error_var"] < 1e-9
        assert fx[shape]["edge_weight"] < 1e-12
    assert fx["large"]["quadrature_rel_error_var"] < 1e-9


def _zscores(name, shape):
    with open(os.path.join(GOLD, name)) as f:
        m = json.load(f)["hmc_moments"]
    ex = _fixture()["shapes"][shape]
    zm = (np.asarray(m["mean"]) - ex["mean"]) / np.asarray(m["mcse_mean"])
    zv = (np.asarray(m["var"]) - ex["var"]) / np.asarray(m["mcse_var"])
    return zm, zv


@pytest.mark.parametrize("name,shape", [("posterior_small.json", "small"),
                                        ("posterior_large.json", "large")])
def test_oracle_hmc_agrees_with_exact(name, shape):
    from scipy.stats import norm

    zm, zv = _zscores(name, shape)
    n = zm.size
    zmax = max(3.0, float(norm.ppf(1.0 - 0.01 / (2.0 * 2 * n))))
    assert np.abs(zm).max() < zmax and np.abs(zv).max() < zmax, (np.abs(zm).max(),
                                                                  np.abs(zv).max())
    if n > 100:     # the spread is that of independent standard normals
        assert 0.8 < np.sqrt(np.mean(zm ** 2)) < 1.3
        assert 0.8 < np.sqrt(np.mean(zv ** 2)) < 1.3


def test_reparam_density_is_the_change_of_variables():
    """workloads.hierarchical_reparam (the exp-transformed scales + their
    log-Jacobian identity terms) is hierarchical's density in (mu, log tau,
    log sigma, theta): log p_reparam(u, v) = log p(e^u, e^v) + u + v, so the
    fixture's (log tau, log sigma) moments are its posterior's."""
    import torch

    G, N = W.SHAPES["small"]
    a, _ = W.hierarchical(W.ns_oracle(), G, N)
    b, _ = W.hierarchical_reparam(W.ns_oracle(), G, N)
    rng = np.random.default_rng(3)
    for _ in range(3):
        mu, u, v = rng.normal(1.0, 0.3), rng.normal(0.3, 0.3), rng.normal(0.0, 0.05)
        th = torch.tensor(rng.normal(1.0, 1.0, G), dtype=torch.float64)
        pa = {"mu": torch.tensor(mu, dtype=torch.float64),
              "tau": torch.tensor(np.exp(u), dtype=torch.float64),
              "sigma": torch.tensor(np.exp(v), dtype=torch.float64), "theta": th}
        pb = {"mu": pa["mu"], "log_tau": torch.tensor(u, dtype=torch.float64),
              "log_sigma": torch.tensor(v, dtype=torch.float64), "theta": th}
        with torch.no_grad():
            np.testing.assert_allclose(float(b(pb)), float(a(pa)) + u + v, rtol=1e-12)
