"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by mlx_mcmc_amd/).

CPU restatements the device diagnostics (csrc/diag.h) are checked against:

  compute_ess   examples/06_nuts_comparison.py:22-41, verbatim semantics
                (oracle.samplers.compute_ess); ``ess_batch`` is the same rule
                vectorised over columns.
  compute_ess_02  the variant of examples/02_hmc_comparison.py:111-128 that
                produced the published example-02 ESS (PROGRESS.md:78-80): it
                stops at the first rho < 0.05 only from lag 2 on, and has no
                constant-series guard.
  split_rhat    Gelman et al., Bayesian Data Analysis 3rd ed., eq. 11.4 on
                split chains (first and last floor(S/2) draws).  The
                reference has no R-hat (roadmap only, README.md:214), so this
                is parity unpinned against the reference; it is pinned by
                hand-computed known answers in tests/test_oracle_pins.py.
  summary       mlx_mcmc/inference/mcmc.py:191-227 verbatim: np.mean / np.std
                / np.median / np.percentile over every value of a parameter.
"""
from __future__ import annotations

import numpy as np

from .samplers import compute_ess  # noqa: F401  (re-exported)


def compute_ess_02(samples) -> float:
    """examples/02_hmc_comparison.py:111-128 (restated)."""
    x = np.asarray(samples, np.float64)
    n = len(x)
    mean = np.mean(x)
    c0 = np.mean((x - mean) ** 2)
    acf = []
    for lag in range(1, min(n // 2, 100)):
        acf.append(np.mean((x[:-lag] - mean) * (x[lag:] - mean)) / c0)
        if len(acf) > 1 and acf[-1] < 0.05:
            break
    return n / (1 + 2 * np.sum(acf))


def ess_batch(x) -> np.ndarray:
    """x: [n, m] — m independent series of length n -> ESS per series [m]."""
    x = np.asarray(x, dtype=np.float64)
    n, m = x.shape
    mean = x.mean(axis=0)
    var = x.var(axis=0)
    xc = x - mean
    acf_sum = np.zeros(m)
    active = var != 0
    safe_var = np.where(active, var, 1.0)
    for lag in range(1, min(n // 2, 100)):
        if not active.any():
            break
        c = np.mean(xc[:-lag] * xc[lag:], axis=0) / safe_var
        acf_sum = np.where(active, acf_sum + c, acf_sum)
        active = active & ~(c < 0.05)
    ess = n / (1.0 + 2.0 * acf_sum)
    return np.where(var == 0, float(n), ess)


def mcse_batch(x, n_batches: int = 20):
    """x: [C, S, D] draws -> (MCSE of the pooled mean, MCSE of the pooled
    variance) per parameter by non-overlapping batch means (n_batches per
    chain): robust to the antithetic HMC draws for which the reference's
    autocorrelation rule (compute_ess) gives ESS <= 0.  Test infrastructure
    for SURVEY 8(d)'s parity rule."""
    x = np.asarray(x, dtype=np.float64)
    C, S, D = x.shape
    b = S // n_batches
    xb = x[:, :b * n_batches].reshape(C, n_batches, b, D)
    mean = x.reshape(-1, D).mean(0)
    m1 = xb.mean(2).reshape(-1, D)                       # batch means
    m2 = ((xb - mean) ** 2).mean(2).reshape(-1, D)       # batch second moments
    nb = C * n_batches
    return m1.std(0, ddof=1) / np.sqrt(nb), m2.std(0, ddof=1) / np.sqrt(nb)


def split_rhat(x) -> float:
    """x: [C, S] draws of one scalar -> split R-hat (BDA3 11.4)."""
    x = np.asarray(x, dtype=np.float64)
    C, S = x.shape
    h = S // 2
    halves = np.concatenate([x[:, :h], x[:, S - h:]], axis=0)   # [2C, h]
    m, n = halves.shape
    means = halves.mean(axis=1)
    W = halves.var(axis=1, ddof=1).mean()
    B = n * means.var(ddof=1)
    var_plus = (n - 1) / n * W + B / n
    return float(np.sqrt(var_plus / W))


def summary(samples: dict, credible_interval: float = 0.95) -> dict:
    """mcmc.py:191-227."""
    alpha = 1 - credible_interval
    lower_pct = 100 * alpha / 2
    upper_pct = 100 * (1 - alpha / 2)
    out = {}
    for name, s in samples.items():
        out[name] = {
            'mean': float(np.mean(s)),
            'std': float(np.std(s)),
            'median': float(np.median(s)),
            f'{lower_pct:.1f}%': float(np.percentile(s, lower_pct)),
            f'{upper_pct:.1f}%': float(np.percentile(s, upper_pct)),
        }
    return out
