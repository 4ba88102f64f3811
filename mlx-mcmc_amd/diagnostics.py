"""Sample diagnostics used by the bench: the reference's ESS definition.

``compute_ess`` restates examples/06_nuts_comparison.py:22-41: ESS =
n / (1 + 2 sum rho_k) over lags 1 .. min(n//2, 100) - 1, stopping at (and
including) the first autocorrelation below 0.05; a zero-variance series has
ESS = n.  ``ess_batch`` evaluates the same rule for many series at once
(post-processing of device samples; not on the sampling hot path).
"""
from __future__ import annotations

import numpy as np


def compute_ess(samples) -> float:
    x = np.asarray(samples, dtype=np.float64)
    return float(ess_batch(x[:, None])[0])


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
