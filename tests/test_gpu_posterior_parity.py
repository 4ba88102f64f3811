"""Posterior parity against the reference restatement (SURVEY 8(d) "Parity").

Per parameter, |mean_gpu - mean_ref| <= max(1 % of |mean_ref|, 3 MCSE) and
the same for the variance, with the MCSE of both runs combined (batch means,
20 batches per chain: oracle/diag.py mcse_batch — the reference's
autocorrelation ESS rule breaks down on antithetic HMC draws).  The reference side is the CPU oracle's
HMC (hmc.py:7-206) on the small hierarchical shape at a fixed step size and
its Metropolis-Hastings (metropolis.py:6-101) on example 01's model (8 and 4
chains), held as moments in tests/golden/posterior_small.json
(scripts/gen_posterior.py says why the step size is fixed).  The GPU runs the
same sampler settings on 64 chains through the product API (HMC on the
lane-resident kernel, MH on k_mh).
"""
import json
import os

import numpy as np
import pytest

import workloads as W

pytestmark = pytest.mark.gpu

FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "posterior_small.json")


def _ref(kind):
    with open(FIXTURE) as f:
        fx = json.load(f)
    return fx[kind], {k: np.asarray(v) for k, v in fx[kind + "_moments"].items()}


def _flat(samples, init):
    """Product samples {name: [C, S, *shape]} -> [C, S, D] in layout order."""
    C, S = np.asarray(samples[next(iter(init))]).shape[:2]
    return np.concatenate([np.asarray(samples[k], np.float64).reshape(C, S, -1) for k in init],
                          axis=2)


def _moments(x):
    from oracle.diag import mcse_batch

    pooled = x.reshape(-1, x.shape[-1])
    mcse_m, mcse_v = mcse_batch(x)
    return {"mean": pooled.mean(0), "var": pooled.var(0), "mcse_mean": mcse_m,
            "mcse_var": mcse_v}


def _check(g, r):
    tol_m = np.maximum(0.01 * np.abs(r["mean"]),
                       3.0 * np.hypot(g["mcse_mean"], r["mcse_mean"]))
    tol_v = np.maximum(0.01 * r["var"], 3.0 * np.hypot(g["mcse_var"], r["mcse_var"]))
    dm = np.abs(g["mean"] - r["mean"])
    dv = np.abs(g["var"] - r["var"])
    assert np.all(dm <= tol_m), f"means: |diff| {dm} > tol {tol_m}"
    assert np.all(dv <= tol_v), f"variances: |diff| {dv} > tol {tol_v}"


def test_hmc_posterior_matches_oracle_small_hierarchical(gpu):
    import mlx_mcmc_amd as m

    cfg, ref = _ref("hmc")
    lp, init = W.hierarchical(W.ns_product(), *W.SHAPES["small"])
    s, rate = m.hmc(lp, init, num_samples=cfg["num_samples"], num_warmup=cfg["num_warmup"],
                    step_size=cfg["step_size"], num_leapfrog_steps=cfg["num_leapfrog_steps"],
                    adapt_step_size=cfg["adapt_step_size"], key=m.random.key(0), num_chains=64,
                    progress=False)
    _check(_moments(_flat(s, init)), ref)


def test_mh_posterior_matches_oracle_example01(gpu):
    import mlx_mcmc_amd as m

    cfg, ref = _ref("mh")
    lp, init = W.simple_normal(W.ns_product())
    s, rate = m.metropolis_hastings(lp, init, num_samples=cfg["num_samples"],
                                    proposal_scale=cfg["proposal_scale"], random_seed=0,
                                    num_chains=64)
    _check(_moments(_flat(s, init)), ref)
